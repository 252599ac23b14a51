"""Newton-count histogram of a split QP launch (the metric config and BASELINE C5): per count, how
many problems stopped there, how many of those were polished / had a polish rejected, and how many
ran in the tail launch.  Steady state (after warm-up launches).  Usage: python scripts/diag_newton_hist.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch

for cfg, N, B in (('trot', 100, 1024), ('mixed', 150, 1024)):
    pb = make_batch('trot', N, B, seed_offset=0, mixed=('pace', 'trot') if cfg == 'mixed' else None)
    s = Solver(pb.robot, N, B, 'fp64')
    s.upload(pb)
    for _ in range(4):
        s.scp_iterate(fixed_iters=True)
    s.synchronize()
    z, _, st, it = s.qp_solution(with_y=False)
    tail, pol = s.qp_exit()
    print('%s N=%d B=%d kernel %s status %s' % (cfg, N, B, s.qp_kernel(), dict(zip(*np.unique(st, return_counts=True)))))
    for k in np.unique(it):
        m = it == k
        print('  newton %2d: %4d problems  polished %4d  rejected %3d  tail %4d' %
              (k, m.sum(), (pol[m] > 0).sum(), (pol[m] < 0).sum(), (tail[m] > 0).sum()))
    s.close()
