"""One-wave vs two-wave QP workgroups: Newton iteration differences and solution differences."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch


def run(pb, waves):
    s = Solver(pb.robot, pb.N, pb.B, 'fp64')
    s.set_qp_settings(waves_per_problem=waves)
    s.upload(pb)
    s.scp_iterate(fixed_iters=True)
    z, _, st, it = s.qp_solution(with_y=False)
    s.close()
    return z, st, it


for cfg, N in [('trot', 200), ('talos', 100), ('talos', 127), ('talos', 200)]:
    pb = make_batch(cfg, N, 16, seed_offset=31)
    z1, s1, i1 = run(pb, 1)
    z1b, s1b, i1b = run(pb, 1)
    z2, s2, i2 = run(pb, 2)
    err = (np.abs(z1 - z2).max(axis=1) / np.abs(z1).max(axis=1)).max()
    rep = (np.abs(z1 - z1b).max(axis=1) / np.abs(z1).max(axis=1)).max()
    print(cfg, N, 'status', np.unique(s1), np.unique(s2), 'd_it', np.abs(i1 - i2).max(), 'it1', i1.mean(), 'it2', i2.mean(),
          'z err %.2e' % err, 'repeat err %.2e' % rep, flush=True)
