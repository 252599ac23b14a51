"""Diagnostics: one golden fixture's device solve_scp with the per-iteration QP statuses."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd'), os.path.join(ROOT, 'tests')]
import numpy as np
from cmpc._lib import Solver
from helpers import golden_batch, golden_fp32
tag = sys.argv[1]
g = dict(np.load(os.path.join(ROOT, 'tests/golden/golden_%s.npz' % tag)))
pb = golden_batch(tag, g)
for prec in ('fp32', 'fp64'):
    s = Solver(pb.robot, pb.N, 1, prec)
    s.upload(pb)
    for it in range(3):
        s.scp_iterate(fixed_iters=False)
        z, _, st, its = s.qp_solution(with_y=False)
        merit, nref = s.qp_info()
        log = s.iteration_log()
        print(prec, it, 'qp status', st, 'iters', its, 'merit', merit, 'nref', nref, {k: v[0] for k, v in log.items()})
    sol = s.solution()
    print(prec, 'scp status', sol['status'], 'n_acc', sol['n_accepted'], 'iterations', sol['iterations'])
    s.close()
