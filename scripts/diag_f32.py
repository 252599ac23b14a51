"""Diagnostics: fp32 QP exits on synthetic batches of each gait (status histogram, Newton steps)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
for cfg, N, B in (('trot', 20, 64), ('trot', 100, 256), ('bound', 20, 64), ('pace', 40, 64)):
    pb = make_batch(cfg, N, B)
    for prec in ('fp32',):
        s = Solver(pb.robot, N, B, prec)
        s.upload(pb)
        s.linearize(); s.assemble(); s.qp_solve()
        z, _, st, its = s.qp_solution(with_y=False)
        merit, nref = s.qp_info()
        u, c = np.unique(st, return_counts=True)
        print(cfg, N, B, prec, dict(zip(u.tolist(), c.tolist())), 'iters mean %.1f max %d' % (its.mean(), its.max()),
              'merit max', float(np.nanmax(merit)), 'nref', int(nref.sum()), flush=True)
        s.close()
