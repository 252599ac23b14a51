"""Starting-point floors of the Solo12 IPM (cmpc_qp_settings init_floor_s / _l) over whole
batches: per setting the mean / max Newton steps, the statuses and the QP time of one launch.
floor 0 = CVXOPT's shift."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np

from cmpc._lib import Solver
from cmpc.synth import make_batch

CASES = [('trot', 100, 1024, 1.0), ('bound', 100, 1024, 1.0), ('pace', 100, 1024, 1.0), ('trot', 100, 1024, 5.0),
         ('bound', 60, 1024, 5.0)]
FLOORS = [(0.0, 0.0), (0.1, 0.1), (0.1, 0.03), (0.2, 0.1), (0.1, 0.2), (0.3, 0.3), (0.15, 0.15)]
for cfg, N, B, wmul in CASES:
    pb = make_batch(cfg, N, B)
    if wmul != 1.0:
        for p in pb.params:
            p.scp_params = dict(p.scp_params, omega0=p.scp_params.get('omega0', 100.0) * wmul)
    s = Solver(pb.robot, N, B, 'fp64')
    s.upload(pb)
    out = []
    for fs, fl in FLOORS:
        s.set_qp_settings(init_floor_s=fs, init_floor_l=fl)
        s.linearize(); s.assemble()
        s.synchronize()
        t0 = time.perf_counter()
        s.qp_solve()
        s.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        _, _, st, it = s.qp_solution(with_y=False)
        out.append('(%.2f,%.2f) %.2f/%d %s %.2fms' % (fs, fl, it.mean(), it.max(), '' if np.all(st == 1) else
                                                      'ST%s' % np.unique(st).tolist(), ms))
    s.close()
    print(cfg, N, B, 'w x%g' % wmul, ' | '.join(out), flush=True)
