"""Solution polishing on the GPU (qp_ipm.hip phase_polish_prep): per configuration, the QP's Newton
steps, polishing outcomes and QP time with the robot's polish_eps against polishing off
(CMPC_QP_POLISH_EPS=0), same batch, same box.  Usage: python scripts/diag_polish.py"""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch

CASES = [('trot', 100, 1024), ('talos', 200, 512), ('trot', 100, 256), ('bound', 100, 1024)]
for cfg, N, B in CASES:
    pb = make_batch(cfg, N, B, seed_offset=0)
    for peps in (None, '0'):
        if peps is None:
            os.environ.pop('CMPC_QP_POLISH_EPS', None)
        else:
            os.environ['CMPC_QP_POLISH_EPS'] = peps
        s = Solver(pb.robot, N, B, 'fp64')
        s.upload(pb)
        for _ in range(3):
            s.scp_iterate(fixed_iters=True)
        s.synchronize()
        t0 = time.perf_counter()
        s.timing_begin()
        for _ in range(5):
            s.scp_iterate(fixed_iters=True)
        tim = s.timing_end()
        z, _, st, it = s.qp_solution(with_y=False)
        tail, pol = s.qp_exit()
        print('%-6s N=%d B=%d polish_eps=%-8s kernel %-14s status %s newton mean %.3f max %d  polish +%d -%d  '
              'tail>0 %d  qp_ms %.3f' % (cfg, N, B, 'robot' if peps is None else peps, s.qp_kernel(),
                                         dict(zip(*np.unique(st, return_counts=True))), it.mean(), it.max(),
                                         (pol > 0).sum(), (pol < 0).sum(), (tail > 0).sum(),
                                         tim['qp_ms'] / max(tim['iterations'], 1)), flush=True)
        s.close()
os.environ.pop('CMPC_QP_POLISH_EPS', None)
