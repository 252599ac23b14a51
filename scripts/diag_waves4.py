"""Diagnostics: one vs four waves per problem on a small batch (statuses, Newton steps, solution
difference), then one timed bench-like pass per wave count at the strong-scaling shard sizes."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
cfg, N, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
pb = make_batch(cfg, N, B, seed_offset=41)
res = {}
for w in (1, 2, 4):
    s = Solver(pb.robot, N, B, 'fp64')
    s.set_qp_settings(waves_per_problem=w)
    s.upload(pb)
    s.scp_iterate(fixed_iters=True)
    z, _, st, it = s.qp_solution(with_y=False)
    merit, nref = s.qp_info()
    for _ in range(2):
        s.scp_iterate(fixed_iters=True)
    s.synchronize()
    s.timing_begin()
    t0 = time.perf_counter()
    for _ in range(10):
        s.scp_iterate(fixed_iters=True)
    s.synchronize()
    dt = (time.perf_counter() - t0) / 10
    tim = s.timing_end()
    res[w] = z
    u, c = np.unique(st, return_counts=True)
    print('waves', w, 'status', dict(zip(u.tolist(), c.tolist())), 'iters mean %.2f max %d' % (it.mean(), it.max()),
          'merit max %.3g' % merit.max(), 'step %.3f ms qp %.3f ms' % (dt * 1e3, tim['qp_ms'] / tim['iterations']), flush=True)
    s.close()
for w in (2, 4):
    err = np.abs(res[w] - res[1]).max(axis=1) / np.abs(res[1]).max(axis=1)
    print('waves', w, 'vs 1: max rel diff %.3g' % err.max())
