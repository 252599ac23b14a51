"""Diagnostic: QP exit statuses, final merits and refinement counts of K fixed-K SCP iterations of a
synthetic batch.  Usage: python scripts/qp_exits.py <cfg> <N> <B> <iters> [fp64|fp32] [eps ...]
(several eps values: one run per value, each timed: QP ms from HIP events; a value written
eta=<v> sets the step fraction instead of eps)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
cfg, N, B, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
prec = sys.argv[5] if len(sys.argv) > 5 else 'fp64'
epss = sys.argv[6:] or [None]
pb = make_batch(cfg, N, B) if cfg != 'mixed' else make_batch('trot', N, B, mixed=('pace', 'trot'))
s = Solver(pb.robot, N, B, prec)
for eps in epss:
  if eps is not None and eps.startswith('eta='):
    s.set_qp_settings(step_fraction=float(eps[4:]))
  elif eps is not None:
    s.set_qp_settings(eps_abs=float(eps), eps_rel=float(eps))
  s.upload(pb)
  print('eps', eps)
  for k in range(K):
    s.timing_begin()
    s.scp_iterate(fixed_iters=True)
    tm = s.timing_end()
    _, _, st, it = s.qp_solution(with_y=False)
    merit, nref = s.qp_info()
    log = s.iteration_log()
    u, c = np.unique(st, return_counts=True)
    print('iter %d status %s | ipm it mean %.2f p99 %d max %d | merit max %.3g | refine: %d problems, %d steps | qp %.3f ms'
          % (k, dict(zip(u.tolist(), c.tolist())), it.mean(), np.percentile(it, 99), it.max(), merit.max(),
             (nref > 0).sum(), nref.sum(), tm['qp_ms']))
    print('   decisions', dict(zip(*[a.tolist() for a in np.unique(log['decision'], return_counts=True)])))
    bad = np.nonzero(st != 1)[0]
    for b in bad[:10]:
        print('   problem %d status %d it %d merit %.3g nref %d' % (b, st[b], it[b], merit[b], nref[b]))
s.close()
