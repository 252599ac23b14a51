"""Diagnostic: TALOS N=200 x 512, two fixed-K SCP iterations; report problems whose second QP
does not reach 'solved' and check that QP with the oracle's sparse IPM (test infrastructure)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle.kkt import kkt_residuals
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
N, B = 200, 512
pb = make_batch('talos', N, B)
s = Solver(pb.robot, N, B, 'fp64'); s.upload(pb)
for k in range(3):
    s.scp_iterate(fixed_iters=True); s.synchronize()
    z, y, st, it = s.qp_solution(with_y=True)
    log = s.iteration_log()
    bad = np.nonzero(st != 1)[0]
    print('scp iter', k, 'status counts', dict(zip(*[a.tolist() for a in np.unique(st, return_counts=True)])),
          'ipm it max', int(it.max()), 'argmax', int(it.argmax()), 'p99', float(np.percentile(it, 99)),
          'decisions', dict(zip(*[a.tolist() for a in np.unique(log['decision'], return_counts=True)])), flush=True)
    for b in list(bad[:2]) + ([int(it.argmax())] if len(bad) == 0 else []):
        P, q, A, l, u = s.export_qp(int(b))
        kk = kkt_residuals(P, q, A, l, u, z[b], y[b])
        ref = sparse_ipm_qp(P, q, A, l, u)
        nx = 9 * (N + 1)
        err = np.abs(z[b][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max()
        print('  b', int(b), 'st', int(st[b]), 'it', int(it[b]), 'kkt', {kq: '%.2e' % float(v) for kq, v in kk.items() if np.ndim(v) == 0},
              'oracle status', getattr(ref, 'status', getattr(getattr(ref, 'info', None), 'status', '?')),
              'rel err vs oracle %.2e' % err, flush=True)
s.close()
