"""Per-phase cycle shares of the QP kernel (diagnostic library, CMPC_LIB_VARIANT=diag)."""
import os, sys, time
os.environ.setdefault('CMPC_LIB_VARIANT', 'diag')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
cfg = sys.argv[1] if len(sys.argv) > 1 else 'trot'
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100
B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
W = int(sys.argv[4]) if len(sys.argv) > 4 else 0   # QP waves per problem (0: the library's choice)
pb = make_batch(cfg, N, B)
s = Solver(pb.robot, N, B, 'fp64'); s.set_qp_settings(waves_per_problem=W); s.upload(pb)
s.scp_iterate(True); s.synchronize()
s.timing_begin(); s.scp_iterate(True); t = s.timing_end()
st = s.debug_stamps().astype(float)
names = ['residual', 'factor+w_pred', 'sblock+rhs_pred', 'seq_factor+elim', 'w_corr', 'rhs_corr', 'seq_solve', 'dz', 'update']
its = s.qp_iterations_total() / B
tot = st[:, :9].sum(axis=1).mean()
print('B', B, 'N', N, 'qp_ms', t['qp_ms'], 'ipm iters', its, 'cycles/problem %.3g' % tot)
_, _, _, itv = s.qp_solution(with_y=False)
print('  ipm iterations of the last solve: mean %.2f  p50 %d  p90 %d  p99 %d  max %d' % (
    itv.mean(), np.percentile(itv, 50), np.percentile(itv, 90), np.percentile(itv, 99), itv.max()))
tq = st[:, :9].sum(axis=1)
print('  per-problem QP cycles of the timed solve: p50 %.3g  p90 %.3g  max %.3g' % (
    np.percentile(tq, 50), np.percentile(tq, 90), tq.max()))
for i, n in enumerate(names):
    print('  %-11s %5.1f%%  %.3g cycles/IPM-iter' % (n, 100 * st[:, i].mean() / tot, st[:, i].mean() / its))
# tw_factor_ends sub-steps (top wave; accumulated over the warm-up and the timed iteration)
sub = st[:, 12:16].mean(axis=0) / 2.0
if W == 4:   # four-wave kernel: top chain, barrier wait, separator system, interior chain (per IPM iteration)
    print('  four-wave factorization (cycles/IPM-iter): top chain %.0f  wait %.0f  separators %.0f  interior chain %.0f'
          % tuple(sub / its))
else:
    nst = its * (N + 2) // 2
    print('  factor step sub-phases (cycles/step): X+A %.0f  GJ %.0f  tail %.0f  land %.0f' % tuple(sub / nst))
lin = st[:, 9:11].mean(axis=0)
print('  k_linearize per problem: knots (wave 0) %.3g cycles, covariance scan %.3g cycles' % tuple(lin))
