"""Straggler structure of the QP launches over consecutive SCP iterations (diagnostic library):
per problem and iteration the QP cycles (stamps) and IPM iterations; compares the sum over
iterations of the per-launch maxima (what per-iteration launches pay) with the maximum over
problems of the per-problem sums (what a launch running every problem's iterations back to back
would pay)."""
import os
import sys

os.environ['CMPC_LIB_VARIANT'] = 'diag'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np

from cmpc._lib import Solver
from cmpc.synth import make_batch

cfg = sys.argv[1] if len(sys.argv) > 1 else 'trot'
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
K = int(sys.argv[4]) if len(sys.argv) > 4 else 6
pb = make_batch(cfg, N, B)
s = Solver(pb.robot, N, B, 'fp64')
s.upload(pb)
cyc, its, dec = [], [], []
for i in range(K):
    s.scp_iterate(True)
    st = s.debug_stamps().astype(float)
    cyc.append(st[:, :9].sum(axis=1))
    its.append(s.qp_solution(with_y=False)[3].copy())
    dec.append(s.iteration_log()['decision'].copy())
# stamps accumulate per solve inside the kernel (reset per launch)
cyc = np.array(cyc)
its = np.array(its)
print('per-iteration max / p50 cycles:', ['%.3g/%.3g' % (c.max(), np.median(c)) for c in cyc])
print('per-iteration IPM its max / mean:', ['%d/%.2f' % (x.max(), x.mean()) for x in its])
print('sum of maxima %.4g   max of sums %.4g   ratio %.3f   mean-sum %.4g' % (
    cyc.max(axis=1).sum(), cyc.sum(axis=0).max(), cyc.sum(axis=0).max() / cyc.max(axis=1).sum(), cyc.sum(axis=0).mean()))
c = np.corrcoef(cyc)
print('correlation of per-problem cycles between consecutive iterations:',
      ['%.2f' % c[i, i + 1] for i in range(K - 1)])
print('decisions per iteration:', [np.bincount(d + 1, minlength=5).tolist() for d in dec])

# Pairing model (a two-wave workgroup holding two problems, one per wave; when one finishes, both
# waves finish the other at r x the one-wave time per step): launch time = max over pairs of
# min + (max - min) * r, pairs from the previous iteration's cycles (slowest with fastest) or random.
R = float(os.environ.get('PAIR_R', '0.61'))
rng = np.random.default_rng(0)
for i in range(1, K):
    pred, act = cyc[i - 1], cyc[i]
    o = np.argsort(pred)
    sorted_pairs = [(o[j], o[B - 1 - j]) for j in range(B // 2)]
    rp = rng.permutation(B)
    rand_pairs = [(rp[2 * j], rp[2 * j + 1]) for j in range(B // 2)]
    oracle_o = np.argsort(act)
    oracle_pairs = [(oracle_o[j], oracle_o[B - 1 - j]) for j in range(B // 2)]
    def t(pairs):
        return max(min(act[a], act[b]) + abs(act[a] - act[b]) * R for a, b in pairs)
    print('iter %d: single %.4g  sorted-by-prev %.4g (%.3f)  random %.4g (%.3f)  perfect %.4g (%.3f)' % (
        i, act.max(), t(sorted_pairs), t(sorted_pairs) / act.max(), t(rand_pairs), t(rand_pairs) / act.max(),
        t(oracle_pairs), t(oracle_pairs) / act.max()))
