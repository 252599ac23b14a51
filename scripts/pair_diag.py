"""Paired QP workgroups (k_qp_pair): per-problem Newton steps
with pairing on and off, the pair order k_qp_order builds (restated here from the previous
iteration's Newton steps), and the launch's slowest pair."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np

from cmpc._lib import Solver
from cmpc.synth import make_batch

N, B, K = 100, 1024, 5
pb = make_batch('trot', N, B, seed_offset=777)


def order_of(prev):
    key = np.clip(prev, 0, 15)
    srt = np.argsort(key, kind='stable')
    o = np.empty(B, int)
    o[0::2] = srt[::-1][:B // 2]
    o[1::2] = srt[:B // 2]
    return o


for mode in ('0', '1'):
    os.environ['CMPC_QP_PAIR'] = mode
    s = Solver(pb.robot, N, B, 'fp64')
    s.upload(pb)
    prev = np.zeros(B, int)
    for i in range(K):
        s.scp_iterate(True)
        its = s.qp_solution(with_y=False)[3].copy()
        cyc = its.astype(float)   # Newton steps as the cost proxy (no stamps in the default library)
        msg = 'pair=%s iter %d: its mean %.2f max %d  cycles max %.3g p50 %.3g  cyc/it %.3g' % (
            mode, i, its.mean(), its.max(), cyc.max(), np.median(cyc), (cyc / np.maximum(its, 1)).mean())
        if mode == '1':
            o = order_of(prev)
            a, b = o[0::2], o[1::2]
            pair_max = np.maximum(cyc[a], cyc[b])
            j = int(np.argmax(pair_max))
            msg += '  slowest pair its (%d,%d) cycles (%.3g,%.3g)' % (its[a[j]], its[b[j]], cyc[a[j]], cyc[b[j]])
            # problems that finished first in their pair ran one-wave only: their cycles per step
            first = np.where(cyc[a] <= cyc[b], a, b)
            msg += '  one-wave-only cyc/it %.3g' % (cyc[first] / np.maximum(its[first], 1)).mean()
        print(msg, flush=True)
        prev = its
    s.close()
