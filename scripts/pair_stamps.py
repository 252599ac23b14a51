"""Paired QP workgroups on the diagnostic library (metric config): per problem the QP cycles
(one-wave part + two-wave part), Newton steps, and the steps and cycles spent on both waves
(stamp slots 9, 10 of k_qp_pair); the slowest pairs of the last launch."""
import os
import sys

os.environ['CMPC_LIB_VARIANT'] = 'diag'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np

from cmpc._lib import Solver
from cmpc.synth import make_batch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
pb = make_batch('trot', N, B, seed_offset=777)
s = Solver(pb.robot, N, B, 'fp64')
s.upload(pb)
prev = None
for i in range(3):
    s.scp_iterate(True)
    st = s.debug_stamps().astype(float)
    its = s.qp_solution(with_y=False)[3].copy()
    cyc = st[:, :9].sum(axis=1)
    bc, bi = st[:, 9], st[:, 10]
    print('iter %d: cycles max %.4g p50 %.4g mean %.4g | its mean %.2f max %d | problems finished on both waves %d'
          % (i, cyc.max(), np.median(cyc), cyc.mean(), its.mean(), its.max(), int((bi > 0).sum())), flush=True)
    one = bi == 0
    print('   one-wave cycles per Newton step (problems never shared) mean %.4g' % (cyc[one] / np.maximum(its[one], 1)).mean())
    sh = bi > 0
    if sh.any():
        print('   two-wave cycles per Newton step mean %.4g over %d problems (%.2f steps each)'
              % ((bc[sh] / bi[sh]).mean(), sh.sum(), bi[sh].mean()))
    top = np.argsort(cyc)[-5:][::-1]
    for b in top:
        print('   slow problem %d: cycles %.4g its %d, both-wave steps %d cycles %.4g' % (b, cyc[b], its[b], bi[b], bc[b]))
    st[:, 9:11] = 0
    prev = its
s.close()
