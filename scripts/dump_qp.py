"""Diagnostic: run K fixed-K SCP iterations of a synthetic batch and save one problem's exported
QP (reference row order, CSC parts) plus the GPU's solution and status to an .npz.
Usage: python scripts/dump_qp.py <cfg> <N> <B> <iters> <problem|argmax> <out.npz>"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
cfg, N, B, K, which, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6]
pb = make_batch(cfg, N, B)
s = Solver(pb.robot, N, B, 'fp64'); s.upload(pb)
for _ in range(K):
    s.scp_iterate(fixed_iters=True)
s.synchronize()
z, y, st, it = s.qp_solution(with_y=True)
b = int(it.argmax()) if which == 'argmax' else int(which)
P, q, A, l, u = s.export_qp(b)
np.savez_compressed(out, P_data=P.data, P_indices=P.indices, P_indptr=P.indptr, P_shape=P.shape,
                    A_data=A.data, A_indices=A.indices, A_indptr=A.indptr, A_shape=A.shape,
                    q=q, l=l, u=u, z=z[b], y=y[b], status=st[b], ipm_iters=it[b], problem=b)
print('saved problem', b, 'status', int(st[b]), 'ipm iterations', int(it[b]), '->', out)
s.close()
