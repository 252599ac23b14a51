"""Headline-size parity diagnosis (GPU): trot N=100 x 1024, two fixed-K SCP iterations, then a third
QP launch phase by phase; for the 16 slowest and 16 random problems: Newton steps, tail steps, merit,
KKT residuals of the reference-form QP, and |X - X_oracle| / |X| against the sparse IPM.  Writes
gpurun_out/diag_headline_<tag>.json and the exported QPs + GPU solutions of the 4 worst problems.
Usage: python scripts/diag_headline.py <tag> [B]"""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from scipy import sparse
from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle.kkt import kkt_residuals
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp

tag = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
N = 100
pb = make_batch('trot', N, B, seed_offset=0)
s = Solver(pb.robot, N, B, 'fp64')
s.upload(pb)
kern = s.qp_kernel()
s.scp_iterate(True); s.scp_iterate(True)
s.linearize(); s.assemble(); s.qp_solve()
z, y, st, it = s.qp_solution(with_y=True)
merit, nref = s.qp_info()
try:
    tail = s.qp_tail()
except Exception:
    tail = np.full(B, -1, np.int32)
slow = [int(b) for b in np.argsort(-it, kind='stable')[:16]]
rng = np.random.default_rng(0)
rand = [int(b) for b in rng.choice(np.setdiff1d(np.arange(B), slow), 16, replace=False)]
nxu = 9 * (N + 1) + 12 * N
rows = []
qps = {}
for b in slow + rand + [170]:
    P, q, A, l, u = s.export_qp(b)
    k = kkt_residuals(P, q, A, l, u, z[b], y[b])
    ref = sparse_ipm_qp(P, q, A, l, u)
    err = float(np.abs(z[b][:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max())
    rows.append(dict(b=b, it=int(it[b]), tail=int(tail[b]), merit=float(merit[b]), nref=int(nref[b]),
                     prim=float(k['prim']), dual=float(k['dual']), sign=float(k['sign']), err=err,
                     ref_status=ref.info.status, arg=int(np.abs(z[b][:nxu] - ref.x[:nxu]).argmax())))
    qps[b] = (P, q, A, l, u, z[b].copy(), y[b].copy(), ref.x)
s.close()
worst = sorted(rows, key=lambda r: -r['err'])[:4]
out = dict(tag=tag, kernel=kern, B=B, it_hist=np.bincount(it).tolist(), status=np.unique(st).tolist(),
           merit_max=float(merit.max()), rows=rows, worst=[r['b'] for r in worst])
os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'diag_headline_%s.json' % tag), 'w'), indent=1)
arr = {}
for r in worst:
    P, q, A, l, u, zb, yb, xr = qps[r['b']]
    P = sparse.csc_matrix(P); A = sparse.csc_matrix(A)
    pre = 'b%d_' % r['b']
    arr.update({pre + 'P_data': P.data, pre + 'P_indices': P.indices, pre + 'P_indptr': P.indptr,
                pre + 'A_data': A.data, pre + 'A_indices': A.indices, pre + 'A_indptr': A.indptr,
                pre + 'A_shape': np.array(A.shape), pre + 'q': q, pre + 'l': l, pre + 'u': u,
                pre + 'z': zb, pre + 'y': yb, pre + 'xref': xr})
np.savez_compressed(os.path.join(ROOT, 'gpurun_out', 'diag_headline_%s.npz' % tag), **arr)
print(json.dumps({k: out[k] for k in ('tag', 'kernel', 'it_hist', 'merit_max', 'worst')}))
for r in sorted(rows, key=lambda r: -r['err'])[:8]:
    print(r)
