"""GPU: the headline launch of tests/test_gpu_headline.py (trot N=100 x 1024, third QP launch after two
fixed-K iterations), dumping the sampled problems' reference-form QPs, GPU solutions and exit data to
gpurun_out/headline_dump.npz for CPU analysis (oracle tolerance, polishing outcome)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd'), os.path.join(ROOT, 'tests')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch

N, B = 100, 1024
pb = make_batch('trot', N, B, seed_offset=0)
s = Solver(pb.robot, N, B, 'fp64')
s.upload(pb)
s.scp_iterate(fixed_iters=True)
s.scp_iterate(fixed_iters=True)
s.linearize(); s.assemble(); s.qp_solve()
z, y, st, it = s.qp_solution(with_y=True)
merit, nref = s.qp_info()
tail, pol = s.qp_exit()
slow = [int(b) for b in np.argsort(-it, kind='stable')[:8]]
rng = np.random.default_rng(0)
rest = np.setdiff1d(np.arange(B), slow)
rand = [int(b) for b in rng.choice(rest, 8, replace=False)]
out = dict(iters=it, status=st, merit=merit, nref=nref, polish=pol, sample=np.array(slow + rand))
for b in slow + rand:
    P, q, A, l, u = s.export_qp(b)
    P, A = P.tocsc(), A.tocsc()
    out['P_data_%d' % b] = P.data; out['P_ind_%d' % b] = P.indices; out['P_ptr_%d' % b] = P.indptr
    out['A_data_%d' % b] = A.data; out['A_ind_%d' % b] = A.indices; out['A_ptr_%d' % b] = A.indptr
    out['A_shape_%d' % b] = np.array(A.shape)
    out['q_%d' % b] = q; out['l_%d' % b] = l; out['u_%d' % b] = u
    out['z_%d' % b] = z[b]; out['y_%d' % b] = y[b]
os.makedirs('gpurun_out', exist_ok=True)
np.savez_compressed('gpurun_out/headline_dump.npz', **out)
print('polish outcomes (all problems):', dict(zip(*np.unique(pol, return_counts=True))))
print('iters:', dict(zip(*np.unique(it, return_counts=True))))
for b in slow + rand:
    print(b, 'iters', int(it[b]), 'polish', int(pol[b]), 'nref', int(nref[b]), 'merit %.3f' % merit[b])
s.close()
