"""Developer probe: run each GPU phase on a few small problems and compare with the oracle."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc.synth import make_batch
from cmpc._lib import Solver
from oracle import model as M, transcription as T, ipm_mirror as IM
from oracle.kkt import kkt_residuals

cfg = sys.argv[1] if len(sys.argv) > 1 else 'trot'
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
B = int(sys.argv[3]) if len(sys.argv) > 3 else 3
prec = sys.argv[4] if len(sys.argv) > 4 else 'fp64'
pb = make_batch(cfg, N, B)
s = Solver(pb.robot, N, B, prec)
s.upload(pb)
t0 = time.time(); s.linearize(); s.synchronize(); print('linearize %.3fs' % (time.time() - t0), flush=True)
lin = s.linearization()
print('NaN counts K', np.isnan(lin['K']).sum(), 'Sigma', np.isnan(lin['Sigma']).sum(), 'K[0,0,:3,:3]', lin['K'][0,0,:3,:3], flush=True)
for b in range(B):
    prob = pb.oracle_problem(b); prm = prob['prm']
    td = M.compute_trajectory_data(prob['Xbar'], prob['Ubar'], prob['logic'], prob['pos'], prob['rot'], prm)
    errs = dict(f=np.abs(lin['f'][b] - td['dynamics'].T).max(), A=np.abs(lin['A'][b] - td['f_x']).max(),
                B=np.abs(lin['Bu'][b] - td['f_u']).max(), C=np.abs(lin['C'][b] - td['f_w']).max(),
                K=np.abs(lin['K'][b] - td['LQR_gains']).max() / np.abs(td['LQR_gains']).max(),
                S=np.abs(lin['Sigma'][b] - td['Covs']).max() / np.abs(td['Covs']).max())
    print('b', b, 'lin errs', {k: '%.2e' % v for k, v in errs.items()}, flush=True)
s.assemble(); s.synchronize()
for b in range(B):
    prob = pb.oracle_problem(b); prm = prob['prm']
    td = M.compute_trajectory_data(prob['Xbar'], prob['Ubar'], prob['logic'], prob['pos'], prob['rot'], prm)
    P, q, A, l, u = s.export_qp(b)
    P0, q0 = T.build_cost(N, prm, prob['Xbar'])
    A0, l0, u0 = T.build_constraints(N, prm, prob['logic'], prob['pos'], prob['rot'], prob['Xbar'], prob['Ubar'], td, 100., 100.)
    print('b', b, 'assembly: P %.1e q %.1e A %.1e (shape %s vs %s) l %.1e u %.1e' % (
        abs(P - P0).max(), np.abs(q - q0).max(), abs(A - A0).max() if A.shape == A0.shape else -1, A.shape, A0.shape,
        np.nanmax(np.abs(np.where(np.isfinite(l0), l - l0, 0))), np.nanmax(np.abs(np.where(np.isfinite(u0), u - u0, 0)))), flush=True)
t0 = time.time(); s.qp_solve(); s.synchronize(); print('qp %.3fs' % (time.time() - t0), flush=True)
z, y, st, it = s.qp_solution()
print('qp status', st, 'iters', it, flush=True)
for b in range(B):
    prob = pb.oracle_problem(b); prm = prob['prm']
    td = M.compute_trajectory_data(prob['Xbar'], prob['Ubar'], prob['logic'], prob['pos'], prob['rot'], prm)
    P0, q0 = T.build_cost(N, prm, prob['Xbar'])
    A0, l0, u0 = T.build_constraints(N, prm, prob['logic'], prob['pos'], prob['rot'], prob['Xbar'], prob['Ubar'], td, 100., 100.)
    k = kkt_residuals(P0, q0, A0, l0, u0, z[b], y[b])
    p = pb.params[pb.class_id[b]]
    qp = IM.StructQP.from_arrays(N, pb.robot, pb.nc, p.Wx, p.Wu, pb.Xbar[b], pb.Ubar[b], td['f_x'], td['f_u'],
                                 td['dynamics'].T, pb.logic[b], pb.rot[b], p.mu, 100., 100., p.tracking,
                                 foot_range=p.foot_range)
    sol = IM.solve(qp, eps=1e-10)
    zm = IM.to_z(qp, sol)
    n_xu = 9 * (N + 1) + 12 * N
    print('b', b, 'kkt prim %.2e dual %.2e compl %.2e sign %.2e | mirror iters %d, |z-zm| %.2e (rel %.2e)' % (
        k['prim'], k['dual'], k['compl'], k['sign'], sol['iters'], np.abs(z[b][:n_xu] - zm[:n_xu]).max(),
        np.abs(z[b][:n_xu] - zm[:n_xu]).max() / np.abs(zm[:n_xu]).max()), flush=True)
s.accept(False); s.synchronize()
print('log', s.iteration_log(), flush=True)
s2 = Solver(pb.robot, N, B, prec); s2.upload(pb)
t0 = time.time(); n = s2.solve_scp(False); print('solve_scp iterations', n, '%.3fs' % (time.time() - t0))
sol = s2.solution(); print({k: sol[k] for k in ('n_accepted', 'iterations', 'status', 'weight', 'radius')})
s2.scp_iterate(True); s2.synchronize(); print('timing', s2.timing())
