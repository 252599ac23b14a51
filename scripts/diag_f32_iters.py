"""Diagnostics: the fp32 QP's residual components after m Newton steps (max_iter = m), from the
device iterate and multipliers against the exported reference-form QP (oracle.kkt), per row family."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')]
import numpy as np
from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle.kkt import kkt_residuals
cfg, N = sys.argv[1], int(sys.argv[2])
pb = make_batch(cfg, N, 1)
nc = pb.nc
for prec in ('fp32', 'fp64'):
    for m in range(1, 16):
        s = Solver(pb.robot, N, 1, prec)
        s.upload(pb)
        s.set_qp_settings(max_iter=m)
        s.linearize(); s.assemble(); s.qp_solve()
        z, y, st, its = s.qp_solution(with_y=True)
        merit, nref = s.qp_info()
        P, q, A, l, u = s.export_qp(0)
        s.close()
        k = kkt_residuals(P, q, A, l, u, z[0], y[0])
        Az = A @ z[0]
        viol = np.maximum(Az - u, 0) + np.maximum(l - Az, 0)
        fam = {'init': (0, 9), 'dyn': (9, 9 + 9 * N), 'fin': (9 + 9 * N, 18 + 9 * N)}
        mc = 2 * nc * N if pb.robot != 'solo12' else 0
        r = 18 + 9 * N
        if mc: fam['cop'] = (r, r + mc); r += mc
        fam['fric'] = (r, r + 5 * nc * N); r += 5 * nc * N
        fam['tr'] = (r, r + 8 * (N + 1)); r += 8 * (N + 1)
        fam['sl'] = (r, r + N + 1)
        pv = {f: float(viol[a:b].max()) for f, (a, b) in fam.items()}
        g = P @ z[0] + q + A.T @ y[0]
        nxx = 9 * (N + 1); nuu = 12 * N
        dv = {'x': float(np.abs(g[:nxx]).max()), 'u': float(np.abs(g[nxx:nxx + nuu]).max()), 't': float(np.abs(g[nxx + nuu:nxx + nuu + N + 1]).max())}
        print(prec, m, 'st', int(st[0]), 'it', int(its[0]), 'merit %.3g' % merit[0], 'prim', {a: '%.2e' % b for a, b in pv.items()},
              'dual', {a: '%.2e' % b for a, b in dv.items()}, 'comp %.2e' % k['compl'], flush=True)
        if st[0] != -2:
            break
