"""Oracle: QP cost and constraint matrices in the reference's exact row order.  TEST INFRASTRUCTURE.

Restates src/cost.py, src/constraints.py and src/scp_solver.py:10-48 of the reference.
Variable layout z = [x_0..x_N (9 each) | u_0..u_{N-1} (nu each) | t_0..t_N | s_0..s_{N-1}]
(src/centroidal_model.py:25-26, src/optimizer.py:5-133).

``prm`` keys used here (in addition to oracle.model's): Wx (9x9), Wu (nu x nu), mu,
beta_u, stochastic (bool), tracking (bool: solo12 with DYNAMICS_FIRST False, quirk Q10),
foot_range (lxp, lxn, lyp, lyn) for TALOS.
"""
import math
import numpy as np
from scipy import sparse
from scipy.stats import norm


def n_vars(N, nu):
    return 9 * (N + 1) + nu * N + (N + 1) + N


def x_idx(k):
    return 9 * k


def u_idx(N, nu, k):
    return 9 * (N + 1) + nu * k


def t_idx(N, nu, k):
    return 9 * (N + 1) + nu * N + k


def penum_mat():
    """Slack_optimizer._penum_mat for nx-6 = 3 (src/optimizer.py:104-112): s_j[i] = (-1)^(j // 2^i)."""
    M = np.zeros((8, 3))
    for i in range(3):
        M[:, i] = [(-1) ** (j // (2 ** i)) for j in range(8)]
    return M


def friction_pyramid(mu):
    """src/utils.py:9-16 (inner pyramid, mu' = mu / sqrt 2)."""
    ml = mu / np.sqrt(2)
    return np.array([[1., 0., -ml], [-1., 0., -ml], [0., 1., -ml], [0., -1., -ml], [0., 0., -1.]])


def chance_xi(beta_u):
    """xi = Phi^-1(1 - beta_u / 5 * 3) (src/constraints.py:157)."""
    return float(norm.ppf(1 - (beta_u / 5 * 3)))


def build_cost(N, prm, Xbar):
    """P, q of sum_up_all_costs (src/scp_solver.py:10-26; src/cost.py:9-39)."""
    nu = prm['nu']; n = n_vars(N, nu)
    Wx = np.asarray(prm['Wx'], float); Wu = np.asarray(prm['Wu'], float)
    P = sparse.block_diag([sparse.kron(sparse.eye(N + 1), Wx), sparse.kron(sparse.eye(N), Wu),
                           sparse.csc_matrix((N + 1, N + 1)), sparse.csc_matrix((N, N))], format='csc')
    P.eliminate_zeros()
    q = np.zeros(n)
    if prm.get('tracking', True) and prm['robot'] == 'solo12':
        for k in range(N + 1):
            q[x_idx(k): x_idx(k) + 9] = -Wx @ np.asarray(Xbar, float)[:, k]
    q[t_idx(N, nu, 0): t_idx(N, nu, 0) + N + 1] = 1.0
    return P, q


class _Rows:
    """COO accumulator that keeps the reference's row order."""

    def __init__(self, n):
        self.n = n; self.r = []; self.c = []; self.v = []; self.lb = []; self.ub = []; self.m = 0

    def add(self, cols, vals, lb, ub):
        for cc, vv in zip(cols, vals):
            if vv != 0.0:
                self.r.append(self.m); self.c.append(cc); self.v.append(float(vv))
        self.lb.append(lb); self.ub.append(ub); self.m += 1

    def mat(self):
        return sparse.csc_matrix((self.v, (self.r, self.c)), shape=(self.m, self.n))


def build_constraints(N, prm, logic, pos, rot, Xbar, Ubar, traj_data, weight, radius, Xinit=None):
    """A, l, u of stack_up_all_constraints (src/scp_solver.py:28-48).

    (Xbar, Ubar) is the linearization point (traj_tuple); the initial / final state rows use the
    warm start ``Xinit`` (model._init_trajectories, src/centroidal_model.py:87-89), which is Xbar
    itself in the reference's loop (quirk Q1) and the default here.

    Row order: init (9) | dynamics (9N) | final (9) | [TALOS CoP: per contact N x-rows then
    N y-rows] | friction (per contact, per knot, 5 rows, rows 0-3 filled when active) |
    TR L1 (8 per knot k=0..N) | TR slack (N+1).
    """
    nu = prm['nu']; nc = prm['nc']; nupc = nu // nc
    n = n_vars(N, nu)
    Xbar = np.asarray(Xbar, float); Ubar = np.asarray(Ubar, float)
    Xi = Xbar if Xinit is None else np.asarray(Xinit, float)
    rows = _Rows(n)
    # initial constraints (src/constraints.py:11-17): x_init = X_npz[0] = Xinit[:, 0]
    for i in range(9):
        rows.add([i], [1.0], Xi[i, 0], Xi[i, 0])
    # dynamics (src/constraints.py:19-50): [A_k  B_k  -I] z = A_k xbar_k + B_k ubar_k - f_k (+-1e-12)
    fdt = traj_data['f_x'].dtype
    for k in range(N):
        A = traj_data['f_x'][k]; B = traj_data['f_u'][k]; f = traj_data['dynamics'][:, k]
        r = A @ Xbar[:, k].astype(fdt) + B @ Ubar[:, k].astype(fdt) - f
        lo = (r - fdt.type(1e-12)).astype(float); hi = (r + fdt.type(1e-12)).astype(float)
        for i in range(9):
            cols = list(range(x_idx(k), x_idx(k) + 9)) + list(range(u_idx(N, nu, k), u_idx(N, nu, k) + nu)) \
                + [x_idx(k + 1) + i]
            vals = list(np.asarray(A[i], float)) + list(np.asarray(B[i], float)) + [-1.0]
            # A_k block and -I may share no column; keep reference's dense-then-sparse nnz pattern
            rows.add(cols, vals, lo[i], hi[i])
    # final constraints (src/constraints.py:103-109)
    for i in range(9):
        rows.add([x_idx(N) + i], [1.0], Xi[i, N], Xi[i, N])
    # TALOS CoP (src/constraints.py:111-145)
    if prm['robot'] == 'TALOS':
        lxp, lxn, lyp, lyn = prm['foot_range']
        for i in range(nc):
            for d, (lo, hi) in enumerate([(-lxn, lxp), (-lyn, lyp)]):
                for k in range(N):
                    if logic[k, i]:
                        rows.add([u_idx(N, nu, k) + nupc * i + d], [1.0], lo, hi)
                    else:
                        rows.add([], [], 0.0, 0.0)
    # friction pyramid (src/constraints.py:153-217)
    Fmu = friction_pyramid(prm['mu'])
    xi = chance_xi(prm['beta_u'])
    fofs = 0 if prm['robot'] == 'solo12' else 2
    for i in range(nc):
        for k in range(N):
            fcol = u_idx(N, nu, k) + nupc * i + fofs
            if logic[k, i]:
                G = Fmu @ np.asarray(rot[k, i], float).T
                for j in range(5):
                    if j < 4:
                        ub = 0.0
                        if prm.get('stochastic', False) and k > 0:
                            # only the constant back-off survives: the Sigma-gradient terms are
                            # exactly zero (quirk Q3); K rows 3*idx..3*idx+2 (quirk, also TALOS)
                            Kc = np.asarray(traj_data['LQR_gains'][k], float)[3 * i: 3 * i + 3, :]
                            KSK = Kc @ np.asarray(traj_data['Covs'][k], float) @ Kc.T
                            for uu in range(3):
                                s = math.sqrt(KSK[uu, uu])
                                if G[j, uu] > 1e-6 and s > 1e-6:
                                    ub -= xi * (2 * G[j, uu] * s)
                        rows.add([fcol, fcol + 1, fcol + 2], list(G[j]), -np.inf, ub)
                    else:
                        rows.add([], [], -np.inf, 0.0)  # row 4 allocated, never filled (quirk Q4)
            else:
                for j in range(5):
                    rows.add([], [], -np.inf, 0.0)
    # state trust region, L1 on angular momentum (src/constraints.py:260-293)
    S = penum_mat()
    for k in range(N + 1):
        for j in range(8):
            rows.add([x_idx(k) + 6, x_idx(k) + 7, x_idx(k) + 8, t_idx(N, nu, k)],
                     [S[j, 0], S[j, 1], S[j, 2], -1.0 / weight], -np.inf, radius + S[j] @ Xbar[6:, k])
    for k in range(N + 1):
        rows.add([t_idx(N, nu, k)], [-1.0], -np.inf, 0.0)
    return rows.mat(), np.array(rows.lb), np.array(rows.ub)


def get_qp_solution(N, nu, z):
    """src/scp_solver.py:89-93 (Fortran-order reshapes)."""
    X = np.reshape(z[:9 * (N + 1)], (9, N + 1), order='F')
    U = np.reshape(z[9 * (N + 1): 9 * (N + 1) + nu * N], (nu, N), order='F')
    return X, U


def interpolate_scp_solution(X, U, N_inner=10):
    """src/scp_solver.py:95-111: linear interpolation, N_inner = 10 sub-steps per interval."""
    Xi = np.zeros((X.shape[0], (X.shape[1] - 1) * N_inner))
    Ui = np.zeros((U.shape[0], (U.shape[1] - 1) * N_inner))
    for i in range(U.shape[1] - 1):
        du = (U[:, i + 1] - U[:, i]) / float(N_inner)
        for j in range(N_inner):
            Ui[:, i * N_inner + j] = U[:, i] + j * du
    for i in range(X.shape[1] - 1):
        dx = (X[:, i + 1] - X[:, i]) / float(N_inner)
        for j in range(N_inner):
            Xi[:, i * N_inner + j] = X[:, i] + j * dx
    return Xi, Ui
