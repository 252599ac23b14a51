"""Oracle: centroidal dynamics, linearization, LQR gains, covariance scan.  TEST INFRASTRUCTURE.

Restates src/centroidal_model.py of the reference (file:line cited per function).
Inputs use the reference's orientation: X is (9, N+1), U is (nu, N); contact data are
``logic`` (N, nc) int, ``pos`` (N, 3*nc), ``rot`` (N, nc, 3, 3) exactly as built by
``Centroidal_model.__fill_contact_data`` (src/centroidal_model.py:127-156).

``prm`` is a dict with keys: robot ('solo12' | 'TALOS'), m, g, dt, nc, nu, nw, Q, R,
cov_w, cov_eta.  ``dtype`` selects the arithmetic type: the reference runs this whole
file in float32 (JAX default, no x64 flag anywhere); the oracle defaults to float64 and
offers float32 to mimic the reference.
"""
import numpy as np


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1],
                     a[2] * b[0] - a[0] * b[2],
                     a[0] * b[1] - a[1] * b[0]], dtype=np.result_type(a, b))


def skew(v):
    """[v]x such that [v]x @ w == v x w."""
    return np.array([[0.0, -v[2], v[1]],
                     [v[2], 0.0, -v[0]],
                     [-v[1], v[0], 0.0]], dtype=v.dtype)


def integrate_one_step(x, u, p, a, R, prm, dtype=np.float64):
    """x+ = x + dt * F(x, u; p, a, R)   (src/centroidal_model.py:189-212).

    F = [l/m ; m g e_z + sum_i a_i f_i ; sum_i a_i (p_i - c) x f_i (+ TALOS CoP/torque terms)].
    """
    t = dtype
    x = np.asarray(x, t); u = np.asarray(u, t); p = np.asarray(p, t)
    R = np.asarray(R, t)
    m = t(prm['m']); nc = prm['nc']
    inv_m = t(1.0) / m
    F = np.array([inv_m * x[3], inv_m * x[4], inv_m * x[5], 0., 0., m * t(prm['g']), 0., 0., 0.], dtype=t)
    nupc = u.shape[0] // nc
    c = x[0:3]
    for i in range(nc):
        ai = t(a[i])
        ui = u[nupc * i: nupc * (i + 1)]
        pc = p[3 * i: 3 * i + 3] - c
        if prm['robot'] == 'solo12':
            f = ui[0:3]
            F[3:6] += ai * f
            F[6:9] += ai * _cross(pc, f)
        else:  # TALOS: u_i = [cop_x, cop_y, fx, fy, fz, tau_z]  (:204-208)
            f = ui[2:5]
            Ri = R[i]
            F[3:6] += ai * f
            F[6:9] += ai * (_cross(pc, f) + _cross(Ri[:, 0:2] @ ui[0:2], f) + Ri[:, 2] * ui[5])
    return x + F * t(prm['dt'])


def jacobians(x, u, p, a, R, prm, dtype=np.float64):
    """Closed-form A = dx+/dx, B = dx+/du, C = dx+/dp.

    Replaces the three ``jax.jacfwd`` traces at src/centroidal_model.py:230-232.  The
    dynamics are linear in each argument separately, so these are exact.
    """
    t = dtype
    x = np.asarray(x, t); u = np.asarray(u, t); p = np.asarray(p, t); R = np.asarray(R, t)
    nc = prm['nc']; nu = u.shape[0]; nupc = nu // nc
    dt = t(prm['dt']); m = t(prm['m'])
    c = x[0:3]
    A = np.eye(9, dtype=t)
    B = np.zeros((9, nu), dtype=t)
    C = np.zeros((9, 3 * nc), dtype=t)
    A[0, 3] = A[1, 4] = A[2, 5] = dt * (t(1.0) / m)
    for i in range(nc):
        ai = t(a[i])
        ui = u[nupc * i: nupc * (i + 1)]
        pc = p[3 * i: 3 * i + 3] - c
        if prm['robot'] == 'solo12':
            f = ui[0:3]
            fcols = slice(nupc * i, nupc * i + 3)
            lever = pc
        else:
            f = ui[2:5]
            fcols = slice(nupc * i + 2, nupc * i + 5)
            Ri = R[i]
            lever = pc + Ri[:, 0:2] @ ui[0:2]
            # d/dcop [(R2 cop) x f] = -[f]x R2 ; d/dtau = R[:,2]
            B[6:9, nupc * i: nupc * i + 2] = dt * ai * (-skew(f) @ Ri[:, 0:2])
            B[6:9, nupc * i + 5] = dt * ai * Ri[:, 2]
        # d/dc [(p - c) x f] = [f]x
        A[6:9, 0:3] += dt * ai * skew(f)
        B[3:6, fcols] = dt * ai * np.eye(3, dtype=t)
        B[6:9, fcols] = dt * ai * skew(lever)
        C[6:9, 3 * i: 3 * i + 3] = -dt * ai * skew(f)
    return A, B, C


def lqr_gain(A, B, Q, R, niter=2, dtype=np.float64):
    """K = -(R + B'P B)^-1 B'P A after ``niter`` Riccati steps from P = Q.

    src/centroidal_model.py:217-228 (compute_lqr_feedback_gains / compute_DARE).
    """
    t = dtype
    A = np.asarray(A, t); B = np.asarray(B, t); Q = np.asarray(Q, t); R = np.asarray(R, t)
    P = Q.copy()
    for _ in range(niter):
        AtP = A.T @ P
        AtPA = AtP @ A
        AtPB = AtP @ B
        RBPB = R + B.T @ P @ B
        P = (Q + AtPA) - AtPB @ np.linalg.solve(RBPB, AtPB.T)
    return -np.linalg.solve(R + B.T @ P @ B, B.T @ P @ A)


def sigma_next(A, B, C, K, Sigma, cov_w, cov_eta, dtype=np.float64):
    """Covariance propagation, src/centroidal_model.py:234-238 (written as the reference does)."""
    t = dtype
    A, B, C, K, Sigma = (np.asarray(v, t) for v in (A, B, C, K, Sigma))
    S_Kt = Sigma @ K.T
    AB = np.hstack([A, B])
    S_xu = np.vstack([np.hstack([Sigma, S_Kt]), np.hstack([S_Kt.T, K @ S_Kt])])
    return AB @ S_xu @ AB.T + C @ np.asarray(cov_w, t) @ C.T + np.asarray(cov_eta, t)


def sigma_next_closed_loop(A, B, C, K, Sigma, cov_w, cov_eta, dtype=np.float64):
    """The same covariance step in the kernel's association (csrc/linearize.hip scan):
    Acl Sigma Acl' + (C cov_w C' + cov_eta) with Acl = A + B K.  Algebraically identical to
    ``sigma_next`` ([A B] [[S, S K'], [K S, K S K']] [A B]' = (A + B K) S (A + B K)'); the two
    roundings differ, and where A + B K has spectral radius ~1 (TALOS with the reference's warm
    start, quirk Q11) the scan amplifies that difference over the horizon."""
    t = dtype
    A, B, C, K, Sigma = (np.asarray(v, t) for v in (A, B, C, K, Sigma))
    Acl = A + B @ K
    Qw = C @ np.asarray(cov_w, t) @ C.T + np.asarray(cov_eta, t)
    return Acl @ Sigma @ Acl.T + Qw


def compute_trajectory_data(X, U, logic, pos, rot, prm, dtype=np.float64, assoc='reference'):
    """Per-knot linearization + LQR + covariance scan (src/centroidal_model.py:257-291).

    The reference also propagates Cov_dx / Cov_du tensors of shape (N+1, 9, 9, {9,nu}, N+1);
    they are identically zero (``Sigma_next_fun`` is a constant closure, :239-240), so the
    oracle returns them only when ``with_cov_grads`` is requested by a test.
    Returns dict(dynamics (9,N), LQR_gains (N,nu,9), f_x (N,9,9), f_u (N,9,nu),
    f_w (N,9,3nc), Covs (N+1,9,9)).  ``assoc='closed_loop'`` evaluates the covariance step in the
    kernel's association (``sigma_next_closed_loop``) instead of the reference's.
    """
    t = dtype
    N = U.shape[1]; nu = U.shape[0]; nc = prm['nc']
    dyn = np.zeros((9, N), t)
    K_all = np.zeros((N, nu, 9), t)
    fx = np.zeros((N, 9, 9), t); fu = np.zeros((N, 9, nu), t); fw = np.zeros((N, 9, 3 * nc), t)
    Covs = np.zeros((N + 1, 9, 9), t)
    for k in range(N):
        x, u = X[:, k], U[:, k]
        f = integrate_one_step(x, u, pos[k], logic[k], rot[k], prm, t)
        A, B, C = jacobians(x, u, pos[k], logic[k], rot[k], prm, t)
        K = lqr_gain(A, B, prm['Q'], prm['R'], 2, t)
        step = sigma_next if assoc == 'reference' else sigma_next_closed_loop
        Covs[k + 1] = step(A, B, C, K, Covs[k], prm['cov_w'], prm['cov_eta'], t)
        dyn[:, k] = f; fx[k] = A; fu[k] = B; fw[k] = C; K_all[k] = K
    return dict(dynamics=dyn, LQR_gains=K_all, f_x=fx, f_u=fu, f_w=fw, Covs=Covs)


def integrate_dynamics_trajectory(X, U, logic, pos, rot, prm, dtype=np.float64):
    """Nonlinear rollout for k = 0..N (src/centroidal_model.py:243-255).

    At k = N the reference indexes past the end of U and the contact arrays; JAX clamps
    the gather index, so the last control / contact row is reused (quirk Q9).
    """
    N1 = X.shape[1]; N = U.shape[1]
    out = np.zeros((X.shape[0], N1), dtype)
    for k in range(N1):
        kk = min(k, N - 1)
        out[:, k] = integrate_one_step(X[:, k], U[:, kk], pos[kk], logic[kk], rot[kk], prm, dtype)
    return out


def compute_model_accuracy(X_sol, U_sol, X_prev, U_prev, traj_data, logic, pos, rot, prm,
                           dtype=np.float64):
    """rho = sum ||nl[6:] - lin[6:]||^2 / sum ||lin||^2 over k < N (src/scp_solver.py:71-87)."""
    t = dtype
    nl = integrate_dynamics_trajectory(np.asarray(X_sol, t), np.asarray(U_sol, t), logic, pos, rot, prm, t)
    N = U_sol.shape[1]
    num = t(0.0); den = t(0.0)
    f_prev = np.asarray(traj_data['dynamics'], t)
    A_prev = np.asarray(traj_data['f_x'], t); B_prev = np.asarray(traj_data['f_u'], t)
    Xs = np.asarray(X_sol, t); Us = np.asarray(U_sol, t)
    Xp = np.asarray(X_prev, t); Up = np.asarray(U_prev, t)
    for k in range(N):
        dx = Xs[:, k] - Xp[:, k]
        du = Us[:, k] - Up[:, k]
        lin = f_prev[:, k] + A_prev[k] @ dx + B_prev[k] @ du
        err = nl[6:, k] - lin[6:]
        num += err @ err
        den += lin @ lin
    return num / den


def spectral_norm(M):
    """Largest singular value, as np.linalg.norm(M, 2) in src/scp_solver.py:151."""
    return float(np.linalg.norm(np.asarray(M, np.float64), 2))
