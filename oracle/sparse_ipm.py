"""Oracle: generic sparse primal-dual interior-point QP solver.  TEST INFRASTRUCTURE.

An independent check on the GPU's structured interior-point kernel: it knows nothing about
stages, knots or the dual Schur complement; it factorizes the full regularized augmented KKT
matrix of   min 1/2 x'Px + q'x  s.t.  l <= Ax <= u   with scipy's sparse LU every iteration
(Mehrotra predictor-corrector), then (polish=True) solves the equality-constrained QP on the
identified active set exactly and keeps it when it verifies (``_polish``).  Used where the OSQP
restatement (``osqp_admm``, the reference's algorithm) needs too many ADMM iterations for a tight
answer (TALOS), and as a second opinion elsewhere.  Returns the same Result(x, y, info) shape as ``osqp_admm``.
"""
import numpy as np
from scipy import sparse
from scipy.sparse.linalg import splu

from .osqp_admm import Info, Result


def _polish(P, q, Ae, be, G, h, x, s, z, eps, sc_p, sc_d):
    """The equality-constrained QP on the active set of the converged iterate (rows whose multiplier
    exceeds their slack), solved exactly with a sparse LU of its KKT matrix (plus two refinement
    steps); kept when every active multiplier is >= -eps * sc_d and every inactive row holds to
    eps * sc_p.  On degenerate problems (the objective nearly flat along some direction, as on Solo12
    trot) the interior-point iterate alone can sit 1e-5 away from the minimizer while its KKT
    residuals are small; the polished point is the minimizer itself.  Returns (x, yv, z) or None."""
    n, me = P.shape[0], Ae.shape[0]
    act = z > s
    Ga = G[act]
    ma = Ga.shape[0]
    K = sparse.bmat([[P, Ae.T, Ga.T], [Ae, None, None], [Ga, None, None]], format='csc')
    Kr = K + sparse.diags(np.concatenate([np.full(n, 1e-14), np.full(me + ma, -1e-14)]))
    rhs = np.concatenate([-q, be, h[act]])
    try:
        lu = splu(Kr.tocsc())
    except RuntimeError:
        return None
    sol = lu.solve(rhs)
    for _ in range(3):
        sol = sol + lu.solve(rhs - K @ sol)
    if not np.all(np.isfinite(sol)):
        return None
    xp, ye, za = sol[:n], sol[n:n + me], sol[n + me:]
    zp = np.zeros_like(z)
    zp[act] = za
    viol = G[~act] @ xp - h[~act] if (~act).any() else np.zeros(0)
    if (za.min() if ma else 0.0) < -eps * sc_d or (viol.max() if viol.size else 0.0) > eps * sc_p:
        return None
    return xp, ye, zp


def solve_qp(P, q, A, l, u, eps=1e-11, max_iter=300, eta=0.99, reg=1e-12, polish=True):
    P = sparse.csc_matrix(P); A = sparse.csr_matrix(A)
    n, m = P.shape[0], A.shape[0]
    l = np.asarray(l, float); u = np.asarray(u, float)
    eq = np.isfinite(l) & np.isfinite(u) & (np.abs(u - l) <= 1e-9)
    up = np.isfinite(u) & ~eq
    lo = np.isfinite(l) & ~eq
    nz = np.asarray(abs(A).sum(axis=1)).ravel() > 0
    up &= nz; lo &= nz                          # all-zero rows (e.g. unfilled friction rows) are trivial
    Ae = A[eq]; be = 0.5 * (l[eq] + u[eq])
    G = sparse.vstack([A[up], -A[lo]]).tocsr(); h = np.concatenate([u[up], -l[lo]])
    me, mi = Ae.shape[0], G.shape[0]
    x = np.zeros(n); yv = np.zeros(me); s = np.maximum(h - G @ x, 1.0); z = np.ones(mi)
    status = -2
    it = 0
    for it in range(max_iter):
        rd = P @ x + q + Ae.T @ yv + G.T @ z
        re = Ae @ x - be
        ri = G @ x + s - h
        mu = s @ z / max(mi, 1)
        sc_d = max(1.0, np.abs(P @ x).max(), np.abs(q).max())
        sc_p = max(1.0, np.abs(be).max() if me else 1.0, np.abs(h).max() if mi else 1.0)
        if (np.abs(rd).max() <= eps * sc_d and (np.abs(re).max() if me else 0) <= eps * sc_p
                and (np.abs(ri).max() if mi else 0) <= eps * sc_p and (s * z).max() <= eps * sc_d):
            status = 1
            if polish:   # the exact minimizer on the identified active set, when it verifies
                pol = _polish(P, q, Ae, be, G, h, x, s, z, eps * 1e3, sc_p, sc_d)
                if pol is not None:
                    x, yv, z = pol
            break
        D = z / s
        H = (P + G.T @ sparse.diags(D) @ G).tocsc()
        K = sparse.bmat([[H + reg * sparse.eye(n), Ae.T], [Ae, -reg * sparse.eye(me)]], format='csc')
        K0 = sparse.bmat([[H, Ae.T], [Ae, None]], format='csc')
        lu = splu(K)

        def newton(rc):
            rhs1 = -(rd + G.T @ (D * ri - rc / s))
            sol = lu.solve(np.concatenate([rhs1, -re]))
            for _ in range(2):   # iterative refinement against the unregularized system
                res = np.concatenate([rhs1, -re]) - K0 @ sol
                sol = sol + lu.solve(res)
            dx = sol[:n]; dy = sol[n:]
            dz = D * (G @ dx + ri) - rc / s
            ds = -ri - G @ dx
            return dx, dy, dz, ds

        def step(v, dv):
            neg = dv < 0
            return min(1.0, float(np.min(-v[neg] / dv[neg]))) if np.any(neg) else 1.0

        dx, dy, dz, ds = newton(s * z)
        a = min(step(s, ds), step(z, dz))
        sigma = (((s + a * ds) @ (z + a * dz)) / max(mi, 1) / max(mu, 1e-300)) ** 3
        dx, dy, dz, ds = newton(s * z + ds * dz - sigma * mu)
        a = min(1.0, eta * min(step(s, ds), step(z, dz)))
        x += a * dx; yv += a * dy; z += a * dz; s += a * ds
    y = np.zeros(m)
    y[np.nonzero(eq)[0]] = yv
    zi = z[:up.sum()]; zl = z[up.sum():]
    y[np.nonzero(up)[0]] += zi
    y[np.nonzero(lo)[0]] -= zl
    obj = 0.5 * x @ (P @ x) + q @ x
    st = {1: 'solved', -2: 'maximum iterations reached'}[status]
    return Result(x, y, Info(st, status, it, obj, 0.0, 0.0, 0, 0))
