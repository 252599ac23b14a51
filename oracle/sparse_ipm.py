"""Oracle: generic sparse primal-dual interior-point QP solver.  TEST INFRASTRUCTURE.

An independent check on the GPU's structured interior-point kernel: it knows nothing about
stages, knots or the dual Schur complement; it factorizes the full regularized augmented KKT
matrix of   min 1/2 x'Px + q'x  s.t.  l <= Ax <= u   with scipy's sparse LU every iteration
(Mehrotra predictor-corrector).  Used where the OSQP restatement (``osqp_admm``, the
reference's algorithm) needs too many ADMM iterations for a tight answer (TALOS), and as a
second opinion elsewhere.  Returns the same Result(x, y, info) shape as ``osqp_admm``.
"""
import numpy as np
from scipy import sparse
from scipy.sparse.linalg import splu

from .osqp_admm import Info, Result


def solve_qp(P, q, A, l, u, eps=1e-11, max_iter=300, eta=0.99, reg=1e-12):
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
