"""Oracle: solver-independent KKT residuals for  min 1/2 z'Pz + q'z  s.t.  l <= Az <= u.  TEST INFRASTRUCTURE.

Used to pin any QP answer (GPU, oracle ADMM) without trusting the solver that produced it.
The QP of the reference has a unique (x, u, t) minimizer (P > 0 on x and u; t is pinned by its
positive linear cost; the control slacks s have zero cost and no rows), so two solutions with
small KKT residuals agree on (x, u, t).
"""
import numpy as np


def kkt_residuals(P, q, A, l, u, z, y=None):
    """Returns dict(prim, dual, compl, sign) in the infinity norm.

    prim: bound violation of Az;  dual: ||Pz + q + A'y||;  compl: max over rows of
    |y_i| * distance of (Az)_i to the bound y_i pushes against.  If y is None the
    multipliers are recovered by a least-squares fit on the rows within 1e-6 of a bound
    (a certificate, not a solver)."""
    z = np.asarray(z, float)
    Az = A @ z
    viol = np.maximum(Az - u, 0) + np.maximum(l - Az, 0)
    prim = float(np.max(np.abs(viol))) if viol.size else 0.0
    g = P @ z + q
    if y is None:
        tol = 1e-6 * (1 + np.abs(Az))
        act = (np.abs(Az - u) <= tol) | (np.abs(Az - l) <= tol)
        idx = np.nonzero(act)[0]
        y = np.zeros(A.shape[0])
        if idx.size:
            At = A[idx].T.toarray()
            sol, *_ = np.linalg.lstsq(At, -g, rcond=None)
            y[idx] = sol
    dual = float(np.max(np.abs(g + A.T @ y)))
    yp = np.maximum(y, 0.0); ym = np.maximum(-y, 0.0)
    fu = np.isfinite(u); fl = np.isfinite(l)
    comp = np.zeros_like(y)
    comp[fu] += yp[fu] * np.abs(u[fu] - Az[fu])
    comp[fl] += ym[fl] * np.abs(Az[fl] - l[fl])
    # a multiplier pushing against an infinite bound is a dual sign violation
    sign = float(max(np.max(yp[~fu], initial=0.0), np.max(ym[~fl], initial=0.0)))
    return dict(prim=prim, dual=dual, compl=float(np.max(comp, initial=0.0)), sign=sign, y=y)
