"""Oracle: restatement of OSQP's published ADMM algorithm.  TEST INFRASTRUCTURE.

The reference solves every SCP subproblem with OSQP (src/scp_solver.py:59-68):
``osqp.OSQP().setup(P, q, A, l, u, warm_start=True, verbose=False, eps_abs=1e-7,
eps_rel=1e-7, polish=True); res = prob.solve()`` and accepts only status 'solved'.
OSQP is a third-party C library that is not vendored in /root/reference and is not
installed here (osqp-python, version unpinned: setup.py:2-6 has no install_requires; the
py3.8-era egg suggests 0.6.x).  This module restates its published algorithm
(Stellato et al., "OSQP: an operator splitting solver for quadratic programs", Math. Prog.
Comp. 2020; osqp 0.6 defaults):

* Ruiz equilibration of the KKT matrix (10 passes) plus cost scaling,
* ADMM with over-relaxation alpha = 1.6, sigma = 1e-6, rho = 0.1, rho_eq = 1e3 rho,
  rho_min = 1e-6 for free rows,
* residual-balancing adaptive rho (tolerance 5).  OSQP's default interval is derived
  from wall-clock timing (non-deterministic); the restatement uses a fixed interval,
* termination on unscaled residuals every ``check_termination`` (25) iterations,
* primal / dual infeasibility certificates,
* solution polishing on the guessed active set with 3 iterative-refinement steps.

The KKT system [P + sigma I, A'; A, -diag(1/rho)] is factorized with scipy's sparse LU.
"""
from collections import namedtuple

import numpy as np
from scipy import sparse
from scipy.sparse.linalg import splu

OSQP_INFTY = 1e30
MIN_SCALING = 1e-4
MAX_SCALING = 1e4
RHO_MIN = 1e-6
RHO_MAX = 1e6
RHO_EQ_OVER_RHO_INEQ = 1e3
RHO_TOL = 1e-4
DIV_TOL = 1e-20

Info = namedtuple('Info', 'status status_val iter obj_val pri_res dua_res rho_updates status_polish')
Result = namedtuple('Result', 'x y info')

STATUS = {1: 'solved', 2: 'solved inaccurate', -2: 'maximum iterations reached',
          -3: 'primal infeasible', -4: 'dual infeasible'}


def _limit(v):
    v = np.array(v, dtype=float, copy=True)
    v[v < MIN_SCALING] = 1.0
    v[v > MAX_SCALING] = MAX_SCALING
    return v


def _col_inf(M):
    M = abs(M).tocsc()
    out = np.zeros(M.shape[1])
    if M.nnz:
        out = np.asarray(M.max(axis=0).todense()).ravel()
    return out


class OSQPRestated:
    def __init__(self, P, q, A, l, u, rho=0.1, sigma=1e-6, alpha=1.6, scaling=10, max_iter=4000,
                 eps_abs=1e-7, eps_rel=1e-7, eps_prim_inf=1e-4, eps_dual_inf=1e-4,
                 adaptive_rho=True, adaptive_rho_interval=25, adaptive_rho_tolerance=5.0,
                 check_termination=25, polish=True, delta=1e-6, polish_refine_iter=3):
        self.n = P.shape[0]; self.m = A.shape[0]
        P = sparse.csc_matrix(P, dtype=float); A = sparse.csc_matrix(A, dtype=float)
        # OSQP keeps only the upper triangle of P and symmetrizes implicitly
        Pu = sparse.triu(P, format='csc')
        self.P_full = (Pu + sparse.triu(Pu, 1).T).tocsc()
        self.A = A.copy(); self.q = np.array(q, float)
        self.l = np.clip(np.array(l, float), -OSQP_INFTY, OSQP_INFTY)
        self.u = np.clip(np.array(u, float), -OSQP_INFTY, OSQP_INFTY)
        self.s = dict(rho=rho, sigma=sigma, alpha=alpha, max_iter=max_iter, eps_abs=eps_abs,
                      eps_rel=eps_rel, eps_prim_inf=eps_prim_inf, eps_dual_inf=eps_dual_inf,
                      adaptive_rho=adaptive_rho, adaptive_rho_interval=adaptive_rho_interval,
                      adaptive_rho_tolerance=adaptive_rho_tolerance, check_termination=check_termination,
                      polish=polish, delta=delta, polish_refine_iter=polish_refine_iter)
        self._scale(scaling)
        self.rho = rho
        self._set_rho_vec()
        self._factor()

    # ---- setup -------------------------------------------------------------------------
    def _scale(self, passes):
        n, m = self.n, self.m
        D = np.ones(n); E = np.ones(m); c = 1.0
        P = self.P_full.copy(); A = self.A.copy(); q = self.q.copy()
        for _ in range(passes):
            Dt = np.maximum(_col_inf(P), _col_inf(A)) if m else _col_inf(P)
            Et = _col_inf(A.T.tocsc()) if m else np.ones(0)
            Dt = 1.0 / np.sqrt(_limit(Dt)); Et = 1.0 / np.sqrt(_limit(Et))
            Dm = sparse.diags(Dt); Em = sparse.diags(Et)
            P = (Dm @ P @ Dm).tocsc(); A = (Em @ A @ Dm).tocsc(); q = Dt * q
            D *= Dt; E *= Et
            ct = float(np.mean(_col_inf(P))) if n else 1.0
            ct = _limit([ct])[0]
            qn = _limit([np.max(np.abs(q)) if n else 1.0])[0]
            ct = _limit([max(ct, qn)])[0]
            ct = 1.0 / ct
            P = P * ct; q = q * ct; c *= ct
        self.Ps, self.As, self.qs = P.tocsc(), A.tocsc(), q
        self.D, self.E, self.c = D, E, c
        self.Dinv, self.Einv, self.cinv = 1.0 / D, 1.0 / E, 1.0 / c
        self.ls = np.where(self.l > -OSQP_INFTY, E * self.l, -OSQP_INFTY)
        self.us = np.where(self.u < OSQP_INFTY, E * self.u, OSQP_INFTY)

    def _set_rho_vec(self):
        l, u = self.ls, self.us
        rv = np.full(self.m, self.rho)
        free = (l < -OSQP_INFTY * MIN_SCALING) & (u > OSQP_INFTY * MIN_SCALING)
        eq = (~free) & (u - l < RHO_TOL)
        rv[free] = RHO_MIN
        rv[eq] = RHO_EQ_OVER_RHO_INEQ * self.rho
        self.rho_vec = rv; self.rho_inv_vec = 1.0 / rv
        self.constr_type = np.where(free, -1, np.where(eq, 1, 0))

    def _factor(self):
        n = self.n
        K = sparse.bmat([[self.Ps + self.s['sigma'] * sparse.eye(n), self.As.T],
                         [self.As, -sparse.diags(self.rho_inv_vec)]], format='csc')
        self.lu = splu(K)

    # ---- helpers -----------------------------------------------------------------------
    def _residuals(self, x, z, y):
        Ax = self.As @ x; Px = self.Ps @ x; Aty = self.As.T @ y
        prim = np.max(np.abs(self.Einv * (Ax - z))) if self.m else 0.0
        eps_p = self.s['eps_abs'] + self.s['eps_rel'] * max(
            np.max(np.abs(self.Einv * Ax)) if self.m else 0.0, np.max(np.abs(self.Einv * z)) if self.m else 0.0)
        dual = self.cinv * np.max(np.abs(self.Dinv * (Px + self.qs + Aty)))
        eps_d = self.s['eps_abs'] + self.s['eps_rel'] * self.cinv * max(
            np.max(np.abs(self.Dinv * Px)), np.max(np.abs(self.Dinv * Aty)) if self.m else 0.0,
            np.max(np.abs(self.Dinv * self.qs)))
        return prim, eps_p, dual, eps_d

    def _rho_estimate(self, x, z, y):
        Ax = self.As @ x; Px = self.Ps @ x; Aty = self.As.T @ y
        pr = np.max(np.abs(Ax - z)) / (max(np.max(np.abs(Ax)), np.max(np.abs(z))) + DIV_TOL)
        dr = np.max(np.abs(Px + self.qs + Aty)) / (
            max(np.max(np.abs(Px)), np.max(np.abs(Aty)), np.max(np.abs(self.qs))) + DIV_TOL)
        est = self.rho * np.sqrt(pr / (dr + DIV_TOL))
        return float(np.clip(est, RHO_MIN, RHO_MAX))

    def _prim_infeasible(self, dy):
        eps = self.s['eps_prim_inf']
        ndy = np.max(np.abs(self.E * dy)) if self.m else 0.0
        if ndy < DIV_TOL:
            return False
        Atdy = self.Dinv * (self.As.T @ dy)
        if np.max(np.abs(Atdy)) > eps * ndy:
            return False
        ub = np.where(self.us < OSQP_INFTY * MIN_SCALING, self.us * np.maximum(dy, 0), 0.0).sum()
        lb = np.where(self.ls > -OSQP_INFTY * MIN_SCALING, self.ls * np.minimum(dy, 0), 0.0).sum()
        return ub + lb < -eps * ndy

    def _dual_infeasible(self, dx):
        eps = self.s['eps_dual_inf']
        ndx = np.max(np.abs(self.D * dx))
        if ndx < DIV_TOL:
            return False
        if self.qs @ dx >= -self.c * eps * ndx:
            return False
        if np.max(np.abs(self.Dinv * (self.Ps @ dx))) > self.c * eps * ndx:
            return False
        Adx = self.Einv * (self.As @ dx)
        tol = eps * ndx
        ok_u = np.where(self.us < OSQP_INFTY * MIN_SCALING, Adx <= tol, True)
        ok_l = np.where(self.ls > -OSQP_INFTY * MIN_SCALING, Adx >= -tol, True)
        return bool(np.all(ok_u & ok_l))

    # ---- solve ---------------------------------------------------------------------------
    def solve(self):
        s = self.s; n, m = self.n, self.m
        x = np.zeros(n); z = np.zeros(m); y = np.zeros(m)
        status = -2; it = 0; rho_updates = 0
        prim = dual = np.inf
        for it in range(1, s['max_iter'] + 1):
            x_prev, z_prev = x, z
            rhs = np.concatenate([s['sigma'] * x_prev - self.qs, z_prev - self.rho_inv_vec * y])
            sol = self.lu.solve(rhs)
            xt = sol[:n]; nu = sol[n:]
            zt = z_prev + self.rho_inv_vec * (nu - y)
            x = s['alpha'] * xt + (1 - s['alpha']) * x_prev
            zr = s['alpha'] * zt + (1 - s['alpha']) * z_prev
            z = np.clip(zr + self.rho_inv_vec * y, self.ls, self.us)
            dy = self.rho_vec * (zr - z)
            y = y + dy
            dx = x - x_prev
            if it % s['check_termination'] == 0 or it == s['max_iter']:
                prim, eps_p, dual, eps_d = self._residuals(x, z, y)
                if prim <= eps_p and dual <= eps_d:
                    status = 1
                    break
                if self._prim_infeasible(dy):
                    status = -3
                    break
                if self._dual_infeasible(dx):
                    status = -4
                    break
            if s['adaptive_rho'] and s['adaptive_rho_interval'] and it % s['adaptive_rho_interval'] == 0:
                est = self._rho_estimate(x, z, y)
                if est > self.rho * s['adaptive_rho_tolerance'] or est < self.rho / s['adaptive_rho_tolerance']:
                    self.rho = est; self._set_rho_vec(); self._factor(); rho_updates += 1
        if status == -2:
            prim, eps_p, dual, eps_d = self._residuals(x, z, y)
            if prim <= 10 * eps_p and dual <= 10 * eps_d:
                status = 2
        status_polish = 0
        if s['polish'] and status == 1:
            px, pz, py, ok = self._polish(x, z, y, prim, dual)
            if ok:
                x, z, y = px, pz, py; status_polish = 1
                prim, _, dual, _ = self._residuals(x, z, y)
            else:
                status_polish = -1
        xu = self.D * x; yu = self.cinv * self.E * y
        obj = 0.5 * xu @ (self.P_full @ xu) + self.q @ xu
        info = Info(STATUS[status], status, it, obj, prim, dual, rho_updates, status_polish)
        return Result(xu, yu, info)

    def _polish(self, x, z, y, prim, dual):
        n = self.n; d = self.s['delta']
        low = (z - self.ls < -y); upp = (self.us - z < y)
        idx_l = np.nonzero(low)[0]; idx_u = np.nonzero(upp)[0]
        Ared = sparse.vstack([self.As[idx_l], self.As[idx_u]], format='csc')
        mr = Ared.shape[0]
        K = sparse.bmat([[self.Ps + d * sparse.eye(n), Ared.T], [Ared, -d * sparse.eye(mr)]], format='csc')
        K0 = sparse.bmat([[self.Ps, Ared.T], [Ared, None]], format='csc') if mr else self.Ps
        b = np.concatenate([-self.qs, self.ls[idx_l], self.us[idx_u]])
        lu = splu(K)
        sol = lu.solve(b)
        for _ in range(self.s['polish_refine_iter']):
            sol = sol + lu.solve(b - K0 @ sol)
        px = sol[:n]; yr = sol[n:]
        py = np.zeros(self.m); py[idx_l] = yr[:len(idx_l)]; py[idx_u] = yr[len(idx_l):]
        pz = np.clip(self.As @ px, self.ls, self.us)
        pp, _, pd, _ = self._residuals(px, pz, py)
        ok = (pp < prim and pd < dual) or (pp < prim and dual < 1e-10) or (pd < dual and prim < 1e-10)
        return px, pz, py, ok


def solve_qp(P, q, A, l, u, **settings):
    """OSQP().setup(...).solve() equivalent; returns Result(x, y, info)."""
    return OSQPRestated(P, q, A, l, u, **settings).solve()
