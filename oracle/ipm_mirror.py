"""CPU mirror of the GPU structured interior-point QP (same algorithm, numpy).  TEST INFRASTRUCTURE.

This is NOT a restatement of the reference; it mirrors the algorithm of the GPU kernel
(centroidal-mpc_amd/csrc/qp_ipm.hip) step by step so that a GPU mismatch can be localized
to one phase.  Parity of the GPU answer itself is checked against ``osqp_admm`` (the
reference's algorithm) and the solver-independent ``kkt`` residuals.

Structured QP per problem (all blocks per knot k):
  min  sum_k 1/2 x_k'Wx x_k + qx_k'x_k + t_k + sum_{k<N} 1/2 u_k'Wu u_k
  s.t. x_0 = xbar_0;  A_k x_k + B_k u_k - x_{k+1} = r_k (k<N);  x_N = xbar_N
       TR:   s_j'L_k + cw t_k <= btr_kj  (j<8),  -t_k <= 0          (L = x[6:9], cw = -1/omega)
       fric: G_kij' f_ki <= h_kij (active contacts, j<4)
       CoP:  lo <= cop_kid <= hi (TALOS, active contacts)
Mehrotra predictor-corrector.  The Newton system is reduced to the dual Schur complement
S = E Phi^-1 E' (Phi = H + G'DG is block diagonal per knot; t is eliminated in each knot),
which is block tridiagonal with N+2 blocks of 9x9 and is factorized by block Cholesky.

Exits (the kernel's status codes, OSQP's values): 1 solved (merit <= 1); 2 solved inaccurate
(the stall guard: mu not halving for 3 iterations within 1e3 of the tolerance; the host maps it
to a failure as the reference does for OSQP's 'solved inaccurate', src/scp_solver.py:65-67);
-3 primal infeasible (Farkas certificate from the multipliers, below); -2 iteration cap;
-10 non-finite.  Dual infeasibility cannot occur: P > 0 on (x, u) and the only other variable t
has cost +1 and t >= 0, so no recession direction lowers the cost.

Iterative refinement: near the solution of a degenerate QP (a force pinned by three or four
active pyramid rows, D = lambda / s ~ 1e9) the push-through solves and the Schur factorization
lose digits, and the corrector direction stops satisfying its own linear system (TALOS N=200
problem 280 at its second SCP iteration: the friction rows' linearized complementarity residual
reaches 3e-5 against mu = 7e-6, the step length collapses to 3e-4 and mu stalls).  When the
corrector's step length is below ``refine_alpha``, or mu did not halve in the previous iteration,
late in the solve (merit < ``refine_merit``),
the residual of the full Newton system is formed with the exact operators and one correction
is solved with the same factorization (one refinement step).
"""
import numpy as np

PENUM = np.array([[(-1) ** (j // (2 ** i)) for i in range(3)] for j in range(8)], float)


class StructQP:
    """Structured subproblem (built by ``from_arrays``)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    @staticmethod
    def from_arrays(N, robot, nc, Wx, Wu, Xbar, Ubar, A, Bm, f, logic, rot, mu, weight, radius,
                    tracking=True, fric_h=None, foot_range=(0.01, 0.01, 0.01, 0.01)):
        """Xbar (N+1,9), Ubar (N,nu), A (N,9,9), Bm (N,9,nu), f (N,9), logic (N,nc), rot (N,nc,3,3)."""
        nu = Ubar.shape[1]
        r = np.einsum('kij,kj->ki', A, Xbar[:N]) + np.einsum('kij,kj->ki', Bm, Ubar) - f
        ml = mu / np.sqrt(2)
        Fmu = np.array([[1., 0., -ml], [-1., 0., -ml], [0., 1., -ml], [0., -1., -ml]])
        G = np.einsum('rj,kimj->kirm', Fmu, rot)          # F_mu R^T  -> (N, nc, 4, 3)
        if fric_h is None:
            fric_h = np.zeros((N, nc, 4))
        qx = -(Wx[None, :] * Xbar) if tracking else np.zeros_like(Xbar)
        btr = radius + Xbar[:, 6:9] @ PENUM.T               # (N+1, 8)
        return StructQP(N=N, robot=robot, nc=nc, nu=nu, nupc=nu // nc, Wx=np.asarray(Wx, float),
                        Wu=np.asarray(Wu, float), qx=qx, A=A, Bm=Bm, r=r, x0=Xbar[0].copy(),
                        xN=Xbar[N].copy(), btr=btr, cw=-1.0 / weight, G=G, fh=fric_h,
                        fmask=logic.astype(bool), foot_range=foot_range, Xbar=Xbar, Ubar=Ubar)


def _chol_floor(S, floor):
    """Cholesky with a pivot floor (modified Cholesky): near the solution of a degenerate QP
    the last Schur blocks are differences of O(M) numbers and may lose positivity by rounding."""
    n = S.shape[0]
    L = np.zeros_like(S)
    for c in range(n):
        d2 = S[c, c] - L[c, :c] @ L[c, :c]
        d = np.sqrt(max(d2, floor[c]))
        L[c, c] = d
        L[c + 1:, c] = (S[c + 1:, c] - L[c + 1:, :c] @ L[c, :c]) / d
    return L


def max_step(v, dv, mk):
    """Largest step in (0, 1] keeping v + a dv >= 0 on the rows of mask mk."""
    neg = (dv < 0) & (mk > 0)
    if not np.any(neg):
        return 1.0
    return min(1.0, float(np.min(-v[neg] / dv[neg])))


def _fslot(qp):
    return 0 if qp.robot == 'solo12' else 2


INIT_FLOOR = 0.1          # s floor of the Solo12 starting point
INIT_FLOOR_L = 0.1        # lambda floor


def robot_defaults(qp):
    """The kernel's default fp64 stopping and polishing tolerances for the QP's robot (cmpc_api.cpp
    qp_eps_default / qp_polish_eps): eps 1e-10; Solo12 polishes at 1e-7, TALOS not (0; the mirror's
    tests of TALOS polishing pass their own tolerance)."""
    return (1e-10, 1e-7) if qp.robot == 'solo12' else (1e-10, 0.0)


def solve(qp, eps=1e-11, max_iter=60, eta=0.999, verbose=False, reg=0.0, piv_floor=1e-13, dcap_rel=1e12,
          refine_alpha=0.5, refine_merit=1e6, eps_pinf=1e-4, init_floor=INIT_FLOOR,
          init_floor_l=INIT_FLOOR_L, fric_floor=1e-9, polish=False, polish_eps=None, polish_rel=1e-14,
          comp_primal=None):
    if polish_eps is None:
        polish_eps = eps
    N, nc, nu, nupc = qp.N, qp.nc, qp.nu, qp.nupc
    fo = _fslot(qp)
    talos = qp.robot != 'solo12'
    # ---- variables ----
    x = qp.Xbar.copy(); u = qp.Ubar.copy(); t = np.zeros(N + 1); nu_ = np.zeros((N + 2, 9))
    fm = qp.fmask[:, :, None].astype(float) * np.ones((1, 1, 4))        # (N, nc, 4)
    cm = qp.fmask[:, :, None, None].astype(float) * np.ones((1, 1, 2, 2)) if talos else None
    lxp, lxn, lyp, lyn = qp.foot_range
    cop_hi = np.array([lxp, lyp]); cop_lo = np.array([-lxn, -lyn])

    def ineq_val(x, u, t):
        """g'z - h for every inequality (so feasibility is <= 0)."""
        L = x[:, 6:9]
        v_tr = L @ PENUM.T + qp.cw * t[:, None] - qp.btr
        v_sl = -t
        f = u.reshape(N, nc, nupc)[:, :, fo:fo + 3]
        v_fr = np.einsum('kirm,kim->kir', qp.G, f) - qp.fh
        out = [v_tr, v_sl, v_fr]
        if talos:
            cop = u.reshape(N, nc, nupc)[:, :, 0:2]
            v_cp = np.stack([cop - cop_hi, -cop + cop_lo], axis=3)         # (N, nc, 2dim, 2side)
            out.append(v_cp)
        return out

    masks = [np.ones((N + 1, 8)), np.ones(N + 1), fm] + ([cm] if talos else [])
    vals = ineq_val(x, u, t)
    s = [np.where(mk > 0, np.maximum(-v, 1.0), 1.0) for v, mk in zip(vals, masks)]
    lam = [mk * 1.0 for mk in masks]
    m_tot = sum(mk.sum() for mk in masks)

    def GT(lams):
        """G' lambda split into (x (N+1,9), t (N+1,), u (N,nu))."""
        gx = np.zeros((N + 1, 9)); gt = np.zeros(N + 1); gu = np.zeros((N, nc, nupc))
        gx[:, 6:9] = lams[0] @ PENUM
        gt += qp.cw * lams[0].sum(axis=1) - lams[1]
        gu[:, :, fo:fo + 3] = np.einsum('kirm,kir->kim', qp.G, lams[2])
        if talos:
            gu[:, :, 0:2] += lams[3][..., 0] - lams[3][..., 1]
        return gx, gt, gu.reshape(N, nu)

    def Gz(dx, du, dt_):
        L = dx[:, 6:9]
        out = [L @ PENUM.T + qp.cw * dt_[:, None], -dt_,
               np.einsum('kirm,kim->kir', qp.G, du.reshape(N, nc, nupc)[:, :, fo:fo + 3])]
        if talos:
            cop = du.reshape(N, nc, nupc)[:, :, 0:2]
            out.append(np.stack([cop, -cop], axis=3))
        return out

    def ET(nv):
        ex = np.zeros((N + 1, 9)); eu = np.zeros((N, nu))
        ex[0] += nv[0]
        ex[:N] += np.einsum('kji,kj->ki', qp.A, nv[1:N + 1])
        ex[1:N + 1] -= nv[1:N + 1]
        ex[N] += nv[N + 1]
        eu += np.einsum('kji,kj->ki', qp.Bm, nv[1:N + 1])
        return ex, eu

    def Ez(x, u):
        e = np.zeros((N + 2, 9))
        e[0] = x[0]
        e[1:N + 1] = np.einsum('kij,kj->ki', qp.A, x[:N]) + np.einsum('kij,kj->ki', qp.Bm, u) - x[1:]
        e[N + 1] = x[N]
        return e

    e_rhs = np.zeros((N + 2, 9)); e_rhs[0] = qp.x0; e_rhs[1:N + 1] = qp.r; e_rhs[N + 1] = qp.xN
    it = 0; status = -2
    hist = []
    s = [mk * 1.0 + (1 - mk) for mk in masks]
    lam = [mk * 1.0 for mk in masks]
    stall = 0; mu_prev = None
    polished_try = False; polish_log = []; last = None
    system_at = lambda *a_: system(*a_)   # (bound below, once per iteration)
    n_refine = 0; merit = np.inf; prim_prev = 0.0
    hs = [qp.btr, np.zeros(N + 1), qp.fh]
    if talos:
        hs.append(np.stack([np.broadcast_to(cop_hi, (N, nc, 2)), np.broadcast_to(-cop_lo, (N, nc, 2))], axis=3))
    for it in range(0, max_iter + 1):
        # iteration 0 is the initialization step: one full Newton step from s = lambda = 1 (an
        # equality-constrained least-squares start).  Solo12: s and lambda are then floored row
        # by row at INIT_FLOOR / INIT_FLOOR_L.  TALOS: CVXOPT's shift of every row by 1 + the largest violation.
        # On Solo12 the shift starts at mu ~ 700, far from the central path (trot N=100: 9.3
        # Newton steps on average, 5.3 with the floors); on TALOS the floors were not robust
        # (N=40: 22-24 steps against 18, one stall).
        init = it == 0
        # ---- residuals ----
        gx, gt, gu = GT(lam)
        ex, eu = ET(nu_)
        rdx = qp.Wx * x + qp.qx + ex + gx
        rdt = 1.0 + gt
        rdu = qp.Wu * u + eu + gu
        rde = Ez(x, u) - e_rhs
        vals = ineq_val(x, u, t)
        rdi = [(v + si) * mk for v, si, mk in zip(vals, s, masks)]
        mu_ = sum((si * li * mk).sum() for si, li, mk in zip(s, lam, masks)) / m_tot
        # ---- termination (OSQP-style relative criteria on the reference problem) ----
        prim = max(np.abs(rde).max(), max(np.maximum(v * mk, 0).max() for v, mk in zip(vals, masks)))
        dual = max(np.abs(rdx).max(), np.abs(rdt).max(), np.abs(rdu).max())
        comp = max((si * li * mk).max() for si, li, mk in zip(s, lam, masks))
        # the kernel's scales (qp_ipm.hip resid_knot: nm.sp, nm.sd): primal -- the dynamics and
        # boundary rows' terms and every present inequality row's |g'z| and |h|; dual -- every term
        # of the dual rows (W z, q, E' nu, G' lambda)
        ineq_sc = max(float(np.max(np.where(mk > 0, np.maximum(np.abs(v + h), np.abs(np.broadcast_to(h, v.shape))), 0)))
                      for v, h, mk in zip(vals, hs, masks))
        scale_p = max(np.abs(Ez(x, u)).max(), np.abs(e_rhs).max(), np.abs(x[0]).max(), np.abs(x[N]).max(), ineq_sc, 1.0)
        scale_d = max(np.abs(qp.Wx * x).max(), np.abs(qp.qx).max(), np.abs(ex).max(), np.abs(gx).max(),
                      np.abs(qp.Wu * u).max(), np.abs(eu).max(), np.abs(gu).max(), 1.0)
        # complementarity against the primal scale on Solo12, the dual scale on TALOS (qp_ipm.hip
        # COMP_PRIMAL_SCALE)
        # (Solo12: 10x the primal tolerance once a polish was rejected, or with polishing off)
        strict = (comp_primal if comp_primal is not None else
                  (not talos and (not polish or any(pl['status'] < 0 for pl in polish_log))))
        scale_c = 10.0 * scale_p if strict else scale_d
        hist.append((it, prim, dual, comp, mu_))
        if verbose:
            print('it %2d prim %.2e dual %.2e comp %.2e mu %.2e' % (it, prim, dual, comp, mu_))
        merit = max(prim / (eps * scale_p), dual / (eps * scale_d), comp / (eps * scale_c))
        if not (merit == merit):
            status = -10
            break
        if not init and merit <= 1.0:
            status = 1
            break
        # (the kernel's second attempt after a rejected guess, once the dual-scale test at eps holds)
        if strict and polish and len(polish_log) == 1 and not init and \
                max(prim / (eps * scale_p), dual / (eps * scale_d), comp / (eps * scale_d)) <= 1.0:
            pol = _polish(qp, masks, x, u, t, nu_, s, lam, last, system_at, GT, ET, Ez, ineq_val, e_rhs,
                          polish_eps, talos, polish_rel)
            polish_log.append(pol)
            if pol['status'] == 1:
                x, u, t, nu_, lam, s = pol['x'], pol['u'], pol['t'], pol['nu'], pol['lam'], pol['s']
                status = 1
                break
        # solution polishing once the iterate meets eps_polish (looser than eps): accepted -> done;
        # rejected -> the interior-point iterations go on to eps
        if polish and not polished_try and not init and it > 1 and merit * eps / polish_eps <= 1.0:
            polished_try = True
            pol = _polish(qp, masks, x, u, t, nu_, s, lam, last, system_at, GT, ET, Ez, ineq_val, e_rhs,
                          polish_eps, talos, polish_rel)
            polish_log.append(pol)
            if pol['status'] == 1:
                x, u, t, nu_, lam, s = pol['x'], pol['u'], pol['t'], pol['nu'], pol['lam'], pol['s']
                status = 1
                break
        # primal infeasibility (Farkas): E'nu + G'lambda -> 0 relative to |(nu, lambda)| while
        # b'nu + h'lambda < 0 (OSQP's test, on the multipliers, which diverge along the certificate)
        # (evaluated, as in the kernel, once the primal residual stagnates away from the solution)
        if not init and it >= 3 and prim > 0.9 * prim_prev and merit > 1e3:
            ay = max(np.abs(ex + gx).max(), np.abs(gt).max(), np.abs(eu + gu).max())
            cy = float((e_rhs * nu_).sum() + sum((h * l * mk).sum() for h, l, mk in zip(hs, lam, masks)))
            ny = max(np.abs(nu_).max(), max(float(l.max()) for l in lam))
            if ay <= eps_pinf * ny and cy <= -eps_pinf * ny:
                status = -3
                break
        prim_prev = prim
        # stall guard: mu no longer decreasing for 3 iterations while within 1e3x of tolerance;
        # reported as 'solved inaccurate' (2), which the SCP loop treats as a failed QP
        stall = stall + 1 if (not init and mu_prev is not None and mu_ >= 0.5 * mu_prev) else 0
        mu_prev = None if init else mu_
        if stall >= 3 and merit <= 1e3:
            status = 2
            break
        # ---- factorization ----
        def system(s, lam, rdx, rdt, rdu, rde, rdi):
            """Factorization of the Newton system at (s, lam); returns newton(rc, ...) and lin_res."""
            D = [li / si * mk for li, si, mk in zip(lam, s, masks)]
            # cap D on the rows handled in D-form (TR, slack, CoP): beyond ~1e12 x the stage
            # curvature the products D * r lose all precision; the capped Newton step is an inexact
            # Newton step on exact residuals (convergence is driven by the residuals)
            dcap = dcap_rel * max(float(np.max(qp.Wx)), 1.0)
            if talos:
                D[3] = np.minimum(D[3], dcap)
            # x/t block: Phi_LL, Phi_Lt, Phi_tt
            # (L, t) block in push-through form.  Unknowns dL (3), dt, dlam_TR (8), dlam_sl:
            #   W dL + G' dlam = vL ;  cw 1'dlam - dlam_sl = vt ;  G dL + cw 1 dt - D^-1 dlam = -rh ;
            #   -dt - D_sl^-1 dlam_sl = -rh_sl
            # eliminated with K = D_TR^-1 + G W^-1 G' (8x8 SPD, floored), k = K^-1 1, kap = 1'k:
            #   dt = (vt + D_sl rh_sl - cw 1'K^-1 a) / (D_sl + cw^2 kap),  a = G W^-1 vL + rh
            #   dlam = K^-1 a + cw dt k ;  dL = W^-1 (vL - G'dlam) ;  dlam_sl = cw 1'dlam - vt
            WLi = 1.0 / qp.Wx[6:9]
            YL = PENUM * WLi[None, :]                                  # G W^-1 (8x3)
            GWG_tr = PENUM @ YL.T                                       # (8x8)
            DinvT = np.where(D[0] > 0, 1.0 / np.maximum(D[0], 1e-300), 1e300)
            kfl = 1e-12 * np.trace(GWG_tr)
            Ktr = GWG_tr[None] + np.maximum(DinvT, kfl)[:, :, None] * np.eye(8)[None]
            Ktr_inv = np.linalg.inv(Ktr)                                # (N+1,8,8)
            kvec = Ktr_inv.sum(axis=2)                                  # K^-1 1
            kap = kvec.sum(axis=1)
            Dsl = D[1]
            den = Dsl + qp.cw ** 2 * kap
            Pm = Ktr_inv - qp.cw ** 2 * np.einsum('ka,kb->kab', kvec, kvec) / den[:, None, None]
            ML = np.diag(WLi)[None] - np.einsum('ja,kjl,lb->kab', YL, Pm, YL)
            Mfull = np.zeros((N + 1, 9, 9))
            Mfull[:, np.arange(6), np.arange(6)] = 1.0 / qp.Wx[:6]
            Mfull[:, 6:9, 6:9] = ML
            # u blocks, computed stably (D can reach 1e15+): with K = D^-1 + G W^-1 G' (4x4 SPD),
            # Phi_u^-1 = W^-1 - W^-1 G' K^-1 G W^-1 and Phi_u^-1 G' D = W^-1 G' K^-1 (push-through).
            Wu_b = qp.Wu.reshape(nc, nupc)
            Winv = np.zeros((N, nc, nupc, nupc)) + np.stack([np.diag(1.0 / Wu_b[i]) for i in range(nc)])[None]
            if talos:
                # CoP rows are bound rows on single coordinates: fold them into the diagonal
                # (D <= 1/lo-side slack, bounded by the box width, so no cancellation)
                dcop = D[3].sum(axis=3)                                   # (N, nc, 2)
                for d in range(2):
                    Winv[:, :, d, d] = 1.0 / (Wu_b[None, :, d] + dcop[:, :, d])
            Gw = np.einsum('kirm,kimn->kirn', qp.G, Winv[:, :, fo:fo + 3, fo:fo + 3])    # G W^-1 (N,nc,4,3)
            Dinv_f = np.where(fm > 0, s[2] / np.where(fm > 0, lam[2], 1.0), 1.0)
            GWG = np.einsum('kirn,kiqn->kirq', Gw, qp.G)
            # floor on D^-1: at a zero force all four pyramid rows are active (degenerate, K -> rank 3);
            # kernel KFLOOR_FR (1e-9; 1e-12 before round 2's TALOS weight cases)
            kfloor = fric_floor * np.trace(GWG, axis1=2, axis2=3)[..., None] + 1e-300
            Kf = GWG + np.maximum(Dinv_f, kfloor)[..., None] * np.eye(4)
            Kf = np.where(fm[..., None] > 0, Kf, np.eye(4))                 # inactive contacts: identity
            Gw = Gw * fm[..., None]
            Kf_inv = np.linalg.inv(Kf)
            Phiuinv = Winv.copy()
            Phiuinv[:, :, fo:fo + 3, fo:fo + 3] -= np.einsum('kirn,kirq,kiqm->kinm', Gw, Kf_inv, Gw)
            # S blocks
            Sd = np.zeros((N + 2, 9, 9)); So = np.zeros((N + 1, 9, 9))
            Sd[0] = Mfull[0]
            Bblk = qp.Bm.reshape(N, 9, nc, nupc)
            BPB = np.einsum('kaic,kicd,kbid->kab', Bblk, Phiuinv, Bblk)
            Sd[1:N + 1] = np.einsum('kai,kij,kbj->kab', qp.A, Mfull[:N], qp.A) + BPB + Mfull[1:]
            Sd[N + 1] = Mfull[N]
            So[0] = Mfull[0] @ qp.A[0].T
            So[1:N] = -np.einsum('kij,kbj->kib', Mfull[1:N], qp.A[1:N])
            So[N] = -Mfull[N]
            # block Cholesky: Lc[j] lower, Lo[j] = S_{j+1,j} Lc[j]^-T
            Lc = np.zeros_like(Sd); Lo = np.zeros_like(So)
            # tiny diagonal regularization of each Schur block: the last blocks are differences of
            # O(M) numbers once the forces are pinned by active rows (cancellation), see DESIGN.md
            for j in range(N + 2):
                Sd[j] += reg * np.trace(Sd[j]) / 9 * np.eye(9)
            Sh = Sd[0].copy()
            for j in range(N + 2):
                Lc[j] = _chol_floor(Sh, piv_floor * np.diag(Sd[j]))
                if j < N + 1:
                    Lo[j] = np.linalg.solve(Lc[j], So[j]).T        # (S_{j,j+1})^T Lc^-T
                    Sh = Sd[j + 1] - Lo[j] @ Lo[j].T

            def tr_local(vL, vt, rh_tr, rh_sl):
                """(dL, dt, dlam_TR, dlam_sl) of the (L, t) block (see the factorization)."""
                a = vL @ YL.T + rh_tr                                   # (N+1, 8)
                ka = np.einsum('kab,kb->ka', Ktr_inv, a)
                dt_ = (vt + Dsl * rh_sl - qp.cw * ka.sum(axis=1)) / den
                dlt = ka + qp.cw * dt_[:, None] * kvec
                dL = WLi[None, :] * (vL - dlt @ PENUM)
                dls = qp.cw * dlt.sum(axis=1) - vt
                return dL, dt_, dlt, dls

            def u_local(vu, rh_f, rh_cp):
                """(du, dlam_fric) of the control blocks: friction rows in push-through form, CoP
                rows folded into the diagonal."""
                vu = vu.reshape(N, nc, nupc).copy()
                if talos:
                    vu[:, :, 0:2] += -(D[3][..., 0] * rh_cp[..., 0] - D[3][..., 1] * rh_cp[..., 1])
                du_ = np.einsum('kiab,kib->kia', Winv, vu)
                vf = vu[:, :, fo:fo + 3]
                z = np.einsum('kirn,kin->kir', Gw, vf) + rh_f
                dlf = np.einsum('kirq,kiq->kir', Kf_inv, z) * fm
                gl = np.einsum('kirm,kir->kim', qp.G, dlf)
                du_[:, :, fo:fo + 3] = np.einsum('kiab,kib->kia', Winv[:, :, fo:fo + 3, fo:fo + 3], vf - gl)
                return du_.reshape(N, nu), dlf

            def phi_solve(vx, vt, vu):
                """Phi^-1 (vx, vt, vu) (no row terms)."""
                dx = vx / qp.Wx[None, :]
                dL, dt_, _, _ = tr_local(vx[:, 6:9], vt, np.zeros((N + 1, 8)), np.zeros(N + 1))
                dx[:, 6:9] = dL
                du_, _ = u_local(vu, np.zeros((N, nc, 4)), np.zeros((N, nc, 2, 2)) if talos else None)
                return dx, dt_, du_

            def newton(rc, rdx=rdx, rdt=rdt, rdu=rdu, rde=rde, rdi=rdi):
                rhat = [(ri - c / np.where(mk > 0, li, 1.0)) * mk for ri, c, li, mk in zip(rdi, rc, lam, masks)]
                rcp = rhat[3] if talos else None
                # particular solution w = Phi^-1 (r_d + G'D rhat): local solves with v = -r_d
                wx = rdx / qp.Wx[None, :]
                dL, dt0, _, _ = tr_local(-rdx[:, 6:9], -rdt, rhat[0], rhat[1])
                wx[:, 6:9] = -dL
                wt = -dt0
                du0, _ = u_local(-rdu, rhat[2], rcp)
                wu = -du0
                rhs = rde - Ez(wx, wu)
                # forward / backward block substitution
                y = np.zeros((N + 2, 9))
                for j in range(N + 2):
                    b = rhs[j] - (Lo[j - 1] @ y[j - 1] if j > 0 else 0)
                    y[j] = np.linalg.solve(Lc[j], b)
                dnu = np.zeros((N + 2, 9))
                for j in range(N + 1, -1, -1):
                    b = y[j] - (Lo[j].T @ dnu[j + 1] if j < N + 1 else 0)
                    dnu[j] = np.linalg.solve(Lc[j].T, b)
                ex_, eu_ = ET(dnu)
                # full direction from the local solves with v = -(r_d + E'dnu)
                vx = -(rdx + ex_); vu = -(rdu + eu_)
                dx = vx / qp.Wx[None, :]
                dL, dt_, dlt, dls = tr_local(vx[:, 6:9], -rdt, rhat[0], rhat[1])
                dx[:, 6:9] = dL
                du, dlf = u_local(vu, rhat[2], rcp)
                gz = Gz(dx, du, dt_)
                dl = [dlt, dls, dlf]
                if talos:
                    dl.append(D[3] * (gz[3] + rhat[3]) * masks[3])
                ds = [(-ri - g) * mk for ri, g, mk in zip(rdi, gz, masks)]
                return dx, dt_, du, dnu, dl, ds

            def lin_res(d, rc):
                """Residual of the Newton system at direction d (the exact operators)."""
                dx, dt_, du, dnu, dl, ds = d
                gx_, gt_, gu_ = GT(dl)
                ex_, eu_ = ET(dnu)
                zx = np.zeros_like(dx); zu = np.zeros_like(du)
                gz = Gz(dx, du, dt_)
                return (qp.Wx * dx + ex_ + gx_ + rdx, gt_ + rdt, qp.Wu * du + eu_ + gu_ + rdu,
                        Ez(dx, du) - Ez(zx, zu) + rde,
                        [(g + dsi + ri) * mk for g, dsi, ri, mk in zip(gz, ds, rdi, masks)],
                        [(si * dli + li * dsi + c) * mk for si, dli, li, dsi, c, mk in zip(s, dl, lam, ds, rc, masks)])
            return newton, lin_res

        newton, lin_res = system(s, lam, rdx, rdt, rdu, rde, rdi)
        rc_aff = [si * li * mk for si, li, mk in zip(s, lam, masks)]
        dx, dt_, du, dnu, dl, ds = newton(rc_aff)
        if init:
            x = x + dx; t = t + dt_; u = u + du; nu_ = nu_ + dnu
            vals = ineq_val(x, u, t)
            s_new = [-v * mk for v, mk in zip(vals, masks)]
            l_new = [(li + dli) * mk for li, dli, mk in zip(lam, dl, masks)]
            if not talos and init_floor > 0:
                # Solo12: per-row floors; rows the least-squares point violates start just inside
                # the cone instead of every row shifting by the largest violation
                s = [np.where(mk > 0, np.maximum(si, init_floor), 1.0) for si, mk in zip(s_new, masks)]
                lam = [np.maximum(li, init_floor_l) * mk for li, mk in zip(l_new, masks)]
            else:
                # TALOS: CVXOPT's shift by 1 + the largest violation
                ap = max(float(-np.min(si[mk > 0])) for si, mk in zip(s_new, masks))
                ad = max(float(-np.min(li[mk > 0])) for li, mk in zip(l_new, masks))
                s = [np.where(mk > 0, si + (1 + ap if ap >= 0 else 0), 1.0) for si, mk in zip(s_new, masks)]
                lam = [(li + (1 + ad if ad >= 0 else 0)) * mk for li, mk in zip(l_new, masks)]
            continue
        a_aff = min(min(max_step(si, dsi, mk) for si, dsi, mk in zip(s, ds, masks)),
                    min(max_step(li, dli, mk) for li, dli, mk in zip(lam, dl, masks)))
        mu_aff = sum(((si + a_aff * dsi) * (li + a_aff * dli) * mk).sum()
                     for si, dsi, li, dli, mk in zip(s, ds, lam, dl, masks)) / m_tot
        sigma = (mu_aff / mu_) ** 3
        rc = [(si * li + dsi * dli - sigma * mu_) * mk for si, li, dsi, dli, mk in zip(s, lam, ds, dl, masks)]
        dx, dt_, du, dnu, dl, ds = newton(rc)
        a = min(min(max_step(si, dsi, mk) for si, dsi, mk in zip(s, ds, masks)),
                min(max_step(li, dli, mk) for li, dli, mk in zip(lam, dl, masks)))
        if (a < refine_alpha or (stall > 0 and refine_alpha > 0)) and merit < refine_merit:
            # one step of iterative refinement of the corrector direction
            d = (dx, dt_, du, dnu, dl, ds)
            r1, r2, r3, r4, r5, r6 = lin_res(d, rc)
            c = newton(r6, rdx=r1, rdt=r2, rdu=r3, rde=r4, rdi=r5)
            dx, dt_, du, dnu = dx + c[0], dt_ + c[1], du + c[2], dnu + c[3]
            dl = [p + q for p, q in zip(dl, c[4])]
            ds = [p + q for p, q in zip(ds, c[5])]
            a = min(min(max_step(si, dsi, mk) for si, dsi, mk in zip(s, ds, masks)),
                    min(max_step(li, dli, mk) for li, dli, mk in zip(lam, dl, masks)))
            n_refine += 1
        a = min(1.0, eta * a)
        x = x + a * dx; t = t + a * dt_; u = u + a * du; nu_ = nu_ + a * dnu
        s = [np.where(mk > 0, si + a * dsi, 1.0) for si, dsi, mk in zip(s, ds, masks)]
        lam = [(li + a * dli) * mk for li, dli, mk in zip(lam, dl, masks)]
        last = (a, ds, dl)
    out = dict(x=x, u=u, t=t, nu=nu_, lam=lam, s=s, status=status, iters=it, hist=hist, merit=merit,
               n_refine=n_refine, polish=polish_log[-1]['status'] if polish_log else 0, polish_log=polish_log)
    return out


def _polish(qp, masks, x, u, t, nu_, s, lam, last, system, GT, ET, Ez, ineq_val, e_rhs, eps, talos, rel):
    """Solution polishing (the reference's osqp setup has polish=True, src/scp_solver.py:62): the
    equality-constrained QP on the active set guessed from the converged iterate, solved with one
    Newton step of the same structured system.  Active set by the Tapia indicators of the last step
    (s_k / s_{k-1} against lambda_k / lambda_{k-1}: on an active row s vanishes while lambda settles,
    on an inactive one the reverse; lambda > s alone misreads rows where both are small).  Active
    rows get s = rel * lambda (D = 1 / rel: the push-through blocks then floor D^-1 as in any
    solve), inactive rows lambda = rel * s (D = rel), and the Newton step with sigma = 0 and a full
    step gives the solution of the reduced KKT system.  Accepted (status 1) when every active row
    keeps lambda >= -eps * scale_d and every inactive row s >= -eps * scale_p; otherwise -1 and the
    interior-point solution stands."""
    N = qp.N
    a, ds, dl = last
    s_prev = [np.where(mk > 0, si - a * dsi, 1.0) for si, dsi, mk in zip(s, ds, masks)]
    l_prev = [(li - a * dli) * mk for li, dli, mk in zip(lam, dl, masks)]
    act = [(mk > 0) & (si * lp < li * sp) for si, li, sp, lp, mk in zip(s, lam, s_prev, l_prev, masks)]
    s1 = [np.where(ac, rel * li, si) for si, li, ac in zip(s, lam, act)]
    l1 = [np.where(ac, li, rel * si) * mk for si, li, ac, mk in zip(s, lam, act, masks)]
    gx, gt, gu = GT(l1)
    ex, eu = ET(nu_)
    rdx = qp.Wx * x + qp.qx + ex + gx
    rdt = 1.0 + gt
    rdu = qp.Wu * u + eu + gu
    rde = Ez(x, u) - e_rhs
    vals = ineq_val(x, u, t)
    rdi = [(v + si) * mk for v, si, mk in zip(vals, s1, masks)]
    newton, _ = system(s1, l1, rdx, rdt, rdu, rde, rdi)
    dx, dt_, du, dnu, dlp, dsp = newton([si * li * mk for si, li, mk in zip(s1, l1, masks)])
    x2, t2, u2, n2 = x + dx, t + dt_, u + du, nu_ + dnu
    s2 = [np.where(mk > 0, si + dsi, 1.0) for si, dsi, mk in zip(s1, dsp, masks)]
    l2 = [(li + dli) * mk for li, dli, mk in zip(l1, dlp, masks)]
    scale_p = max(np.abs(Ez(x2, u2)).max(), np.abs(e_rhs).max(), 1.0)
    scale_d = max(np.abs(qp.Wx * x2).max(), np.abs(qp.Wu * u2).max(), np.abs(qp.qx).max(), 1.0)
    lmin = min(float(np.min(np.where(ac, li, np.inf))) for li, ac in zip(l2, act))
    smin = min(float(np.min(np.where((mk > 0) & ~ac, -v, np.inf)))
               for v, ac, mk in zip(ineq_val(x2, u2, t2), act, masks))
    prim2 = np.abs(Ez(x2, u2) - e_rhs).max()
    # as the kernel (ipm_loop, pm == 2): the primal side 100x tighter than the stopping test
    ok = lmin >= -eps * scale_d and smin >= -0.01 * eps * scale_p and prim2 <= 0.01 * eps * scale_p and np.isfinite(x2).all()
    return dict(status=1 if ok else -1, x=x2, u=u2, t=t2, nu=n2, s=s2, lam=l2, lmin=lmin, smin=smin,
                n_active=int(sum(a_.sum() for a_ in act)))


def to_z(qp, sol):
    """Pack into the reference's z layout [x | u | t | s(=0)]."""
    N = qp.N
    return np.concatenate([sol['x'].ravel(), sol['u'].ravel(), sol['t'], np.zeros(N)])


def to_y(qp, sol):
    """Multipliers in the reference's row layout (init | dyn | final | friction | TR | slack), solo12."""
    N, nc = qp.N, qp.nc
    fr = np.zeros((nc, N, 5))
    fr[:, :, :4] = np.transpose(sol['lam'][2], (1, 0, 2))
    return np.concatenate([sol['nu'][0], sol['nu'][1:N + 1].ravel(), sol['nu'][N + 1], fr.ravel(),
                           sol['lam'][0].ravel(), sol['lam'][1]])
