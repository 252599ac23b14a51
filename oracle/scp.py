"""Oracle: the SCP trust-region state machine of the reference.  TEST INFRASTRUCTURE.

Restates ``solve_scp`` (src/scp_solver.py:118-179) including its quirks:
* the linearization point and ``prev_traj_dict`` are never reassigned (:129-130), so every
  iteration re-linearizes around the warm start and ``convergence`` is identically 0 (Q1);
* a QP status other than 'solved' aborts the whole solve with False (Q13);
* the trust-region test uses the spectral norm of the 9x(N+1) state difference (Q6);
* radius growth is capped at radius0 (Q8).
``fixed_iters=True`` keeps iterating to ``max_iterations`` (acceptance still computed), the
benchmark's fixed-K mode.

``gusto=True`` restates the GuSTO scheme the reference cites (:113-117) but never executes: an
accepted solution becomes the next linearization point (traj_tuple), the previous one
prev_traj_dict, and the loop stops after an accepted iteration once
convergence(traj_tuple, prev_traj_dict) (:51-56, spectral norms) < convergence_threshold.  The
tracking cost and the initial / final state rows stay on the warm start (sum_up_all_costs and
the constraint builders read model._init_trajectories).  This is the device's
CMPC_SCP_MODE_GUSTO.
"""
import numpy as np

from . import model as M
from . import transcription as T
from .osqp_admm import solve_qp


def convergence(Xc, Uc, Xp, Up):
    """src/scp_solver.py:51-56 on (9, N+1) / (nu, N) arrays."""
    return (M.spectral_norm(Uc - Up) / M.spectral_norm(Uc) + M.spectral_norm(Xc - Xp) / M.spectral_norm(Xc))


def solve_scp(prob, scp_params, qp=solve_qp, dtype=np.float64, fixed_iters=False, log=None, gusto=False):
    """prob: dict(prm=..., N=..., logic, pos, rot, Xbar (9,N+1), Ubar (nu,N)).

    Returns the reference's dict(state=[...], control=[...], gains=[...], covs=[...]) or False,
    plus (when ``log`` is a list) one record per iteration."""
    prm = prob['prm']; N = prob['N']; nu = prm['nu']
    Xbar, Ubar = prob['Xbar'], prob['Ubar']
    out = dict(state=[], control=[], gains=[], covs=[])
    rho0, rho1 = scp_params['rho0'], scp_params['rho1']
    omega_max = scp_params['omega_max']
    beta_succ, beta_fail = scp_params['beta_succ'], scp_params['beta_fail']
    max_iter = scp_params['max_iterations']
    conv_thresh = scp_params['convergence_threshold']
    gamma_fail = scp_params['gamma_fail']
    weight = float(scp_params['omega0']); radius = float(scp_params['trust_region_radius0'])
    success = False
    it = 0
    conv = 0.0   # convergence(traj_tuple, prev_traj_dict): identically 0 in the reference (Q1)
    P, q = T.build_cost(N, prm, Xbar)
    Xl, Ul = Xbar, Ubar   # linearization point (traj_tuple)
    while it < max_iter and weight < omega_max and not (
            (not fixed_iters) and it != 0 and success and conv < conv_thresh):
        success = False
        td = M.compute_trajectory_data(Xl, Ul, prob['logic'], prob['pos'], prob['rot'], prm, dtype)
        A, l, u = T.build_constraints(N, prm, prob['logic'], prob['pos'], prob['rot'], Xl, Ul, td,
                                      weight, radius, Xinit=Xbar)
        res = qp(P, q, A, l, u)
        rec = dict(it=it, weight=weight, radius=radius, status=res.info.status, qp_iter=res.info.iter)
        if res.info.status != 'solved':
            if log is not None:
                rec['decision'] = 'qp_failed'; log.append(rec)
            return False
        X, U = T.get_qp_solution(N, nu, res.x)
        tr = M.spectral_norm(X - Xl)
        rec['tr_norm'] = tr
        if tr < radius:
            rho = float(M.compute_model_accuracy(X, U, Xl, Ul, td, prob['logic'], prob['pos'],
                                                 prob['rot'], prm, dtype))
            rec['rho'] = rho
            if rho > rho1:
                radius *= beta_fail
                rec['decision'] = 'reject_rho'
            else:
                out['state'].append(X); out['control'].append(U)
                out['gains'].append(td['LQR_gains']); out['covs'].append(td['Covs'])
                success = True
                rec['decision'] = 'accept'
                if rho < rho0:
                    radius = min(beta_succ * radius, scp_params['trust_region_radius0'])
                if gusto:
                    conv = float(convergence(X, U, Xl, Ul))
                    rec['conv'] = conv
                    Xl, Ul = X, U
        else:
            weight *= gamma_fail
            rec['decision'] = 'reject_tr'
        if log is not None:
            log.append(rec)
        it += 1
    return out
