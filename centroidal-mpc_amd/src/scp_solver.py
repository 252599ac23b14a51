"""Sequential convex programming driver (drop-in for reference src/scp_solver.py:1-179).

Same public functions, arguments and return types as the reference; the work runs in
libcmpc.so on the GPU:

* ``solve_scp(model, scp_params)`` runs the whole GuSTO-style loop on the device
  (cmpc_solve_scp: linearize -> assemble -> batched interior-point QP -> trust-region test and
  accept/reject per iteration) and returns the reference's dict of accepted solutions, or
  False when a QP subproblem fails (quirk Q13).
* ``solve_scp_batch(models, ...)`` is the batched entry: many models (one robot / horizon) in one
  device handle, one result per model.
* ``sum_up_all_costs`` / ``stack_up_all_constraints`` / ``solve_subproblem`` keep the reference's
  step-by-step interface.  The QP they describe is the one assembled on the device, exported
  in the reference's CSC layout; ``solve_subproblem`` solves it with the device QP solver.  A
  QP built elsewhere (plain ``Cost`` / ``Constraint`` in the reference's layout) is decoded into
  the device's structured form by ``cmpc_load_qp`` first; one without the stage structure is
  refused with a ``CmpcError`` naming the offending row.

The reference's OSQP call (eps 1e-7 + polish, src/scp_solver.py:59-68) is replaced by an
interior-point method converged to 1e-10 (fp64; 1e-6 fp32): the QP's minimizer is unique (P > 0 on the
states and controls, slacks priced linearly), so both return the same solution to within the
reference's own tolerance.
"""
from collections import namedtuple
from warnings import warn

import numpy as np

from cmpc._lib import Solver
from cmpc.problem import ProblemBatch
from src import _device
from src.constraints import Constraint
from src.cost import Cost

Info = namedtuple('Info', 'status status_val iter obj_val')
Result = namedtuple('Result', 'x y info')

# device QP status -> OSQP status strings (the reference compares res.info.status to 'solved')
QP_STATUS = {1: 'solved', 2: 'solved inaccurate', -2: 'maximum iterations reached', -3: 'primal infeasible',
             -4: 'dual infeasible', -10: 'unsolved'}
SCP_QP_FAILED = -1


class _DeviceCost(Cost):
    """Cost(Q, p) that remembers the model whose device assembly produced it."""


class _DeviceConstraint(Constraint):
    """Constraint(mat, lb, ub) that remembers the device state that produced it."""


def sum_up_all_costs(model):
    """P, q of the SCP subproblem (reference :10-26)."""
    _, P, q, _, _, _ = _device.export(model)
    c = _DeviceCost(Q=P, p=q)
    c._model = model
    return c


def stack_up_all_constraints(model, traj_tuple, traj_data, trust_region_updates):
    """A, l, u in the reference's row order (reference :28-48).  ``traj_data`` is accepted for
    signature compatibility; the device linearizes at ``traj_tuple`` itself."""
    tr = {'weight': float(np.asarray(trust_region_updates['weight'])),
          'radius': float(np.asarray(trust_region_updates['radius']))}
    _, _, _, A, l, u = _device.export(model, traj_tuple, tr)
    c = _DeviceConstraint(mat=A, lb=l, ub=u)
    c._model, c._traj, c._tr = model, traj_tuple, tr
    return c


def convergence(traj_tuple_curr, traj_tuple_prev):
    """Relative spectral-norm change (reference :51-56)."""
    X_prev, U_prev = traj_tuple_prev['state'], traj_tuple_prev['control']
    X_curr, U_curr = traj_tuple_curr['state'], traj_tuple_curr['control']
    return (np.linalg.norm(U_curr - U_prev, 2) / np.linalg.norm(U_curr, 2) +
            np.linalg.norm(X_curr - X_prev, 2) / np.linalg.norm(X_curr, 2))


_FOREIGN = {}


def _foreign_solver(n, m):
    """A one-problem device handle for a QP of n variables and m rows in the reference's layout:
    n = 23 N + 10 for both robots; m = 38 N + 27 (Solo12) or 32 N + 27 (TALOS)."""
    N = (n - 10) // 23
    if N < 2 or 23 * N + 10 != n:
        raise ValueError('%d variables is not the layout 9(N+1) + 12N + (N+1) + N of any horizon N' % n)
    cfg = 'trot' if m == 38 * N + 27 else 'talos' if m == 32 * N + 27 else None
    if cfg is None:
        raise ValueError('%d rows is neither the Solo12 (%d) nor the TALOS (%d) layout at N = %d'
                         % (m, 38 * N + 27, 32 * N + 27, N))
    s = _FOREIGN.get((cfg, N))
    if s is None:
        from cmpc.synth import make_batch
        pb = make_batch(cfg, N, 1)      # a valid problem to install the handle's sizes; load_qp replaces it
        s = Solver(pb.robot, N, 1, 'fp64')
        s.upload(pb)
        _FOREIGN[(cfg, N)] = s
    return s


def solve_subproblem(cost, constraints):
    """Solve the QP (cost.Q, cost.p, constraints.mat, constraints.lb, constraints.ub) on the device;
    returns (QP_FEASIBILITY, res) with res.x, res.y, res.info.status as OSQP's (reference :59-68).

    QPs built by sum_up_all_costs / stack_up_all_constraints are solved where the device assembled
    them.  Any other QP in the reference's layout is decoded by cmpc_load_qp (csrc/load_qp.cpp: the
    stage structure is checked row by row) into a one-problem handle of its robot and horizon."""
    model = getattr(constraints, '_model', None)
    same = model is not None and getattr(cost, '_model', None) is model
    if model is not None and not same:
        _, P, q, _, _, _ = _device.export(model, constraints._traj, constraints._tr)
        same = (cost.Q.shape == P.shape and abs(cost.Q - P).max() == 0 and
                np.abs(np.asarray(cost.p) - q).max() <= 1e-12 * max(1.0, np.abs(q).max()))
    if same:
        s, P, q, A, l, u = _device.export(model, constraints._traj, constraints._tr)
    else:
        P, q = cost.Q, np.asarray(cost.p, float)
        A, l, u = constraints.mat, np.asarray(constraints.lb, float), np.asarray(constraints.ub, float)
        s = _foreign_solver(A.shape[1], A.shape[0])
        s.load_qp(0, P, q, A, l, u)
    s.qp_solve()
    z, y, st, it = s.qp_solution()
    x = z[0]
    status = QP_STATUS.get(int(st[0]), 'unsolved')
    res = Result(x=x, y=y[0], info=Info(status, int(st[0]), int(it[0]), float(0.5 * x @ (P @ x) + q @ x)))
    if status != 'solved':
        warn('[solve_OSQP]: Problem unfeasible.')
        return False, res
    return True, res


def compute_model_accuracy(model, curr_traj, prev_traj, prev_traj_data):
    """rho = sum_k |x+(X_k, U_k)[6:] - lin_k[6:]|^2 / sum_k |lin_k|^2 with
    lin_k = f_k + A_k dx_k + B_k du_k over k < N (reference :71-87); the rollout runs on the device."""
    nl = model.integrate_dynamics_trajectory(curr_traj)
    N = model._N
    f = np.asarray(prev_traj_data['dynamics'])[:, :N]
    A = np.asarray(prev_traj_data['gradients']['f_x'])
    B = np.asarray(prev_traj_data['gradients']['f_u'])
    dX = (np.asarray(curr_traj['state']) - np.asarray(prev_traj['state']))[:, :N]
    dU = (np.asarray(curr_traj['control']) - np.asarray(prev_traj['control']))[:, :N]
    lin = f.T + np.einsum('kij,jk->ki', A, dX) + np.einsum('kij,jk->ki', B, dU)
    err = nl[6:, :N].T - lin[:, 6:]
    return float((err ** 2).sum() / (lin ** 2).sum())


def get_QP_solution(model, res):
    """X (nx, N+1), U (nu, N) from z (reference :89-93, Fortran-order reshapes)."""
    n_x, n_u, N = model._n_x, model._n_u, model._N
    X_sol = np.reshape(res.x[:n_x * (N + 1)], (n_x, N + 1), order='F')
    U_sol = np.reshape(res.x[n_x * (N + 1):n_x * (N + 1) + n_u * N], (n_u, N), order='F')
    return dict(state=X_sol, control=U_sol)


def interpolate_SCP_solution(solution):
    """Linear interpolation of the last accepted solution, 10 sub-steps per interval
    (reference :95-111): column i*10 + j = v_i + j (v_{i+1} - v_i) / 10, the last knot dropped."""
    N_inner = 10
    X, U = np.asarray(solution['state'][-1]), np.asarray(solution['control'][-1])

    def interp(V):
        d = (V[:, 1:] - V[:, :-1]) / float(N_inner)
        j = np.arange(N_inner, dtype=float)
        out = V[:, :-1, None] + d[:, :, None] * j[None, None, :]
        return out.reshape(V.shape[0], -1)
    return dict(X=interp(X), U=interp(U))


def _results(s, sol, nu, B):
    """The reference's dict of lists per problem: every accepted iterate in acceptance order
    (src/scp_solver.py:162-167; the device keeps them, cmpc_get_accepted), or False (QP failed)."""
    out = []
    n_acc = sol['n_accepted']
    per = [s.accepted(j) for j in range(int(n_acc.max()) if B else 0)]
    for b in range(B):
        if int(sol['status'][b]) == SCP_QP_FAILED:
            out.append(False)
            continue
        r = dict(state=[], control=[], gains=[], covs=[])
        for j in range(int(n_acc[b])):
            a = per[j]
            r['state'].append(a['X'][b].T.copy())
            r['control'].append(a['U'][b][:, :nu].T.copy())
            r['gains'].append(a['K'][b][:, :nu, :].copy())
            r['covs'].append(a['Sigma'][b].copy())
        out.append(r)
    return out


def _print_iterations(records, n):
    """The reference's per-iteration banners and decisions (src/scp_solver.py:135-178), from the
    device's iteration records."""
    for rec in records[:n]:
        print('\n' + '=' * 50)
        print('Iteration ' + str(int(rec['iteration'])))
        print('-' * 50)
        dec = int(rec['decision'])
        if dec == -1:
            print('QP subproblem Failed at iter #' + str(int(rec['iteration'])))
        elif dec == 3:
            print('solution is outside trust region .. rejecting solution and increasing trust region weight')
        else:
            print('solution is inside trust region .. checking model accuracy')
            print("error ratio between linearized and nonlinear dynamics = ", float(rec['rho']))
            if dec == 2:
                print('linearized model is NOT accurate .. rejecting solution and decreasing trust region radius')
            else:
                print('linearized model is accurate enough .. accepting solution ')


def solve_scp(model, scp_params, gusto=False, verbose=True):
    """The reference's SCP loop for one model (reference :118-179), run on the device.
    ``gusto=True`` moves the linearization point to each accepted solution and iterates until
    convergence (the GuSTO scheme the reference cites, :113-117; include/cmpc.h
    CMPC_SCP_MODE_GUSTO); the default reproduces the reference exactly (quirk Q1).

    Returns the reference's dict of lists (state, control, gains, covs), one entry per accepted
    iterate in acceptance order, or False when a QP fails.  In reference mode the loop ends at the
    first accepted iterate (Q1), so the lists hold the reference's one entry; with ``gusto=True``
    every accepted iterate is returned, as the reference's loop appends them.  ``verbose`` prints
    the reference's per-iteration banners from the device's iteration records."""
    s = model._device_solver(None, scp_params)
    s.set_scp_mode('gusto' if gusto else 'reference')
    s.solve_scp(fixed_iters=False)
    sol = s.solution()
    rec, n = s.iteration_history()
    if verbose:
        _print_iterations(rec[0], int(n[0]))
    res = _results(s, sol, model._n_u, 1)[0]
    it = int(sol['iterations'][0])
    if res is False:
        return False
    print('[solve_ccscp] Success: ' + str(int(rec[0][n[0] - 1]['decision']) == 1 if n[0] else False)
          + ', Nb of iterations: ' + str(it))
    return res


def solve_scp_batch(models, scp_params=None, precision='fp64', device=0, fixed_iters=False, gusto=False,
                    n_inner=None):
    """Batched SCP: all ``models`` (one robot and horizon) in one device handle; returns one
    result per model (the reference's dict or False).  ``scp_params`` (optional) overrides every
    model's conf scp_params; ``gusto`` selects the GuSTO mode (see solve_scp); with ``n_inner``
    each result also carries 'interpolated' = interpolate_SCP_solution of its accepted solution
    with n_inner sub-steps, computed on the device."""
    models = list(models)
    if not models:
        return []
    m0 = models[0]
    if any(m._robot != m0._robot or m._N != m0._N for m in models):
        raise ValueError('solve_scp_batch needs models of one robot and horizon')
    pbs = [m.problem_batch(None, scp_params) for m in models]
    # one parameter class per distinct conf parameter set (models built from one conf share it)
    classes, index, cid = [], {}, np.zeros(len(models), np.int32)
    for b, (m, pb) in enumerate(zip(models, pbs)):
        key = id(m._params)
        if key not in index:
            index[key] = len(classes)
            classes.append(pb.params[0])
        cid[b] = index[key]
    cat = lambda name: np.concatenate([getattr(pb, name) for pb in pbs])
    batch = ProblemBatch(m0._robot, m0._N, pbs[0].nc, m0._n_u, cat('logic'), cat('pos'), cat('rot'), cat('Xbar'),
                         cat('Ubar'), cid, classes)
    batch.validate()
    with Solver(m0._robot, m0._N, batch.B, precision, device) as s:
        s.upload(batch)
        s.set_scp_mode('gusto' if gusto else 'reference')
        s.solve_scp(fixed_iters=fixed_iters)
        sol = s.solution()
        interp = s.interpolate(int(n_inner)) if n_inner else None
        res = _results(s, sol, m0._n_u, batch.B)
    if interp is not None:
        for b, r in enumerate(res):
            if r is not False and r['state']:
                r['interpolated'] = dict(X=interp[0][b], U=interp[1][b][:m0._n_u])
    return res
