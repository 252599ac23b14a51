"""CPU: the numpy mirror of the GPU interior-point QP (oracle/ipm_mirror.py) on the cases that
shaped its exits.  The mirror runs the kernel's algorithm step for step, so these pin the
algorithm itself without a GPU; the GPU side is tests/test_gpu_qp_status.py.

* TALOS N=200, problem 280 of the BASELINE C4 shard at its second SCP iteration (the first
  iteration rejects every problem on the trust-region test, so the weight is omega0 * gamma_fail
  = 500 and the radius stays at 100).  Without iterative refinement the corrector direction
  loses its accuracy on the pinned friction rows and mu stalls (round 1's GPU failure, status
  -2 after 60 iterations there; the mirror's stall guard reports it as 'solved inaccurate'); with
  one refinement step where the step length collapses, the IPM converges to merit <= 1 and
  matches an independent sparse IPM on the reference-form QP.
* A primal infeasible trot QP (final vertical momentum below the free-fall bound: the friction
  pyramid keeps every f_z >= 0): the Farkas certificate exits with -3, and the OSQP restatement
  (the reference's QP algorithm) reports 'primal infeasible' on the same QP.
"""
import numpy as np
import pytest

from cmpc.synth import make_batch
from oracle import ipm_mirror as IM
from oracle import model as M, transcription as T
from oracle.osqp_admm import solve_qp as admm_qp
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp


def _struct(cfg, N, b, weight, radius, edit=None):
    pb = make_batch(cfg, N, 1, seed_offset=b)     # seed 1000 * cfg_seed + b: problem b of a batch
    if edit is not None:
        edit(pb)
    p = pb.oracle_problem(0)
    prm = p['prm']
    par = pb.params[0]
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], prm)
    qp = IM.StructQP.from_arrays(N, par.robot, pb.nc, par.Wx, par.Wu, pb.Xbar[0], pb.Ubar[0], td['f_x'], td['f_u'],
                                 td['dynamics'].T, pb.logic[0], pb.rot[0], par.mu, weight, radius,
                                 tracking=par.tracking, foot_range=par.foot_range)
    P, q = T.build_cost(N, prm, p['Xbar'])
    A, l, u = T.build_constraints(N, prm, p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td, weight, radius)
    return qp, (P, q, A, l, u)


def test_talos_problem_280_needs_refinement():
    """Round 1's C4 stall (friction floor 1e-12, as then): it stalls without refinement and solves
    with it; the round-2 friction floor (1e-9) solves it as well."""
    N = 200
    qp, ref_qp = _struct('talos', N, 280, 500.0, 100.0)
    plain = IM.solve(qp, refine_alpha=0.0, fric_floor=1e-12)
    assert plain['status'] == 2 and plain['merit'] > 1.0          # the stall, reproduced on the CPU
    sol = IM.solve(qp, fric_floor=1e-12)
    assert sol['status'] == 1 and sol['merit'] <= 1.0 and sol['n_refine'] >= 1
    assert IM.solve(qp)['status'] == 1
    ref = sparse_ipm_qp(*ref_qp)
    assert ref.info.status == 'solved'
    nx = 9 * (N + 1)
    z = IM.to_z(qp, sol)
    assert np.abs(z[:nx] - ref.x[:nx]).max() <= 1e-8 * np.abs(ref.x[:nx]).max()


@pytest.mark.parametrize('cfg,N,b', [('trot', 100, 3), ('bound', 60, 5)])
def test_refinement_not_triggered_on_regular_problems(cfg, N, b):
    qp, _ = _struct(cfg, N, b, 100.0, 100.0 if cfg == 'trot' else 50.0)
    sol = IM.solve(qp)
    assert sol['status'] == 1 and sol['merit'] <= 1.0 and sol['n_refine'] == 0


def _infeasible(pb):
    N, par = pb.N, pb.params[0]
    pb.Xbar[0, N, 5] = pb.Xbar[0, 0, 5] + N * par.dt * par.mass * par.gravity - 1.0


def test_primal_infeasible_certificate():
    N = 30
    qp, ref_qp = _struct('trot', N, 0, 100.0, 100.0, edit=_infeasible)
    sol = IM.solve(qp)
    # (from the floored start the multipliers diverge along the certificate at ~1.1-1.5x per
    # Newton step, so detection takes ~40 steps at N=30; the iteration cap is 60)
    assert sol['status'] == -3 and sol['iters'] <= 50
    assert admm_qp(*ref_qp).info.status == 'primal infeasible'


def test_talos_zero_force_friction_floor():
    """TALOS with other cost weights (state weights x (2, 2, 0.5, 1, 1, 1, 3, 3, 3), control weights
    x 0.25): contact forces reach the pyramid's apex, where all four friction rows are active and
    K = D^-1 + G W^-1 G' tends to rank 3.  At the old 1e-12 floor the direction's complementarity
    residual stays at 0.1-0.5 and the solve hits the iteration cap; at the kernel's 1e-9 it solves
    and matches the sparse IPM on the same QP."""
    N = 40
    pb = make_batch('talos', N, 1, seed_offset=0)
    p = pb.oracle_problem(0)
    par = pb.params[0]
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    sp = p['scp_params']
    wx = np.asarray(par.Wx) * np.array([2.0, 2.0, 0.5, 1.0, 1.0, 1.0, 3.0, 3.0, 3.0])
    wu = np.asarray(par.Wu) * 0.25
    qp = IM.StructQP.from_arrays(N, par.robot, pb.nc, wx, wu, pb.Xbar[0], pb.Ubar[0], td['f_x'], td['f_u'],
                                 td['dynamics'].T, pb.logic[0], pb.rot[0], par.mu, sp['omega0'],
                                 sp['trust_region_radius0'], tracking=par.tracking, foot_range=par.foot_range)
    assert IM.solve(qp, fric_floor=1e-12)['status'] == -2
    sol = IM.solve(qp)
    assert sol['status'] == 1 and sol['merit'] <= 1.0
    prm = dict(p['prm'])
    prm['Wx'] = np.diag(wx); prm['Wu'] = np.diag(wu)
    P, q = T.build_cost(N, prm, p['Xbar'])
    A, l, u = T.build_constraints(N, prm, p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td, sp['omega0'],
                                  sp['trust_region_radius0'])
    ref = sparse_ipm_qp(P, q, A, l, u)
    assert ref.info.status == 'solved'
    nx = 9 * (N + 1)
    z = IM.to_z(qp, sol)
    assert np.abs(z[:nx] - ref.x[:nx]).max() <= 1e-6 * np.abs(ref.x[:nx]).max()


def _scp0(cfg, N, b):
    pb = make_batch(cfg, N, 1, seed_offset=b)
    sp = pb.oracle_problem(0)['scp_params']
    return _struct(cfg, N, b, sp['omega0'], sp['trust_region_radius0'])


@pytest.mark.parametrize('cfg,N,b', [('talos', 40, 5), ('talos', 40, 4), ('trot', 40, 2), ('trot', 40, 9)])
def test_polish_reaches_the_exact_minimizer(cfg, N, b):
    """Solution polishing (the reference runs OSQP with polish=True, src/scp_solver.py:62), at the
    kernel's robot defaults (Solo12 eps 1e-9, polish 1e-7; TALOS eps 1e-10, polish 1e-7 here, off in
    the kernel by default): once the iterate
    meets polish_eps, the active set guessed from the last step (Tapia indicators) gives a reduced
    KKT system; its solution, verified at eps, is the QP's exact minimizer (<= 1e-8 of an
    independent sparse IPM run to 1e-12, and no farther than the unpolished solve) in fewer Newton
    steps than the unpolished solve."""
    qp, ref_qp = _scp0(cfg, N, b)
    eps, peps = IM.robot_defaults(qp)
    peps = peps or 1e-7   # (TALOS does not polish by default; the algorithm is checked at 1e-7)
    plain = IM.solve(qp, eps=eps)
    pol = IM.solve(qp, eps=eps, polish=True, polish_eps=peps)
    assert plain['status'] == 1 and pol['status'] == 1
    assert pol['polish'] == 1 and pol['iters'] < plain['iters']
    ref = sparse_ipm_qp(*ref_qp, eps=1e-12, max_iter=500)
    nxu = 9 * (N + 1) + 12 * N
    sc = np.abs(ref.x[:nxu]).max()
    err_pol = np.abs(IM.to_z(qp, pol)[:nxu] - ref.x[:nxu]).max() / sc
    err_plain = np.abs(IM.to_z(qp, plain)[:nxu] - ref.x[:nxu]).max() / sc
    assert err_pol <= 1e-8 and err_pol <= max(1.01 * err_plain, 1e-9), (err_pol, err_plain)


def test_rejected_polish_rolls_back():
    """A wrong active-set guess (TALOS problem 8 at polish_eps 1e-9): the verification fails, the
    iterate before the polish is restored and the interior-point iterations finish exactly as
    without polishing."""
    qp, _ = _scp0('talos', 40, 8)
    eps, _ = IM.robot_defaults(qp)
    peps = 1e-9
    plain = IM.solve(qp, eps=eps)
    pol = IM.solve(qp, eps=eps, polish=True, polish_eps=peps)
    assert [p['status'] for p in pol['polish_log']] == [-1] and pol['status'] == 1
    assert pol['iters'] == plain['iters']
    np.testing.assert_array_equal(IM.to_z(qp, pol), IM.to_z(qp, plain))


@pytest.mark.parametrize('b', [3, 12, 17, 36])
def test_solo12_stopping_test_reaches_the_minimizer(b):
    """Solo12's stopping test measures complementarity against the primal scale (qp_ipm.hip
    COMP_PRIMAL_SCALE; round 4): trot N=100 problems whose solves stopped 2e-5 to 7e-5 away from the
    exact minimizer with the dual scale (one friction row left at s lambda ~ 5e-6) land within 1e-6
    of an independent sparse IPM at the defaults."""
    N = 100
    qp, ref_qp = _scp0('trot', N, b)
    eps, peps = IM.robot_defaults(qp)
    sol = IM.solve(qp, eps=eps, polish=True, polish_eps=peps)
    assert sol['status'] == 1
    ref = sparse_ipm_qp(*ref_qp, eps=1e-12, max_iter=500)
    nxu = 9 * (N + 1) + 12 * N
    err = np.abs(IM.to_z(qp, sol)[:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max()
    assert err <= 1e-6, err
