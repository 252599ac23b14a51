"""GPU parity: libcmpc.so (through the C ABI) against the oracle on identical inputs.

Tolerances (stated per quantity):
  * linearization fp64: f/A/B/C bit-for-bit up to 1e-15 abs; K, Sigma 1e-11 relative to their max
    (TALOS Sigma 1e-4 against the kernel's association: the covariance scan is ill-conditioned
    there, see the test).
    fp32: 2e-6 relative (f, A, B) / 1e-3 relative (K, Sigma; fp32 LQR solves).
  * assembly: the exported CSC equals the oracle's (reference row order) to 1e-13 (fp64).
  * QP: the GPU solution's KKT residuals on the reference-form QP (prim <= 1e-8, dual <= 1e-6 x
    cost scale) and |X_gpu - X_oracle|_inf <= 1e-5 * |X|_inf against the OSQP restatement run
    to eps 1e-10 (the reference runs OSQP at 1e-7 + polish; our fp64 IPM stops at 1e-10).
    fp32: KKT primal <= 1e-3, |X| agreement 5e-3 relative.
  * SCP: identical decisions (accept / reject_tr / reject_rho / qp_failed), iterations and
    accepted counts as the oracle's solve_scp; accepted X, U within the QP tolerance.
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle import model as M, transcription as T
from oracle.kkt import kkt_residuals
from oracle.osqp_admm import solve_qp
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
from oracle import scp as OS

pytestmark = pytest.mark.gpu

CASES = [('trot', 30, 4), ('bound', 40, 3), ('pace', 40, 3), ('talos', 50, 2)]


def _solver(cfg, N, B, prec='fp64', stochastic=False, mixed=None):
    pb = make_batch(cfg, N, B, stochastic=stochastic, mixed=mixed)
    s = Solver(pb.robot, N, B, prec)
    s.upload(pb)
    return pb, s


def _oracle_lin(pb, b):
    p = pb.oracle_problem(b)
    return p, M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])


@pytest.mark.parametrize('cfg,N,B', CASES)
def test_linearization_fp64(cfg, N, B):
    pb, s = _solver(cfg, N, B)
    s.linearize()
    lin = s.linearization()
    for b in range(B):
        _, td = _oracle_lin(pb, b)
        np.testing.assert_allclose(lin['f'][b], td['dynamics'].T, rtol=0, atol=1e-13)
        np.testing.assert_allclose(lin['A'][b], td['f_x'], rtol=0, atol=1e-15)
        np.testing.assert_allclose(lin['Bu'][b], td['f_u'], rtol=0, atol=1e-15)
        np.testing.assert_allclose(lin['C'][b], td['f_w'], rtol=0, atol=1e-15)
        np.testing.assert_allclose(lin['K'][b], td['LQR_gains'], rtol=0, atol=1e-11 * np.abs(td['LQR_gains']).max())
        # TALOS: with the reference's TALOS warm start (quirk Q11) the 2-step LQR leaves A + BK with
        # spectral radius 1, and the covariance scan amplifies rounding: the reference's association
        # and the kernel's (A + BK) S (A + BK)' differ by ~8e-6 relative at N=50 in the oracle alone
        # (tests/test_host.py::test_talos_covariance_scan_sensitivity), so the bound is 1e-4 against
        # the oracle evaluated in the kernel's association; Solo12 holds 1e-11 either way
        if cfg == 'talos':
            p = pb.oracle_problem(b)
            cl = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'],
                                           assoc='closed_loop')['Covs']
            np.testing.assert_allclose(lin['Sigma'][b], cl, rtol=0, atol=1e-4 * np.abs(cl).max())
        else:
            np.testing.assert_allclose(lin['Sigma'][b], td['Covs'], rtol=0, atol=1e-11 * np.abs(td['Covs']).max())
    s.close()


def test_linearization_fp32():
    pb, s = _solver('trot', 40, 2, 'fp32')
    s.linearize()
    lin = s.linearization()
    for b in range(2):
        _, td = _oracle_lin(pb, b)
        np.testing.assert_allclose(lin['f'][b], td['dynamics'].T, rtol=0, atol=2e-6 * np.abs(td['dynamics']).max())
        np.testing.assert_allclose(lin['A'][b], td['f_x'], rtol=0, atol=2e-6)
        np.testing.assert_allclose(lin['K'][b], td['LQR_gains'], rtol=0, atol=1e-3 * np.abs(td['LQR_gains']).max())
        np.testing.assert_allclose(lin['Sigma'][b], td['Covs'], rtol=0, atol=1e-3 * np.abs(td['Covs']).max())
    s.close()


@pytest.mark.parametrize('cfg,N,B,stoch', [('trot', 30, 2, False), ('trot', 30, 2, True), ('talos', 40, 2, False),
                                           ('bound', 30, 2, True)])
def test_assembly_matches_reference_order(cfg, N, B, stoch):
    pb, s = _solver(cfg, N, B, stochastic=stoch)
    s.linearize(); s.assemble()
    for b in range(B):
        p, td = _oracle_lin(pb, b)
        P, q, A, l, u = s.export_qp(b)
        P0, q0 = T.build_cost(N, p['prm'], p['Xbar'])
        r0 = p['scp_params']['trust_region_radius0']
        A0, l0, u0 = T.build_constraints(N, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td,
                                         p['scp_params']['omega0'], r0)
        assert P.shape == P0.shape and A.shape == A0.shape
        assert abs(P - P0).max() == 0
        np.testing.assert_allclose(q, q0, rtol=0, atol=1e-12)
        assert abs(A - A0).max() <= 1e-13
        fin = np.isfinite(l0)
        assert np.array_equal(fin, np.isfinite(l)) and np.array_equal(np.isfinite(u0), np.isfinite(u))
        np.testing.assert_allclose(l[fin], l0[fin], rtol=0, atol=1e-11)
        fu = np.isfinite(u0)
        np.testing.assert_allclose(u[fu], u0[fu], rtol=0, atol=1e-11)
    s.close()


@pytest.mark.parametrize('cfg,N,B', CASES)
def test_qp_matches_oracle_fp64(cfg, N, B):
    pb, s = _solver(cfg, N, B)
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    assert np.all(st == 1), st
    nxu = 9 * (N + 1) + 12 * N
    for b in range(B):
        P, q, A, l, u = s.export_qp(b)
        k = kkt_residuals(P, q, A, l, u, z[b], y[b])
        scale = max(1.0, np.abs(P @ z[b]).max(), np.abs(q).max())
        assert k['prim'] <= 1e-8, k['prim']
        assert k['dual'] <= 1e-6 * scale, (k['dual'], scale)
        assert k['sign'] == 0.0
        # the reference's algorithm (OSQP restatement) run tight; for TALOS it needs >1e5 ADMM
        # iterations, so the independent sparse interior-point oracle is the reference there
        if cfg == 'talos':
            ref = sparse_ipm_qp(P, q, A, l, u)
        else:
            ref = solve_qp(P, q, A, l, u, eps_abs=1e-10, eps_rel=1e-10, max_iter=200000)
        assert ref.info.status == 'solved'
        err = np.abs(z[b][:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max()
        assert err <= 1e-5, err
    s.close()


def test_qp_fp32_tolerance():
    pb, s = _solver('bound', 40, 2, 'fp32')
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    assert np.all(st == 1), st
    nxu = 9 * 41 + 12 * 40
    for b in range(2):
        p, td = _oracle_lin(pb, b)
        P, q = T.build_cost(40, p['prm'], p['Xbar'])
        A, l, u = T.build_constraints(40, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td,
                                      p['scp_params']['omega0'], p['scp_params']['trust_region_radius0'])
        k = kkt_residuals(P, q, A, l, u, z[b])
        assert k['prim'] <= 1e-3
        ref = sparse_ipm_qp(P, q, A, l, u)
        err = np.abs(z[b][:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max()
        assert err <= 5e-3, err
    s.close()


@pytest.mark.parametrize('cfg,N,B', [('trot', 50, 1), ('trot', 30, 3), ('bound', 30, 2), ('talos', 40, 2)])
def test_solve_scp_matches_oracle(cfg, N, B):
    """(trot, 50, 1) is BASELINE C1, the reference's own CPU case, on the GPU."""
    pb, s = _solver(cfg, N, B)
    n = s.solve_scp(fixed_iters=False)
    sol = s.solution()
    for b in range(B):
        p = pb.oracle_problem(b)
        log = []
        ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp, log=log)
        assert sol['iterations'][b] == len(log)
        if ref is False:
            assert sol['status'][b] == -1
            continue
        assert sol['n_accepted'][b] == len(ref['state'])
        if len(ref['state']):
            X = sol['X'][b].T
            np.testing.assert_allclose(X, ref['state'][-1], rtol=0, atol=1e-5 * np.abs(ref['state'][-1]).max())
            np.testing.assert_allclose(sol['U'][b].T, ref['control'][-1], rtol=0,
                                       atol=1e-5 * np.abs(ref['control'][-1]).max())
            np.testing.assert_allclose(sol['K'][b], ref['gains'][-1], rtol=0,
                                       atol=1e-11 * np.abs(ref['gains'][-1]).max())
    s.close()


def test_fixed_iteration_mode_is_deterministic():
    pb, s = _solver('trot', 40, 8)
    s.scp_iterate(True); z1, _, st1, it1 = s.qp_solution(with_y=False)
    s.scp_iterate(True); z2, _, st2, it2 = s.qp_solution(with_y=False)
    assert np.array_equal(z1, z2) and np.array_equal(it1, it2)
    s.close()


def test_mixed_batch_pace_trot():
    pb, s = _solver('trot', 60, 6, mixed=('pace', 'trot'))
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    assert np.all(st == 1)
    for b in (0, 1):
        P, q, A, l, u = s.export_qp(b)
        k = kkt_residuals(P, q, A, l, u, z[b], y[b])
        assert k['prim'] <= 1e-8
    s.close()


def test_full_size_metric_config_properties():
    """BASELINE metric size (trot, N=100, 1024 problems): every QP solved; size-independent
    properties on a sample: dynamics rows satisfied, KKT residuals small, SCP decisions valid."""
    pb, s = _solver('trot', 100, 1024)
    s.scp_iterate(fixed_iters=True)
    z, y, st, it = s.qp_solution(with_y=True)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    assert 3 <= it.mean() <= 40
    for b in (0, 511, 1023):
        P, q, A, l, u = s.export_qp(b)
        k = kkt_residuals(P, q, A, l, u, z[b], y[b])
        assert k['prim'] <= 1e-8 and k['sign'] == 0.0
    log = s.iteration_log()
    assert set(np.unique(log['decision'])) <= {1, 2, 3}
    s.close()


def test_edge_single_problem_and_max_horizon():
    pb, s = _solver('talos', 200, 1)          # TALOS N=200 (BASELINE C4 horizon), Schur blocks in HBM
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    P, q, A, l, u = s.export_qp(0)
    k = kkt_residuals(P, q, A, l, u, z[0], y[0])
    assert st[0] == 1 and k['prim'] <= 1e-8
    s.close()


@pytest.mark.parametrize('cfg,N,B', [('trot', 31, 2), ('trot', 2, 2), ('trot', 255, 2), ('talos', 101, 2)])
def test_qp_horizon_edges(cfg, N, B):
    """Horizons at the edges of the half-wave Schur recurrence: odd N (N + 2 odd: both ends take
    the same number of steps), the smallest horizon (N = 2: one step per end) and the largest
    (N = 255: 257 blocks, the workspace pitch KPC).  KKT residuals of the reference-form QP."""
    pb, s = _solver(cfg, N, B)
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    assert np.all(st == 1), st
    for b in range(B):
        P, q, A, l, u = s.export_qp(b)
        k = kkt_residuals(P, q, A, l, u, z[b], y[b])
        scale = max(1.0, np.abs(P @ z[b]).max(), np.abs(q).max())
        assert k['prim'] <= 1e-8, k['prim']
        assert k['dual'] <= 1e-6 * scale, (k['dual'], scale)
        assert k['sign'] == 0.0
    s.close()


@pytest.mark.parametrize('cfg,N,B,prec,mixed', [
    ('trot', 100, 256, 'fp64', None),            # BASELINE C2: two waves per problem, one end of the
                                                 # Schur recurrence per wave (tw_factor_ends<T, 64>)
    ('bound', 100, 1024, 'fp32', None),          # BASELINE C3: fp32 + tolerance check vs CPU
    ('talos', 200, 512, 'fp64', None),           # BASELINE C4: one GPU's shard of 4096
    ('trot', 150, 1024, 'fp64', ('pace', 'trot')),  # BASELINE C5: one GPU's shard of 8192, mixed plans
])
def test_full_size_baseline_configs(cfg, N, B, prec, mixed):
    """Full per-GPU sizes of BASELINE C2-C5: every QP solved; on a sample (first, middle, last
    problem), KKT primal residual of the reference-form QP (fp64 1e-8, fp32 1e-3) and |X| within
    1e-5 (fp64) / 5e-3 (fp32) of the oracle's independent sparse IPM on the same QP."""
    pb, s = _solver(cfg, N, B, prec, mixed=mixed)
    s.scp_iterate(fixed_iters=True)
    z, y, st, it = s.qp_solution(with_y=True)
    assert np.all(st == 1), np.unique(st, return_counts=True)
    nx = 9 * (N + 1)
    tol_prim, tol_x = (1e-3, 5e-3) if prec == 'fp32' else (1e-8, 1e-5)
    for b in (0, B // 2 + 1, B - 1):
        P, q, A, l, u = s.export_qp(b)
        k = kkt_residuals(P, q, A, l, u, z[b])
        assert k['prim'] <= tol_prim, (b, k)
        ref = sparse_ipm_qp(P, q, A, l, u)
        err = np.abs(z[b][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max()
        assert err <= tol_x, (b, err, int(it[b]))
    s.close()


def test_talos_shrunk_trust_region_qp_solves():
    """BASELINE C4 shard (TALOS N=200 x 512) with the trust region of round 1's second fixed-K SCP
    iteration (weight 500 after a trust-region reject at radius 100; since radius0 = 1000 the
    first iteration accepts, so the weight is set directly): every QP reaches 'solved' with merit
    <= 1.  Round 1
    stalled on problem 280 here (60 iterations, status -2); iterative refinement of the corrector
    direction fixes it (tests/test_ipm_mirror.py reproduces the stall and the fix on the CPU).
    The slowest problem matches the oracle's sparse IPM on the same exported QP."""
    N, B = 200, 512
    pb, s = _solver('talos', N, B)
    s.set_trust_region(weight=500.0, radius=100.0)
    s.scp_iterate(fixed_iters=True)
    z, y, st, it = s.qp_solution(with_y=True)
    merit, nref = s.qp_info()
    b = int(it.argmax())
    P, q, A, l, u = s.export_qp(b)
    ref = sparse_ipm_qp(P, q, A, l, u)
    nx = 9 * (N + 1)
    err = np.abs(z[b][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max()
    P2, q2, A2, l2, u2 = s.export_qp(280)
    ref2 = sparse_ipm_qp(P2, q2, A2, l2, u2)
    err2 = np.abs(z[280][:nx] - ref2.x[:nx]).max() / np.abs(ref2.x[:nx]).max()
    s.close()
    assert np.all(st == 1), (np.nonzero(st != 1)[0], int(it.max()))
    assert np.all(merit <= 1.0), merit.max()
    assert it.max() <= 30, int(it.max())
    assert err <= 1e-5, err
    assert err2 <= 1e-5, err2
