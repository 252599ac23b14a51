"""SURVEY.md 8f row f1 on the GPU: GuSTO mode (the linearization point follows each accepted
solution) against the oracle's restatement of the same loop, the reference mode's untouched
linearization point (quirk Q1), and the device interpolate_SCP_solution.

Tolerances: identical iteration counts / accepted counts; accepted X, U and the convergence
measure within 1e-5 of their scale (the QP solutions are 1e-10-accurate on both sides and
feed the next linearization); interpolation bit-for-bit up to 1e-14 relative (same formula).
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle import scp as OS
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('cfg,N,B', [('trot', 30, 3), ('bound', 30, 2)])
def test_gusto_matches_oracle(cfg, N, B):
    pb = make_batch(cfg, N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.set_scp_mode('gusto')
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        Xl, Ul, conv = s.linearization_point()
    multi = 0
    for b in range(B):
        p = pb.oracle_problem(b)
        log = []
        ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp, log=log, gusto=True)
        assert ref is not False
        assert sol['iterations'][b] == len(log), (sol['iterations'][b], [r['decision'] for r in log])
        assert sol['n_accepted'][b] == len(ref['state'])
        multi += len(ref['state']) > 1
        X, U = ref['state'][-1], ref['control'][-1]
        np.testing.assert_allclose(sol['X'][b].T, X, rtol=0, atol=1e-5 * np.abs(X).max())
        np.testing.assert_allclose(sol['U'][b][:, :U.shape[0]].T, U, rtol=0, atol=1e-5 * np.abs(U).max())
        # the device's linearization point is the last accepted solution
        np.testing.assert_allclose(Xl[b].T, X, rtol=0, atol=1e-5 * np.abs(X).max())
        last = [r['conv'] for r in log if 'conv' in r][-1]
        assert abs(conv[b] - last) <= 1e-5 * max(1.0, abs(last))
        if sol['status'][b] == 1:
            assert conv[b] < p['scp_params']['convergence_threshold']
    assert multi >= 1   # the mode does iterate past the reference's single accepted step


def test_reference_mode_keeps_the_warm_start():
    pb = make_batch('trot', 30, 2)
    with Solver(pb.robot, 30, 2, 'fp64') as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        Xl, Ul, conv = s.linearization_point()
        sol = s.solution()
    assert np.array_equal(Xl, pb.Xbar) and np.array_equal(Ul[:, :, :pb.Ubar.shape[2]], pb.Ubar)
    assert np.all(conv == 0.0) and np.all(sol['n_accepted'] <= 1)


def test_device_interpolation_matches_reference_formula():
    N, B, ni = 30, 3, 10
    pb = make_batch('trot', N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        Xi, Ui = s.interpolate(ni)
    for b in range(B):
        X, U = sol['X'][b].T, sol['U'][b].T
        # reference src/scp_solver.py:95-111, loop form
        Xr = np.zeros((9, (X.shape[1] - 1) * ni)); Ur = np.zeros((U.shape[0], (U.shape[1] - 1) * ni))
        for i in range(U.shape[1] - 1):
            du = (U[:, i + 1] - U[:, i]) / float(ni)
            for j in range(ni):
                Ur[:, i * ni + j] = U[:, i] + j * du
        for i in range(X.shape[1] - 1):
            dx = (X[:, i + 1] - X[:, i]) / float(ni)
            for j in range(ni):
                Xr[:, i * ni + j] = X[:, i] + j * dx
        np.testing.assert_allclose(Xi[b], Xr, rtol=1e-14, atol=1e-14)
        np.testing.assert_allclose(Ui[b], Ur, rtol=1e-14, atol=1e-14)


def test_accepted_gains_and_covariances_survive_mode_switch():
    """Reference mode serves an accepted iteration's K and Sigma from the live linearization
    arrays (the linearization point never moves, quirk Q1, so they are that iteration's arrays,
    as the reference keeps references to them); switching to GuSTO mode first copies them, so
    the accepted results are bit-identical before and after the switch and after a GuSTO-mode
    iteration that moves the linearization point."""
    pb = make_batch('trot', 30, 3)
    with Solver(pb.robot, 30, 3, 'fp64') as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        assert np.all(sol['n_accepted'] >= 1)
        lin = s.linearization()
        np.testing.assert_array_equal(sol['K'], lin['K'])
        np.testing.assert_array_equal(sol['Sigma'], lin['Sigma'])
        s.set_scp_mode('gusto')
        sol2 = s.solution()
        np.testing.assert_array_equal(sol2['K'], sol['K'])
        np.testing.assert_array_equal(sol2['Sigma'], sol['Sigma'])
        s.linearize()          # the same inputs: the live arrays are recomputed, the accepted copies stay
        s.set_trust_region(radius=np.full(3, 1e-9))   # every further iteration rejects: nothing new accepted
        s.scp_iterate(fixed_iters=True)
        sol3 = s.solution()
        np.testing.assert_array_equal(sol3['n_accepted'], sol['n_accepted'])
        np.testing.assert_array_equal(sol3['K'], sol['K'])
        np.testing.assert_array_equal(sol3['Sigma'], sol['Sigma'])


@pytest.mark.parametrize('cfg,N,B', [('trot', 30, 3), ('bound', 30, 2)])
def test_gusto_accepted_history_matches_oracle(cfg, N, B):
    """Every accepted iterate, in acceptance order (the reference appends each one,
    src/scp_solver.py:162-167): list lengths equal the oracle's GuSTO loop's, and each accepted X,
    U, K, Sigma matches it (X, U 1e-5 of scale; K, Sigma 1e-5 relative: they are linearized at
    the previous accepted X, U, so they inherit the QP's 1e-10-level differences, amplified by the
    Riccati steps).  The drop-in's solve_scp_batch returns the same lists."""
    pb = make_batch(cfg, N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.set_scp_mode('gusto')
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        acc = [s.accepted(j) for j in range(int(sol['n_accepted'].max()))]
        rec, nrec = s.iteration_history()
    multi = 0
    for b in range(B):
        p = pb.oracle_problem(b)
        log = []
        ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp, log=log, gusto=True)
        assert ref is not False and int(sol['n_accepted'][b]) == len(ref['state'])
        multi += len(ref['state']) > 1
        for j in range(len(ref['state'])):
            X, U, K, S = ref['state'][j], ref['control'][j], ref['gains'][j], ref['covs'][j]
            np.testing.assert_allclose(acc[j]['X'][b].T, X, rtol=0, atol=1e-5 * np.abs(X).max())
            np.testing.assert_allclose(acc[j]['U'][b][:, :U.shape[0]].T, U, rtol=0, atol=1e-5 * np.abs(U).max())
            np.testing.assert_allclose(acc[j]['K'][b][:, :K.shape[1]], K, rtol=0, atol=1e-5 * np.abs(K).max())
            np.testing.assert_allclose(acc[j]['Sigma'][b], S, rtol=0, atol=1e-5 * np.abs(S).max())
        for j in range(len(ref['state']), len(acc)):   # beyond this problem's accepts: zeros
            assert not acc[j]['X'][b].any()
        # one record per iteration, the oracle's decisions, trust regions and norms
        assert int(nrec[b]) == len(log)
        code = {'accept': 1, 'reject_rho': 2, 'reject_tr': 3}
        for i, r in enumerate(log):
            d = rec[b][i]
            assert int(d['iteration']) == i and int(d['decision']) == code[r['decision']]
            assert abs(d['weight'] - r['weight']) <= 1e-12 * r['weight']
            assert abs(d['radius'] - r['radius']) <= 1e-12 * r['radius']
            assert abs(d['tr_norm'] - r['tr_norm']) <= 1e-5 * max(1.0, r['tr_norm'])
            if 'rho' in r:
                assert abs(d['rho'] - r['rho']) <= 1e-5 * max(1e-6, abs(r['rho']))
            else:
                assert np.isnan(d['rho'])
    assert multi >= 1


def test_reference_mode_iteration_history_with_rejects():
    """Reference mode with a radius small enough that the first iterations reject (trust-region
    rejects raise the weight, rho rejects halve the radius): the per-iteration records equal the
    oracle's log of the reference's state machine, and the single accepted iterate is history
    slot 0 (= cmpc_get_solution)."""
    N, B = 30, 3
    pb = make_batch('trot', N, B)
    for p in pb.params:
        p.scp_params = dict(p.scp_params, trust_region_radius0=0.05)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        rec, nrec = s.iteration_history()
        a0 = s.accepted(0)
    code = {'accept': 1, 'reject_rho': 2, 'reject_tr': 3}
    saw_reject = 0
    for b in range(B):
        p = pb.oracle_problem(b)
        log = []
        OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp, log=log)
        assert int(nrec[b]) == len(log) == int(sol['iterations'][b])
        saw_reject += sum(r['decision'] != 'accept' for r in log)
        for i, r in enumerate(log):
            d = rec[b][i]
            assert int(d['decision']) == code[r['decision']], (b, i, d, r)
            assert abs(d['weight'] - r['weight']) <= 1e-12 * r['weight']
            assert abs(d['radius'] - r['radius']) <= 1e-12 * r['radius']
        if sol['n_accepted'][b]:
            np.testing.assert_array_equal(a0['X'][b], sol['X'][b])
            np.testing.assert_array_equal(a0['K'][b], sol['K'][b])
    assert saw_reject >= 1
