"""The oracle restatement against golden vectors produced by the reference's own code
(tests/golden/make_golden.py).  Tolerances: the fixtures were computed by the reference in
float64 under numpy stand-ins (forward-difference Jacobians, exact up to rounding)."""
import numpy as np
import pytest

from oracle import model as M, transcription as T
from oracle.scp import solve_scp
from oracle.osqp_admm import solve_qp
from helpers import golden_batch, golden_csc, golden_P, same_bounds

TAGS = ['trot', 'trot_stoch', 'bound', 'pace', 'talos']


def _prob(tag, golden):
    g = golden[tag]
    return g, golden_batch(tag, g).oracle_problem(0)


@pytest.mark.parametrize('tag', TAGS)
def test_linearization_matches_reference(tag, golden):
    g, p = _prob(tag, golden)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    np.testing.assert_allclose(td['dynamics'], g['dynamics'], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(td['f_x'], g['f_x'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(td['f_u'], g['f_u'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(td['f_w'], g['f_w'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(td['LQR_gains'], g['K'], rtol=1e-7, atol=1e-9 * np.abs(g['K']).max())
    np.testing.assert_allclose(td['Covs'], g['Covs'], rtol=1e-7, atol=1e-9 * np.abs(g['Covs']).max())
    # the reference's covariance-gradient tensors are identically zero (quirk Q3)
    assert g['cov_grad_maxabs'] == 0.0


@pytest.mark.parametrize('tag', TAGS)
def test_cost_matches_reference(tag, golden):
    g, p = _prob(tag, golden)
    P, q = T.build_cost(p['N'], p['prm'], p['Xbar'])
    assert abs(P - golden_P(g)).max() == 0.0
    np.testing.assert_allclose(q, g['q'], rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize('tag', TAGS)
@pytest.mark.parametrize('which', ['c1', 'c2'])
def test_constraints_match_reference(tag, which, golden):
    g, p = _prob(tag, golden)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    w, r = g['tr1'] if which == 'c1' else g['tr2']
    A, l, u = T.build_constraints(p['N'], p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td, w, r)
    A0, l0, u0 = golden_csc(g, which)
    assert A.shape == A0.shape
    assert abs(A - A0).max() <= 1e-12
    assert same_bounds(l, l0, 1e-9) and same_bounds(u, u0, 1e-9)


@pytest.mark.parametrize('tag', TAGS)
def test_rollout_and_model_accuracy(tag, golden):
    g, p = _prob(tag, golden)
    roll = M.integrate_dynamics_trajectory(g['rollout_X'], g['rollout_U'], p['logic'], p['pos'], p['rot'], p['prm'])
    np.testing.assert_allclose(roll, g['rollout'], rtol=1e-13, atol=1e-13)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    rho = M.compute_model_accuracy(g['rollout_X'], g['rollout_U'], p['Xbar'], p['Ubar'], td, p['logic'], p['pos'],
                                   p['rot'], p['prm'])
    assert abs(rho - float(g['rho'])) <= 1e-9 * max(1.0, abs(float(g['rho'])))


@pytest.mark.parametrize('tag', TAGS)
def test_interpolation(tag, golden):
    g = golden[tag]
    Xi, Ui = T.interpolate_scp_solution(g['rollout_X'], g['rollout_U'])
    np.testing.assert_allclose(Xi, g['interp_X'], rtol=0, atol=1e-15)
    np.testing.assert_allclose(Ui, g['interp_U'], rtol=0, atol=1e-15)


@pytest.mark.parametrize('tag', ['trot', 'bound', 'pace', 'talos'])
def test_scp_state_machine_matches_reference(tag, golden):
    """Same QP solver (the oracle restatement) under the reference's solve_scp and the oracle's."""
    g, p = _prob(tag, golden)
    sp = dict(p['scp_params'])
    sol = solve_scp(p, sp, qp=lambda *a: solve_qp(*a, max_iter=20000))
    if not int(g['scp_ok']):
        assert sol is False
        return
    assert sol is not False
    assert len(sol['state']) == int(g['scp_n_accepted'])
    np.testing.assert_allclose(sol['state'][-1], g['scp_X'], rtol=0, atol=1e-9)
    np.testing.assert_allclose(sol['control'][-1], g['scp_U'], rtol=0, atol=1e-9)
