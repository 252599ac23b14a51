"""The oracle restatement against golden vectors produced by the reference's own code
(tests/golden/make_golden.py).

Tolerances.  The float64 fixtures were computed by the reference under numpy stand-ins
(forward-difference Jacobians, exact up to rounding): f, A, B, C to 1e-12, K and Sigma to 1e-7.
The ``*_f32`` fixtures ran the reference at its own float32 precision (JAX's default);
the oracle run in float32 meets them to 1e-6 relative (f, A, B, C, rollout: a few float32 ulps from
a different summation order) and 1e-5 relative (K, Sigma: two Riccati solves and the scan), and
their constraint bounds, which carry the float32 dynamics residual, to 1e-6.
"""
import numpy as np
import pytest

from conftest import GOLDEN_TAGS
from oracle import model as M, transcription as T
from oracle.scp import solve_scp
from helpers import golden_batch, golden_csc, golden_P, golden_fp32, golden_qp, same_bounds

TAGS = list(GOLDEN_TAGS)


def _prob(tag, golden):
    if tag not in golden:
        pytest.skip('fixture %s missing' % tag)
    g = golden[tag]
    return g, golden_batch(tag, g).oracle_problem(0)


def _dtype(g):
    return np.float32 if golden_fp32(g) else np.float64


def _close(a, b, rel):
    a = np.asarray(a, float); b = np.asarray(b, float)
    np.testing.assert_allclose(a, b, rtol=0, atol=rel * max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize('tag', TAGS)
def test_linearization_matches_reference(tag, golden):
    g, p = _prob(tag, golden)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'], _dtype(g))
    if golden_fp32(g):
        for k, ref in (('dynamics', 'dynamics'), ('f_x', 'f_x'), ('f_u', 'f_u'), ('f_w', 'f_w')):
            assert td[k].dtype == np.float32 and g[ref].dtype == np.float32
            _close(td[k], g[ref], 1e-6)
        _close(td['LQR_gains'], g['K'], 1e-5)
        _close(td['Covs'], g['Covs'], 1e-5)
    else:
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
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'], _dtype(g))
    w, r = g['tr1'] if which == 'c1' else g['tr2']
    A, l, u = T.build_constraints(p['N'], p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td, w, r)
    A0, l0, u0 = golden_csc(g, which)
    assert A.shape == A0.shape
    tol_b = 1e-6 if golden_fp32(g) else 1e-9
    assert abs(A - A0).max() <= (1e-7 if golden_fp32(g) else 1e-12)
    assert same_bounds(l, l0, tol_b) and same_bounds(u, u0, tol_b)


@pytest.mark.parametrize('tag', TAGS)
def test_rollout_and_model_accuracy(tag, golden):
    g, p = _prob(tag, golden)
    dt = _dtype(g)
    roll = M.integrate_dynamics_trajectory(g['rollout_X'], g['rollout_U'], p['logic'], p['pos'], p['rot'], p['prm'], dt)
    if golden_fp32(g):
        _close(roll, g['rollout'], 1e-6)
    else:
        np.testing.assert_allclose(roll, g['rollout'], rtol=1e-13, atol=1e-13)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'], dt)
    rho = M.compute_model_accuracy(g['rollout_X'], g['rollout_U'], p['Xbar'], p['Ubar'], td, p['logic'], p['pos'],
                                   p['rot'], p['prm'], dt)
    tol = 1e-3 if golden_fp32(g) else 1e-9
    assert abs(rho - float(g['rho'])) <= tol * max(1.0 if not golden_fp32(g) else 0.0, abs(float(g['rho'])))


@pytest.mark.parametrize('tag', TAGS)
def test_interpolation(tag, golden):
    if tag not in golden:
        pytest.skip('fixture %s missing' % tag)
    g = golden[tag]
    Xi, Ui = T.interpolate_scp_solution(np.asarray(g['rollout_X'], float), np.asarray(g['rollout_U'], float))
    tol = 1e-6 if golden_fp32(g) else 1e-15
    _close(Xi, g['interp_X'], tol)
    _close(Ui, g['interp_U'], tol)


@pytest.mark.parametrize('tag', [t for t in TAGS if t != 'trot_stoch'])
def test_scp_state_machine_matches_reference(tag, golden):
    """The same QP stand-in under the reference's solve_scp and the oracle's.  1e-9 with the
    OSQP restatement (deterministic ADMM on equal matrices); 1e-6 with the sparse IPM, whose
    answer at its 1e-11 stopping test moves by ~1e-7 of max|X| when the matrices differ in the
    last bits (TALOS: momenta ~40, state cost 1e5)."""
    g, p = _prob(tag, golden)
    sp = dict(p['scp_params'])
    sol = solve_scp(p, sp, qp=golden_qp(tag, g), dtype=_dtype(g))
    assert int(g['scp_ok']) == 1, 'every fixture reaches an accepted iterate (TALOS since radius0 = 1000)'
    assert sol is not False
    assert len(sol['state']) == int(g['scp_n_accepted'])
    tol = 1e-9 if tag in ('trot', 'bound', 'pace') else 1e-6
    _close(sol['state'][-1], g['scp_X'], tol)
    _close(sol['control'][-1], g['scp_U'], tol)
