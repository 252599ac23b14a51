"""GPU against the reference's own outputs: the golden fixtures (tests/golden/golden_*.npz, made by
tests/golden/make_golden.py, which runs the reference's src/centroidal_model.py:257-291,
src/scp_solver.py:10-48 and its solve_scp state machine) are uploaded through the C ABI and the
device results are compared with the reference-produced arrays directly, not through the oracle.

Fixtures: N=20 per robot / gait, BASELINE C1's horizon (trot N=50), the metric config's and C2's
(trot N=100), C3's bound N=100, and two float32 fixtures (trot N=20, bound N=100) made at the
reference's own precision (JAX float32), compared with the device's fp32 path.

Tolerances, float64 fixtures (the reference under numpy stand-ins, with forward-difference
Jacobians that are exact up to rounding because the dynamics are bilinear):
  * f, A, B, C: 1e-12 absolute; K, Sigma: 1e-7 relative to their max (the stand-in's finite
    differences perturb the LQR gains at that level; the oracle meets the same bound);
  * exported P, q exactly / 1e-14; constraint matrix 1e-12; bounds 1e-9 (same as the oracle);
  * rollout 1e-13;
  * solve_scp: the same success flag and number of accepted iterations, the accepted X and U
    within 1e-5 relative (the reference's state machine was run with the OSQP restatement; the
    GPU QP is an interior-point method at 1e-10);
  * the device's model-accuracy ratio rho against the reference formula
    (src/scp_solver.py:71-87, restated in oracle.model) evaluated on the device's own QP solution,
    1e-10 relative.
Float32 fixtures against the device's fp32 path: f, A, B, C, rollout 2e-6 relative to each
array's max (a few float32 ulps: different summation order); K, Sigma 1e-4 (two Riccati steps in
information form against the reference's solves, then the scan); exported constraint values and
bounds 2e-6; the accepted X, U of solve_scp 5e-3 (the fp32 QP stops at 1e-6, the fixture's QP ran
in float64 on the float32 data).
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from conftest import GOLDEN_TAGS
from helpers import golden_batch, golden_csc, golden_P, golden_fp32, same_bounds
from oracle import model as M

pytestmark = pytest.mark.gpu

TAGS = list(GOLDEN_TAGS)


def _upload(tag, golden):
    if tag not in golden:
        pytest.skip('fixture %s missing' % tag)
    g = golden[tag]
    pb = golden_batch(tag, g)
    s = Solver(pb.robot, pb.N, 1, 'fp32' if golden_fp32(g) else 'fp64')
    s.upload(pb)
    return g, pb, s


def _close(a, b, rel):
    a = np.asarray(a, float); b = np.asarray(b, float)
    np.testing.assert_allclose(a, b, rtol=0, atol=rel * max(np.abs(b).max(), 1e-300))


@pytest.mark.parametrize('tag', TAGS)
def test_linearization_equals_reference_outputs(tag, golden):
    g, pb, s = _upload(tag, golden)
    s.linearize()
    lin = s.linearization()
    s.close()
    if golden_fp32(g):
        _close(lin['f'][0], g['dynamics'].T, 2e-6)
        _close(lin['A'][0], g['f_x'], 2e-6)
        _close(lin['Bu'][0], g['f_u'], 2e-6)
        _close(lin['C'][0], g['f_w'], 2e-6)
        _close(lin['K'][0], g['K'], 1e-4)
        _close(lin['Sigma'][0], g['Covs'], 1e-4)
        return
    np.testing.assert_allclose(lin['f'][0], g['dynamics'].T, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(lin['A'][0], g['f_x'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['Bu'][0], g['f_u'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['C'][0], g['f_w'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['K'][0], g['K'], rtol=0, atol=1e-7 * np.abs(g['K']).max())
    np.testing.assert_allclose(lin['Sigma'][0], g['Covs'], rtol=0, atol=1e-7 * np.abs(g['Covs']).max())


@pytest.mark.parametrize('tag', TAGS)
@pytest.mark.parametrize('which', ['c1', 'c2'])
def test_exported_qp_equals_reference_matrices(tag, which, golden):
    g, pb, s = _upload(tag, golden)
    w, r = g['tr1'] if which == 'c1' else g['tr2']
    s.set_trust_region(weight=w, radius=r)
    s.linearize(); s.assemble()
    P, q, A, l, u = s.export_qp(0)
    s.close()
    assert abs(P - golden_P(g)).max() == 0.0
    if golden_fp32(g):   # the device forms q = -Wx xbar in float32
        _close(q, g['q'], 2e-7)
    else:
        np.testing.assert_allclose(q, g['q'], rtol=1e-14, atol=1e-14)
    A0, l0, u0 = golden_csc(g, which)
    assert A.shape == A0.shape
    if golden_fp32(g):
        assert abs(A - A0).max() <= 2e-6 * abs(A0).max()
        assert same_bounds(l, l0, 2e-6) and same_bounds(u, u0, 2e-6)
        return
    assert abs(A - A0).max() <= 1e-12
    assert same_bounds(l, l0, 1e-9) and same_bounds(u, u0, 1e-9)


@pytest.mark.parametrize('tag', TAGS)
def test_rollout_equals_reference(tag, golden):
    g, pb, s = _upload(tag, golden)
    out = s.rollout(g['rollout_X'].T[None], g['rollout_U'].T[None])
    s.close()
    if golden_fp32(g):
        _close(out[0].T, g['rollout'], 2e-6)
        return
    np.testing.assert_allclose(out[0].T, g['rollout'], rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize('tag', [t for t in TAGS if t != 'trot_stoch'])
def test_solve_scp_equals_reference_state_machine(tag, golden):
    """The device loop against the reference's own solve_scp run (every fixture accepts; TALOS
    since its synthetic radius0 is 1000, config/conf_talos.py): same success flag and number of
    accepted iterations, and the accepted X, U (for TALOS the accepted K and Sigma too, read back
    through the accept / keep path).  The fixtures hold no per-iteration decision sequence
    (make_golden.py keeps scp_ok, scp_n_accepted, scp_X, scp_U), so the sequence is not compared."""
    g, pb, s = _upload(tag, golden)
    s.solve_scp(fixed_iters=False)
    sol = s.solution()
    s.close()
    assert int(g['scp_ok']) == 1
    assert sol['status'][0] != -1
    assert int(sol['n_accepted'][0]) == int(g['scp_n_accepted'])
    X, U = sol['X'][0].T, sol['U'][0].T
    tol = 5e-3 if golden_fp32(g) else 1e-5
    _close(X, g['scp_X'], tol)
    _close(U, g['scp_U'], tol)
    if not golden_fp32(g):
        _close(sol['K'][0], g['K'], 1e-7)
        _close(sol['Sigma'][0], g['Covs'], 1e-7)


@pytest.mark.parametrize('tag', ['trot', 'bound', 'talos', 'trot_n50', 'trot_n100', 'bound_n100'])
def test_device_rho_matches_reference_formula(tag, golden):
    g, pb, s = _upload(tag, golden)
    s.scp_iterate(fixed_iters=True)
    z, _, st, _ = s.qp_solution(with_y=False)
    rho_dev = float(s.iteration_log()['rho'][0])
    s.close()
    assert st[0] == 1
    p = pb.oracle_problem(0)
    N, nu = p['N'], 12
    X = z[0][:9 * (N + 1)].reshape(N + 1, 9).T
    U = z[0][9 * (N + 1):9 * (N + 1) + nu * N].reshape(N, nu).T
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    rho = M.compute_model_accuracy(X, U, p['Xbar'], p['Ubar'], td, p['logic'], p['pos'], p['rot'], p['prm'])
    assert abs(rho_dev - rho) <= 1e-10 * max(abs(rho), 1e-300), (rho_dev, rho)
