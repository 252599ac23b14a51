"""GPU against the reference's own outputs: the golden fixtures (tests/golden/golden_*.npz, made by
tests/golden/make_golden.py, which runs the reference's src/centroidal_model.py:257-291,
src/scp_solver.py:10-48 and its solve_scp state machine) are uploaded through the C ABI and the
device results are compared with the reference-produced arrays directly, not through the oracle.

Tolerances (the fixtures are the reference computed in float64 under numpy stand-ins, with
forward-difference Jacobians that are exact up to rounding because the dynamics are bilinear):
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
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from helpers import golden_batch, golden_csc, golden_P, same_bounds
from oracle import model as M

pytestmark = pytest.mark.gpu

TAGS = ['trot', 'trot_stoch', 'bound', 'pace', 'talos']


def _upload(tag, g):
    pb = golden_batch(tag, g)
    s = Solver(pb.robot, pb.N, 1, 'fp64')
    s.upload(pb)
    return pb, s


@pytest.mark.parametrize('tag', TAGS)
def test_linearization_equals_reference_outputs(tag, golden):
    g = golden[tag]
    pb, s = _upload(tag, g)
    s.linearize()
    lin = s.linearization()
    s.close()
    np.testing.assert_allclose(lin['f'][0], g['dynamics'].T, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(lin['A'][0], g['f_x'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['Bu'][0], g['f_u'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['C'][0], g['f_w'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(lin['K'][0], g['K'], rtol=0, atol=1e-7 * np.abs(g['K']).max())
    np.testing.assert_allclose(lin['Sigma'][0], g['Covs'], rtol=0, atol=1e-7 * np.abs(g['Covs']).max())


@pytest.mark.parametrize('tag', TAGS)
@pytest.mark.parametrize('which', ['c1', 'c2'])
def test_exported_qp_equals_reference_matrices(tag, which, golden):
    g = golden[tag]
    pb, s = _upload(tag, g)
    w, r = g['tr1'] if which == 'c1' else g['tr2']
    s.set_trust_region(weight=w, radius=r)
    s.linearize(); s.assemble()
    P, q, A, l, u = s.export_qp(0)
    s.close()
    assert abs(P - golden_P(g)).max() == 0.0
    np.testing.assert_allclose(q, g['q'], rtol=1e-14, atol=1e-14)
    A0, l0, u0 = golden_csc(g, which)
    assert A.shape == A0.shape
    assert abs(A - A0).max() <= 1e-12
    assert same_bounds(l, l0, 1e-9) and same_bounds(u, u0, 1e-9)


@pytest.mark.parametrize('tag', TAGS)
def test_rollout_equals_reference(tag, golden):
    g = golden[tag]
    pb, s = _upload(tag, g)
    out = s.rollout(g['rollout_X'].T[None], g['rollout_U'].T[None])
    s.close()
    np.testing.assert_allclose(out[0].T, g['rollout'], rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize('tag', ['trot', 'bound', 'pace', 'talos'])
def test_solve_scp_equals_reference_state_machine(tag, golden):
    """TALOS: the fixture's run returned False because its QP stand-in (the OSQP restatement,
    capped at 20000 ADMM iterations) did not converge on the TALOS subproblems, not because a
    subproblem is infeasible; so the device loop is compared with the reference's state machine
    restated by the oracle and fed an exact QP solver (sparse IPM) on the same inputs."""
    g = golden[tag]
    pb, s = _upload(tag, g)
    s.solve_scp(fixed_iters=False)
    sol = s.solution()
    log = s.iteration_log()
    s.close()
    if tag == 'talos':
        from oracle import scp as OS
        from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
        assert int(g['scp_ok']) == 0
        p = pb.oracle_problem(0)
        olog = []
        ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp, log=olog)
        assert ref is not False and int(sol['status'][0]) != -1
        assert int(sol['iterations'][0]) == len(olog)
        assert int(sol['n_accepted'][0]) == len(ref['state'])
        return
    ok = int(g['scp_ok'])
    assert (sol['status'][0] != -1) == bool(ok)
    if not ok:
        return
    assert int(sol['n_accepted'][0]) == int(g['scp_n_accepted'])
    X, U = sol['X'][0].T, sol['U'][0].T
    np.testing.assert_allclose(X, g['scp_X'], rtol=0, atol=1e-5 * np.abs(g['scp_X']).max())
    np.testing.assert_allclose(U, g['scp_U'], rtol=0, atol=1e-5 * np.abs(g['scp_U']).max())


@pytest.mark.parametrize('tag', ['trot', 'bound', 'talos'])
def test_device_rho_matches_reference_formula(tag, golden):
    g = golden[tag]
    pb, s = _upload(tag, g)
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
