"""GPU: QPs in the reference's CSC layout that the device did not assemble (cmpc_load_qp, the
drop-in solve_subproblem on plain Cost / Constraint tuples; reference src/scp_solver.py:59-68).

* round trip: a device-assembled QP exported with cmpc_export_qp and loaded into another handle
  solves to the same answer (same Newton steps, 1e-9 relative): the decoder recovers the stage
  record, the weights and dt / mass;
* foreign QPs: the reference-form QP built by the oracle's transcription, then edited the way a
  caller might (tighter friction bounds, another trust-region radius and weight, another initial
  state, other cost weights), solved on the device and by the oracle's sparse IPM on the same CSC
  data: 1e-5 relative, as every QP parity test;
* QPs without the stage structure (an off-pattern dynamics entry, an off-diagonal cost term, a
  control gradient) are refused with an error naming the problem, not solved wrongly.
"""
import numpy as np
import pytest
from scipy import sparse

from cmpc._lib import CmpcError, Solver
from cmpc.synth import make_batch
from oracle import model as M, transcription as T
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp

pytestmark = pytest.mark.gpu


def _ref_qp(cfg, N, b=0, stochastic=False, weight=None, radius=None):
    pb = make_batch(cfg, N, 1, stochastic=stochastic, seed_offset=b)
    p = pb.oracle_problem(0)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    sp = p['scp_params']
    P, q = T.build_cost(N, p['prm'], p['Xbar'])
    A, l, u = T.build_constraints(N, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td,
                                  weight or sp['omega0'], radius or sp['trust_region_radius0'])
    return pb, p, [P, q, A, l, u]


def _device_solve(pb, qp):
    s = Solver(pb.robot, pb.N, 1, 'fp64')
    s.upload(pb)
    s.load_qp(0, *qp)
    s.qp_solve()
    z, _, st, it = s.qp_solution(with_y=False)
    s.close()
    return z[0], int(st[0]), int(it[0])


@pytest.mark.parametrize('cfg,N,stoch', [('trot', 30, False), ('trot', 30, True), ('bound', 40, False),
                                         ('talos', 40, False)])
def test_exported_qp_round_trip(cfg, N, stoch):
    pb = make_batch(cfg, N, 2, stochastic=stoch, seed_offset=5)
    s = Solver(pb.robot, N, 2, 'fp64')
    s.upload(pb)
    s.linearize(); s.assemble(); s.qp_solve()
    z0, _, st0, it0 = s.qp_solution(with_y=False)
    qp = s.export_qp(0)
    s.load_qp(1, *qp)          # problem 1's slot now holds problem 0's QP
    s.qp_solve()
    z1, _, st1, it1 = s.qp_solution(with_y=False)
    s.close()
    assert st0[0] == 1 and st1[1] == 1
    if cfg != 'talos':         # TALOS's Newton path moves with last-bit changes (test_gpu_qp_waves.py)
        assert it1[1] == it0[0]
    err = np.abs(z1[1] - z0[0]).max() / np.abs(z0[0]).max()
    assert err <= (1e-5 if cfg == 'talos' else 1e-9), err


def _edit_friction(pb, qp):     # tighter friction cones: every filled friction row's bound -= 0.5
    P, q, A, l, u = qp
    nf = 5 * pb.nc * pb.N
    r0 = A.shape[0] - 9 * (pb.N + 1) - nf
    rows = np.arange(r0, r0 + nf)
    filled = np.diff(A.tocsr().indptr)[rows] > 0
    u = u.copy()
    u[rows[filled]] -= 0.5
    return [P, q, A, l, u]


def _edit_x0(pb, qp):          # another initial state (the init rows' bounds)
    P, q, A, l, u = qp
    l, u = l.copy(), u.copy()
    d = np.array([0.01, -0.02, 0.005, 0.3, -0.2, 0.1, 0.05, -0.04, 0.02])
    l[:9] += d; u[:9] += d
    return [P, q, A, l, u]


def _edit_weights(pb, qp):     # other cost weights (a new parameter class) and a shifted tracking gradient
    P, q, A, l, u = qp
    n = P.shape[0]
    d = P.diagonal().copy()
    nx, nu = 9 * (pb.N + 1), 12 * pb.N
    d[:nx] *= np.tile([2.0, 2.0, 0.5, 1.0, 1.0, 1.0, 3.0, 3.0, 3.0], pb.N + 1)
    d[nx:nx + nu] *= 0.25
    q = q.copy()
    q[:nx] *= 1.5
    return [sparse.diags(d, format='csc', shape=(n, n)), q, A, l, u]


@pytest.mark.parametrize('cfg,N,edit', [('trot', 30, 'friction'), ('trot', 30, 'x0'), ('trot', 30, 'weights'),
                                        ('bound', 30, 'tr'), ('talos', 40, 'friction'), ('talos', 40, 'weights')])
def test_foreign_qp_matches_sparse_ipm(cfg, N, edit):
    if edit == 'tr':           # another trust-region radius and weight than the handle's SCP state
        pb, p, qp = _ref_qp(cfg, N, weight=350.0, radius=0.7)
    else:
        pb, p, qp = _ref_qp(cfg, N)
        qp = {'friction': _edit_friction, 'x0': _edit_x0, 'weights': _edit_weights}[edit](pb, qp)
    z, st, _ = _device_solve(pb, qp)
    ref = sparse_ipm_qp(*qp)
    assert ref.info.status == 'solved' and st == 1, (ref.info.status, st)
    nxu = 9 * (N + 1) + 12 * N
    err = np.abs(z[:nxu] - ref.x[:nxu]).max() / np.abs(ref.x[:nxu]).max()
    assert err <= 1e-5, err


def test_qp_without_stage_structure_is_refused():
    pb, p, (P, q, A, l, u) = _ref_qp('trot', 20)
    s = Solver(pb.robot, 20, 1, 'fp64')
    s.upload(pb)
    A1 = A.tolil(); A1[9 + 3, 2] = 0.7          # dynamics row 3 of knot 0 on a position column
    with pytest.raises(CmpcError, match='centroidal form'):
        s.load_qp(0, P, q, A1.tocsc(), l, u)
    P1 = P.tolil(); P1[0, 1] = P1[1, 0] = 0.1   # coupled cost
    with pytest.raises(CmpcError, match='off-diagonal'):
        s.load_qp(0, P1.tocsc(), q, A, l, u)
    q1 = q.copy(); q1[9 * 21 + 2] = 1.0          # control gradient
    with pytest.raises(CmpcError, match='zero on the controls'):
        s.load_qp(0, P, q1, A, l, u)
    s.close()


def test_dropin_solve_subproblem_on_plain_tuples():
    """The reference's call with Cost / Constraint built outside the drop-in's assembly."""
    from src.constraints import Constraint
    from src.cost import Cost
    from src.scp_solver import solve_subproblem
    pb, p, qp = _ref_qp('trot', 30)
    P, q, A, l, u = _edit_friction(pb, qp)
    ok, res = solve_subproblem(Cost(Q=P, p=q), Constraint(mat=A, lb=l, ub=u))
    assert ok and res.info.status == 'solved'
    ref = sparse_ipm_qp(P, q, A, l, u)
    nxu = 9 * 31 + 12 * 30
    assert np.abs(res.x[:nxu] - ref.x[:nxu]).max() <= 1e-5 * np.abs(ref.x[:nxu]).max()


@pytest.mark.parametrize('cfg,N', [('trot', 30), ('talos', 40)])
def test_load_after_linearize_then_export(cfg, N):
    """Loading into a handle that has already linearized (reference mode: the stage record is
    written, the dense A, Bu are not) must not let a later export or getter rerun the
    linearization over the loaded problem: the export of problem 1 equals the QP loaded into it,
    problem 0's export is unchanged, and the next QP solve solves the loaded QP."""
    pb = make_batch(cfg, N, 2, seed_offset=9)
    s = Solver(pb.robot, N, 2, 'fp64')
    s.upload(pb)
    s.linearize(); s.assemble()
    _, p, qp = _ref_qp(cfg, N, b=3, radius=0.5)
    qp0 = s.export_qp(0)
    s.load_qp(1, *qp)
    P1, q1, A1, l1, u1 = s.export_qp(1)
    P0, q0, A0, l0, u0 = s.export_qp(0)
    lin = s.linearization()
    s.qp_solve()
    z, _, st, _ = s.qp_solution(with_y=False)
    s.close()
    P, q, A, l, u = qp
    assert abs(P1 - P).max() == 0.0 and np.abs(q1 - q).max() <= 1e-12 * np.abs(q).max()
    assert abs(A1 - A).max() <= 1e-12 * abs(A).max()
    fin = np.isfinite(u)
    assert np.array_equal(np.isfinite(u1), fin) and np.abs(u1[fin] - u[fin]).max() <= 1e-9 * (1 + np.abs(u[fin]).max())
    for a, b_ in zip((P0, A0), (qp0[0], qp0[2])):
        assert abs(a - b_).max() == 0.0
    assert np.array_equal(q0, qp0[1])
    # the getter's dense A of the loaded problem is the loaded one
    Adyn = A.tocsr()[9:9 + 9 * N][:, :9 * (N + 1)].toarray()
    for k in (0, N // 2, N - 1):
        assert np.abs(lin['A'][1][k] - Adyn[9 * k:9 * k + 9, 9 * k:9 * k + 9]).max() <= 1e-12
    ref = sparse_ipm_qp(*qp)
    nx = 9 * (N + 1)
    assert st[1] == 1
    assert np.abs(z[1][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max() <= 1e-5
