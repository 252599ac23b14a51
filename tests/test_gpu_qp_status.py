"""GPU: the QP's exit statuses (OSQP's codes, include/cmpc.h) through the C ABI.

* 'solved' (1) means merit <= 1 for every problem, at the metric config and at BASELINE C3's
  fp32 size, so no problem leaves through the stall guard ('solved inaccurate', 2);
* a primal infeasible subproblem (final vertical momentum below the free-fall bound) exits early
  with -3, the status the reference's OSQP returns for it (the OSQP restatement agrees on the
  exported QP), and the SCP loop records a failed QP for that problem only (quirk Q13);
* iterative refinement is rare on regular problems.
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch
from oracle.kkt import kkt_residuals
from oracle.osqp_admm import solve_qp as admm_qp

pytestmark = pytest.mark.gpu


def _solver(cfg, N, B, prec='fp64', edit=None):
    pb = make_batch(cfg, N, B)
    if edit is not None:
        edit(pb)
    s = Solver(pb.robot, N, B, prec)
    s.upload(pb)
    return pb, s


def test_metric_config_exits_are_genuine():
    pb, s = _solver('trot', 100, 1024)
    s.scp_iterate(fixed_iters=True)
    z, y, st, it = s.qp_solution(with_y=False)
    merit, nref = s.qp_info()
    s.close()
    assert np.all(st == 1), np.unique(st, return_counts=True)
    assert np.all(merit <= 1.0), merit.max()
    assert nref.sum() <= 0.01 * it.sum(), (nref.sum(), it.sum())


def test_fp32_bound_c3_exits_are_genuine():
    """BASELINE C3 (bound, N=100, 1024 problems, fp32): every QP meets the fp32 tolerance (1e-6
    relative) with merit <= 1, not through the stall guard."""
    pb, s = _solver('bound', 100, 1024, 'fp32')
    s.scp_iterate(fixed_iters=True)
    z, y, st, it = s.qp_solution(with_y=False)
    merit, nref = s.qp_info()
    s.close()
    assert np.all(st == 1), np.unique(st, return_counts=True)
    assert np.all(merit <= 1.0), merit.max()


def _infeasible_odd(pb):
    N, par = pb.N, pb.params[0]
    for b in range(1, pb.B, 2):
        pb.Xbar[b, N, 5] = pb.Xbar[b, 0, 5] + N * par.dt * par.mass * par.gravity - 1.0


def test_primal_infeasible_detected():
    N, B = 30, 4
    pb, s = _solver('trot', N, B, edit=_infeasible_odd)
    s.linearize(); s.assemble(); s.qp_solve()
    z, y, st, it = s.qp_solution()
    assert list(st) == [1, -3, 1, -3], st
    assert it[1] <= 55 and it[3] <= 55, it   # before the 60-step cap (mirror: 36-40)
    P, q, A, l, u = s.export_qp(1)
    assert admm_qp(P, q, A, l, u).info.status == 'primal infeasible'
    P, q, A, l, u = s.export_qp(0)
    assert kkt_residuals(P, q, A, l, u, z[0], y[0])['prim'] <= 1e-8
    s.close()


def test_infeasible_problem_fails_only_itself_in_solve_scp():
    N, B = 30, 4
    pb, s = _solver('trot', N, B, edit=_infeasible_odd)
    s.solve_scp(fixed_iters=False)
    sol = s.solution()
    log = s.iteration_log()
    s.close()
    assert list(sol['status'][1::2]) == [-1, -1]
    assert list(log['qp_status'][1::2]) == [-3, -3]
    assert all(v != -1 for v in sol['status'][0::2])
