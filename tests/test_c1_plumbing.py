"""BASELINE C1 on the CPU: conf_solo12_trot, N=50, one problem, through the reference's CPU path as
restated by the oracle (numpy linearization, reference-order CSC assembly, the OSQP algorithm at
the reference's eps 1e-7 with polish, the solve_scp state machine of src/scp_solver.py:118-179).
The GPU runs the same case in tests/test_gpu_parity.py::test_solve_scp_matches_oracle[trot-50-1].

Checks the plumbing: the reference's return format (lists of accepted states (9, N+1), controls
(nu, N), gains (N, nu, 9) and covariances (N+1, 9, 9)), the loop's exit after the first accepted
iteration (quirk Q1), and the accepted QP solution's KKT residuals on the reference-form QP."""
import numpy as np

from cmpc.synth import make_batch
from oracle import model as M, transcription as T
from oracle import scp as OS
from oracle.kkt import kkt_residuals
from oracle.osqp_admm import solve_qp


def test_c1_trot_n50_single_problem():
    N = 50
    pb = make_batch('trot', N, 1)
    p = pb.oracle_problem(0)
    log = []
    sol = OS.solve_scp(p, p['scp_params'], qp=lambda *a: solve_qp(*a, max_iter=20000), log=log)
    assert sol is not False
    assert set(sol) >= {'state', 'control', 'gains', 'covs'}
    assert len(sol['state']) == 1 and log[-1]['decision'] == 'accept'      # Q1: exits after the first accept
    X, U = sol['state'][0], sol['control'][0]
    assert X.shape == (9, N + 1) and U.shape == (12, N)
    assert sol['gains'][0].shape == (N, 12, 9) and sol['covs'][0].shape == (N + 1, 9, 9)
    # the accepted iterate solves the QP of its iteration (weight / radius of that iteration)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    P, q = T.build_cost(N, p['prm'], p['Xbar'])
    A, l, u = T.build_constraints(N, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td,
                                  log[-1]['weight'], log[-1]['radius'])
    z = np.concatenate([X.ravel(order='F'), U.ravel(order='F'), np.zeros(2 * N + 1)])
    res = solve_qp(P, q, A, l, u, max_iter=20000)
    z[9 * (N + 1) + 12 * N:] = res.x[9 * (N + 1) + 12 * N:]
    assert kkt_residuals(P, q, A, l, u, z)['prim'] <= 1e-6
