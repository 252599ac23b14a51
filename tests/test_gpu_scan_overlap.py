"""GPU: the covariance scan off the critical path (cmpc_api.cpp launch_phase).

Inside cmpc_scp_iterate a deterministic batch whose QP leaves SIMDs free (two-wave workgroups, or
fewer QP waves than SIMDs) runs k_cov_scan on a low-priority side stream, joined behind the QP;
when the QP fills the device with one wave per SIMD, the QP kernel's workgroups run the scans
from a job counter once their own problem has converged (k_qp_ipm, cov_scan.hpp).  The
phase-by-phase entry points (cmpc_linearize, cmpc_assemble, cmpc_qp_solve, cmpc_accept) keep the
scan kernel in order on the main stream.  All orders must give bit-identical X, U, K and Sigma:
the scan reads only what k_lin_knots wrote, runs the same code on every path, and nothing else in
the step reads Sigma.  Cases: two-wave batch at the metric horizon (side stream), a small
one-wave batch (side stream), the metric-size batch (scans inside the QP kernel) and a
stochastic batch (Sigma feeds the assembly: in order).
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


def _run(pb, fused, steps=2):
    s = Solver(pb.robot, pb.N, pb.B, 'fp64')
    s.upload(pb)
    for _ in range(steps):
        if fused:
            s.scp_iterate(fixed_iters=True)
        else:
            s.linearize(); s.assemble(); s.qp_solve(); s.accept(fixed_iters=True)
    sol = s.solution()
    lin = s.linearization()
    s.close()
    return sol, lin


@pytest.mark.parametrize('cfg,N,B,stochastic', [('trot', 100, 256, False), ('trot', 40, 16, False),
                                                ('trot', 100, 1024, False), ('trot', 60, 32, True)])
def test_overlapped_scan_matches_in_order(cfg, N, B, stochastic):
    pb = make_batch(cfg, N, B, stochastic=stochastic, seed_offset=11)
    fused, lin_f = _run(pb, True)
    plain, lin_p = _run(pb, False)
    assert np.all(fused['status'] == plain['status'])
    for k in ('X', 'U', 'K', 'Sigma'):
        np.testing.assert_array_equal(fused[k], plain[k], err_msg=k)
    np.testing.assert_array_equal(lin_f['Sigma'], lin_p['Sigma'])
    assert np.abs(lin_f['Sigma'][:, -1]).max() > 0   # the scan ran to the last knot


@pytest.mark.parametrize('N,B', [(100, 1024), (100, 256)])
def test_overlapped_scan_early_exit_path(N, B):
    """The reference's early-exit loop (fixed_iters=False, only the active problems iterate): every
    other problem gets a tiny trust-region radius and keeps rejecting, the rest accept at the first
    iteration and leave the loop.  With problems inactive, the QP workgroups of inactive problems
    return before the scan-job loop (1024: scans inside the QP kernel) and the side-stream scan
    skips them (256); X, U, K, Sigma must equal the phase-by-phase order bit for bit."""
    pb = make_batch('trot', N, B, seed_offset=23)
    radius = np.where(np.arange(B) % 2 == 0, 1e-9, pb.params[0].scp_params['trust_region_radius0'])

    def run(fused):
        s = Solver(pb.robot, N, B, 'fp64')
        s.upload(pb)
        s.set_trust_region(radius=radius)
        for _ in range(3):
            if fused:
                s.scp_iterate(fixed_iters=False)
            else:
                s.linearize(); s.assemble(); s.qp_solve(); s.accept(fixed_iters=False)
        sol = s.solution()
        s.close()
        return sol

    f, p = run(True), run(False)
    assert np.all(f['n_accepted'][1::2] == 1) and np.all(f['n_accepted'][0::2] == 0)
    assert np.all(f['iterations'][1::2] == 1) and np.all(f['iterations'][0::2] == 3)
    for k in ('X', 'U', 'K', 'Sigma', 'iterations', 'status', 'weight', 'radius'):
        np.testing.assert_array_equal(f[k], p[k], err_msg=k)
