"""GPU: the QP kernel's one-wave and two-wave workgroups (cmpc_qp_settings.waves_per_problem)
solve the same problems to the same answers.

With two waves the per-knot phases run one knot per thread over 128 threads and the Schur
recurrence stays on the first wave; the fused right-hand side's last term then crosses a wave
boundary and goes through an LDS side array (qp_ipm.hip add_wx).  The two variants differ only
in the summation order of the block-wide reductions.  On Solo12 problems statuses, Newton
iteration counts and SCP decisions must agree and the solutions to 1e-9 relative.  TALOS QPs are
ill-conditioned: a last-bit change in mu moves the Newton path (measured with
scripts/waves_diag.py: +-1..2 Newton steps and 0.4-3.6e-6 relative solution differences at
N = 100, 127 and 200, identically at one knot pass per thread, while each variant repeats
bit-exactly), so there both must solve, iteration counts agree within 2 and solutions within the
1e-5 parity bar of the oracle tests.  Horizons cover one knot pass (N = 63),
exactly two waves (N = 127), the metric horizon, and TALOS at BASELINE C4's N = 200 (two passes
of 128 knots); the last knot block straddles the wave boundary in all of them.
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import make_batch

pytestmark = pytest.mark.gpu


def _run(pb, waves, steps=2):
    s = Solver(pb.robot, pb.N, pb.B, 'fp64')
    s.set_qp_settings(waves_per_problem=waves)
    s.upload(pb)
    out = []
    for _ in range(steps):
        s.scp_iterate(fixed_iters=True)
        z, _, st, it = s.qp_solution(with_y=False)
        out.append((z.copy(), st.copy(), it.copy(), s.iteration_log()['decision'].copy()))
    s.close()
    return out


@pytest.mark.parametrize('cfg,N,B', [('trot', 63, 8), ('trot', 127, 8), ('trot', 100, 64), ('talos', 200, 16),
                                     ('bound', 100, 8)])
def test_two_wave_workgroup_matches_one_wave(cfg, N, B):
    pb = make_batch(cfg, N, B, seed_offset=31)
    one, two = _run(pb, 1), _run(pb, 2)
    talos = cfg == 'talos'
    for (z1, s1, i1, d1), (z2, s2, i2, d2) in zip(one, two):
        assert np.all(s1 == 1) and np.all(s2 == 1), (s1, s2)
        if talos:
            assert np.abs(i1 - i2).max() <= 2, (i1, i2)
        else:
            np.testing.assert_array_equal(i1, i2)
        np.testing.assert_array_equal(d1, d2)
        err = np.abs(z1 - z2).max(axis=1) / np.abs(z1).max(axis=1)
        assert err.max() <= (1e-5 if talos else 1e-9), err.max()


@pytest.mark.parametrize('cfg,N,B', [('trot', 40, 8), ('trot', 100, 64), ('trot', 255, 4), ('bound', 100, 8),
                                     ('talos', 200, 16), ('pace', 150, 8)])
def test_four_wave_partitioned_recurrence(cfg, N, B):
    """Four-wave workgroups factor the Schur system as four chains around three separators
    (schur_pt.hpp), a different elimination order from the two-ended recurrence, so results agree
    to rounding: every QP solved, Newton counts within one (TALOS two), SCP decisions equal,
    solutions within 1e-7 (TALOS 1e-5) of the one-wave kernel's, and the first and last problems
    within 1e-5 of the oracle's sparse IPM on the exported QP."""
    from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
    pb = make_batch(cfg, N, B, seed_offset=41)
    one, four = _run(pb, 1), _run(pb, 4)
    talos = cfg == 'talos'
    for (z1, s1, i1, d1), (z4, s4, i4, d4) in zip(one, four):
        assert np.all(s1 == 1) and np.all(s4 == 1), (s1, s4)
        assert np.abs(i1 - i4).max() <= (2 if talos else 1), (i1, i4)
        np.testing.assert_array_equal(d1, d4)
        err = np.abs(z1 - z4).max(axis=1) / np.abs(z1).max(axis=1)
        assert err.max() <= (1e-5 if talos else 1e-7), err.max()
    s = Solver(pb.robot, N, B, 'fp64')
    s.set_qp_settings(waves_per_problem=4)
    s.upload(pb)
    s.scp_iterate(fixed_iters=True)
    z, _, st, _ = s.qp_solution(with_y=False)
    nx = 9 * (N + 1)
    for b in (0, B - 1):
        P, q, A, l, u = s.export_qp(b)
        ref = sparse_ipm_qp(P, q, A, l, u)
        assert np.abs(z[b][:nx] - ref.x[:nx]).max() / np.abs(ref.x[:nx]).max() <= 1e-5
    s.close()


def test_waves_setting_is_validated():
    """waves_per_problem: 0 (auto, the default), 1, 2 or 4; anything else is refused."""
    pb = make_batch('trot', 20, 2)
    s = Solver(pb.robot, 20, 2, 'fp64')
    s.set_qp_settings(waves_per_problem=0)
    s.set_qp_settings(waves_per_problem=4)
    with pytest.raises(Exception):
        s.set_qp_settings(waves_per_problem=3)
    with pytest.raises(Exception):
        s.set_qp_settings(waves_per_problem=8)
    s.close()


@pytest.mark.parametrize('cfg,N,eta', [('trot', 40, 0.999), ('talos', 40, 0.995)])
def test_step_fraction_default_is_per_robot(cfg, N, eta):
    """step_fraction 0 (the default) resolves to the robot's value (cmpc_api.cpp qp_step_fraction):
    a default run and one with that value set explicitly are bit-identical; 0.9 differs."""
    pb = make_batch(cfg, N, 4, seed_offset=7)

    def run(**kw):
        s = Solver(pb.robot, N, pb.B, 'fp64')
        if kw:
            s.set_qp_settings(**kw)
        s.upload(pb)
        s.scp_iterate(fixed_iters=True)
        z, _, st, it = s.qp_solution(with_y=False)
        s.close()
        return z, st, it

    z0, s0, i0 = run()
    z1, s1, i1 = run(step_fraction=eta)
    assert np.all(s0 == 1)
    np.testing.assert_array_equal(i0, i1)
    np.testing.assert_array_equal(z0, z1)
    z2, _, _ = run(step_fraction=0.9)
    assert not np.array_equal(z0, z2)
    s = Solver(pb.robot, N, pb.B, 'fp64')
    with pytest.raises(Exception):
        s.set_qp_settings(step_fraction=-0.5)
    with pytest.raises(Exception):
        s.set_qp_settings(step_fraction=1.0)
    s.close()
