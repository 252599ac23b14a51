"""SURVEY.md 8f row f2 on the GPU: contact plans built on the device from the gait templates
(cmpc_generate_contact_plans) against the host construction that follows the reference
(src/contact_plan.py:40-48, 112-264; pinned by the golden fixtures in test_oracle_golden), and
the device warm-start controls (src/centroidal_model.py:176-183).

Tolerance: bit-for-bit (logic, positions, rotations, controls; the foot advance is the same
sequence of float additions), and an SCP iteration on device-built plans returns exactly the
QP solution of the host-uploaded batch.
"""
import numpy as np
import pytest

from cmpc._lib import Solver
from cmpc.synth import CONFIGS, load_conf, make_batch, plan_spec

pytestmark = pytest.mark.gpu


def _specs(names, N, B):
    gaits, feet = [], []
    for b in range(B):
        name = names[(0 if b % 2 == 1 else 1) if len(names) > 1 else 0]
        rng = np.random.default_rng(1000 * CONFIGS[name][1] + b)
        g, f0, _, _ = plan_spec(load_conf(name), N, rng)
        gaits.append(g)
        feet.append(f0)
    return gaits, np.array(feet)


@pytest.mark.parametrize('cfg,N,B', [('trot', 100, 16), ('bound', 100, 8), ('pace', 60, 8), ('talos', 150, 4)])
def test_device_plans_match_host(cfg, N, B):
    pb = make_batch(cfg, N, B)
    gaits, feet = _specs([cfg], N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.generate_contact_plans(gaits, feet)
        lg, pos, rot = s.contact_plans()
        s.upload_states(pb.params, pb.class_id, pb.Xbar)        # controls built on the device
        _, U = s.warm_start()
    assert np.array_equal(lg, pb.logic)
    assert np.array_equal(pos, pb.pos)
    assert np.array_equal(rot, pb.rot)
    assert np.array_equal(U[:, :, :pb.Ubar.shape[2]], pb.Ubar)


def test_mixed_pace_trot_batch_solves_identically():
    N, B = 100, 8
    pb = make_batch('trot', N, B, mixed=('pace', 'trot'))
    gaits, feet = _specs(['pace', 'trot'], N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.scp_iterate(True)
        z0, _, st0, _ = s.qp_solution(with_y=False)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.generate_contact_plans(gaits, feet)
        s.upload_states(pb.params, pb.class_id, pb.Xbar)
        s.scp_iterate(True)
        z1, _, st1, _ = s.qp_solution(with_y=False)
    assert np.all(st0 == 1) and np.array_equal(st0, st1)
    assert np.array_equal(z0, z1)


def test_plan_validation():
    with Solver('TALOS', 40, 1, 'fp64') as s:
        g = dict(type='TROT', nbSteps=4, stepKnots=10, supportKnots=5, stepLength=0.1)
        with pytest.raises(Exception, match='PACE only'):
            s.generate_contact_plans([g], np.zeros((1, 2, 3)))
        g = dict(type='PACE', nbSteps=1, stepKnots=5, supportKnots=5, stepLength=0.0)
        with pytest.raises(Exception, match='shorter than the horizon'):
            s.generate_contact_plans([g], np.zeros((1, 2, 3)))


def test_accepted_gains_kept_across_new_plans():
    """Reference mode serves the accepted K / Sigma from the live arrays; new contact plans change
    what a later linearization computes, so they are copied first: after regenerating the plans
    (a different gait) and linearizing, the accepted results still equal those of the solve."""
    N, B = 60, 4
    pb = make_batch('trot', N, B)
    gaits, feet = _specs(['bound'], N, B)
    with Solver(pb.robot, N, B, 'fp64') as s:
        s.upload(pb)
        s.solve_scp(fixed_iters=False)
        sol = s.solution()
        assert np.all(sol['n_accepted'] >= 1)
        s.generate_contact_plans(gaits, feet)
        s.linearize()
        after = s.solution()
        np.testing.assert_array_equal(after['K'], sol['K'])
        np.testing.assert_array_equal(after['Sigma'], sol['Sigma'])
        assert not np.array_equal(s.linearization()['K'], sol['K'])   # the live arrays did change
