"""Host-side logic of the product (no GPU): contact plans, configs, problem packing."""
import numpy as np
import pytest

from cmpc.synth import load_conf, contact_plan, make_batch, warm_start_controls
from cmpc.problem import ModelParams
from src.contact_plan import create_contact_sequence, create_contact_trajectory, contact_arrays, plan_length


@pytest.mark.parametrize('tag', ['trot', 'bound', 'pace', 'talos'])
def test_contact_plan_matches_reference(tag, golden):
    """Product gait rules == reference create_contact_sequence/_fill_contact_data (golden)."""
    g = golden[tag]
    N = int(g['N'])
    logic, pos, rot = contact_plan(load_conf(tag), N, rng=None)
    np.testing.assert_array_equal(logic, g['logic'])
    np.testing.assert_allclose(pos.reshape(N, -1), g['pos'], rtol=0, atol=1e-15)
    np.testing.assert_allclose(rot, g['rot'], rtol=0, atol=1e-15)


@pytest.mark.parametrize('tag', ['trot', 'bound', 'pace', 'talos'])
def test_warm_start_control_rule(tag, golden):
    """Ubar = [1e-3, 1e-3, m*9.81/#active] at rows 3i (reference rule, incl. the TALOS slot quirk)."""
    g = golden[tag]
    p = ModelParams.from_conf(load_conf(tag))
    U = warm_start_controls(g['logic'], p.mass, p.gravity, g['Ubar'].shape[0])
    np.testing.assert_allclose(U.T, g['Ubar'], rtol=1e-15, atol=1e-15)


def test_native_horizons():
    """N of the stock configs: trot/bound 165, pace 107, TALOS 165."""
    assert load_conf('trot').N == 165 and load_conf('bound').N == 165
    assert load_conf('pace').N == 107 and load_conf('talos').N == 165


def test_contact_index_order():
    conf = load_conf('trot')
    traj = create_contact_trajectory(conf)
    assert list(traj.keys()) == ['FR', 'FL', 'HR', 'HL']      # quirk Q12
    assert [traj[c][0].idx for c in traj] == [0, 1, 2, 3]


def test_batch_shapes_and_validation():
    pb = make_batch('trot', 40, 3)
    pb.validate()
    assert pb.Xbar.shape == (3, 41, 9) and pb.Ubar.shape == (3, 40, 12)
    bad = pb.subset(0, 1)
    bad.logic = bad.logic.copy(); bad.logic[0, 5] = 0
    with pytest.raises(ValueError):
        bad.validate()


def test_mixed_batch_alternates_classes():
    pb = make_batch('trot', 60, 4, mixed=('pace', 'trot'))
    assert list(pb.class_id) == [1, 0, 1, 0]
    assert pb.params[0].scp_params['trust_region_radius0'] == 50


def test_synthetic_problems_are_deterministic():
    a = make_batch('trot', 30, 2)
    b = make_batch('trot', 30, 2)
    np.testing.assert_array_equal(a.Xbar, b.Xbar)
    np.testing.assert_array_equal(a.pos, b.pos)


def test_talos_covariance_scan_sensitivity():
    """Why the TALOS covariance parity bound is 1e-4 (tests/test_gpu_parity.py): with the
    reference's TALOS warm start (quirk Q11) A + BK has spectral radius 1 and the scan amplifies
    rounding.  The reference's association of the step and the kernel's (A + BK) S (A + BK)' are
    the same algebra, yet differ by ~1e-5 relative at N=50 in float64 on the CPU alone; Solo12's
    scan is contractive and they agree to 1e-14."""
    from oracle import model as M

    def diff(cfg, N):
        pb = make_batch(cfg, N, 1)
        p = pb.oracle_problem(0)
        a = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])['Covs']
        c = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'],
                                      assoc='closed_loop')['Covs']
        return np.abs(a - c).max() / np.abs(a).max()

    assert diff('trot', 100) <= 1e-14
    assert 1e-7 <= diff('talos', 50) <= 1e-4
