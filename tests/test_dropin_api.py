"""Drop-in Python API (src.centroidal_model / src.scp_solver / src.cost / src.constraints /
src.optimizer): host-side behaviour that needs no GPU.  Index conventions are checked against
the oracle's restatement of the reference layout (src/optimizer.py, src/centroidal_model.py:25-26)."""
import numpy as np
import pytest

from helpers import dropin_model, model_oracle_problem
from oracle import model as M, transcription as T
from src import _device, optimizer as O
from src import scp_solver as S
from src.constraints import Constraint
from src.cost import Cost


def test_optimizer_indices_match_reference_layout():
    N, nu = 30, 12
    for i, name in enumerate(['com_x', 'com_y', 'com_z', 'lin_mom_x', 'lin_mom_y', 'lin_mom_z', 'ang_mom_x',
                              'ang_mom_y', 'ang_mom_z']):
        o = O.State_optimizer(name, 9, N)
        assert o._optimizer_idx == i
        assert np.array_equal(o._optimizer_idx_vector, [T.x_idx(k) + i for k in range(N + 1)])
    for c in range(4):
        for j, name in enumerate(['fx', 'fy', 'fz']):
            o = O.Control_optimizer(name, c, 'solo12', 9, nu, N)
            assert np.array_equal(o._optimizer_idx_vector, [T.u_idx(N, nu, k) + 3 * c + j for k in range(N)])
    for c in range(2):
        for j, name in enumerate(['cop_x', 'cop_y', 'fx', 'fy', 'fz', 'tau_z']):
            o = O.Control_optimizer(name, c, 'TALOS', 9, nu, N)
            assert np.array_equal(o._optimizer_idx_vector, [T.u_idx(N, nu, k) + 6 * c + j for k in range(N)])
    s = O.Slack_optimizer('state', 9, nu, 1, N)
    assert np.array_equal(s._penum_mat, T.penum_mat())
    assert s._nb_slack_constraints == 8
    assert np.array_equal(s._slack_optimizers_idx_vector, [T.t_idx(N, nu, k) for k in range(N + 1)])
    d = O.Dynamics_optimizer('dynamics', 9, nu, N)
    assert np.array_equal(d._u_idx_vector, [T.u_idx(N, nu, k) for k in range(N)])
    # the reference's Control_optimizer('fz', 2, 'solo12', 9, 12, 4) (SURVEY 8c probe)
    assert list(O.Control_optimizer('fz', 2, 'solo12', 9, 12, 4)._optimizer_idx_vector) == [53, 65, 77, 89]


# Module-level names of the reference's config/conf_*.py.  `robot` (a pinocchio RobotWrapper,
# example_robot_data / robot_properties_solo) is the one name left out: the whole-body stage that
# needs it is out of scope.
_REF_CONF_NAMES = ['ee_frame_names', 'rmodel', 'rdata', 'robot_mass', 'gravity_constant', 'dt', 'dt_ctrl',
                   'gait', 'q0', 'gait_templates', 'contact_sequence', 'N', 'N_ctrl', 'n_u_per_contact',
                   'nb_contacts', 'n_u', 'n_x', 'n_t', 'n_w', 'Q', 'R', 'cov_w', 'cov_white_noise', 'beta_u',
                   'state_cost_weights', 'control_cost_weights', 'whole_body_task_weights', 'scp_params',
                   'cameraTF', 'WITHDISPLAY', 'mu', 'DYNAMICS_FIRST']


@pytest.mark.parametrize('name', ['conf_solo12_trot', 'conf_solo12_bound', 'conf_solo12_pace', 'conf_talos'])
def test_config_modules_keep_reference_names(name):
    import importlib
    conf = importlib.import_module('config.' + name)
    missing = [a for a in _REF_CONF_NAMES if not hasattr(conf, a)]
    assert not missing, missing
    assert set(conf.whole_body_task_weights) >= {'footTrack', 'comTrack', 'stateReg', 'ctrlReg', 'frictionCone',
                                                 'centroidalTrack', 'contactForceTrack'}
    assert len(conf.cameraTF) == 7


@pytest.mark.parametrize('cfg', ['trot', 'talos'])
def test_model_attributes_and_row_blocks(cfg):
    N = 20
    m = dropin_model(cfg, N)
    assert m._N == N and m._total_nb_optimizers == T.n_vars(N, m._n_u)
    assert m._contact_data['contacts_logic'].shape == (N, len(m._contact_trajectory))
    assert np.array_equal(m._x_init, m._init_trajectories['state'][:, 0])
    p = model_oracle_problem(m)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    A, l, u = T.build_constraints(N, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td, 100., 1.)
    blocks = _device.row_blocks(m)
    assert blocks['initial'][0] == 0 and max(b[1] for b in blocks.values()) == A.shape[0]
    spans = sorted(blocks.values())
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    m.close()


def test_interpolation_and_solution_reshape_match_oracle():
    rng = np.random.default_rng(3)
    X, U = rng.normal(size=(9, 31)), rng.normal(size=(12, 30))
    got = S.interpolate_SCP_solution(dict(state=[X], control=[U]))
    Xi, Ui = T.interpolate_scp_solution(X, U)
    assert np.allclose(got['X'], Xi, rtol=0, atol=1e-15) and np.allclose(got['U'], Ui, rtol=0, atol=1e-15)
    m = dropin_model('trot', 30)
    z = rng.normal(size=T.n_vars(30, 12))
    sol = S.get_QP_solution(m, S.Result(x=z, y=None, info=None))
    X0, U0 = T.get_qp_solution(30, 12, z)
    assert np.array_equal(sol['state'], X0) and np.array_equal(sol['control'], U0)
    assert S.convergence(dict(state=X, control=U), dict(state=X, control=U)) == 0.0


def test_qp_of_no_layout_is_rejected_and_missing_warm_start_raises(tmp_path, monkeypatch):
    from scipy import sparse
    with pytest.raises(ValueError, match='variables'):   # before any device call
        S.solve_subproblem(Cost(Q=sparse.eye(3), p=np.zeros(3)), Constraint(mat=sparse.eye(3), lb=-np.ones(3),
                                                                            ub=np.ones(3)))
    import types
    from cmpc.synth import load_conf
    from src.centroidal_model import Centroidal_model
    conf0 = load_conf('trot')
    conf = types.SimpleNamespace(**{k: getattr(conf0, k) for k in dir(conf0) if not k.startswith('__')})
    conf.N = 20
    monkeypatch.chdir(tmp_path)     # no wholeBody_to_centroidal_traj.npz here
    with pytest.raises(FileNotFoundError):
        Centroidal_model(conf)


def test_foreign_qp_layout_inference_rejects_other_sizes():
    """solve_subproblem on a QP not built by the drop-in infers robot and horizon from the
    reference's layout (n = 23 N + 10; m = 38 N + 27 Solo12, 32 N + 27 TALOS) before any device
    call, and refuses sizes of no layout."""
    from src.scp_solver import _foreign_solver
    with pytest.raises(ValueError, match='variables'):
        _foreign_solver(23 * 30 + 11, 38 * 30 + 27)
    with pytest.raises(ValueError, match='rows'):
        _foreign_solver(23 * 30 + 10, 38 * 30 + 28)


def test_export_cache_key_follows_content_and_trust_region():
    """The drop-in keeps the last exported QP (the reference asks for the cost and every
    constraint family of one QP separately); its key is the linearization point's content and
    the trust region, so an in-place edit or another radius is a different QP."""
    m = dropin_model('trot', 20)
    tr = {'weight': 100.0, 'radius': 100.0}
    k0 = _device._key(m, None, tr)
    assert _device._key(m, None, dict(tr)) == k0
    assert _device._key(m, None, {'weight': 100.0, 'radius': 50.0}) != k0
    traj = {k: np.array(v, copy=True) for k, v in m._init_trajectories.items()}
    assert _device._key(m, traj, tr) == k0
    traj['state'][3, 7] += 1e-9
    assert _device._key(m, traj, tr) != k0
    m.close()
