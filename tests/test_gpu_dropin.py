"""Drop-in API on the GPU: the reference's functions (src.centroidal_model, src.scp_solver,
src.cost, src.constraints) answered by libcmpc.so, compared with the oracle on the same inputs.

Tolerances: linearization 1e-15 abs (f, A, B, C) / 1e-11 relative (K, Sigma); rollout 1e-13;
QP matrices exact (P) / 1e-13 (A) / 1e-11 (bounds); QP solution 1e-5 relative to the OSQP
restatement run to 1e-10; rho 1e-9 relative; SCP results as in test_gpu_parity."""
import numpy as np
import pytest

from helpers import dropin_model, model_oracle_problem
from oracle import model as M, transcription as T, scp as OS
from oracle.osqp_admm import solve_qp
from oracle.sparse_ipm import solve_qp as sparse_ipm_qp
from src import constraints as Cn, cost as Co, scp_solver as S

pytestmark = pytest.mark.gpu


def _oracle(m):
    p = model_oracle_problem(m)
    td = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'])
    return p, td


@pytest.mark.parametrize('cfg', ['trot', 'talos'])
def test_trajectory_data_and_rollout(cfg):
    m = dropin_model(cfg, 30)
    p, td = _oracle(m)
    got = m.compute_trajectory_data(m._init_trajectories)
    assert np.allclose(got['dynamics'], td['dynamics'], rtol=0, atol=1e-13)
    for k in ('f_x', 'f_u', 'f_w'):
        assert np.allclose(got['gradients'][k], td[k], rtol=0, atol=1e-15)
    assert np.allclose(got['LQR_gains'], td['LQR_gains'], rtol=0, atol=1e-11 * np.abs(td['LQR_gains']).max())
    if cfg == 'talos':   # the kernel's association, 1e-4 (see test_gpu_parity.test_linearization_fp64)
        cl = M.compute_trajectory_data(p['Xbar'], p['Ubar'], p['logic'], p['pos'], p['rot'], p['prm'],
                                       assoc='closed_loop')['Covs']
        assert np.allclose(got['Covs'], cl, rtol=0, atol=1e-4 * np.abs(cl).max())
    else:
        assert np.allclose(got['Covs'], td['Covs'], rtol=0, atol=1e-11 * np.abs(td['Covs']).max())
    assert got['Covs_gradients']['Cov_dx'].shape == (31, 9, 9, 9, 31) and not got['Covs_gradients']['Cov_du'].any()
    rng = np.random.default_rng(0)
    traj = dict(state=p['Xbar'] + 1e-3 * rng.normal(size=p['Xbar'].shape),
                control=p['Ubar'] + 1e-2 * rng.normal(size=p['Ubar'].shape))
    nl = m.integrate_dynamics_trajectory(traj)
    ref = M.integrate_dynamics_trajectory(traj['state'], traj['control'], p['logic'], p['pos'], p['rot'], p['prm'])
    assert np.allclose(nl, ref, rtol=0, atol=1e-13 * max(1.0, np.abs(ref).max()))
    m.close()


@pytest.mark.parametrize('cfg', ['trot', 'talos'])
def test_cost_constraints_and_subproblem(cfg):
    N = 30
    m = dropin_model(cfg, N)
    p, td = _oracle(m)
    tr = {'weight': 500.0, 'radius': 50.0}
    cost = S.sum_up_all_costs(m)
    cons = S.stack_up_all_constraints(m, m._init_trajectories, None, tr)
    P0, q0 = T.build_cost(N, p['prm'], p['Xbar'])
    A0, l0, u0 = T.build_constraints(N, p['prm'], p['logic'], p['pos'], p['rot'], p['Xbar'], p['Ubar'], td,
                                     tr['weight'], tr['radius'])
    assert abs(cost.Q - P0).max() == 0 and np.allclose(cost.p, q0, rtol=0, atol=1e-12)
    assert cons.mat.shape == A0.shape and abs(cons.mat - A0).max() <= 1e-13
    fin = np.isfinite(u0)
    assert np.array_equal(fin, np.isfinite(cons.ub)) and np.allclose(cons.ub[fin], u0[fin], rtol=0, atol=1e-11)
    # the same QP asked again is served from the drop-in's last export: no device call
    ep = m._solver._epoch
    cons2 = S.stack_up_all_constraints(m, {k: np.array(v, copy=True) for k, v in m._init_trajectories.items()}, None, tr)
    assert m._solver._epoch == ep and abs(cons2.mat - cons.mat).max() == 0 and np.array_equal(cons2.ub, cons.ub)
    # the per-family functions stack up to the same matrix
    fams = [Cn.construct_initial_constraints(m), Cn.construct_dynamics_constraints(m, m._init_trajectories, None),
            Cn.construct_final_constraints(m)]
    if cfg == 'talos':
        fams.append(Cn.construct_cop_constraints(m))
    fams += [Cn.construct_friction_pyramid_constraints(m, m._init_trajectories, None),
             Cn.construct_state_trust_region_constraints(m, m._init_trajectories, tr)]
    from scipy import sparse
    Ast = sparse.vstack([f.mat for f in fams]).tocsc()
    assert abs(Ast - cons.mat).max() == 0
    q_parts = Co.construct_total_cost(m).p + Co.construct_state_trust_region_cost(m).p
    if cfg == 'trot':
        q_parts = q_parts + Co.construct_state_tracking_cost(m).p
    assert np.allclose(q_parts, cost.p, rtol=0, atol=1e-12)
    ok, res = S.solve_subproblem(cost, cons)
    assert ok and res.info.status == 'solved'
    ref = sparse_ipm_qp(P0, q0, A0, l0, u0) if cfg == 'talos' else \
        solve_qp(P0, q0, A0, l0, u0, eps_abs=1e-10, eps_rel=1e-10, max_iter=200000)
    nxu = 9 * (N + 1) + 12 * N
    assert np.abs(res.x[:nxu] - ref.x[:nxu]).max() <= 1e-5 * np.abs(ref.x[:nxu]).max()
    sol = S.get_QP_solution(m, res)
    rho = S.compute_model_accuracy(m, sol, m._init_trajectories, m.compute_trajectory_data(m._init_trajectories))
    rho0 = M.compute_model_accuracy(sol['state'], sol['control'], p['Xbar'], p['Ubar'], td, p['logic'], p['pos'],
                                    p['rot'], p['prm'])
    assert abs(rho - rho0) <= 1e-9 * abs(rho0)
    m.close()


@pytest.mark.parametrize('cfg', ['trot', 'bound'])
def test_solve_scp_and_batch(cfg):
    N = 30
    models = [dropin_model(cfg, N, seed=s) for s in range(3)]
    batch = S.solve_scp_batch(models)
    for m, rb in zip(models, batch):
        p = model_oracle_problem(m)
        ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp)
        got = S.solve_scp(m, p['scp_params'])
        if ref is False:
            assert got is False and rb is False
            continue
        assert len(got['state']) == len(ref['state']) == len(rb['state'])
        if ref['state']:
            sc = np.abs(ref['state'][-1]).max()
            assert np.allclose(got['state'][-1], ref['state'][-1], rtol=0, atol=1e-5 * sc)
            assert np.allclose(rb['state'][-1], got['state'][-1], rtol=0, atol=1e-9 * sc)
            assert np.allclose(got['gains'][-1], ref['gains'][-1], rtol=0, atol=1e-11 * np.abs(ref['gains'][-1]).max())
            it = S.interpolate_SCP_solution(got)
            assert it['X'].shape == (9, N * 10)
        m.close()


def test_npz_chain_ddp_to_gpu_scp_to_ddp(tmp_path, monkeypatch):
    """SURVEY 8f row f3 end to end: a DDP-style ``wholeBody_to_centroidal_traj.npz`` in the working
    directory (key 'X', (N+1, 9)) -> the drop-in ``Centroidal_model`` reads it (no
    init_trajectories, reference src/centroidal_model.py:80-89,174) -> solve_scp on the GPU ->
    ``centroidal_to_wholeBody_traj.npz`` (X (9, N+1), U (nu, N), trot_demo.ipynb:61) as the
    whole-body stage loads it (src/whole_body_control.py:41-44).  The written trajectory equals the
    oracle's solve_scp from the same file."""
    import types
    from cmpc import npz_io
    from cmpc.synth import CONFIGS, load_conf, warm_start
    from cmpc.problem import ModelParams
    from src.centroidal_model import Centroidal_model
    from src.contact_plan import create_contact_trajectory, contact_arrays
    N = 40
    conf0 = load_conf('trot')
    conf = types.SimpleNamespace(**{k: getattr(conf0, k) for k in dir(conf0) if not k.startswith('__')})
    conf.N = N
    logic, pos, rot = contact_arrays(create_contact_trajectory(conf), N)
    prm = ModelParams.from_conf(conf)
    X = warm_start(conf, logic, pos, np.random.default_rng(1000 * CONFIGS['trot'][1] + 7), prm.mass, 0.24,
                   prm.gravity, prm.robot)
    monkeypatch.chdir(tmp_path)
    npz_io.save_warm_start(npz_io.WARM_START, X)                      # the DDP stage's output
    m = Centroidal_model(conf)                                       # reads it from the CWD
    assert np.array_equal(m._init_trajectories['state'], X.T)
    sol = S.solve_scp(m, conf.scp_params)
    assert sol is not False and sol['state']
    paths = npz_io.save_to_whole_body(npz_io.TO_WHOLE_BODY, sol)
    Xw, Uw = npz_io.load_tracking(paths[0])                         # what the whole-body stage loads
    assert Xw.shape == (9, N + 1) and Uw.shape == (12, N)
    p = model_oracle_problem(m)
    ref = OS.solve_scp(p, p['scp_params'], qp=sparse_ipm_qp)
    assert ref is not False and len(ref['state']) == len(sol['state'])
    assert np.allclose(Xw, ref['state'][-1], rtol=0, atol=1e-5 * np.abs(ref['state'][-1]).max())
    assert np.allclose(Uw, ref['control'][-1], rtol=0, atol=1e-5 * np.abs(ref['control'][-1]).max())
    m.close()
