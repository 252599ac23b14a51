"""Shared test helpers: build oracle problems from golden fixtures / synthetic batches."""
import numpy as np
from scipy import sparse

from cmpc.problem import ModelParams, ProblemBatch
from cmpc.synth import load_conf

KIND_CONF = {'trot': 'trot', 'trot_stoch': 'trot', 'bound': 'bound', 'pace': 'pace', 'talos': 'talos',
             'trot_n50': 'trot', 'trot_n100': 'trot', 'bound_n100': 'bound', 'trot_f32': 'trot',
             'bound_n100_f32': 'bound'}


def golden_fp32(g):
    """True for the fixtures made at the reference's own float32 precision (``*_f32``)."""
    return bool(int(g['fp32'])) if 'fp32' in g else False


def golden_qp(tag, g):
    """The QP stand-in the fixture's solve_scp ran with (tests/golden/make_golden.py FIXTURES):
    the OSQP restatement for the N=20 Solo12 fixtures, the sparse IPM for the others."""
    from oracle.osqp_admm import solve_qp
    from oracle.sparse_ipm import solve_qp as sparse_ipm
    if tag in ('trot', 'trot_stoch', 'bound', 'pace'):
        return lambda *a: solve_qp(*a, max_iter=20000)
    return sparse_ipm


def golden_params(tag, g):
    conf = load_conf(KIND_CONF[tag])
    return ModelParams.from_conf(conf, stochastic=bool(g['stochastic']))


def golden_batch(tag, g):
    """ProblemBatch (B=1) holding the golden problem's inputs."""
    p = golden_params(tag, g)
    N = int(g['N'])
    nc = g['logic'].shape[1]
    nu = g['Ubar'].shape[0]
    pos = g['pos'].reshape(N, nc, 3)
    pb = ProblemBatch(p.robot, N, nc, nu, g['logic'][None].astype(np.int8), pos[None], g['rot'][None],
                      g['Xbar'].T[None].copy(), g['Ubar'].T[None].copy(), np.zeros(1, np.int32), [p])
    pb.validate()
    return pb


def golden_csc(g, tag):
    n_rows = tuple(g[tag + '_A_shape'])
    A = sparse.csc_matrix((g[tag + '_A_data'], g[tag + '_A_indices'], g[tag + '_A_indptr']), shape=n_rows)
    return A, g[tag + '_l'], g[tag + '_u']


def golden_P(g):
    n = int(g['n'])
    return sparse.csc_matrix((g['P_data'], g['P_indices'], g['P_indptr']), shape=(n, n))


def same_bounds(a, b, tol=1e-12):
    a = np.asarray(a, float); b = np.asarray(b, float)
    fin = np.isfinite(a) & np.isfinite(b)
    return bool(np.all(np.isfinite(a) == np.isfinite(b)) and np.all(np.sign(a[~fin]) == np.sign(b[~fin]))
                and np.allclose(a[fin], b[fin], rtol=tol, atol=tol))


def dropin_model(cfg, N, seed=0, stochastic=False, precision='fp64'):
    """A drop-in ``Centroidal_model`` built from the config module with the horizon truncated to N
    (the reference's behaviour when conf.N < plan length) and a synthetic warm start passed as
    ``init_trajectories`` (the DDP npz of the reference is not available)."""
    import types
    from cmpc.synth import CONFIGS, warm_start, warm_start_controls
    from src.centroidal_model import Centroidal_model
    from src.contact_plan import create_contact_trajectory, contact_arrays
    conf0 = load_conf(cfg)
    conf = types.SimpleNamespace(**{k: getattr(conf0, k) for k in dir(conf0) if not k.startswith('__')})
    conf.N = N
    logic, pos, rot = contact_arrays(create_contact_trajectory(conf), N)
    p = ModelParams.from_conf(conf)
    rng = np.random.default_rng(1000 * CONFIGS[cfg][1] + seed)
    com_z = 0.24 if p.robot == 'solo12' else 0.87
    X = warm_start(conf, logic, pos, rng, p.mass, com_z, p.gravity, p.robot)
    U = warm_start_controls(logic, p.mass, p.gravity, conf.n_u)
    model = Centroidal_model(conf, STOCHASTIC_OCP=stochastic, init_trajectories=dict(state=X.T, control=U.T),
                             precision=precision)
    return model


def model_oracle_problem(model):
    """The oracle's problem dict for a drop-in model."""
    return model.problem_batch().oracle_problem(0)
