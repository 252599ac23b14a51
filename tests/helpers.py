"""Shared test helpers: build oracle problems from golden fixtures / synthetic batches."""
import numpy as np
from scipy import sparse

from cmpc.problem import ModelParams, ProblemBatch
from cmpc.synth import load_conf

KIND_CONF = {'trot': 'trot', 'trot_stoch': 'trot', 'bound': 'bound', 'pace': 'pace', 'talos': 'talos'}


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
