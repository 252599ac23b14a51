"""QP cost terms (drop-in for reference src/cost.py:1-47), answered from the GPU assembly.

The full cost is blkdiag(I_{N+1} (x) W_x, I_N (x) W_u, 0, 0) with gradient -W_x xbar_k on the
state slots (solo12 tracking, quirk Q10) and 1 on every trust-region slack t_k.  Each function
returns its own term in the reference's ``Cost(Q, p)`` form, sliced from the QP that
cmpc_assemble built on the device for the model's warm start.
"""
from collections import namedtuple

import numpy as np
from scipy import sparse

from src import _device

Cost = namedtuple('Cost', 'Q, p')


def _P_q(model):
    _, P, q, _, _, _ = _device.export(model)
    return P, q


def construct_total_cost(model):
    """Quadratic part (reference :9-16)."""
    P, _ = _P_q(model)
    return Cost(Q=P, p=np.zeros(model._total_nb_optimizers))


def construct_state_tracking_cost(model):
    """-W_x xbar_k on the x_k slots (reference :21-29; solo12 with DYNAMICS_FIRST False)."""
    n = model._total_nb_optimizers
    _, q = _P_q(model)
    p = np.zeros(n)
    nxs = model._n_x * (model._N + 1)
    p[:nxs] = q[:nxs]
    return Cost(Q=sparse.csc_matrix((n, n)), p=p)


def construct_state_trust_region_cost(model):
    """Unit L1 penalty on the trust-region slacks t_0..t_N (reference :34-39)."""
    n, N = model._total_nb_optimizers, model._N
    t0 = model._n_x * (N + 1) + model._n_u * N
    p = np.zeros(n)
    p[t0:t0 + N + 1] = 1.0
    return Cost(Q=sparse.csc_matrix((n, n)), p=p)


def construct_control_trust_region_cost(model):
    """Unit penalty on the (unused) control slacks (reference :44-47)."""
    n, N = model._total_nb_optimizers, model._N
    p = np.zeros(n)
    p[n - N:] = 1.0
    return Cost(Q=sparse.csc_matrix((n, n)), p=p)
