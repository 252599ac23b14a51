"""QP constraint families (drop-in for reference src/constraints.py), answered from the GPU
assembly: each function returns its rows of the QP that cmpc_assemble built on the device,
in the reference's ``Constraint(mat, lb, ub)`` form and exact row order.

``traj_data`` arguments are accepted for signature compatibility; the device recomputes the
linearization at ``prev_traj_tuple`` itself (identical to the caller's traj_data, which is
cmpc_linearize's output when it came from Centroidal_model.compute_trajectory_data).
"""
from collections import namedtuple

import numpy as np

from src import _device

Constraint = namedtuple('Constraint', 'mat, lb, ub')


def _family(model, name, traj_tuple=None, trust_region=None):
    _, _, _, A, l, u = _device.export(model, traj_tuple, trust_region)
    r0, r1 = _device.row_blocks(model)[name]
    return Constraint(*_device.rows(A, l, u, r0, r1))


def construct_initial_constraints(model):
    """x_0 = x_init (reference :11-17)."""
    return _family(model, 'initial')


def construct_dynamics_constraints(model, prev_traj_tuple, traj_data=None):
    """A_k x_k + B_k u_k - x_{k+1} = A_k xbar_k + B_k ubar_k - f_k (reference :19-50)."""
    return _family(model, 'dynamics', prev_traj_tuple)


def construct_final_constraints(model):
    """x_N = x_final (reference :103-109)."""
    return _family(model, 'final')


def construct_cop_constraints(model):
    """TALOS centre-of-pressure box, per contact x rows then y rows (reference :111-145)."""
    if model._robot != 'TALOS':
        raise ValueError('CoP constraints exist for TALOS only')
    return _family(model, 'cop')


def construct_friction_pyramid_constraints(model, prev_traj_tuple=None, traj_data=None):
    """Linearized friction pyramid, 5 rows per (contact, knot) with rows 0-3 filled for active
    contacts (quirk Q4); stochastic back-off when the model is STOCHASTIC_OCP (reference :153-217)."""
    return _family(model, 'friction', prev_traj_tuple)


def construct_state_trust_region_constraints(model, prev_traj_tuple, trust_region):
    """L1 trust region on the angular momentum with slack t_k / omega, then -t_k <= 0
    (reference :260-293)."""
    _, _, _, A, l, u = _device.export(model, prev_traj_tuple, trust_region)
    blocks = _device.row_blocks(model)
    r0, r1 = blocks['trust_region'][0], blocks['slack'][1]
    return Constraint(*_device.rows(A, l, u, r0, r1))


def check_symmetric(a, rtol=1e-05, atol=1e-08):
    return np.allclose(a, a.T, rtol=rtol, atol=atol)
