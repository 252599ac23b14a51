"""Index book-keeping of the QP decision vector (drop-in for reference src/optimizer.py:1-133).

The QP variable layout is z = [x_0 .. x_N (9 each) | u_0 .. u_{N-1} (nu each) | t_0 .. t_N |
s_0 .. s_{N-1}] (reference src/centroidal_model.py:25-26).  The classes keep the reference's
attribute names (``_optimizer_idx``, ``_optimizer_idx_vector``, ``_penum_mat`` ...) because
demo and plotting code reads them directly; the indices are computed in closed form.
"""
import numpy as np

_STATE_NAMES = ('com_x', 'com_y', 'com_z', 'lin_mom_x', 'lin_mom_y', 'lin_mom_z', 'ang_mom_x', 'ang_mom_y',
                'ang_mom_z')
_CONTROL_NAMES = {'solo12': ('fx', 'fy', 'fz'), 'TALOS': ('cop_x', 'cop_y', 'fx', 'fy', 'fz', 'tau_z')}


def _sign_enumeration(n):
    """(2^n, n) matrix whose row j holds the signs (-1)^bit_i(j) (reference _penum_mat)."""
    j = np.arange(2 ** n)[:, None]
    return np.where((j >> np.arange(n)[None, :]) & 1, -1.0, 1.0)


class State_optimizer:
    """Global indices of one state coordinate over knots 0..N (reference src/optimizer.py:5-33)."""

    def __init__(self, OPTIMIZER_IDENTIFIER, nb_x_optimizers, horizon_length):
        self._name = OPTIMIZER_IDENTIFIER
        self.nx = nb_x_optimizers
        self.N = horizon_length
        self._optimizer_idx = None
        self._optimizer_idx_vector = np.zeros(self.N + 1, dtype=int)
        if self._name in _STATE_NAMES:
            self._optimizer_idx = _STATE_NAMES.index(self._name)
            self._optimizer_idx_vector = np.arange(self.N + 1) * self.nx + self._optimizer_idx
        else:
            print('this is not a state optimizer name !')


class Control_optimizer:
    """Global indices of one control coordinate of one contact over knots 0..N-1
    (reference src/optimizer.py:35-70; per-contact width 3 for solo12, 6 for TALOS)."""

    def __init__(self, OPTIMIZER_IDENTIFIER, contact_idx, robot_name, nb_x_optimizers, nb_u_ptimizers,
                 horizon_length):
        self._name = OPTIMIZER_IDENTIFIER
        self.nx = nb_x_optimizers
        self.nu = nb_u_ptimizers
        self.N = horizon_length
        self._optimizer_idx = None
        self._optimizer_idx_vector = np.zeros(self.N, dtype=int)
        names = _CONTROL_NAMES.get(robot_name)
        if names is None or self._name not in names:
            print('this is not a control optimizer name !')
            return
        self._optimizer_idx = names.index(self._name)
        width = len(names)
        self._optimizer_idx_vector = (self.nx * (self.N + 1) + np.arange(self.N) * self.nu + width * contact_idx +
                                      self._optimizer_idx)


class Dynamics_optimizer:
    """Start indices of x_k and u_k (reference src/optimizer.py:72-88)."""

    def __init__(self, OPTIMIZER_IDENTIFIER, nx_optimizers, nu_optimizers, horizon_length):
        self._name = OPTIMIZER_IDENTIFIER
        self.nx = nx_optimizers
        self.nu = nu_optimizers
        self.N = horizon_length
        self._x_idx_vector = np.zeros(self.N + 1, dtype=int)
        self._u_idx_vector = np.zeros(self.N, dtype=int)
        if self._name == 'dynamics':
            self._x_idx_vector = np.arange(self.N + 1) * self.nx
            self._u_idx_vector = self.nx * (self.N + 1) + np.arange(self.N) * self.nu
        else:
            print('this not a dynamics optimizer name !')


class Slack_optimizer:
    """Trust-region slack bookkeeping (reference src/optimizer.py:90-133).  'state': one slack t_k
    per knot and the 2^(nx-6) sign rows of the L1 ball on the angular momentum x[6:9];
    'control': one slack per control knot over all nu coordinates."""

    def __init__(self, OPTIMIZER_IDENTIFIER, nx_optimizers, nu_optimizers, nt_optimizers, horizon_length):
        self._name = OPTIMIZER_IDENTIFIER
        self.N = horizon_length
        self.nx = nx_optimizers
        self.nu = nu_optimizers
        self.nt = nt_optimizers
        first_slack = self.nx * (self.N + 1) + self.nu * self.N
        if self._name == 'state':
            self._nb_slack_constraints = self.nt * (2 ** (self.nx - 6))
            self._penum_mat = _sign_enumeration(self.nx - 6)
            self._x0_optimizer_idx_vector = np.arange(self.N + 1) * self.nx
            self._slack_optimizers_idx_vector = first_slack + np.arange(self.N + 1)
        elif self._name == 'control':
            self._nb_slack_constraints = self.nt * (2 ** self.nu)
            self._penum_mat = _sign_enumeration(self.nu)
            self._u0_optimizer_idx_vector = self.nx * (self.N + 1) + np.arange(self.N) * self.nu
            self._slack_optimizers_idx_vector = first_slack + self.nt * (self.N + 1) + np.arange(self.N)
        else:
            print('this not a slack optimizer name !')
