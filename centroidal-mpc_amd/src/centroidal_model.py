"""Centroidal model, GPU-backed (drop-in for reference src/centroidal_model.py:13-291).

Keeps the reference's constructor signature, protected attributes (``_N``, ``_n_u``,
``_contact_data``, ``_init_trajectories``, the optimizer index dictionaries ...) and the two
public methods the SCP loop uses.  The arithmetic runs in libcmpc.so on the GPU:

* ``compute_trajectory_data`` -> ``cmpc_linearize`` (f, A, B, C, LQR gains, covariance scan);
* ``integrate_dynamics_trajectory`` -> ``cmpc_rollout``.

There is no CPU path: without the HIP library or a GPU every method raises ``CmpcError``.
The returned dictionaries use the reference's keys and layouts (dynamics (nx, N), gradients
f_x (N, nx, nx) / f_u (N, nx, nu) / f_w (N, nx, nw), LQR_gains (N, nu, nx), Covs (N+1, nx, nx)).
``Covs_gradients`` are identically zero in the reference (quirk Q3: ``Sigma_next_fun`` is a
constant, src/centroidal_model.py:239-240) and are returned as zero arrays of the same shapes.
"""
import dataclasses
import os

import numpy as np

from cmpc._lib import Solver
from cmpc.problem import ModelParams, ProblemBatch
from src.contact_plan import create_contact_trajectory, contact_arrays
from src.optimizer import Control_optimizer, Slack_optimizer, State_optimizer

WARM_START_FILE = 'wholeBody_to_centroidal_traj.npz'


class Centroidal_model:
    def __init__(self, conf, STOCHASTIC_OCP=False, init_trajectories=None, precision='fp64', device=0):
        """``init_trajectories``: optional dict(state=(nx, N+1), control=(nu, N)).  Without it the
        states come from ``wholeBody_to_centroidal_traj.npz`` in the working directory (key 'X',
        (N+1, nx)), as the reference does when DYNAMICS_FIRST is False, and the controls follow the
        reference rule [1e-3, 1e-3, m*|g|/#active] (src/centroidal_model.py:158-187)."""
        self._DYNAMICS_FIRST = conf.DYNAMICS_FIRST
        self._robot = conf.robot_name
        self._n_x = conf.n_x
        self._n_u_per_contact = conf.n_u_per_contact
        self._n_u = conf.n_u
        self._n_w = conf.n_w
        self._n_t = conf.n_t
        self._N = conf.N
        self._total_nb_optimizers = (self._n_x * (self._N + 1) + self._n_u * self._N + self._n_t * (self._N + 1) +
                                     self._n_t * self._N)
        self._max_leg_length = conf.max_leg_length
        self._m = conf.robot_mass
        self._g = conf.gravity_constant
        self._dt = conf.dt
        self._state_cost_weights = conf.state_cost_weights
        self._control_cost_weights = conf.control_cost_weights
        self._linear_friction_coefficient = conf.mu
        self._Q = conf.Q
        self._R = conf.R
        if self._robot == 'TALOS':
            self._robot_foot_range = {'x': np.array([conf.lxp, conf.lxn]), 'y': np.array([conf.lyp, conf.lyn])}
        self._STOCHASTIC_OCP = STOCHASTIC_OCP
        self._beta_u = conf.beta_u
        self._Cov_w = conf.cov_w
        self._Cov_eta = conf.cov_white_noise
        self._params = ModelParams.from_conf(conf, STOCHASTIC_OCP)
        self._precision = precision
        self._device = device
        self._solver = None
        self._fill_contact_data(conf)
        self._fill_optimizer_indices()
        self._fill_initial_trajectory(conf, init_trajectories)

    # ------------------------------------------------------------------ construction
    def _fill_contact_data(self, conf):
        self._contact_trajectory = create_contact_trajectory(conf)
        logic, pos, rot = contact_arrays(self._contact_trajectory, self._N)
        self._logic, self._pos, self._rot = logic, pos, rot
        self._contact_data = dict(contacts_logic=logic.astype(int), contacts_orient=rot,
                                  contacts_position=pos.reshape(self._N, -1))

    def _fill_optimizer_indices(self):
        names = ['com_x', 'com_y', 'com_z', 'lin_mom_x', 'lin_mom_y', 'lin_mom_z', 'ang_mom_x', 'ang_mom_y',
                 'ang_mom_z']
        states = [State_optimizer(n, self._n_x, self._N) for n in names]
        # the reference's grouping (src/centroidal_model.py:100-102) is kept as is
        self._state_optimizers_indices = {'coms': states[:2], 'lin_moms': states[2:5], 'ang_moms': states[5:]}
        controls = ['fx', 'fy', 'fz'] if self._robot == 'solo12' else ['cop_x', 'cop_y', 'fx', 'fy', 'fz', 'tau_z']
        self._control_optimizers_indices = {}
        for ci, contact in enumerate(self._contact_trajectory):
            opt = [Control_optimizer(n, ci, self._robot, self._n_x, self._n_u, self._N) for n in controls]
            if self._robot == 'TALOS':
                self._control_optimizers_indices[contact] = {'cops': opt[:2], 'forces': opt[2:5], 'moment': opt[5:]}
            else:
                self._control_optimizers_indices[contact] = {'forces': opt}
        self._state_slack_optimizers_indices = Slack_optimizer('state', self._n_x, self._n_u, self._n_t, self._N)

    def _fill_initial_trajectory(self, conf, init_trajectories):
        N = self._N
        if init_trajectories is not None:
            X = np.asarray(init_trajectories['state'], float)
            U = np.asarray(init_trajectories['control'], float)
        elif self._DYNAMICS_FIRST:
            X = np.zeros((self._n_x, N + 1))
            U = np.zeros((self._n_u, N))
        else:
            if not os.path.exists(WARM_START_FILE):
                raise FileNotFoundError('%s not found: the reference warm-starts from the whole-body DDP '
                                        'trajectory; pass init_trajectories=dict(state=..., control=...) '
                                        'instead' % WARM_START_FILE)
            X = np.asarray(np.load(WARM_START_FILE)['X'], float).T
            U = np.zeros((self._n_u, N))
            weight = -self._m * self._g
            for k in range(N):
                act = np.nonzero(self._logic[k])[0]
                for i in act:
                    # TALOS too writes at 3*i (reference quirk Q11)
                    U[3 * i:3 * i + 3, k] = [1e-3, 1e-3, weight / len(act)]
        if X.shape != (self._n_x, N + 1) or U.shape != (self._n_u, N):
            raise ValueError('init trajectories must be state (%d, %d) and control (%d, %d)'
                             % (self._n_x, N + 1, self._n_u, N))
        if self._DYNAMICS_FIRST:
            self._x_init, self._x_final = np.asarray(conf.x_init, float), np.asarray(conf.x_final, float)
        else:
            self._x_init, self._x_final = X[:, 0].copy(), X[:, -1].copy()
        self._init_trajectories = {'state': X, 'control': U}

    # ------------------------------------------------------------------ device plumbing
    def problem_batch(self, traj_tuple=None, scp_params=None):
        """This model (and a linearization point) as a one-problem ``ProblemBatch``; ``scp_params``
        overrides the conf's SCP parameters for this batch only."""
        traj = self._init_trajectories if traj_tuple is None else traj_tuple
        params = self._params if scp_params is None else dataclasses.replace(self._params, scp_params=dict(scp_params))
        X = np.asarray(traj['state'], float)
        U = np.asarray(traj['control'], float)
        return ProblemBatch(self._robot, self._N, self._logic.shape[1], self._n_u, self._logic[None], self._pos[None],
                            self._rot[None], np.ascontiguousarray(X.T)[None], np.ascontiguousarray(U.T)[None],
                            np.zeros(1, np.int32), [params])

    def _device_solver(self, traj_tuple=None, scp_params=None):
        """The model's GPU handle with (traj_tuple or the warm start) uploaded as linearization point."""
        if self._solver is None:
            self._solver = Solver(self._robot, self._N, 1, self._precision, self._device)
        self._solver.upload(self.problem_batch(traj_tuple, scp_params))
        return self._solver

    # ------------------------------------------------------------------ reference methods
    def integrate_dynamics_trajectory(self, traj_tuple):
        """x+_k for k = 0..N along traj_tuple (reference :243-255), (nx, N+1)."""
        s = self._device_solver(traj_tuple)
        X = np.ascontiguousarray(np.asarray(traj_tuple['state'], float).T)[None]
        U = np.ascontiguousarray(np.asarray(traj_tuple['control'], float).T)[None]
        return s.rollout(X, U)[0].T

    def compute_trajectory_data(self, traj_tuple):
        """Linearization along traj_tuple (reference :257-291) computed by cmpc_linearize."""
        s = self._device_solver(traj_tuple)
        s.linearize()
        lin = s.linearization()
        nx, nu, N = self._n_x, self._n_u, self._N
        return dict(dynamics=lin['f'][0].T.copy(), LQR_gains=lin['K'][0],
                    gradients={'f_x': lin['A'][0], 'f_u': lin['Bu'][0], 'f_w': lin['C'][0]},
                    Covs=lin['Sigma'][0],
                    Covs_gradients={'Cov_dx': np.zeros((N + 1, nx, nx, nx, N + 1)),
                                    'Cov_du': np.zeros((N + 1, nx, nx, nu, N + 1))})

    def close(self):
        if self._solver is not None:
            self._solver.close()
            self._solver = None
