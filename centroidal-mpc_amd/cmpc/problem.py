"""Host-side problem description shared by the drop-in API and the batched API.

A batch holds B independent SCP problems that share one robot/horizon (``Dims``) and
reference one of a few parameter classes (``ModelParams``; e.g. trot and pace configs in
one mixed batch).  Array layouts are knot-major, C-contiguous, float64 on the host:

=========  ====================  ==================================================
logic      (B, N, nc)   int8     contact active flags   (reference _contact_data)
pos        (B, N, nc, 3)         contact positions      (zeros when inactive)
rot        (B, N, nc, 3, 3)      contact orientations   (zeros when inactive)
Xbar       (B, N+1, 9)           warm-start states      (npz 'X' layout)
Ubar       (B, N, nu)            warm-start controls
class_id   (B,)         int32    parameter class per problem
=========  ====================  ==================================================
"""
from dataclasses import dataclass, field

import numpy as np

ROBOT_SOLO12 = 0
ROBOT_TALOS = 1


@dataclass
class ModelParams:
    """Per-class parameters (the conf_* attributes the hot path reads)."""
    robot: str
    mass: float
    gravity: float
    dt: float
    mu: float
    beta_u: float
    Wx: np.ndarray            # (9,) diag of state_cost_weights
    Wu: np.ndarray            # (nu,) diag of control_cost_weights
    Q: np.ndarray             # (9, 9) LQR
    R: np.ndarray             # (nu, nu) LQR
    cov_w: np.ndarray         # (nw, nw)
    cov_eta: np.ndarray       # (9, 9)
    foot_range: tuple = (0.01, 0.01, 0.01, 0.01)   # lxp, lxn, lyp, lyn
    stochastic: bool = False
    tracking: bool = True
    scp_params: dict = field(default_factory=dict)

    @staticmethod
    def from_conf(conf, stochastic=False):
        Wx = np.asarray(conf.state_cost_weights, float)
        Wu = np.asarray(conf.control_cost_weights, float)
        for W, name in ((Wx, 'state_cost_weights'), (Wu, 'control_cost_weights')):
            if np.count_nonzero(W - np.diag(np.diag(W))):
                raise ValueError('%s must be diagonal (all reference configs are)' % name)
        return ModelParams(
            robot=conf.robot_name, mass=float(conf.robot_mass), gravity=float(conf.gravity_constant),
            dt=float(conf.dt), mu=float(conf.mu), beta_u=float(conf.beta_u),
            Wx=np.diag(Wx).copy(), Wu=np.diag(Wu).copy(), Q=np.asarray(conf.Q, float),
            R=np.asarray(conf.R, float), cov_w=np.asarray(conf.cov_w, float),
            cov_eta=np.asarray(conf.cov_white_noise, float),
            foot_range=(float(getattr(conf, 'lxp', 0.01)), float(getattr(conf, 'lxn', 0.01)),
                        float(getattr(conf, 'lyp', 0.01)), float(getattr(conf, 'lyn', 0.01))),
            stochastic=bool(stochastic),
            tracking=(conf.robot_name == 'solo12' and not conf.DYNAMICS_FIRST),
            scp_params=dict(conf.scp_params))

    @property
    def robot_id(self):
        return ROBOT_SOLO12 if self.robot == 'solo12' else ROBOT_TALOS

    def as_prm(self, nc, nu):
        """Dict in the oracle's ``prm`` format (tests only)."""
        return dict(robot=self.robot, m=self.mass, g=self.gravity, dt=self.dt, nc=nc, nu=nu, nw=3 * nc,
                    Q=self.Q, R=self.R, cov_w=self.cov_w, cov_eta=self.cov_eta, Wx=np.diag(self.Wx),
                    Wu=np.diag(self.Wu), mu=self.mu, beta_u=self.beta_u, stochastic=self.stochastic,
                    tracking=self.tracking, foot_range=self.foot_range)


@dataclass
class ProblemBatch:
    robot: str
    N: int
    nc: int
    nu: int
    logic: np.ndarray
    pos: np.ndarray
    rot: np.ndarray
    Xbar: np.ndarray
    Ubar: np.ndarray
    class_id: np.ndarray
    params: list

    @property
    def B(self):
        return self.logic.shape[0]

    def subset(self, lo, hi):
        return ProblemBatch(self.robot, self.N, self.nc, self.nu, self.logic[lo:hi], self.pos[lo:hi],
                            self.rot[lo:hi], self.Xbar[lo:hi], self.Ubar[lo:hi], self.class_id[lo:hi],
                            self.params)

    def validate(self):
        B, N, nc, nu = self.B, self.N, self.nc, self.nu
        exp = dict(logic=(B, N, nc), pos=(B, N, nc, 3), rot=(B, N, nc, 3, 3), Xbar=(B, N + 1, 9),
                   Ubar=(B, N, nu), class_id=(B,))
        for k, shp in exp.items():
            a = getattr(self, k)
            if tuple(a.shape) != shp:
                raise ValueError('%s has shape %s, expected %s' % (k, a.shape, shp))
        if nu % nc or (self.robot == 'solo12' and nu != 3 * nc) or (self.robot == 'TALOS' and nu != 6 * nc):
            raise ValueError('inconsistent nu=%d nc=%d for %s' % (nu, nc, self.robot))
        if self.class_id.min() < 0 or self.class_id.max() >= len(self.params):
            raise ValueError('class_id out of range')
        if np.any(self.logic.sum(axis=2) == 0):
            raise ValueError('a knot without any active contact (the reference divides by zero there)')

    def oracle_problem(self, b):
        """Problem b in the oracle's format (reference orientation X (9, N+1), U (nu, N))."""
        p = self.params[int(self.class_id[b])]
        return dict(prm=p.as_prm(self.nc, self.nu), N=self.N, logic=self.logic[b],
                    pos=self.pos[b].reshape(self.N, 3 * self.nc), rot=self.rot[b],
                    Xbar=self.Xbar[b].T.copy(), Ubar=self.Ubar[b].T.copy(), scp_params=p.scp_params)
