"""Deterministic synthetic SCP problems for the benchmark configurations.

The reference's inputs come from pinocchio forward kinematics (foot positions) and a
whole-body DDP warm start (``wholeBody_to_centroidal_traj.npz``); neither is available
here, so problems are synthesized:

* contact plan: the reference gait rules (src/contact_plan.py:112-264) applied to the conf
  gait dict; nbSteps is raised until the plan covers N knots, then the plan is truncated to
  N (what the reference does when conf.N < plan length); per-problem foot xy jitter
  U(-0.01, 0.01) m and, for trot/bound, stepLength ~ U(0.08, 0.16);
* warm start (N+1, 9): CoM xy follows the centroid of the stance feet (smoothed), CoM z
  = nominal height + N(0, 0.003^2), linear momentum = m * finite-difference velocity,
  angular momentum smoothed N(0, 0.01^2)
  (all noise terms are 9-tap moving averages, so the warm start is smooth);
* Ubar: the reference rule [1e-3, 1e-3, m*9.81/#active] at rows 3i..3i+2 of every active
  contact (src/centroidal_model.py:176-183; also for TALOS, quirk Q11).
Seed: numpy default_rng(1000 * cfg_seed + b).
"""
import copy
import importlib

import numpy as np

from src.contact_plan import create_contact_sequence, create_contact_trajectory, contact_arrays, plan_length
from .problem import ModelParams, ProblemBatch

CONFIGS = {'trot': ('config.conf_solo12_trot', 1), 'bound': ('config.conf_solo12_bound', 2),
           'pace': ('config.conf_solo12_pace', 3), 'talos': ('config.conf_talos', 4)}


def load_conf(name):
    return importlib.import_module(CONFIGS[name][0])


class _PlanConf:
    def __init__(self, dt, seq):
        self.dt = dt
        self.contact_sequence = seq


def contact_plan(conf, N, rng=None, jitter=True):
    """(logic, pos, rot) of N knots for one problem of config ``conf``."""
    gait = dict(conf.gait)
    robot = copy.deepcopy(conf.rmodel)
    if rng is not None and jitter:
        for k in robot.foot_positions:
            robot.foot_positions[k][:2] += rng.uniform(-0.01, 0.01, 2)
        if gait['type'] in ('TROT', 'BOUND'):
            gait['stepLength'] = float(rng.uniform(0.08, 0.16))
    while True:
        _, seq = create_contact_sequence(conf.dt, gait, conf.ee_frame_names, robot, robot, conf.q0)
        if plan_length(seq, conf.dt) >= N:
            break
        gait['nbSteps'] += 1
    traj = create_contact_trajectory(_PlanConf(conf.dt, seq))
    return contact_arrays(traj, N)


def warm_start(conf, logic, pos, rng, mass, com_z):
    """Synthetic DDP-like centroidal warm start, (N+1, 9)."""
    N, nc = logic.shape
    cxy = np.zeros((N + 1, 2))
    for k in range(N):
        act = logic[k] > 0
        cxy[k] = pos[k, act, :2].mean(axis=0)
    cxy[N] = cxy[N - 1]
    # moving-average smoothing, edge-padded
    w = 9
    pad = np.pad(cxy, ((w // 2, w // 2), (0, 0)), mode='edge')
    ker = np.ones(w) / w
    cxy = np.stack([np.convolve(pad[:, i], ker, mode='valid') for i in range(2)], axis=1)
    X = np.zeros((N + 1, 9))
    X[:, 0:2] = cxy
    sm = lambda v: np.convolve(v, np.ones(9) / 9, mode='valid')
    X[:, 1] += sm(rng.normal(0, 0.005, N + 9))
    X[:, 2] = com_z + sm(rng.normal(0, 0.003, N + 9))
    vel = np.zeros((N + 1, 3))
    vel[:-1] = np.diff(X[:, 0:3], axis=0) / conf.dt
    vel[-1] = vel[-2]
    X[:, 3:6] = mass * vel
    kn = rng.normal(0, 0.01, (N + 9, 3))
    X[:, 6:9] = np.stack([sm(kn[:, i]) for i in range(3)], axis=1)
    return X


def warm_start_controls(logic, mass, gravity, nu):
    """Reference rule src/centroidal_model.py:176-183 (Ubar, (N, nu))."""
    N, nc = logic.shape
    U = np.zeros((N, nu))
    w = -mass * gravity
    for k in range(N):
        per = w / np.sum(logic[k])
        for i in range(nc):
            if logic[k, i]:
                U[k, 3 * i: 3 * i + 3] = [1e-3, 1e-3, per]
    return U


def make_batch(cfg, N, B, stochastic=False, seed_offset=0, mixed=None):
    """B synthetic problems of config ``cfg`` ('trot' | 'bound' | 'pace' | 'talos').

    ``mixed=('pace', 'trot')`` alternates configs by problem index (odd b -> first),
    which is the BASELINE C5 workload; all configs of one batch must share the robot."""
    names = list(mixed) if mixed else [cfg]
    confs = [load_conf(n) for n in names]
    params = [ModelParams.from_conf(c, stochastic) for c in confs]
    robot = params[0].robot
    if any(p.robot != robot for p in params):
        raise ValueError('a batch must share one robot')
    nc = len(create_contact_trajectory(confs[0]))
    nu = confs[0].n_u
    com_z = 0.24 if robot == 'solo12' else 0.87
    logic = np.zeros((B, N, nc), np.int8); pos = np.zeros((B, N, nc, 3)); rot = np.zeros((B, N, nc, 3, 3))
    Xbar = np.zeros((B, N + 1, 9)); Ubar = np.zeros((B, N, nu)); cid = np.zeros(B, np.int32)
    for b in range(B):
        c = (0 if b % 2 == 1 else 1) if len(names) > 1 else 0
        conf = confs[c]
        rng = np.random.default_rng(1000 * CONFIGS[names[c]][1] + b + seed_offset)
        lg, ps, rt = contact_plan(conf, N, rng)
        logic[b], pos[b], rot[b] = lg, ps, rt
        Xbar[b] = warm_start(conf, lg, ps, rng, params[c].mass, com_z)
        Ubar[b] = warm_start_controls(lg, params[c].mass, params[c].gravity, nu)
        cid[b] = c
    pb = ProblemBatch(robot, N, nc, nu, logic, pos, rot, Xbar, Ubar, cid, params)
    pb.validate()
    return pb
