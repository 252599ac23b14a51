"""Deterministic synthetic SCP problems for the benchmark configurations.

The reference's inputs come from pinocchio forward kinematics (foot positions) and a
whole-body DDP warm start (``wholeBody_to_centroidal_traj.npz``); neither is available
here, so problems are synthesized:

* contact plan: the reference gait rules (src/contact_plan.py:112-264) applied to the conf
  gait dict; nbSteps is raised until the plan covers N knots, then the plan is truncated to
  N (what the reference does when conf.N < plan length); per-problem foot xy jitter
  U(-0.01, 0.01) m and, for trot/bound, stepLength ~ U(0.08, 0.16);
* warm start (N+1, 9): a rollout of the centroidal dynamics (src/centroidal_model.py:189-212)
  whose contact forces track the smoothed stance-foot centroid and the nominal CoM height
  inside the friction pyramid (so the SCP subproblem is feasible, as with a DDP warm start),
  plus smooth noise under a sin^2(pi k / N) envelope that vanishes at both ends;
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


def plan_spec(conf, N, rng=None, jitter=True):
    """(gait, foot0) of one problem: the conf gait dict with the per-problem stepLength and the
    nbSteps that covers N knots, and the initial foot positions (nc, 3) in the contact order
    FR, FL, HR, HL / FR, FL (what cmpc_generate_contact_plans takes)."""
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
    trans = [robot.foot_positions[n] for n in conf.ee_frame_names]
    feet = {'FL': trans[0], 'FR': trans[1]}
    order = ('FR', 'FL')
    if len(trans) == 4:
        feet['HL'], feet['HR'] = trans[2], trans[3]
        order = ('FR', 'FL', 'HR', 'HL')
    foot0 = np.array([feet[c] for c in order], float)
    return gait, foot0, robot, seq


def contact_plan(conf, N, rng=None, jitter=True):
    """(logic, pos, rot) of N knots for one problem of config ``conf``."""
    _, _, _, seq = plan_spec(conf, N, rng, jitter)
    traj = create_contact_trajectory(_PlanConf(conf.dt, seq))
    return contact_arrays(traj, N)


def warm_start(conf, logic, pos, rng, mass, com_z, gravity=-9.81, robot='solo12'):
    """Synthetic DDP-like centroidal warm start, (N+1, 9).

    A whole-body DDP warm start is dynamically consistent; a synthetic one must be too, or the
    SCP subproblem is infeasible (a random final state is unreachable under the friction
    pyramid).  So the states are a rollout of the centroidal dynamics driven by contact
    forces that track the smoothed stance-foot centroid (PD on the CoM, forces kept strictly
    inside the friction pyramid), plus smooth noise that vanishes at both ends."""
    N, nc = logic.shape
    dt = conf.dt
    nupc = 3 if robot == 'solo12' else 6
    fo = 0 if robot == 'solo12' else 2
    cd = np.zeros((N + 2, 2))
    for k in range(N):
        cd[k] = pos[k, logic[k] > 0, :2].mean(axis=0)
    cd[N:] = cd[N - 1]
    w = 15
    pad = np.pad(cd, ((w // 2, w // 2), (0, 0)), mode='edge')
    cd = np.stack([np.convolve(pad[:, i], np.ones(w) / w, mode='valid') for i in range(2)], axis=1)
    X = np.zeros((N + 1, 9))
    X[0, 0:2] = cd[0]
    X[0, 2] = com_z
    g = -gravity
    kp, kd = 40.0, 12.0
    for k in range(N):
        x = X[k]
        c, v = x[0:3], x[3:6] / mass
        a_ff = (cd[k + 2] - 2 * cd[k + 1] + cd[k]) / dt ** 2 if k + 2 <= N + 1 else np.zeros(2)
        axy = a_ff + kp * (cd[k] - c[:2]) + kd * ((cd[k + 1] - cd[k]) / dt - v[:2])
        az = kp * (com_z - c[2]) - kd * v[2]
        act = np.nonzero(logic[k])[0]
        fz = mass * (g + az) / len(act)
        fxy = mass * axy / len(act)
        lim = 0.25 * fz
        nrm = np.linalg.norm(fxy)
        if nrm > lim:
            fxy = fxy * lim / nrm
        F = np.zeros(9)
        F[0:3] = v
        F[5] = mass * gravity
        for i in act:
            f = np.array([fxy[0], fxy[1], fz])
            F[3:6] += f
            F[6:9] += np.cross(pos[k, i] - c, f)
        X[k + 1] = x + dt * F
    sm = lambda v_: np.convolve(v_, np.ones(9) / 9, mode='valid')
    env = np.sin(np.pi * np.arange(N + 1) / N) ** 2
    X[:, 0:3] += env[:, None] * np.stack([sm(rng.normal(0, 0.002, N + 9)) for _ in range(3)], axis=1)
    X[:, 3:6] += mass * env[:, None] * np.stack([sm(rng.normal(0, 0.02, N + 9)) for _ in range(3)], axis=1)
    X[:, 6:9] += env[:, None] * np.stack([sm(rng.normal(0, 0.01, N + 9)) for _ in range(3)], axis=1)
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
        Xbar[b] = warm_start(conf, lg, ps, rng, params[c].mass, com_z, params[c].gravity, robot)
        Ubar[b] = warm_start_controls(lg, params[c].mass, params[c].gravity, nu)
        cid[b] = c
    pb = ProblemBatch(robot, N, nc, nu, logic, pos, rot, Xbar, Ubar, cid, params)
    pb.validate()
    return pb
