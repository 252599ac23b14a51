"""Gait template -> contact sequence -> per-knot contact trajectory (host side, setup only).

Drop-in for the reference's src/contact_plan.py (``Debris`` :8-37,
``create_contact_trajectory`` :40-48, ``create_contact_sequence`` :112-264).  Clean-room:
the behaviour (phase templates, swing/stance assignment, foot advance after each step,
contact index mapping FR=0, FL=1, HR=2, HL=3) follows the reference; pinocchio is optional.
When pinocchio is absent the caller passes a ``FootFrames`` object as ``rmodel``/``rdata``
holding the foot translations that the reference reads from forward kinematics.
"""
import numpy as np

_CONTACT_IDX = {'RF': 0, 'FR': 0, 'LF': 1, 'FL': 1, 'HR': 2, 'HL': 3}


def _angle_axis(angle, axis3):
    """Rotation matrix of an angle-axis pair (Rodrigues), = pin.AngleAxis(angle, axis).matrix()."""
    a = np.asarray(axis3, float)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * (K @ K)


class SE3:
    """Minimal pose (rotation, translation) standing in for pinocchio.SE3."""

    def __init__(self, rotation, translation):
        self.rotation = np.asarray(rotation, float)
        self.translation = np.asarray(translation, float)


class Debris:
    """One contact of one phase (reference src/contact_plan.py:8-37)."""

    def __init__(self, CONTACT, t_start=0.0, t_end=1.0, x=None, y=None, z=None, axis=None,
                 angle=None, ACTIVE=False):
        if ACTIVE:
            ax = np.array(axis, np.float64)
            ax /= np.linalg.norm(ax)
            self.axis = ax
            self.pose = SE3(_angle_axis(angle, np.concatenate([ax, [0.0]])), np.array([x, y, z], float))
        self.t_start = t_start
        self.t_end = t_end
        self.CONTACT = CONTACT
        self.ACTIVE = ACTIVE
        self.idx = _CONTACT_IDX.get(CONTACT)


class FootFrames:
    """Pinocchio-free robot description: ``name`` ('solo' | 'talos') and foot translations by
    frame name.  Acts as both ``rmodel`` and ``rdata`` for create_contact_sequence."""

    def __init__(self, name, foot_positions):
        self.name = name
        self.foot_positions = {k: np.array(v, float) for k, v in foot_positions.items()}


def _foot_translations(ee_frame_names, rmodel, rdata, q0):
    if isinstance(rmodel, FootFrames):
        return [rmodel.foot_positions[n].copy() for n in ee_frame_names]
    import pinocchio as pin  # only when a real pinocchio model is handed in
    pin.forwardKinematics(rmodel, rdata, q0)
    pin.updateFramePlacements(rmodel, rdata)
    return [rdata.oMf[rmodel.getFrameId(n)].translation.copy() for n in ee_frame_names]


def gait_templates_for(gait, robot_name):
    """Phase templates per gait type (reference src/contact_plan.py:113-149)."""
    steps = gait['nbSteps']
    if gait['type'] == 'TROT':
        cyc = ['rflhStep', 'lfrhStep']
    elif gait['type'] == 'PACE':
        cyc = ['rfrhStep', 'lflhStep'] if robot_name == 'solo' else ['rfStep', 'lfStep']
    elif gait['type'] == 'BOUND':
        cyc = ['rflfStep', 'rhlhStep']
    else:
        raise ValueError('unknown gait type %r' % gait['type'])
    out = []
    for s in range(steps):
        tpl = ['doubleSupport', cyc[0], 'doubleSupport', cyc[1]]
        if s == steps - 1:
            tpl = tpl + ['doubleSupport']
        out.append(tpl)
    return out


# phase -> (swing contacts, contacts whose foot advances by stepLength after the phase)
_SOLO_PHASES = {
    'rflhStep': (('FR', 'HL'), ('FR', 'HL')),
    'lfrhStep': (('FL', 'HR'), ('FL', 'HR')),
    'rfrhStep': (('FR', 'HR'), ('FR', 'HR')),
    'lflhStep': (('FL', 'HL'), ('FL', 'HL')),
    'rflfStep': (('FR', 'FL'), ('FR', 'FL')),
    'rhlhStep': (('HR', 'HL'), ('HR', 'HL')),
}
_TALOS_PHASES = {'rfStep': (('FR',), ('FR',)), 'lfStep': (('FL',), ('FL',))}


def create_contact_sequence(dt, gait, ee_frame_names, rmodel, rdata, q0=None):
    """Reference src/contact_plan.py:112-264.  Returns (gait_templates, contact_sequence)."""
    name = rmodel.name
    templates = gait_templates_for(gait, name)
    trans = _foot_translations(ee_frame_names, rmodel, rdata, q0)
    # reference: fl = ee[0], fr = ee[1], hl = ee[2], hr = ee[3] (for TALOS ee = [right, left],
    # so the contact named FR sits on ee[1]; kept as the reference does)
    feet = {'FL': trans[0], 'FR': trans[1]}
    if name == 'solo':
        feet['HL'] = trans[2]
        feet['HR'] = trans[3]
        order = ('FR', 'FL', 'HR', 'HL')
        phases = _SOLO_PHASES
    else:
        order = ('FR', 'FL')
        phases = _TALOS_PHASES
    stepKnots, supportKnots = gait['stepKnots'], gait['supportKnots']
    L = gait['stepLength']
    t_start = 0.0
    seq = []
    for tpl in templates:
        for phase in tpl:
            if phase == 'doubleSupport':
                t_end = t_start + supportKnots * dt
                swing, advance = (), ()
            else:
                t_end = t_start + stepKnots * dt
                if phase not in phases:
                    swing, advance = order, order  # reference's fall-through branch (:254-263)
                else:
                    swing, advance = phases[phase]
            seq_k = []
            for c in order:
                if c in swing:
                    seq_k.append(Debris(CONTACT=c, t_start=t_start, t_end=t_end, ACTIVE=False))
                else:
                    p = feet[c]
                    seq_k.append(Debris(CONTACT=c, t_start=t_start, t_end=t_end, x=p[0], y=p[1], z=p[2],
                                        axis=[-1, 0], angle=0.0, ACTIVE=True))
            for c in advance:
                feet[c][0] += L
            t_start = t_end
            seq.append(seq_k)
    return templates, seq


def create_contact_trajectory(conf):
    """Expand phases into per-knot contact lists (reference src/contact_plan.py:40-48)."""
    seq = conf.contact_sequence
    traj = dict([(c.CONTACT, []) for c in seq[0]])
    for contacts in seq:
        for c in contacts:
            dur = int(round((c.t_end - c.t_start) / conf.dt))
            for _ in range(dur):
                traj[c.CONTACT].append(c)
    return traj


def plan_length(contact_sequence, dt):
    """N as the configs compute it: int(round(t_end_last / dt, 2))."""
    return int(round(contact_sequence[-1][0].t_end / dt, 2))


def contact_arrays(contact_trajectory, N):
    """logic (N, nc) int8, pos (N, nc, 3), rot (N, nc, 3, 3): the arrays built by
    Centroidal_model.__fill_contact_data (reference src/centroidal_model.py:127-156); zeros
    for inactive contacts."""
    names = list(contact_trajectory.keys())
    nc = len(names)
    logic = np.zeros((N, nc), np.int8)
    pos = np.zeros((N, nc, 3))
    rot = np.zeros((N, nc, 3, 3))
    for k in range(N):
        for i, c in enumerate(names):
            d = contact_trajectory[c][k]
            if d.ACTIVE:
                logic[k, i] = 1
                pos[k, i] = d.pose.translation
                rot[k, i] = d.pose.rotation
    return logic, pos, rot
