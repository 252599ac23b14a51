"""Solo12 pace (reference config/conf_solo12_pace.py, same attribute names and values)."""
import numpy as np

from src.contact_plan import create_contact_sequence, plan_length
from config import _robots

# walking parameters (:7-19)
DYNAMICS_FIRST = False
dt = 0.01
dt_ctrl = 0.001
gait = {'type': 'PACE', 'stepLength': 0.0, 'stepHeight': 0.05, 'stepKnots': 10, 'supportKnots': 3,
        'nbSteps': 4}
mu = 0.5

# robot model and parameters (:21-36)
robot_name = 'solo12'
ee_frame_names = ['FL_FOOT', 'FR_FOOT', 'HL_FOOT', 'HR_FOOT']
rmodel, rdata, q0, robot_mass = _robots.solo12()
gravity_constant = -9.81
max_leg_length = 0.34
foot_scaling = 1.
lxp = lxn = lyp = lyn = 0.01

# centroidal state and control dimensions (:38-43)
n_u_per_contact = 3
nb_contacts = 4
n_u = nb_contacts * n_u_per_contact
n_x = 9
n_t = 1

gait_templates, contact_sequence = create_contact_sequence(dt, gait, ee_frame_names, rmodel, rdata, q0)
N = plan_length(contact_sequence, dt)
N_ctrl = int((N - 1) * (dt / dt_ctrl))

# LQR gains (:55-62)
Q = np.diag([1e4, 1e4, 1e4, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3])
R = np.diag([1e2, 5e2, 1e1] * 4)

# noise (:66-77)
n_w = nb_contacts * 3
cov_w = np.diag([0.4 ** 2, 0.4 ** 2, 0.3 ** 2] * 4)
cov_white_noise = dt * np.diag(np.array([0.7 ** 2, 0.5 ** 2, 0.01 ** 2, 0.8 ** 2, 0.6 ** 2, 0.01 ** 2,
                                         0.7 ** 2, 0.5 ** 2, 0.01 ** 2]))
beta_u = 0.01

# cost weights (:81-85)
state_cost_weights = np.diag([1e4, 1e4, 1e4, 1e3, 1e3, 1e3, 1e5, 1e5, 1e5])
control_cost_weights = np.diag([1e2, 1e2, 1e1] * 4)

# whole-body task weights (conf_solo12_pace.py:90-92): read by the whole-body stage only (out of scope),
# kept so scripts that read the attribute run unchanged
whole_body_task_weights = {'footTrack': {'swing': 1e5, 'impact': 1e6}, 'impulseVel': 20, 'comTrack': 1000, 'stateBounds': 0e3,
                           'stateReg': {'stance': 0.1, 'impact': 1}, 'ctrlReg': {'stance': 1, 'impact': 10}, 'frictionCone': 2,
                           'centroidalTrack': 1e4, 'contactForceTrack': 100}

# SCP solver parameters (conf_solo12_pace.py:96-98)
scp_params = {'trust_region_radius0': 50, 'omega0': 100, 'omega_max': 1e10, 'epsilon': 1e-6, 'rho0': 0.4,
              'rho1': 1.5, 'beta_succ': 2., 'beta_fail': 0.5, 'gamma_fail': 5, 'convergence_threshold': 1e-3,
              'max_iterations': 20}

WITHDISPLAY = False
WITH_MESHCAT_DISPLAY = False
WITH_PYBULLET_SIMULATION = False
WITHPLOT = False
SAVEDAT = False
cameraTF = [2., 2.68, 0.84, 0.2, 0.62, 0.72, 0.22]  # viewer camera (conf_solo12_pace.py:101)
