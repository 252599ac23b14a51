"""TALOS biped (reference config/conf_talos.py).

The reference config defines only the robot, dt, gait, mu and the contact sequence
(config/conf_talos.py:6-40); it lacks every centroidal parameter, so
``Centroidal_model(conf_talos)`` raises AttributeError in the reference
(src/centroidal_model.py:18).  The centroidal parameters below are SYNTHETIC (same
structure as the solo12 configs, scaled to a 90 kg biped with 6-D contact controls
[cop_x, cop_y, fx, fy, fz, tau_z]); parity for TALOS is therefore relative to these values.
"""
import numpy as np

from src.contact_plan import create_contact_sequence, plan_length
from config import _robots

rmodel, rdata, q0, robot_mass = _robots.talos()
ee_frame_names = ['right_sole_link', 'left_sole_link']
DYNAMICS_FIRST = False
dt = 0.03
dt_ctrl = 0.001
gait = {'type': 'PACE', 'stepLength': 0., 'stepHeight': 0.1, 'stepKnots': 15, 'supportKnots': 5, 'nbSteps': 4}
mu = 0.5
gait_templates, contact_sequence = create_contact_sequence(dt, gait, ee_frame_names, rmodel, rdata, q0)
N = plan_length(contact_sequence, dt)
N_ctrl = int((N - 1) * (dt / dt_ctrl))

# whole-body task weights (conf_talos.py:26-28): read by the whole-body stage only (out of scope),
# kept so scripts that read the attribute run unchanged
whole_body_task_weights = {'footTrack': {'swing': 1e8, 'impact': 1e8}, 'impulseVel': 1e6, 'comTrack': 1e6, 'stateBounds': 0e3,
                           'stateReg': {'stance': 1e1, 'impact': 1e1}, 'ctrlReg': {'stance': 1e-3, 'impact': 1e-3}, 'frictionCone': 10,
                           'centroidalTrack': 1e4, 'contactForceTrack': 100}

# ---- synthetic centroidal parameters (absent from the reference config) ----
robot_name = 'TALOS'
gravity_constant = -9.81
max_leg_length = 1.0
lxp, lxn, lyp, lyn = 0.1, 0.05, 0.05, 0.05   # foot CoP box
n_u_per_contact = 6
nb_contacts = 2
n_u = nb_contacts * n_u_per_contact
n_x = 9
n_t = 1
n_w = nb_contacts * 3
Q = np.diag([1e4, 1e4, 1e4, 1e3, 1e3, 1e3, 1e3, 1e3, 1e3])
R = np.diag([1e2, 1e2, 1e-1, 1e-1, 1e-2, 1e1] * 2)
cov_w = np.diag([0.4 ** 2, 0.4 ** 2, 0.1 ** 2] * 2)
cov_white_noise = dt * np.diag(np.array([0.85 ** 2, 0.4 ** 2, 0.01 ** 2, 0.75 ** 2, 0.4 ** 2, 0.01 ** 2,
                                         0.85 ** 2, 0.4 ** 2, 0.01 ** 2]))
beta_u = 0.01
state_cost_weights = np.diag([1e4, 1e4, 1e4, 1e3, 1e3, 1e3, 1e5, 1e5, 1e5])
control_cost_weights = np.diag([1e3, 1e3, 1e-1, 1e-1, 1e-2, 1e1] * 2)
# trust_region_radius0: the solve_scp acceptance test is the spectral norm of the whole 9 x (N+1)
# state change (quirk Q6), and for a 90 kg robot with no tracking cost (Q10) that change is
# dominated by the linear and angular momenta the state cost pulls toward zero: 500-530 on the
# BASELINE C4 problems (N=200), whatever the trust-region weight (the QP's L1 trust region binds
# only x[6:9], per knot).  The Solo12 value 100 would reject every iteration until
# max_iterations ("TALOS acceptance"); 1000 accepts at the first iteration with
# rho 0.38-0.41.
scp_params = {'trust_region_radius0': 1000, 'omega0': 100, 'omega_max': 1e10, 'epsilon': 1e-6, 'rho0': 0.4,
              'rho1': 1.5, 'beta_succ': 2., 'beta_fail': 0.5, 'gamma_fail': 5, 'convergence_threshold': 1e-3,
              'max_iterations': 10}
WITHDISPLAY = False
cameraTF = [3., 3.68, 0.84, 0.2, 0.62, 0.72, 0.22]  # viewer camera (conf_talos.py:42)
