"""Robot constants used when pinocchio / example_robot_data are not installed.

Synthetic values (the reference computes them by forward kinematics on the URDF):
* solo12: total mass 2.5 kg; feet at the initial configuration (x = +-0.1946,
  y = +-0.14695 (src/simulate_solo.py:56), z = 0).
* TALOS (legs): total mass 90 kg; soles at y = -+0.085, x = z = 0.
"""
import numpy as np

from src.contact_plan import FootFrames

SOLO12_MASS = 2.5
SOLO12_FEET = {'FL_FOOT': (0.1946, 0.14695, 0.0), 'FR_FOOT': (0.1946, -0.14695, 0.0),
               'HL_FOOT': (-0.1946, 0.14695, 0.0), 'HR_FOOT': (-0.1946, -0.14695, 0.0)}
TALOS_MASS = 90.0
TALOS_FEET = {'right_sole_link': (0.0, -0.085, 0.0), 'left_sole_link': (0.0, 0.085, 0.0)}


def solo12():
    try:  # the reference's path (config/conf_solo12_trot.py:25-28)
        import example_robot_data
        import pinocchio
        from robot_properties_solo.solo12wrapper import Solo12Config
        robot = example_robot_data.load('solo12')
        rmodel = robot.model
        q0 = np.array(Solo12Config.initial_configuration.copy()); q0[0] = 0.0
        return rmodel, rmodel.createData(), q0, pinocchio.computeTotalMass(rmodel)
    except ImportError:
        ff = FootFrames('solo', SOLO12_FEET)
        return ff, ff, None, SOLO12_MASS


def talos():
    try:
        import example_robot_data
        import pinocchio
        robot = example_robot_data.load('talos_legs')
        rmodel = robot.model; rmodel.name = 'talos'
        q0 = rmodel.referenceConfigurations['half_sitting'].copy()
        return rmodel, rmodel.createData(), q0, pinocchio.computeTotalMass(rmodel)
    except ImportError:
        ff = FootFrames('talos', TALOS_FEET)
        return ff, ff, None, TALOS_MASS
