"""Problem configurations with the reference's attribute names (config/conf_*.py).

The reference configs load the robot with example_robot_data / pinocchio at import time
(e.g. config/conf_solo12_trot.py:23-28,45-47).  Those packages are optional here: when
they are absent, robot mass and foot positions come from the synthetic constants in
``_robots.py`` (documented in DESIGN.md; parity for these two quantities is unpinned).
"""
