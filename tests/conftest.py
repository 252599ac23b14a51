import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')
# tests/golden/make_golden.py FIXTURES: N=20 per robot / gait, BASELINE C1 (trot N=50), the metric
# horizon (trot N=100), C3's bound N=100, and float32 runs at the reference's own precision
GOLDEN_TAGS = ('trot', 'trot_stoch', 'bound', 'pace', 'talos', 'trot_n50', 'trot_n100', 'bound_n100',
               'trot_f32', 'bound_n100_f32')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libcmpc.so)')
    config.addinivalue_line('markers', 'slow: longer CPU test')


@pytest.fixture(scope='session')
def golden():
    import numpy as np
    out = {}
    for tag in GOLDEN_TAGS:
        path = os.path.join(GOLDEN, 'golden_%s.npz' % tag)
        if os.path.exists(path):
            out[tag] = dict(np.load(path, allow_pickle=False))
    if not out:
        pytest.skip('golden fixtures missing')
    return out
