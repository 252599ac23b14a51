import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'centroidal-mpc_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through libcmpc.so)')
    config.addinivalue_line('markers', 'slow: longer CPU test')


@pytest.fixture(scope='session')
def golden():
    import numpy as np
    out = {}
    for tag in ('trot', 'trot_stoch', 'bound', 'pace', 'talos'):
        path = os.path.join(GOLDEN, 'golden_%s.npz' % tag)
        if os.path.exists(path):
            out[tag] = dict(np.load(path, allow_pickle=False))
    if not out:
        pytest.skip('golden fixtures missing')
    return out
