"""libcmpc.so: builds for gfx950, loads, exports every symbol of include/cmpc.h; fails loudly
without a GPU (no CPU fallback)."""
import os
import re

import pytest

from cmpc import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, 'include', 'cmpc.h')).read()
    return sorted(set(re.findall(r'^(?:int|const char \*)\s*\*?(cmpc_\w+)\s*\(', src, re.M)))


def test_header_declares_expected_api():
    syms = header_symbols()
    assert 'cmpc_create' in syms and 'cmpc_qp_solve' in syms and 'cmpc_export_qp' in syms
    assert set(syms) == set(_lib.EXPORTS)


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert lib.cmpc_version() == 1


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, 'rb').read()
    assert b'gfx950' in data


@pytest.mark.skipif(os.path.exists('/dev/kfd'), reason='GPU present')
def test_no_gpu_fails_loudly():
    with pytest.raises(_lib.CmpcError):
        _lib.Solver('solo12', 20, 2)


def test_default_qp_settings():
    lib = _lib.load()
    s = _lib.QPSettings()
    assert lib.cmpc_default_qp_settings(0, s) == 0
    # tolerances 0 = the robot's (cmpc_api.cpp qp_eps_default), polishing < 0 = the robot's
    assert s.eps_abs == 0.0 and s.eps_rel == 0.0 and s.max_iter > 0 and s.waves_per_problem == 0
    assert s.polish_eps < 0
    assert lib.cmpc_default_qp_settings(1, s) == 0 and s.eps_abs == 0.0
