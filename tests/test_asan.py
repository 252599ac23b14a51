"""Host AddressSanitizer build of the C ABI (`make -C centroidal-mpc_amd/csrc asan`,
run by __graft_entry__.build()): the host code of cmpc_api.cpp, load_qp.cpp and comm.cpp with
-fsanitize=address, linked as libcmpc_asan.so.
  * csrc/asan_harness.cpp drives the validation and error paths of every entry point (all of them
    without a device; handle creation, uploads, cmpc_load_qp's CSC checks and the getters with one);
  * the CPU suite's library tests (tests/test_library.py: loading, exports, the no-GPU failure, the
    default settings) run again against the ASan library (CMPC_LIB_VARIANT=asan, the ASan runtime
    preloaded into the interpreter).
GPU ASan is not available on gfx950 here, so the kernels themselves are not instrumented."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CMPC = os.path.join(ROOT, 'centroidal-mpc_amd', 'cmpc')
HARNESS = os.path.join(CMPC, 'asan_harness')
LIB = os.path.join(CMPC, 'libcmpc_asan.so')
CLANG = '/opt/rocm/lib/llvm/bin/clang++'

pytestmark = pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.exists(LIB)),
                                reason='ASan build absent (make -C centroidal-mpc_amd/csrc asan)')


def _runtime():
    return subprocess.run([CLANG, '-print-file-name=libclang_rt.asan-x86_64.so'], capture_output=True,
                          text=True, check=True).stdout.strip()


def test_harness_clean_under_asan():
    r = subprocess.run([HARNESS], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0'))
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'ERROR: AddressSanitizer' not in r.stderr and 'ERROR: LeakSanitizer' not in r.stderr, r.stderr
    assert 'asan harness: ok' in r.stdout


def test_library_tests_under_asan():
    env = dict(os.environ, CMPC_LIB_VARIANT='asan', LD_PRELOAD=_runtime(),
               ASAN_OPTIONS='detect_leaks=0:abort_on_error=0')   # (the interpreter's own allocations)
    r = subprocess.run([sys.executable, '-m', 'pytest', '-q', '-p', 'no:cacheprovider',
                        os.path.join(ROOT, 'tests', 'test_library.py')], capture_output=True, text=True,
                       timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert 'ERROR: AddressSanitizer' not in r.stderr, r.stderr[-3000:]
