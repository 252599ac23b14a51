#!/bin/bash
# GPU tests of a selection (no -x: every failure of the selection is reported), e.g.
#   gpurun -- 'bash scripts/gpu_sel.sh tests/test_gpu_golden.py tests/test_gpu_load_qp.py'
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest "$@" -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_sel.log | tail -40
exit $rc
