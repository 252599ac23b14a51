#!/bin/bash
# GPU test suite only (time-limited; per-test timeout names a hang).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | sed 's/ *\[.*%\]//' | awk '{print $2, $1}' | sort | uniq -c | sort -rn | head -3
grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -30
tail -3 gpurun_out/pytest_gpu.log
exit $rc
