#!/bin/bash
# The full GPU test suite as the driver runs it (one process, per-test timeout), log in gpurun_out.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/suite.log 2>&1
rc=$?
tail -30 gpurun_out/suite.log
exit $rc
