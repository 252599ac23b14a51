#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_pair.py -x -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_pair.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_pair.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 scripts/stamps.py trot 20 4 > gpurun_out/stamps_small.log 2>&1; rc=$?
tail -20 gpurun_out/stamps_small.log; exit $rc
