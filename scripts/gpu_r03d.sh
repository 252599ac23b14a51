#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_pair.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { tail -20 gpurun_out/pytest_pair.log; exit 1; }
tail -1 gpurun_out/pytest_pair.log
bash scripts/gpu_ab.sh prev > gpurun_out/ab_prev.log 2>&1 || { cat gpurun_out/ab_prev.log; exit 1; }
tail -4 gpurun_out/ab_prev.log
timeout -k 10 200 python3 scripts/pair_stamps.py 100 1024 > gpurun_out/pair_stamps.log 2>&1 || { cat gpurun_out/pair_stamps.log; exit 1; }
tail -9 gpurun_out/pair_stamps.log
