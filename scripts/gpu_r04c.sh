#!/bin/bash
# Round 4: the flat-scratch fix (forced inlining, separators by value) with T1-T3, grouped tests first
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_pair.py -x -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_pair.log 2>&1 || { tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf --deselect tests/test_gpu_headline.py::test_metric_config_kernel_matches_oracle --deselect "tests/test_gpu_headline.py::test_metric_shards_match_oracle" > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/gpu_ab.sh r03 || exit 1
timeout -k 10 200 python scripts/stamps.py trot 100 1024 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
