#!/bin/bash
# Quick GPU iteration: GPU parity tests, per-phase cycle stamps, a short bench line.
# Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python scripts/stamps.py trot 100 1024 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
