#!/bin/bash
# GPU session: tests -> stamps -> bench (each step time-limited, stop at first failure)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
timeout -k 10 200 python3 scripts/stamps.py trot 100 256 || exit 1
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
