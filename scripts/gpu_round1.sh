#!/bin/bash
# probe + first bench + rocprof kernel stats (each GPU step time-limited; stop at first failure)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python3 scripts/gpu_probe.py trot 30 2 fp64 > gpurun_out/probe3.log 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 400 python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo bench failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { echo rocprof failed; exit 1; }
echo done
