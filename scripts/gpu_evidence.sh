#!/bin/bash
# Round evidence at HEAD: GPU suite, profile session (rocprofv3 stats, PMC traffic / counters,
# default bench line with CPU baseline), BASELINE configs, strong-scaling shards.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r03f}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
bash scripts/gpu_profile.sh $TAG > gpurun_out/profile_$TAG.log 2>&1 || { tail -30 gpurun_out/profile_$TAG.log; exit 1; }
tail -3 gpurun_out/profile_$TAG.log
bash scripts/gpu_configs.sh > gpurun_out/configs_$TAG.log 2>&1 || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
for B in 128 256 512; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batch $B > gpurun_out/shard_$B.json 2>&1 || exit 1
done
echo done
