#!/bin/bash
# Round-end evidence at HEAD: cycle stamps, rocprof + PMC passes and the default bench line
# (scripts/gpu_profile.sh), the other BASELINE configs (scripts/gpu_configs.sh) and one GPU's step
# at the strong-scaling shard sizes (512 / 256 / 128 problems of the metric config).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02c}
timeout -k 10 200 python scripts/stamps.py trot 100 1024 > gpurun_out/stamps_$TAG.log 2>&1 || { tail -20 gpurun_out/stamps_$TAG.log; exit 1; }
bash scripts/gpu_profile.sh $TAG || exit 1
bash scripts/gpu_configs.sh > gpurun_out/configs_$TAG.jsonl || exit 1
for nb in 512 256 128; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --batch $nb > gpurun_out/shard_$nb.json 2> gpurun_out/shard_$nb.err || { tail -20 gpurun_out/shard_$nb.err; exit 1; }
done
cat gpurun_out/shard_*.json
