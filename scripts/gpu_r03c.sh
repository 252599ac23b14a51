#!/bin/bash
# A/B (default vs libcmpc_prev.so), pair stamps at the metric config, phase stamps of the
# four-wave shards (128, 256 problems)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_ab.sh prev > gpurun_out/ab_prev.log 2>&1 || { cat gpurun_out/ab_prev.log; exit 1; }
tail -4 gpurun_out/ab_prev.log
timeout -k 10 200 python3 scripts/pair_stamps.py 100 1024 > gpurun_out/pair_stamps.log 2>&1 || { cat gpurun_out/pair_stamps.log; exit 1; }
cat gpurun_out/pair_stamps.log
for B in 128 256; do
  timeout -k 10 200 python3 scripts/stamps.py trot 100 $B 4 > gpurun_out/stamps4_$B.log 2>&1 || { cat gpurun_out/stamps4_$B.log; exit 1; }
  cat gpurun_out/stamps4_$B.log
done
