#!/bin/bash
# Per-GPU bench lines for BASELINE.json's other configs (C2..C5, one GPU's shard of each).
# Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() {  # name, bench args...
    local name=$1; shift
    timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || { tail -20 gpurun_out/cfg_$name.err; exit 1; }
    cat gpurun_out/cfg_$name.json
}
run c2_trot_n100_b256_fp64 --config trot --N 100 --batch 256
run c3_bound_n100_b1024_fp32 --config bound --N 100 --batch 1024 --precision fp32
run c4_talos_n200_b512_fp64 --config talos --N 200 --batch 512
run c5_mixed_n150_b1024_fp64 --config mixed --N 150 --batch 1024
