#!/bin/bash
# Round 4: rocprofv3 kernel traces of BASELINE C4 (TALOS N=200 x 512) and C5 (mixed N=150 x 1024),
# so the head / tail split of their QP launches is on record next to the metric's.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04f_c4 -o trace -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --config talos --N 200 --batch 512 > gpurun_out/prof_r04f_c4.log 2>&1 || { tail -20 gpurun_out/prof_r04f_c4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04f_c5 -o trace -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --config mixed --N 150 > gpurun_out/prof_r04f_c5.log 2>&1 || { tail -20 gpurun_out/prof_r04f_c5.log; exit 1; }
for c in c4 c5; do head -4 gpurun_out/prof_r04f_$c/trace_kernel_stats.csv | cut -c1-160; done
