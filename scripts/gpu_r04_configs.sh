#!/bin/bash
# Round 4 measurements: split tests, BASELINE C2..C5 per-GPU lines, the metric's 1-GPU shards
# (strong-scaling projection), and the fresh-batch prior A/B on the early-exit leg.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_qp_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k_split.log 2>&1 || { tail -40 gpurun_out/k_split.log; exit 1; }
tail -1 gpurun_out/k_split.log
run() {  # name, bench args...
    local name=$1; shift
    timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/r04_$name.json 2> gpurun_out/r04_$name.err || { tail -20 gpurun_out/r04_$name.err; exit 1; }
}
run c2_trot_n100_b256_fp64 --config trot --N 100 --batch 256 --no-extras
run c3_bound_n100_b1024_fp32 --config bound --N 100 --batch 1024 --precision fp32 --no-extras
run c4_talos_n200_b512_fp64 --config talos --N 200 --batch 512 --no-extras
run c5_mixed_n150_b1024_fp64 --config mixed --N 150 --batch 1024 --no-extras
run shard512 --batch 512 --no-extras
run shard128 --batch 128 --no-extras
run metric_prior
CMPC_QP_SPLIT_FRESH=0 run metric_noprior
python3 - <<'PY'
import json
for t in ('c2_trot_n100_b256_fp64', 'c3_bound_n100_b1024_fp32', 'c4_talos_n200_b512_fp64', 'c5_mixed_n150_b1024_fp64', 'shard512', 'shard128', 'metric_prior', 'metric_noprior'):
    d = json.load(open('gpurun_out/r04_%s.json' % t))
    ee = d.get('early_exit', {})
    print(t, round(d['value']), 'ms/step %.3f' % d['ms_per_step'], 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'],
          'newton %.2f' % d['qp_ipm_iterations_mean'], d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'],
          'early_exit %s' % (round(ee['value']) if ee else '-'))
PY
