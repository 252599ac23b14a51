#!/bin/bash
# Round 4: suite + smoke + default bench, then the per-GPU config lines and shards.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_final.sh || exit 1
run() {  # name, bench args...
    local name=$1; shift
    timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/r04e_$name.json 2> gpurun_out/r04e_$name.err || { tail -20 gpurun_out/r04e_$name.err; exit 1; }
}
run c2_trot_n100_b256_fp64 --config trot --N 100 --batch 256 --no-extras
run c3_bound_n100_b1024_fp32 --config bound --N 100 --batch 1024 --precision fp32 --no-extras
run c4_talos_n200_b512_fp64 --config talos --N 200 --batch 512 --no-extras
run c5_mixed_n150_b1024_fp64 --config mixed --N 150 --batch 1024 --no-extras
run shard512 --batch 512 --no-extras
run shard256 --batch 256 --no-extras
run shard128 --batch 128 --no-extras
python3 - <<'PY'
import json
for t in ('c2_trot_n100_b256_fp64', 'c3_bound_n100_b1024_fp32', 'c4_talos_n200_b512_fp64', 'c5_mixed_n150_b1024_fp64', 'shard512', 'shard256', 'shard128'):
    d = json.load(open('gpurun_out/r04e_%s.json' % t))
    print(t, round(d['value']), 'ms/step %.3f' % d['ms_per_step'], 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'],
          'newton %.2f' % d['qp_ipm_iterations_mean'], d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'],
          'pol +%d -%d' % (d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected']))
PY
