#!/bin/bash
# GPU suite, then the two-wave configurations: BASELINE C2 / C4 lines and one GPU's step at the
# strong-scaling shard sizes (512 / 256 / 128 problems of the metric config), plus stamps of C2.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 200 python scripts/stamps.py trot 100 256 > gpurun_out/stamps_c2.log 2>&1 || { tail -20 gpurun_out/stamps_c2.log; exit 1; }
tail -2 gpurun_out/stamps_c2.log
for a in "c2 --config trot --N 100 --batch 256" "c4 --config talos --N 200 --batch 512" "s512 --batch 512" "s128 --batch 128"; do
  set -- $a; n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/sb_$n.json 2> gpurun_out/sb_$n.err || { tail -20 gpurun_out/sb_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sb_$n.json'));print('$n', round(d['value']), 'ms/step %.3f' % d['ms_per_step'], 'qp %.3f' % d['phase_ms_per_step']['qp_ms'])"
done
