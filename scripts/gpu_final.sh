#!/bin/bash
# Round-end check at HEAD: smoke, GPU suite, default bench line; then the two-wave group A/B
# (on / unshared / off, CMPC_QP_GROUP2W=1) on the 512-problem shard.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'], 'early', round(d['early_exit']['value']))"
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --batch 512"
for i in 1 2; do
  CMPC_QP_GROUP2W=1 timeout -k 10 200 $B > gpurun_out/g2_on_$i.json 2>&1 || exit 1
  CMPC_QP_GROUP2W=1 CMPC_QP_PAIR=2 timeout -k 10 200 $B > gpurun_out/g2_noshare_$i.json 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/g2_off_$i.json 2>&1 || exit 1
done
for f in gpurun_out/g2_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'qp_ms %.4f' % d['phase_ms_per_step']['qp_ms'], d['roofline']['kernel'])"; done
