#!/bin/bash
# Uniformity variants of k_qp_pair (libcmpc_v<k>.so): smoke (B = 3, both modes) then the metric
# bench, one variant after the other, stopping at the first failure.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  echo "== $v"
  CMPC_LIB_VARIANT=$v timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$v.log 2>&1 || { tail -5 gpurun_out/smoke_$v.log; exit 1; }
  tail -1 gpurun_out/smoke_$v.log
  CMPC_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/bench_$v.json 2>&1 || { tail -5 gpurun_out/bench_$v.json; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['phase_ms_per_step']['qp_ms'])"
done
