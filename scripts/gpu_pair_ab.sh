#!/bin/bash
# Paired QP workgroups: GPU suite, then same-box A/B of the metric config with pairing (default)
# against CMPC_QP_PAIR=0 (one wave per problem), bench lines A B A B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/pair_on_$i.json 2>&1 || exit 1
  CMPC_QP_PAIR=0 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/pair_off_$i.json 2>&1 || exit 1
  CMPC_QP_PAIR=2 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/pair_noshare_$i.json 2>&1 || exit 1
done
for f in gpurun_out/pair_o*.json gpurun_out/pair_noshare_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['phase_ms_per_step'], d['qp_ipm_iterations_mean'], d['qp_exit'])"; done
timeout -k 10 300 python3 scripts/pair_diag.py > gpurun_out/pair_diag.log 2>&1 || exit 1
cat gpurun_out/pair_diag.log
for v in 1 0; do
  CMPC_QP_PAIR=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --config bound --precision fp32 > gpurun_out/pair_c3_$v.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/pair_c3_$v.json').read().strip().splitlines()[-1]); print('C3 pair=$v', round(d['value']), d['phase_ms_per_step']['qp_ms'], d['qp_exit'])"
done
