#!/bin/bash
# Grouped QP workgroups: pair/group tests, then same-box bench lines quads (default) / pairs
# (CMPC_QP_GROUP=2) / one wave per problem (CMPC_QP_PAIR=0), twice; group stamps.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_pair.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { tail -30 gpurun_out/pytest_pair.log; exit 1; }
tail -1 gpurun_out/pytest_pair.log
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/grp_quad_$i.json 2>&1 || exit 1
  CMPC_QP_GROUP=2 timeout -k 10 200 $B > gpurun_out/grp_pair_$i.json 2>&1 || exit 1
  CMPC_QP_PAIR=0 timeout -k 10 200 $B > gpurun_out/grp_off_$i.json 2>&1 || exit 1
done
for f in gpurun_out/grp_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'qp_ms %.4f' % d['phase_ms_per_step']['qp_ms'], d['qp_exit']['status_counts'])"; done
timeout -k 10 200 python3 scripts/pair_stamps.py 100 1024 > gpurun_out/group_stamps.log 2>&1 || { cat gpurun_out/group_stamps.log; exit 1; }
tail -9 gpurun_out/group_stamps.log
