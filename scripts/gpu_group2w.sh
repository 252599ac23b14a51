#!/bin/bash
# Two-wave groups (k_qp_group<.., 2, 2>, LDS half-workgroup barrier; CMPC_QP_GROUP2W=1): unshared bit-identity first
# (short timeout: a barrier mismatch would hang), then the group tests, then the 512 shard A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 90 python -u -m pytest tests/test_gpu_qp_pair.py -x -v -k "unshared and trot-100-11" --timeout 60 --timeout-method thread > gpurun_out/pytest_g2w_a.log 2>&1 || { tail -30 gpurun_out/pytest_g2w_a.log; exit 1; }
tail -1 gpurun_out/pytest_g2w_a.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_pair.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_g2w.log 2>&1 || { tail -30 gpurun_out/pytest_g2w.log; exit 1; }
tail -1 gpurun_out/pytest_g2w.log
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --batch 512"
for i in 1 2; do
  CMPC_QP_GROUP2W=1 timeout -k 10 200 $B > gpurun_out/g2w_on_$i.json 2>&1 || exit 1
  CMPC_QP_GROUP2W=1 CMPC_QP_PAIR=2 timeout -k 10 200 $B > gpurun_out/g2w_noshare_$i.json 2>&1 || exit 1
  CMPC_QP_PAIR=0 timeout -k 10 200 $B > gpurun_out/g2w_off_$i.json 2>&1 || exit 1
done
CMPC_QP_GROUP2W=1 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --config talos --N 200 --batch 512 > gpurun_out/g2w_c4_on.json 2>&1 || exit 1
CMPC_QP_PAIR=0 timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --config talos --N 200 --batch 512 > gpurun_out/g2w_c4_off.json 2>&1 || exit 1
for f in gpurun_out/g2w_*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'qp_ms %.4f' % d['phase_ms_per_step']['qp_ms'], d['roofline']['kernel'], d['qp_exit']['status_counts'])"; done
