#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_qp_waves.py tests/test_gpu_qp_pair.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || { tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
for B in 128 256; do
  timeout -k 10 200 python3 scripts/stamps.py trot 100 $B 4 > gpurun_out/stamps4_$B.log 2>&1 || { cat gpurun_out/stamps4_$B.log; exit 1; }
  head -12 gpurun_out/stamps4_$B.log
done
for B in 128 256 512 1024; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --batch $B > gpurun_out/shard_$B.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/shard_$B.json').read().strip().splitlines()[-1]); print('B=$B', round(d['value']), 'ms/step %.4f' % d['ms_per_step'], d['phase_ms_per_step'])"
done
