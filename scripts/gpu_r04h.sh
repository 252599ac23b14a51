#!/bin/bash
# Round 4: split launches with two-wave heads -- split tests, C4 (TALOS N=200 x 512) A/B, metric bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_qp_split.py -x -v --timeout 200 --timeout-method thread > gpurun_out/h_split.log 2>&1 || { tail -40 gpurun_out/h_split.log; exit 1; }
tail -3 gpurun_out/h_split.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 --config talos --N 200 --batch 512 > gpurun_out/h_c4_on$i.json 2> gpurun_out/h_c4_on$i.err || { tail -20 gpurun_out/h_c4_on$i.err; exit 1; }
  CMPC_QP_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 --config talos --N 200 --batch 512 > gpurun_out/h_c4_off$i.json 2> gpurun_out/h_c4_off$i.err || { tail -20 gpurun_out/h_c4_off$i.err; exit 1; }
done
python - <<'PY'
import json
for t in ('on1', 'off1', 'on2', 'off2'):
    d = json.load(open('gpurun_out/h_c4_%s.json' % t))
    print('C4', t, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'ms/step %.3f' % d['ms_per_step'],
          'newton %.3f' % d['qp_ipm_iterations_mean'], d['qp_exit'], d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'])
PY
