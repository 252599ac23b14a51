#!/bin/bash
# Round 4: headline dump (sampled QPs + exits), same-box A/B of the split launches and the configs'
# QP diagnostics on the current build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/dump_headline.py > gpurun_out/g_dump.log 2>&1 || { tail -30 gpurun_out/g_dump.log; exit 1; }
cat gpurun_out/g_dump.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/g_bench_on$i.json 2> gpurun_out/g_bench_on$i.err || { tail -20 gpurun_out/g_bench_on$i.err; exit 1; }
  CMPC_QP_SPLIT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/g_bench_off$i.json 2> gpurun_out/g_bench_off$i.err || { tail -20 gpurun_out/g_bench_off$i.err; exit 1; }
done
python - <<'PY'
import json
for t in ('on1', 'off1', 'on2', 'off2'):
    d = json.load(open('gpurun_out/g_bench_%s.json' % t))
    print(t, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'ms/step %.3f' % d['ms_per_step'],
          'newton %.3f' % d['qp_ipm_iterations_mean'], d['qp_exit'], d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'])
PY
timeout -k 10 300 python -u scripts/diag_polish.py > gpurun_out/g_polish.log 2>&1 || { tail -30 gpurun_out/g_polish.log; exit 1; }
cat gpurun_out/g_polish.log
