#!/bin/bash
# Round 4: polishing build with the grouped kernel off -- smoke, the headline-kernel oracle test,
# polishing diagnostics, then a same-box A/B (polishing on / off) on the metric config.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/e_smoke.log 2>&1 || { tail -30 gpurun_out/e_smoke.log; exit 1; }
tail -1 gpurun_out/e_smoke.log
timeout -k 10 300 python -u scripts/dump_headline.py > gpurun_out/e_dump.log 2>&1 || { tail -30 gpurun_out/e_dump.log; exit 1; }
cat gpurun_out/e_dump.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 250 --timeout-method thread > gpurun_out/e_headline.log 2>&1 || { tail -40 gpurun_out/e_headline.log; exit 1; }
tail -3 gpurun_out/e_headline.log
timeout -k 10 300 python -u scripts/diag_polish.py > gpurun_out/e_polish.log 2>&1 || { tail -30 gpurun_out/e_polish.log; exit 1; }
cat gpurun_out/e_polish.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/e_bench_pol$i.json 2> gpurun_out/e_bench_pol$i.err || { tail -20 gpurun_out/e_bench_pol$i.err; exit 1; }
  CMPC_QP_POLISH_EPS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/e_bench_off$i.json 2> gpurun_out/e_bench_off$i.err || { tail -20 gpurun_out/e_bench_off$i.err; exit 1; }
done
python - <<'PY'
import json
for t in ('pol1', 'off1', 'pol2', 'off2'):
    d = json.load(open('gpurun_out/e_bench_%s.json' % t))
    print(t, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'ms/step %.3f' % d['ms_per_step'],
          'newton %.3f' % d['qp_ipm_iterations_mean'], d['qp_exit'], d['roofline']['kernel'], 'frac %.3f' % d['roofline']['frac'])
PY
