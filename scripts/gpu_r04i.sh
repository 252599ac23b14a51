#!/bin/bash
# Round 4: BASELINE C4 (TALOS N=200 x 512) polishing-tolerance sweep, same box.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for pe in 1e-7 1e-8 1e-9 0; do
  CMPC_QP_POLISH_EPS=$pe timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 10 --warmup 3 --config talos --N 200 --batch 512 > gpurun_out/i_c4_$pe.json 2> gpurun_out/i_c4_$pe.err || { tail -20 gpurun_out/i_c4_$pe.err; exit 1; }
done
for pe in 1e-7 1e-8 0; do
  CMPC_QP_POLISH_EPS=$pe timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/i_m_$pe.json 2> gpurun_out/i_m_$pe.err || { tail -20 gpurun_out/i_m_$pe.err; exit 1; }
done
python - <<'PY'
import json
for tag in ('c4_1e-7', 'c4_1e-8', 'c4_1e-9', 'c4_0', 'm_1e-7', 'm_1e-8', 'm_0'):
    d = json.load(open('gpurun_out/i_%s.json' % tag))
    print(tag, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'newton %.3f' % d['qp_ipm_iterations_mean'],
          d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected'], d['roofline']['kernel'])
PY
