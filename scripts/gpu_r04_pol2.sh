#!/bin/bash
# Round 4: polishing tolerance on the metric (split) and C2 (four waves per problem, no split).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for pe in 1e-7 3e-8 1e-8 1e-6; do
  CMPC_QP_POLISH_EPS=$pe timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > gpurun_out/p2_m_$pe.json 2>/dev/null || exit 1
  CMPC_QP_POLISH_EPS=$pe timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --config trot --N 100 --batch 256 > gpurun_out/p2_c2_$pe.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for pe in ('1e-7', '3e-8', '1e-8', '1e-6'):
    for c in ('m', 'c2'):
        d = json.load(open('gpurun_out/p2_%s_%s.json' % (c, pe)))
        print(c, pe, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'newton %.3f' % d['qp_ipm_iterations_mean'],
              'pol +%d -%d' % (d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected']))
PY
