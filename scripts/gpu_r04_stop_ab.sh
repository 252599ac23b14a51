#!/bin/bash
# Round 4: same-box A/B of the stopping test -- the shipped one (Solo12: complementarity against the
# primal scale at 1e-9) against round 3's (dual scale at 1e-10, diagnostic build libcmpc_cd.so),
# both with polishing, on the metric config, C2 and C5; then the fp32 C3 line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() {  # tag, env..., -- bench args
    local tag=$1; shift
    timeout -k 10 300 env "$@" > gpurun_out/s_$tag.json 2> gpurun_out/s_$tag.err || { tail -20 gpurun_out/s_$tag.err; exit 1; }
}
for i in 1 2; do
  run m_new$i python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5
  run m_old$i CMPC_LIB_VARIANT=cd CMPC_QP_EPS=1e-10 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5
done
run c5_new python3 bench.py --no-cpu-baseline --no-extras --config mixed --N 150 --batch 1024
run c5_old CMPC_LIB_VARIANT=cd CMPC_QP_EPS=1e-10 python3 bench.py --no-cpu-baseline --no-extras --config mixed --N 150 --batch 1024
run c2_new python3 bench.py --no-cpu-baseline --no-extras --config trot --N 100 --batch 256
run c2_old CMPC_LIB_VARIANT=cd CMPC_QP_EPS=1e-10 python3 bench.py --no-cpu-baseline --no-extras --config trot --N 100 --batch 256
run c3 python3 bench.py --no-cpu-baseline --no-extras --config bound --N 100 --batch 1024 --precision fp32
python3 - <<'PY'
import json
for t in ('m_new1', 'm_old1', 'm_new2', 'm_old2', 'c5_new', 'c5_old', 'c2_new', 'c2_old', 'c3'):
    d = json.load(open('gpurun_out/s_%s.json' % t))
    print(t, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'newton %.3f' % d['qp_ipm_iterations_mean'],
          'pol +%d -%d' % (d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected']), d['roofline']['kernel'])
PY
