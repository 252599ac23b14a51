#!/bin/bash
# Round 4: split-launch tail shape A/B (host-side knobs only: CMPC_QP_TAIL_WAVES, CMPC_QP_SPLIT_CAP)
# on the metric config and BASELINE C5, same box, A B A B order for the default.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
run() {   # run <tag> <env...> -- <bench args>
    local tag=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 ${ARGS} > gpurun_out/tab_$tag.json 2> gpurun_out/tab_$tag.err \
        || { tail -5 gpurun_out/tab_$tag.err; return 1; }
}
ARGS="" run m_def0 X=0 || exit 1
ARGS="" run m_t2 CMPC_QP_TAIL_WAVES=2 || exit 1
ARGS="" run m_c192 CMPC_QP_SPLIT_CAP=192 || exit 1
ARGS="" run m_def1 X=0 || exit 1
ARGS="" run m_c128 CMPC_QP_SPLIT_CAP=128 || exit 1
ARGS="" run m_t2c384 CMPC_QP_TAIL_WAVES=2 CMPC_QP_SPLIT_CAP=384 || exit 1
ARGS="--config mixed --N 150" run c5_def X=0 || exit 1
ARGS="--config mixed --N 150" run c5_t2 CMPC_QP_TAIL_WAVES=2 || exit 1
ARGS="--config mixed --N 150" run c5_c192 CMPC_QP_SPLIT_CAP=192 || exit 1
python3 - <<'PY'
import json
for t in ('m_def0', 'm_t2', 'm_c192', 'm_def1', 'm_c128', 'm_t2c384', 'c5_def', 'c5_t2', 'c5_c192'):
    d = json.load(open('gpurun_out/tab_%s.json' % t))
    print(t, round(d['value']), d['roofline']['kernel'], 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'],
          'newton %.3f' % d['qp_ipm_iterations_mean'], 'status', d['qp_exit']['status_counts'],
          'merit %.3f' % d['qp_exit']['merit_max'], 'pol +%d -%d' % (d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected']))
PY
