#!/bin/bash
# GPU profiling session (one round's evidence for profiles/):
#   smoke -> rocprofv3 kernel trace/stats of the bench -> PMC passes, one counter group per run
#   (FETCH_SIZE, WRITE_SIZE, SQ timing/MFMA group, SQ LDS/VMEM group; kernel-trace only) on the
#   metric config and the HBM passes on BASELINE C5 -> summaries -> default bench line (CPU baseline).
# Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
# PMC passes on the steady state: two warm-up launches first, so the profiled QP dispatches group
# problems by real Newton counts as the timed steps do (the first launch orders by index); only
# the dispatches after the warm-up are averaged (pmc_traffic.py skips the first W of each kernel)
export PMC_BENCH_CMD="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extras"
export CMPC_HEAD=${CMPC_HEAD:-?}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/prof_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_bench_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_bench_$TAG.log
pmc() {   # pmc <name> <counters> <bench args>
    local name=$1 ctr=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${TAG}_$name -o pmc -- \
        python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extras "$@" > gpurun_out/pmc_bench_${TAG}_$name.log 2>&1 \
        || { tail -20 gpurun_out/pmc_bench_${TAG}_$name.log; return 1; }
}
pmc FETCH_SIZE FETCH_SIZE || exit 1
pmc WRITE_SIZE WRITE_SIZE || exit 1
pmc SQ_A "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
pmc SQ_B "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE" || exit 1
pmc C5_FETCH_SIZE FETCH_SIZE --config mixed --N 150 || exit 1
pmc C5_WRITE_SIZE WRITE_SIZE --config mixed --N 150 || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE gpurun_out/qp_pmc_traffic_$TAG.json || exit 1
python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_C5_FETCH_SIZE gpurun_out/pmc_${TAG}_C5_WRITE_SIZE gpurun_out/qp_pmc_traffic_c5_$TAG.json || exit 1
python3 scripts/pmc_counters.py gpurun_out/pmc_${TAG}_SQ_A gpurun_out/pmc_${TAG}_SQ_B > gpurun_out/pmc_counters_$TAG.json || exit 1
cat gpurun_out/pmc_counters_$TAG.json
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
