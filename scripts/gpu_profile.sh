#!/bin/bash
# GPU session: smoke -> rocprofv3 kernel trace/stats of the bench -> PMC passes (FETCH_SIZE and
# WRITE_SIZE separately; kernel-trace only) -> traffic summary -> default bench line with the CPU
# baseline.  Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r01}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_bench_$TAG.log; exit 1; }
tail -1 gpurun_out/prof_bench_$TAG.log
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${TAG}_$C -o pmc -- \
        python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_bench_${TAG}_$C.log 2>&1 || { tail -20 gpurun_out/pmc_bench_${TAG}_$C.log; exit 1; }
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE gpurun_out/qp_pmc_traffic_$TAG.json || exit 1
cp gpurun_out/qp_pmc_traffic_$TAG.json profiles/qp_pmc_traffic.json
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
