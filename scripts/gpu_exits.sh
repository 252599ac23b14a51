set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/qp_exits.py talos 200 512 2 > gpurun_out/ex_talos.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py trot 100 1024 1 > gpurun_out/ex_trot.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py bound 100 1024 1 fp32 > gpurun_out/ex_bound32.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py mixed 150 1024 1 > gpurun_out/ex_mixed.log 2>&1
grep -h "^iter" gpurun_out/ex_*.log
