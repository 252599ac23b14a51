set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for B in 256 512 1024 2048; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bs_$B -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --batch $B > gpurun_out/bs_$B.log 2>&1 || exit 1
done
