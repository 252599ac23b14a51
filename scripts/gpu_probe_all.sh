#!/bin/bash
# developer probe across configs (each step time-limited)
mkdir -p gpurun_out
for args in "trot 30 3 fp64" "talos 50 2 fp64" "bound 50 2 fp64" "trot 50 2 fp32"; do
  echo "=== $args"
  timeout -k 10 240 python3 scripts/gpu_probe.py $args || { echo "FAILED rc=$?"; exit 1; }
done
