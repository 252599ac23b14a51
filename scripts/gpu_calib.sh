#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/calib/fetch_calib.hip) and the counter list of gfx950.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || { tail -5 gpurun_out/counters_list.txt; }
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d gpurun_out/calib_$C -o pmc -- ./scripts/calib/fetch_calib > gpurun_out/calib_$C.log 2>&1 || { tail -20 gpurun_out/calib_$C.log; exit 1; }
done
cat gpurun_out/calib_FETCH_SIZE.log
for C in FETCH_SIZE WRITE_SIZE; do f=$(find gpurun_out/calib_$C -name '*counter_collection.csv' | head -1); python3 - "$f" "$C" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if r['Counter_Name'] == sys.argv[2]:
        tot[r['Kernel_Name'].split('(')[0]] += float(r['Counter_Value'])
for k, v in tot.items():
    print(sys.argv[2], k, '%.0f KB = %.4f GiB' % (v, v * 1024 / 2**30))
PY
done
grep -E "SQ_VALU_MFMA|SQ_WAIT_ANY|SQ_WAVE_CYCLES|SQ_BUSY_CYCLES|SQ_ACTIVE_INST|SQ_INSTS_VALU_MFMA|GRBM_GUI_ACTIVE|SQ_WAVES\b|SQ_INSTS_LDS|SQ_LDS_BANK|MFMA_MOPS|SQ_INST_CYCLES_VMEM|SQ_INSTS_VMEM" gpurun_out/counters_list.txt | head -60
