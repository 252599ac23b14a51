"""Summarize rocprofv3 SQ/GRBM PMC passes into per-dispatch averages and derived ratios for the hot
kernels (k_qp_ipm, k_linearize, k_accept, k_assemble).  Usage: python pmc_counters.py <dir> [<dir> ...]

Derived (MI355X_MICROARCH.md units: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES in cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs):
  clock_ghz          GRBM_GUI_ACTIVE / 8 / kernel duration
  mfma_busy_pct      SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  f64_mfma_tflops    SQ_INSTS_VALU_MFMA_MOPS_F64 * 512 / duration, against the 78.6 TFLOP/s fp64 matrix peak
  wait_pct / issue_stall_pct / active_pct   SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  lds_bank_conflict_pct   SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ('k_qp_group', 'k_qp_ipm', 'k_linearize', 'k_accept', 'k_assemble')
F64_MATRIX_PEAK_TFLOPS = 78.6


def load(d):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = {}
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].split('(')[0].split('<')[0].split('::')[-1]
        if name not in KERNELS:
            continue
        vals[name][r['Counter_Name']] += float(r['Counter_Value'])
        disp[name].add(r['Dispatch_Id'])
        if 'End_Timestamp' in r and r.get('Start_Timestamp'):
            dur[(name, r['Dispatch_Id'])] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
    out = {}
    for k in vals:
        n = len(disp[k])
        d_s = [v for (kk, _), v in dur.items() if kk == k]
        out[k] = dict(dispatches=n, **{c: v / n for c, v in vals[k].items()})
        if d_s:
            out[k]['duration_s'] = sum(d_s) / len(d_s)
    return out


def main():
    res = collections.defaultdict(dict)
    for d in sys.argv[1:]:
        for k, v in load(d).items():
            res[k].update(v)
    for k, v in res.items():
        der = {}
        g = v.get('GRBM_GUI_ACTIVE')
        t = v.get('duration_s')
        if g and t:
            der['clock_ghz'] = g / 8 / t / 1e9
        if g and 'SQ_VALU_MFMA_BUSY_CYCLES' in v:
            der['mfma_busy_pct'] = 100 * v['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024)
        if t and 'SQ_INSTS_VALU_MFMA_MOPS_F64' in v:
            tf = v['SQ_INSTS_VALU_MFMA_MOPS_F64'] * 512 / t / 1e12
            der['f64_mfma_tflops'] = tf
            der['f64_mfma_frac_of_peak'] = tf / F64_MATRIX_PEAK_TFLOPS
        wc = v.get('SQ_WAVE_CYCLES')
        if wc:
            for c, nm in (('SQ_WAIT_ANY', 'wait_pct'), ('SQ_WAIT_INST_ANY', 'issue_stall_pct'),
                          ('SQ_ACTIVE_INST_ANY', 'active_pct'), ('SQ_ACTIVE_INST_VALU', 'valu_active_pct')):
                if c in v:
                    der[nm] = 100 * v[c] / wc
        if v.get('SQ_ACTIVE_INST_LDS'):
            der['lds_bank_conflict_pct'] = 100 * v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_ACTIVE_INST_LDS']
        if v.get('SQ_WAVES') and g and t:
            der['waves_per_dispatch'] = v['SQ_WAVES']
        v['derived'] = der
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
