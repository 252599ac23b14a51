"""Summarize rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, separate runs) into per-launch HBM
bytes of the QP kernel -> profiles/qp_pmc_traffic.json (read by bench.py's roofline.traffic).

FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 reports half the bytes of wide reads);
both counters are in KB.  Usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> [out]
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')


def per_kernel(d, counter, skip=0):
    """{kernel: (sum of the counter, dispatches)} over each kernel's dispatches after its first
    `skip` (the warm-up launches, in dispatch order)."""
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != counter:
            continue
        name = r['Kernel_Name'].split('(')[0]
        per[name][int(r['Dispatch_Id'])] += float(r['Counter_Value'])
    out = {}
    for k, disp in per.items():
        ids = sorted(disp)
        ids = ids[skip:] if len(ids) > skip else ids
        out[k] = (sum(disp[i] for i in ids), len(ids))
    return out


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), '..', 'profiles',
                                                              'qp_pmc_traffic.json')
    skip = int(os.environ.get('PMC_SKIP', '2'))   # warm-up launches of the profiled bench run
    fe, wr = per_kernel(fdir, 'FETCH_SIZE', skip), per_kernel(wdir, 'WRITE_SIZE', skip)
    # the QP launch: its kernels (split launches: k_qp_split, the head and the tail k_qp_ipm; grouped:
    # k_qp_order and k_qp_group), each averaged over its dispatches and summed
    qks = sorted(k for k in fe if any(t in k for t in ('k_qp_ipm', 'k_qp_group', 'k_qp_split', 'k_qp_order')))
    qp = ' + '.join(qks)
    fkb = sum(fe[k][0] / fe[k][1] for k in qks); fn = min(fe[k][1] for k in qks)
    wkb = sum(wr[k][0] / wr[k][1] for k in qks if k in wr); wn = min(wr[k][1] for k in qks if k in wr)
    per_launch = (2.0 * fkb + wkb) * 1024.0
    lib = os.path.join(ROOT, 'centroidal-mpc_amd', 'cmpc', 'libcmpc.so')
    res = {'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)',
           'command': os.environ.get('PMC_BENCH_CMD', '?'),
           'head': os.environ.get('CMPC_HEAD', '?'),
           'lib_sha16': hashlib.sha256(open(lib, 'rb').read()).hexdigest()[:16] if os.path.exists(lib) else None,
           'note': 'average over the QP dispatches of the run; with --warmup >= 2 the dispatches measured '
                   'group problems by the previous launch\'s Newton counts (the timed steady state)',
           'skipped_warmup_dispatches': skip,
           'kernel': qp, 'dispatches': {'FETCH_SIZE': fn, 'WRITE_SIZE': wn},
           'fetch_size_kb_per_launch': fkb, 'write_size_kb_per_launch': wkb,
           'correction': 'FETCH_SIZE x2 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half of the bytes of wide '
                         'reads); counters in KB',
           'hbm_bytes_per_launch': per_launch,
           'per_kernel_kb_per_launch': {c: {k: v[0] / v[1] for k, v in d.items()} for c, d in
                                        (('FETCH_SIZE', fe), ('WRITE_SIZE', wr))}}
    json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps({'kernel': qp, 'hbm_bytes_per_launch': per_launch}))


if __name__ == '__main__':
    main()
