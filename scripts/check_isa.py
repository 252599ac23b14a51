"""Static checks on the QP kernels' device assembly (hipcc --offload-device-only -S qp_ipm.hip):
no flat memory instruction anywhere (every pointer is global- or LDS-qualified; an outlined phase
taking Ctx by reference once did all its accesses through flat pointers to the caller's scratch and
faulted, see qp_ipm.hip PHASE_ATTR), and per kernel the outlined callees and scratch bytes per lane.
Usage: python scripts/check_isa.py qp_ipm.s"""
import re
import sys

txt = open(sys.argv[1]).read()
flat = re.findall(r'\n\s+(flat_\w+)', txt)
print('flat memory instructions:', len(flat))
for m in re.finditer(r'\n\t\.set (_ZN4cmpc\w*k_qp_\w+)\.private_seg_size, (\d+)\+max\(([^)]*)\)', txt):
    callees = sorted(set(re.sub(r'^\.L_ZN4cmpc\d+', '', c.strip()).split('.')[0][:28] for c in m.group(3).split(',')))
    print(m.group(1)[9:60], 'own scratch', m.group(2), 'callees', callees)
sys.exit(1 if flat else 0)
