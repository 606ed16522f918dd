#!/usr/bin/env python3
"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks (one row per
kernel / noinline function): VGPRs, AGPRs, scratch bytes per lane, occupancy,
VGPR/SGPR spills.  usage: resource_table.py [resource.txt]"""
import re
import subprocess
import sys

path = sys.argv[1] if len(sys.argv) > 1 else 'mitsuba0.6_amd/_build/path_kernel.resource.txt'
rows, cur = [], None
for line in open(path):
    m = re.search(r'remark: (.+?): (.*?) \[-Rpass', line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2).strip()
    if key == 'Function Name':
        cur = {'name': val}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
names = [r['name'] for r in rows]
try:
    dem = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True).stdout.split('\n')
except OSError:
    dem = names
print('%-60s %5s %5s %7s %4s %6s %6s' % ('function', 'VGPR', 'AGPR', 'scratch', 'occ', 'vspill', 'sspill'))
for r, d in zip(rows, dem):
    d = d.replace('(MtsgLaunch)', '')
    print('%-60s %5s %5s %7s %4s %6s %6s' % (d[:60], r.get('VGPRs', '?'), r.get('AGPRs', '?'),
          r.get('ScratchSize [bytes/lane]', '?'), r.get('Occupancy [waves/SIMD]', '?'),
          r.get('VGPRs Spill', '?'), r.get('SGPRs Spill', '?')))
