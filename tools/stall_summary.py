#!/usr/bin/env python3
"""Summarise the stall-attribution passes (tools/gpu_runs/r06/call2.sh) of the path
kernel per config into profiles/<round>_stalls_<cfg>.json: instruction counts per
sample by kind (VMEM, SMEM, LDS, SALU), their average latencies (rocprofv3's
VmemLatency / SmemLatency / LdsLatency: in-flight level accumulated per cycle /
instructions, in cycles), and the active-issue cycles of each kind per wave cycle.
usage: stall_summary.py <pass dir> <round> [samples-per-launch scale=1/4 of the rows]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, rnd = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAMPLES = {'C2': 1280 * 720 * 512, 'C3': 1280 * 720 * 512, 'C4': 1280 * 720 * 256, 'C5': 1280 * 720 * 1024,
           'C2g': 1280 * 720 * 512}
sha = None
if os.path.exists(os.path.join(src, 'lib.sha256')):
    sha = open(os.path.join(src, 'lib.sha256')).read().split()[0]


def counters(d):
    acc = defaultdict(float)
    n = defaultdict(set)
    durs = {}
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'path_kernel' in r['Kernel_Name']:
                durs[r['Dispatch_Id']] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'path_kernel' in r['Kernel_Name'] and r['Kernel_Name'].startswith('void path_kernel<false'):
                acc[r['Counter_Name']] += float(r['Counter_Value'])
                n[r['Counter_Name']].add(r['Dispatch_Id'])
                kname = r['Kernel_Name']
    return acc, n, durs


for cfg in ('C2', 'C3', 'C4', 'C5', 'C2g'):
    a, na, da = counters(os.path.join(src, 'stall_%s_A' % cfg))
    b, nb, db = counters(os.path.join(src, 'stall_%s_B' % cfg))
    c, nc, dc = counters(os.path.join(src, 'stall_%s_C' % cfg))
    if not a or not b or not c:
        continue
    smp = SAMPLES[cfg] / 4.0   # prof_run.py <cfg> 1 4: a quarter of the rows, one launch
    launches = len(next(iter(na.values())))
    per = lambda v: v / launches / smp
    t = sum(da.values()) / max(1, len(da)) * 1e-9
    clk = a['GRBM_GUI_ACTIVE'] / launches / 8 / t
    wc = b['SQ_WAVE_CYCLES'] / len(next(iter(nb.values())))
    out = {
        'config': cfg, 'kernel': 'path_kernel<false, ...> (bench instantiation)', 'lib_sha256': sha,
        'rows': '1/4 (tools/prof_run.py %s 1 4)' % cfg, 'clock_ghz': round(clk / 1e9, 3),
        'per_sample': {'vmem_insts': round(per(a['SQ_INSTS_VMEM']), 2), 'smem_insts': round(per(a['SQ_INSTS_SMEM']), 2),
                       'lds_insts': round(per(a['SQ_INSTS_LDS']), 2), 'salu_insts': round(per(a['SQ_INSTS_SALU']), 2)},
        'latency_cycles': {'vmem': round(b.get('VmemLatency', 0) / len(nb.get('VmemLatency', [1])), 1),
                           'smem': round(c.get('SmemLatency', 0) / len(nc.get('SmemLatency', [1])), 1),
                           'lds': round(c.get('LdsLatency', 0) / len(nc.get('LdsLatency', [1])), 1)},
        # SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES count quad-cycles (MI355X_MICROARCH.md)
        'active_frac_of_wave_cycles': {'vmem': round(a['SQ_ACTIVE_INST_VMEM'] / launches / wc, 4),
                                       'lds': round(a['SQ_ACTIVE_INST_LDS'] / launches / wc, 4),
                                       'scalar': round(a['SQ_ACTIVE_INST_SCA'] / launches / wc, 4)},
        'wait_inst_lds_frac_of_wave_cycles': round(a['SQ_WAIT_INST_LDS'] / launches / wc, 4),
        'note': 'SQ pass A: INSTS_VMEM/SMEM/LDS/SALU, WAIT_INST_LDS, ACTIVE_INST_VMEM/LDS/SCA; pass B: VmemLatency + '
                'SQ_WAVE_CYCLES; pass C: SmemLatency + LdsLatency (derived: accumulated in-flight level / instructions)',
    }
    json.dump(out, open(os.path.join(REPO, 'profiles', '%s_stalls_%s.json' % (rnd, cfg)), 'w'), indent=1)
    print(json.dumps(out))
