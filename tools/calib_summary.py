#!/usr/bin/env python3
"""Summarise the VALU calibration (tools/valu_calib.hip: pure v_fma_f32 / packed
v_pk_* chains at 1-8 waves/SIMD, its plain timing log and one rocprofv3 SQ pass)
into profiles/<round>_valu_calib.json, the peak bench.py's valu roofline is
measured against.  Per launch: SIMD-cycles per wave VALU instruction (1024 SIMDs x
the pass's clock x kernel time / SQ_INSTS_VALU), VALU-busy (4 x
SQ_ACTIVE_INST_VALU / SIMD-cycles: SQ_ACTIVE_* count quad-cycles) and the f32
lane-operation rate.
usage: calib_summary.py <pass dir (valu_calib.log + calib_SQ/)> <round>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, rnd = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
plain = [json.loads(l) for l in open(os.path.join(src, 'valu_calib.log')) if l.startswith('{')]
acc = defaultdict(lambda: defaultdict(float))
names = {}
for f in glob.glob(os.path.join(src, 'calib_SQ', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
        names[r['Dispatch_Id']] = r['Kernel_Name'].split('(')[0].replace('void ', '')
dur = {}
for f in glob.glob(os.path.join(src, 'calib_SQ', '**', '*kernel_trace.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
launches = []
# each kernel runs a warm-up launch (1/8 of the iterations) and the measured one: keep the longer
longest = {}
for did in acc:
    if names[did] not in longest or dur[did] > dur[longest[names[did]]]:
        longest[names[did]] = did
for did in sorted(longest.values(), key=int):
    c, t = acc[did], dur[did]
    clk = c['GRBM_GUI_ACTIVE'] / 8 / t
    simd_cycles = 1024 * clk * t
    k = names[did]
    packed = 'valu_calib_pk' in k
    launches.append({'kernel': k, 'kernel_s': round(t, 5), 'clock_ghz': round(clk / 1e9, 4),
                     'waves_per_simd': int(k.split('<')[1].split(',')[0].rstrip('>')),
                     'simd_cycles_per_wave_valu_inst': round(simd_cycles / c['SQ_INSTS_VALU'], 4),
                     'valu_busy_per_simd': round(4 * c['SQ_ACTIVE_INST_VALU'] / simd_cycles, 4),
                     'f32_lane_ops_per_simd_cycle': round(c['SQ_INSTS_VALU'] * 64 * (2 if packed else 1) / simd_cycles, 3),
                     'active_inst_valu_per_inst': round(c['SQ_ACTIVE_INST_VALU'] / c['SQ_INSTS_VALU'], 4)})
scalar = [l for l in launches if 'valu_calib_pk' not in l['kernel']]
best = min(scalar, key=lambda l: l['simd_cycles_per_wave_valu_inst'])
out = {'round': rnd, 'source': 'tools/valu_calib.hip (rocprofv3 SQ pass + plain timing)', 'launches': launches,
       'plain_timing': plain,
       'peak': {'simd_cycles_per_wave_valu_inst': best['simd_cycles_per_wave_valu_inst'],
                'valu_busy_per_simd': best['valu_busy_per_simd'], 'waves_per_simd': best['waves_per_simd'],
                'kernel': best['kernel']},
       'note': 'independent v_fma_f32 chains saturate at ~4.2 SIMD-cycles per wave64 VALU instruction (VALU-busy '
               '~0.95), not the 2 cycles MI355X_MICROARCH.md lists; v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 '
               'issue at the same instruction rate, so the 157 TF f32 spec (32 lane-FMA / SIMD / cycle) needs packed '
               'instructions: unpacked f32 code tops out at half of it'}
json.dump(out, open(os.path.join(REPO, 'profiles', '%s_valu_calib.json' % rnd), 'w'), indent=1)
print(json.dumps(out['peak']))
for l in launches:
    print(l)
