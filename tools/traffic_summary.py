#!/usr/bin/env python3
"""Summarise a prof_round.sh output directory into profiles/<round>_*.

For each config: the path kernel's per-launch FETCH_SIZE / WRITE_SIZE (KiB, as
rocprofv3 reports them) and HBM bytes corrected per MI355X_MICROARCH.md: on
gfx950 FETCH_SIZE counts half the bytes of wide reads (x2), WRITE_SIZE is
exact.  Writes profiles/<round>_traffic_<cfg>.json and copies the kernel
stats CSVs of the bench runs.  From the SQ pass, profiles/<round>_valu_<cfg>.json:
the wave-cycle budget (SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_ANY +
WAIT_INST_ANY, MI355X_MICROARCH.md "rocprofv3 PMC slots"), the VALU issue
fraction per wave, and VALU-busy per SIMD = 4 x ACTIVE_INST_VALU (quad-cycles)
/ (SIMDs x GRBM_GUI_ACTIVE / 8): rocprofv3 sums GRBM_GUI_ACTIVE over the 8
XCDs (it reads 8x the dispatch's duration in shader cycles)."""
import csv
import glob
import json
import os
import shutil
import sys

src, rnd = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(REPO, 'profiles')
# sha256 of the libmtsgpu.so the passes ran (prof_round.sh): bench.py drops profiles of other builds
_sha = os.path.join(src, 'lib.sha256')
LIB_SHA = open(_sha).read().split()[0] if os.path.exists(_sha) else None


def counter(path_glob, name):
    vals = []
    for f in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == name and 'path_kernel' in r['Kernel_Name']:
                vals.append(float(r['Counter_Value']))
    return vals


# samples per profiled launch (one full frame = one launch; C5's 1024 spp fit one splat buffer since r03)
SAMPLES = {'C2': 1280 * 720 * 512, 'C3': 1280 * 720 * 512, 'C4': 1280 * 720 * 256, 'C5': 1280 * 720 * 1024,
           'C2g': 1280 * 720 * 512}

for cfg in ('C2', 'C3', 'C4', 'C5', 'C2g'):
    fetch = counter(os.path.join(src, 'pmc_%s_FETCH_SIZE' % cfg, '**', '*counter_collection.csv'), 'FETCH_SIZE')
    write = counter(os.path.join(src, 'pmc_%s_WRITE_SIZE' % cfg, '**', '*counter_collection.csv'), 'WRITE_SIZE')
    if fetch and write:
        f, w = sum(fetch) / len(fetch), sum(write) / len(write)
        samples = SAMPLES.get(cfg)
        out = {'config': cfg, 'kernel': 'path_kernel', 'lib_sha256': LIB_SHA, 'launches': len(fetch), 'FETCH_SIZE_KiB': f, 'WRITE_SIZE_KiB': w,
               'hbm_bytes_per_launch': 2 * f * 1024 + w * 1024,
               'hbm_bytes_per_launch_fetch_raw': f * 1024 + w * 1024,
               'hbm_bytes_per_sample': (2 * f * 1024 + w * 1024) / samples if samples else None,
               'write_bytes_per_sample': w * 1024 / samples if samples else None,
               'read_bytes_per_sample_raw': f * 1024 / samples if samples else None,
               'note': 'one full frame (tools/prof_run.py %s 1 1). hbm_bytes_per_launch doubles FETCH_SIZE '
                       '(MI355X_MICROARCH.md: gfx950 counts half of 16 B/lane streaming reads), an upper bound '
                       'for the scattered node/triangle reads whose width is uncalibrated; '
                       'hbm_bytes_per_launch_fetch_raw is the undoubled lower bound. WRITE_SIZE as reported '
                       '(exact for 16 B/lane stores and float atomics)' % cfg}
        json.dump(out, open(os.path.join(prof, '%s_traffic_%s.json' % (rnd, cfg)), 'w'), indent=1)
        print(cfg, out)
    for f in glob.glob(os.path.join(src, 'bench_%s' % cfg, '**', '*kernel_stats.csv'), recursive=True):
        shutil.copy(f, os.path.join(prof, '%s_bench_%s_kernel_stats.csv' % (rnd, cfg)))
        print('copied', f)
    log = os.path.join(src, 'bench_%s.log' % cfg)
    if os.path.exists(log):
        shutil.copy(log, os.path.join(prof, '%s_bench_%s.log' % (rnd, cfg)))

SIMDS, XCDS = 256 * 4, 8
for cfg in ('C2', 'C3', 'C4', 'C5', 'C2g'):
    base = os.path.join(src, 'pmc_%s_SQ' % cfg, '**', '*counter_collection.csv')
    names = ['SQ_WAVES', 'SQ_WAVE_CYCLES', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_ANY',
             'SQ_WAIT_INST_ANY', 'SQ_INSTS_VALU', 'SQ_BUSY_CYCLES', 'GRBM_GUI_ACTIVE']
    v = {n: counter(base, n) for n in names}
    if not all(v.values()):
        continue
    c = {n: sum(x) / len(x) for n, x in v.items()}
    wc = c['SQ_WAVE_CYCLES']
    # the pass's kernel durations (its --kernel-trace) give the shader clock:
    # GRBM_GUI_ACTIVE / 8 XCDs cycles over the dispatch's duration
    durs = []
    for f in glob.glob(os.path.join(src, 'pmc_%s_SQ' % cfg, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'path_kernel' in r['Kernel_Name']:
                durs.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
    pass_samples = SAMPLES[cfg] // 4          # tools/prof_run.py <cfg> 1 4: a quarter of the rows
    out = {'config': cfg, 'kernel': 'path_kernel', 'lib_sha256': LIB_SHA, 'counters': c,
           'valu_busy_per_simd': 4 * c['SQ_ACTIVE_INST_VALU'] / (SIMDS * c['GRBM_GUI_ACTIVE'] / XCDS),
           'valu_issue_frac_per_wave': c['SQ_ACTIVE_INST_VALU'] / wc,
           'any_issue_frac_per_wave': c['SQ_ACTIVE_INST_ANY'] / wc,
           'wait_frac_per_wave': c['SQ_WAIT_ANY'] / wc,
           'issue_stall_frac_per_wave': c['SQ_WAIT_INST_ANY'] / wc,
           'valu_insts_per_wave': c['SQ_INSTS_VALU'] / max(1.0, c['SQ_WAVES']),
           'valu_insts_per_sample': c['SQ_INSTS_VALU'] / pass_samples,
           'valu_busy_cycles_per_sample': 4 * c['SQ_ACTIVE_INST_VALU'] / pass_samples,
           'kernel_s': sum(durs) / len(durs) if durs else None,
           'clock_hz': c['GRBM_GUI_ACTIVE'] / XCDS / (sum(durs) / len(durs)) if durs else None,
           'note': '1/4 of the rows (tools/prof_run.py %s 1 4); SQ cycle counters in quad-cycles' % cfg}
    json.dump(out, open(os.path.join(prof, '%s_valu_%s.json' % (rnd, cfg)), 'w'), indent=1)
    print(cfg, {k: out[k] for k in out if k.endswith('frac_per_wave') or k.startswith('valu_busy')})
