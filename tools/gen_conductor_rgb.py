#!/usr/bin/env python3
"""Generate mitsuba0.6_amd/data/conductor_rgb.json: the RGB complex IOR the
reference's roughconductor derives for `material="<name>"` (roughconductor.cpp:
172-190: InterpolatedSpectrum(data/ior/<name>.{eta,k}.spd) -> Spectrum::
fromContinuousSpectrum, RGB build).

Dev-time only (reads /root/reference; runs in the survey container).  The CIE
1931 tables and the .spd samples are read as numbers; tools/spectrum_rgb.c
restates the conversion in single precision.  The committed JSON holds only
the resulting float32 values (hex and decimal)."""
import json
import os
import re
import subprocess
import sys
import tempfile

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), 'mitsuba0.6_amd', 'data', 'conductor_rgb.json')


def table(src, name):
    i = src.index(name + ' = {')
    j = src.index('{', i)
    k = src.index('};', j)
    return re.findall(r'[-+]?\d*\.?\d+(?:[eE][-+]?\d+)?', src[j + 1:k])


def spd(path):
    rows = []
    for line in open(path):
        line = line.strip()
        if not line or line[0] == '#':
            continue
        parts = line.split()
        if len(parts) < 2:
            break
        rows.append((parts[0], parts[1]))
    return rows


def main():
    src = open(os.path.join(REF, 'src/libcore/spectrum.cpp')).read()
    w = table(src, 'const Float CIE_wavelengths[CIE_samples]')
    x = table(src, 'const Float CIE_X_entries[CIE_samples]')
    y = table(src, 'const Float CIE_Y_entries[CIE_samples]')
    z = table(src, 'const Float CIE_Z_entries[CIE_samples]')
    assert len(w) == len(x) == len(y) == len(z) == 471
    lines = ['471'] + ['%s %s %s %s' % t for t in zip(w, x, y, z)]
    names = sorted({f[:-len('.eta.spd')] for f in os.listdir(os.path.join(REF, 'data/ior')) if f.endswith('.eta.spd')})
    for n in names:
        for part in ('eta', 'k'):
            rows = spd(os.path.join(REF, 'data/ior', '%s.%s.spd' % (n, part)))
            lines.append('%s.%s %d' % (n, part, len(rows)))
            lines += ['%s %s' % r for r in rows]
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, 'spectrum_rgb')
        subprocess.run(['gcc', '-O2', '-ffp-contract=off', '-fno-fast-math', '-o', exe,
                        os.path.join(HERE, 'spectrum_rgb.c'), '-lm'], check=True)
        out = subprocess.run([exe], input='\n'.join(lines) + '\n', capture_output=True, text=True, check=True).stdout
    res = {}
    for line in out.splitlines():
        key, r, g, b = line.split()
        n, part = key.rsplit('.', 1)
        vals = [float.fromhex(v) for v in (r, g, b)]
        res.setdefault(n, {})[part] = vals
        res[n][part + '_hex'] = [r, g, b]
    meta = {'source': 'roughconductor.cpp:172-190 + spectrum.cpp:171-190 restated (tools/spectrum_rgb.c); '
                      'inputs: data/ior/*.spd and the CIE 1931 tables of src/libcore/spectrum.cpp',
            'materials': res}
    json.dump(meta, open(OUT, 'w'), indent=0, sort_keys=True)
    print('wrote', OUT, len(res), 'materials; Cu =', res.get('Cu'))


if __name__ == '__main__':
    sys.exit(main())
