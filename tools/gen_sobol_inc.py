#!/usr/bin/env python3
"""Build step: embed mitsuba0.6_amd/data/sobol_joe_kuo_1024.txt (Joe & Kuo
parameters) into libmtsgpu.so as a C array (written to the build directory)."""
import sys

src, dst = sys.argv[1], sys.argv[2]
vals = []
for line in open(src):
    if line.startswith('#') or not line.strip():
        continue
    parts = [int(x) for x in line.split()]
    d, s, a, m = parts[0], parts[1], parts[2], parts[3:]
    assert len(m) == s
    vals += [d, s, a] + m
with open(dst, 'w') as f:
    f.write('// generated from %s -- do not edit\n' % src.split('/')[-1])
    f.write('static const unsigned int kJoeKuoParams[] = {\n')
    for i in range(0, len(vals), 16):
        f.write('    ' + ', '.join(str(v) for v in vals[i:i + 16]) + ',\n')
    f.write('};\n')
