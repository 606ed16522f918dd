#!/usr/bin/env python3
"""Recover the Joe-Kuo Sobol' parameters (degree s, polynomial a, initial m_i)
from the direction-number table vendored in the reference
(/root/reference/src/samplers/sobolseq.cpp:33, `Matrices::matrices64`; the
table is Joe & Kuo's public "new-joe-kuo-6.21201" data expanded to 52 bits,
see sobolseq.cpp:21-27).

Dev-time tool: runs only in the survey container (the reference is absent on
the GPU box).  Output: mitsuba0.6_amd/data/sobol_joe_kuo_1024.txt in the
published Joe-Kuo text layout ("d s a m_1 .. m_s").  The product and the
oracle regenerate every direction number from this file with the Sobol'
recurrence; tests/test_sobol.py pins the regenerated values against golden
vectors extracted from the reference table (tests/golden/make_sobol_golden.py).
"""
import re, sys, os

SRC = '/root/reference/src/samplers/sobolseq.cpp'
BITS = 52


def parse_array(src, name):
    i = src.index(name)
    j = src.index('{', i)
    k = src.index('};', j)
    return [int(x.rstrip('ULul'), 16) for x in re.findall(r'0x[0-9a-fA-F]+', src[j:k])]


def gen_m(s, a, minit, n):
    m = list(minit)
    for k in range(s, n):
        v = m[k - s] ^ (m[k - s] << s)
        for i in range(1, s):
            if (a >> (s - 1 - i)) & 1:
                v ^= m[k - i] << i
        m.append(v)
    return m


def main():
    src = open(SRC).read()
    m64 = parse_array(src, 'Matrices::matrices64[')
    assert len(m64) == 1024 * BITS
    out = []
    for d in range(1024):
        cols = m64[d * BITS:(d + 1) * BITS]
        # column k (0-based) holds m_{k+1} << (BITS-k-1)
        mvals = [cols[k] >> (BITS - k - 1) for k in range(BITS)]
        assert all(cols[k] == mvals[k] << (BITS - k - 1) for k in range(BITS))
        if d == 0:
            assert all(v == 1 for v in mvals)
            out.append((1, 0, 0, [1]))
            continue
        found = None
        for s in range(1, 20):
            for a in range(1 << (s - 1)):
                if gen_m(s, a, mvals[:s], BITS) == mvals:
                    found = (s, a, mvals[:s])
                    break
            if found:
                break
        assert found, d
        out.append((d + 1, found[0], found[1], found[2]))
    dst = os.path.join(os.path.dirname(__file__), '..', 'mitsuba0.6_amd', 'data',
                       'sobol_joe_kuo_1024.txt')
    with open(dst, 'w') as f:
        f.write('# Joe & Kuo Sobol parameters (new-joe-kuo-6.21201), dimensions 2..1024.\n')
        f.write('# d s a m_1 .. m_s   (dimension 1 is the van der Corput sequence)\n')
        for d, s, a, m in out[1:]:
            f.write('%d %d %d %s\n' % (d, s, a, ' '.join(map(str, m))))
    print('wrote', dst)


if __name__ == '__main__':
    main()
