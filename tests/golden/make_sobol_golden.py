#!/usr/bin/env python3
"""Generate tests/golden/sobol_golden.json from the reference's own Sobol tables.

Runs only in the survey container (reads /root/reference).  The vectors are
computed from the reference's vendored tables (src/samplers/sobolseq.cpp:
Matrices::matrices32, vdc_sobol_matrices, vdc_sobol_matrices_inv) by a direct
transcription of sobol::sampleSingle and sobol::look_up
(src/samplers/sobolseq.h:43-57, 93-125).  The committed JSON holds only
inputs and expected outputs.
"""
import json, os, re, random, struct, hashlib

SRC = '/root/reference/src/samplers/sobolseq.cpp'


def arr(src, name):
    i = src.index(name)
    j = src.index('{', i)
    k = src.index('};', j)
    return [int(x, 16) for x in re.findall(r'0x([0-9a-fA-F]+)', src[j:k])]


def rows(src, name):
    # ragged C aggregate: one '{ // m = k' block per resolution, zero-padded to 52
    i = src.index(name)
    j = src.index('{', i)
    k = src.index('};', j)
    body = src[j + 1:k]
    out = []
    for blk in body.split('{')[1:]:
        vals = [int(x, 16) for x in re.findall(r'0x([0-9a-fA-F]+)', blk.split('}')[0])]
        out.extend(vals + [0] * (52 - len(vals)))
    return out


def main():
    src = open(SRC).read()
    m32 = arr(src, 'Matrices::matrices32[')
    vdc = rows(src, 'Matrices::vdc_sobol_matrices[][52]')
    vdci = rows(src, 'Matrices::vdc_sobol_matrices_inv[][52]')
    assert len(m32) == 1024 * 52 and len(vdc) % 52 == 0
    nres = min(len(vdc), len(vdci)) // 52

    def sample_single(index, dim, scramble=0):
        r = scramble
        i = dim * 52
        while index:
            if index & 1:
                r ^= m32[i]
            index >>= 1
            i += 1
        f = struct.unpack('f', struct.pack('f', float(r)))[0]   # (float) uint32
        v = f * 2.0 ** -32
        one_minus = struct.unpack('f', bytes.fromhex('ffff7f3f'))[0]
        return min(v, one_minus)

    def look_up(m, frame, px, py, scramble):
        m2 = m << 1
        index = frame << m2
        delta = 0
        c = 0
        f = frame
        while f:
            if f & 1:
                delta ^= vdc[(m - 1) * 52 + c]
            f >>= 1
            c += 1
        scr = (scramble & 0xFFFFFFFF) >> (32 - m)
        b = ((((px ^ scr) << m) | (py ^ scr)) ^ delta) & 0xFFFFFFFFFFFFFFFF
        c = 0
        while b:
            if b & 1:
                index ^= vdci[(m - 1) * 52 + c]
            b >>= 1
            c += 1
        return index

    rng = random.Random(0x5EED)
    out = {'source': 'src/samplers/sobolseq.cpp (tables) + sobolseq.h:43-125',
           'dim_hash': [], 'samples': [], 'lookups': []}
    for d in range(1024):
        h = hashlib.sha1(struct.pack('<52I', *m32[d * 52:(d + 1) * 52])).hexdigest()[:16]
        out['dim_hash'].append(h)
    for _ in range(3000):
        dim = rng.randrange(1024) if rng.random() < 0.7 else rng.randrange(8)
        index = rng.getrandbits(rng.choice([8, 16, 24, 31, 32]))
        scr = rng.getrandbits(32) if rng.random() < 0.2 else 0
        v = sample_single(index, dim, scr)
        out['samples'].append([index, dim, scr, struct.unpack('<I', struct.pack('<f', v))[0]])
    for m in range(1, min(nres, 14) + 1):
        for _ in range(150):
            frame = rng.randrange(1 << rng.choice([1, 4, 9, 10]))
            if m * 2 + frame.bit_length() > 52:
                continue
            px, py = rng.randrange(1 << m), rng.randrange(1 << m)
            scr = rng.getrandbits(32) if rng.random() < 0.2 else 0
            out['lookups'].append([m, frame, px, py, scr, look_up(m, frame, px, py, scr)])
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sobol_golden.json')
    json.dump(out, open(dst, 'w'))
    print('wrote', dst, len(out['samples']), 'samples', len(out['lookups']), 'lookups', 'vdc resolutions', nres)


if __name__ == '__main__':
    main()
