"""The device's transcendentals (csrc/glibc_f32.h through dmath.h's d_*, built
for gfx950) against the host's libm.so.6, bit for bit: all 2^32 float inputs
of sin/cos (sincosf), expf, acosf, atanf, tanf and of math::fastexp/fastlog
((float)exp/log of the double, include/mitsuba/core/math.h:185-199), and 2^24
seeded pairs of atan2f and powf.  NaN results compare as a class.  The host
values come from oracle/libm_check.c (test infrastructure, glibc_eval /
glibc_compare_range); CPU-side bit-exactness of the same header is
tests/test_glibc_f32.py."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNK = 1 << 27


@pytest.fixture(scope='module')
def glibc():
    so = os.path.join(REPO, 'oracle', '_build', 'liblibm_check.so')
    if not os.path.exists(so):
        subprocess.check_call(['make', '-s', '-C', os.path.join(REPO, 'oracle')])
    L = C.CDLL(so)
    P = C.POINTER(C.c_float)
    L.glibc_eval.argtypes = [C.c_int, P, P, P, C.c_long]
    L.glibc_compare_range.argtypes = [C.c_int, C.c_uint32, C.c_long, P, C.POINTER(C.c_long)]
    L.glibc_compare_range.restype = C.c_long
    return L


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


@pytest.mark.parametrize('fn', ['sin', 'cos', 'expf', 'acosf', 'atanf', 'tanf', 'fastexp', 'fastlog'])
def test_device_libm_exhaustive(gpu_ctx, glibc, fn):
    fid = gpu_ctx.LIBM_FNS.index(fn)
    total = 0
    for first in range(0, 1 << 32, CHUNK):
        dev = gpu_ctx.debug_libm(fn, first=first, n=CHUNK)
        fb = C.c_long(-1)
        bad = glibc.glibc_compare_range(fid, first, CHUNK, _fp(dev), C.byref(fb))
        if bad:
            x = np.uint32(first + fb.value).view(np.float32)
            pytest.fail('%s: %d mismatches in [%#x, +%#x), first x=%r (bits %#x) device=%r' %
                        (fn, bad, first, CHUNK, float(x), first + fb.value, float(dev[fb.value])))
        total += CHUNK
    assert total == 1 << 32


def _pairs(n, seed, fn):
    rng = np.random.default_rng(seed)
    q = n // 4
    a = [rng.integers(0, 1 << 32, q, dtype=np.uint64).astype(np.uint32).view(np.float32),
         rng.uniform(-8, 8, q).astype(np.float32),
         rng.uniform(0, 2, q).astype(np.float32),
         rng.uniform(0, 1, q).astype(np.float32)]
    b = [rng.integers(0, 1 << 32, q, dtype=np.uint64).astype(np.uint32).view(np.float32),
         rng.uniform(-8, 8, q).astype(np.float32),
         rng.uniform(-128, 128, q).astype(np.float32),
         (np.where(rng.random(q) < 0.5, 0.25, 1.0 + rng.uniform(0, 256, q)) if fn == 'powf'
          else rng.uniform(-1e-3, 1e-3, q)).astype(np.float32)]
    return np.concatenate(a), np.concatenate(b)


@pytest.mark.parametrize('fn', ['atan2f', 'powf'])
def test_device_libm_pairs(gpu_ctx, glibc, fn):
    a, b = _pairs(1 << 24, 7, fn)
    dev = gpu_ctx.debug_libm(fn, a, b)
    ref = np.empty_like(a)
    glibc.glibc_eval(gpu_ctx.LIBM_FNS.index(fn), _fp(a), _fp(b), _fp(ref), a.size)
    same = (dev.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(dev) & np.isnan(ref))
    bad = np.flatnonzero(~same)
    assert bad.size == 0, '%s: %d mismatches, e.g. (%r, %r) device %r glibc %r' % (
        fn, bad.size, a[bad[0]], b[bad[0]], dev[bad[0]], ref[bad[0]])
