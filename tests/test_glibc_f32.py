"""The product's glibc restatement (mitsuba0.6_amd/csrc/glibc_f32.h) against
this machine's libm.so.6, bit for bit, on the CPU: all 2^32 inputs of each
unary function (sincosf's sine and cosine, expf, acosf, atanf, tanf) and 2^28
seeded pairs for atan2f and powf (random bit patterns, [-8, 8] values, and the
bases/exponents the path uses).  NaN results compare as a class.

The header is the device's code (tests/test_gpu_libm.py runs the device build);
here gcc compiles it for the host (oracle/libm_check.c).  glibc's x86_64 ifuncs
pick the FMA builds of sincosf/expf/powf on a CPU with FMA and AVX2, which is
what the restatement follows; on a CPU without them the check is skipped."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(REPO, 'oracle', '_build', 'libm_check')


def _cpu_has_fma():
    try:
        flags = open('/proc/cpuinfo').read()
    except OSError:
        return False
    return re.search(r'\bfma\b', flags) is not None and re.search(r'\bavx2\b', flags) is not None


@pytest.fixture(scope='module')
def checker():
    subprocess.check_call(['make', '-s', '-C', os.path.join(REPO, 'oracle')])
    if not _cpu_has_fma():
        pytest.skip('host CPU lacks FMA/AVX2: glibc selects its non-FMA builds there')
    return CHECK


@pytest.mark.parametrize('fn', ['sincosf', 'expf', 'acosf', 'atanf', 'tanf', 'atan2f', 'powf'])
def test_glibc_restatement_bit_exact(checker, fn):
    r = subprocess.run([checker, fn], capture_output=True, text=True, timeout=600)
    out = r.stdout
    m = re.search(r'checked=(\d+) mismatches=(\d+)', out)
    assert m, out + r.stderr
    checked, bad = int(m.group(1)), int(m.group(2))
    assert checked >= (1 << 28)
    assert bad == 0 and r.returncode == 0, out
