import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU')


def host_has_fma():
    """glibc picks its FMA/AVX2 builds of sinf/expf/powf/... on such hosts; those are
    what csrc/glibc_f32.h restates (tests/test_glibc_f32.py)."""
    import re
    try:
        flags = open('/proc/cpuinfo').read()
    except OSError:
        return False
    return re.search(r'\bfma\b', flags) is not None and re.search(r'\bavx2\b', flags) is not None


def pytest_collection_modifyitems(config, items):
    # GPU-vs-oracle parity runs the oracle in glibc mode (libm_mode=0: the host's
    # libm.so.6); on a host without FMA/AVX2 glibc's non-FMA builds round
    # differently from the device restatement, which would read as device bugs
    if host_has_fma():
        return
    skip = pytest.mark.skip(reason='host CPU lacks FMA/AVX2: the oracle\'s libm differs from glibc_f32.h')
    for item in items:
        if item.get_closest_marker('gpu') is not None and 'oracle' in getattr(item, 'fixturenames', ()):
            item.add_marker(skip)


@pytest.fixture(scope='session')
def mts():
    return mitsuba_amd()


@pytest.fixture(scope='session')
def oracle():
    import oracle.binding as ob
    ob.lib()
    return ob


@pytest.fixture(scope='session')
def c5_reference_tables(tmp_path_factory):
    """A directory holding a ggx.dat whose eta layers at C5's relative IOR are the
    reference's own (tests/golden/rtrans_c5_ggx_layers.npz, made by
    make_rtrans_layers.py from data/microfacet/ggx.dat) and whose other layers
    are the generated table's.  setEta reads only those layers
    (spline.cpp:379-450), so C5's reduced 2D tables are the reference file's."""
    import numpy as np
    from mitsuba_amd import rtrans
    fx = np.load(os.path.join(REPO, 'tests', 'golden', 'rtrans_c5_ggx_layers.npz'))
    raw = open(os.path.join(rtrans.GENERATED_DIR, 'ggx.dat'), 'rb').read()
    hdr = fx['header'].tobytes()
    assert raw[:len(hdr)] == hdr, 'generated ggx.dat header differs from the reference file'
    t = np.frombuffer(raw, '<f4', offset=len(hdr)).copy().reshape((-1,) + fx['layers'].shape[1:])
    t[fx['rows']] = fx['layers']
    d = tmp_path_factory.mktemp('c5_reference_tables')
    (d / 'ggx.dat').write_bytes(hdr + t.astype('<f4').tobytes())
    return str(d)


@pytest.fixture(scope='session')
def gpu_ctx():
    from mitsuba_amd.integrator import Context
    return Context()
