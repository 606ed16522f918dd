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


@pytest.fixture(scope='session')
def mts():
    return mitsuba_amd()


@pytest.fixture(scope='session')
def oracle():
    import oracle.binding as ob
    ob.lib()
    return ob


@pytest.fixture(scope='session')
def gpu_ctx():
    from mitsuba_amd.integrator import Context
    return Context()
