"""The committed rocprofv3 kernel-stats profile of each bench configuration timed the
kernel that tests/test_gpu_bench_kernels.py compares with the oracle (its KERNELS
table, e.g. path_kernel<false, false, 336, 4> for C4), and its per-sample profiles
are stamped with the library the kernel-stats run used.  Checked on the CPU: the
profiles' CSVs are not sent to the GPU box, where that test's own check is skipped."""
import importlib.util
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_kernels_module():
    spec = importlib.util.spec_from_file_location(
        'bench_kernels_table', os.path.join(REPO, 'tests', 'test_gpu_bench_kernels.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize('cfg', ['C2', 'C2g', 'C3', 'C4', 'C5'])
def test_profiled_kernel_is_the_parity_tested_one(cfg):
    m = _bench_kernels_module()
    prof = m._profiled_kernel(cfg)
    assert prof is not None, 'no committed kernel-stats profile for %s' % cfg
    assert prof == m.KERNELS[cfg], (cfg, prof)


@pytest.mark.parametrize('cfg', ['C2', 'C2g', 'C3', 'C4', 'C5'])
def test_round_profiles_share_one_build(cfg):
    """traffic, valu and stall summaries of the newest round describe one library."""
    import glob
    shas = set()
    for kind in ('traffic', 'valu', 'stalls'):
        files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_%s_%s.json' % (kind, cfg))))
        assert files, (kind, cfg)
        shas.add(json.load(open(files[-1])).get('lib_sha256'))
    assert len(shas) == 1 and None not in shas, shas
