"""bench.py's roofline line only trusts per-sample profiles taken on the
library build it times: tools/prof_round.sh stamps each
profiles/<round>_{traffic,valu}_<cfg>.json with the sha256 of libmtsgpu.so, and
a profile of another build yields `frac: null` with the reason."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(REPO, 'bench.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


TRAFFIC = {'hbm_bytes_per_sample': 500.0, 'write_bytes_per_sample': 40.0, 'source': 'rX_traffic_C2.json'}
VALU = {'valu_busy_cycles_per_sample': 700.0, 'clock_hz': 2.4e9, 'valu_insts_per_sample': 180.0,
        'wait_frac_per_wave': 0.4, 'source': 'rX_valu_C2.json'}


def _line(monkeypatch, stamp_t, stamp_v, lib):
    b = _bench()
    profs = {'traffic': dict(TRAFFIC, lib_sha256=stamp_t), 'valu': dict(VALU, lib_sha256=stamp_v)}
    monkeypatch.setattr(b, 'measured_profile', lambda kind, cfg: dict(profs[kind]) if kind in profs else None)
    return b.roofline_line(2000.0, 4.7e8, 0.18, 'C2', lib)


def test_matching_stamp_gives_frac(monkeypatch):
    ln = _line(monkeypatch, 'abc', 'abc', 'abc')
    assert ln['bound'] == 'valu' and ln['frac'] is not None and 0 < ln['frac'] < 1
    assert 'frac_null_reason' not in ln and ln['lib_sha256'] == 'abc'


def test_mismatched_stamp_gives_null_frac(monkeypatch):
    ln = _line(monkeypatch, 'old', None, 'new')
    assert ln['frac'] is None
    assert 'rX_traffic_C2.json' in ln['frac_null_reason'] and 'rX_valu_C2.json' in ln['frac_null_reason']
    assert ln['hbm'] is None and ln['valu'] is None and ln['hbm_model']['achieved'] > 0


def test_one_stale_profile_is_dropped(monkeypatch):
    ln = _line(monkeypatch, 'new', 'old', 'new')
    assert ln['bound'] == 'hbm' and ln['frac'] is not None and ln['valu'] is None
    assert any('rX_valu_C2.json' in x for x in ln['stale_profiles_ignored'])


def test_valu_frac_is_against_the_calibrated_issue_peak(monkeypatch):
    """the valu roof is the instruction rate a pure-VALU kernel
    sustains (profiles/r*_valu_calib.json), not the 4-cycle busy metric."""
    b = _bench()
    cal = b.valu_calibration()
    assert cal is not None and 3.5 < cal['peak']['simd_cycles_per_wave_valu_inst'] < 5.0
    ln = _line(monkeypatch, 'abc', 'abc', 'abc')
    v = ln['valu']
    rate = VALU['valu_insts_per_sample'] * 4.7e8 / 0.18
    peak = 1024 * VALU['clock_hz'] / cal['peak']['simd_cycles_per_wave_valu_inst']
    assert abs(v['frac'] - rate / peak) < 1e-4 and v['calibration']['source'] == cal['source']
    assert abs(v['busy']['frac'] - VALU['valu_busy_cycles_per_sample'] * 4.7e8 / 0.18 / (1024 * 2.4e9)) < 1e-4
    assert v['spec_lane_issue']['frac'] < v['frac']


def test_lib_sha256_is_the_file_hash(tmp_path):
    import hashlib
    p = tmp_path / 'lib.so'
    p.write_bytes(b'\x7fELF' + bytes(range(256)) * 9000)
    assert _bench().lib_sha256(str(p)) == hashlib.sha256(p.read_bytes()).hexdigest()
