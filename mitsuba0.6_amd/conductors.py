"""Named conductor IORs (roughconductor `material=...`).

The reference converts data/ior/<name>.{eta,k}.spd to RGB at plugin
construction (roughconductor.cpp:172-190, Spectrum::fromContinuousSpectrum in
the RGB build, spectrum.cpp:171-190).  data/conductor_rgb.json holds those RGB
values for every material the reference ships, computed by the dev-time
generator tools/gen_conductor_rgb.py (single-precision restatement of the
conversion, tools/spectrum_rgb.c); the values are stored as exact float32 hex.
"""
import json
import os

_TABLE = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'conductor_rgb.json')


def _table():
    global _TABLE
    if _TABLE is None:
        _TABLE = json.load(open(_PATH))['materials']
    return _TABLE


def materials():
    return sorted(_table())


def conductor_rgb(name):
    """(eta_rgb, k_rgb) of a named material, as the reference's ctor computes them.
    'none' is the perfect mirror (eta 0, k 1).  Unknown names raise like the
    reference's failing file lookup."""
    if name.lower() == 'none':
        return (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)
    t = _table()
    if name not in t:
        raise ValueError('roughconductor: unknown material "%s" (data/ior/%s.eta.spd does not exist)' % (name, name))
    e = t[name]
    return (tuple(float.fromhex(v) for v in e['eta_hex']), tuple(float.fromhex(v) for v in e['k_hex']))
