"""Rough-transmittance tables for `roughplastic` (RoughTransmittance, src/bsdfs/rtrans.h:46-150).

The reference resolves `data/microfacet/<distribution>.dat` through its
FileResolver (the Mitsuba installation's data directory) when a roughplastic
BSDF is configured.  This module resolves the same file name, in order:

1. an explicit directory (`BSDF.rtransDir`, or the XML scene's directory),
2. `$MTSGPU_MICROFACET_DIR`, then `$MITSUBA_DIR/data/microfacet`,
3. the tables generated in-tree by `tools/rtrans_nd.c` (build() writes them
   to `mitsuba0.6_amd/_build/microfacet/`): the reference's generator
   (src/utils/rdielprec.cpp) with its own adaptive cubature (NDIntegrator,
   src/libcore/quad.cpp) restated.  They match the shipped files bit for bit
   in 54-66% of the entries and to 1e-5 in 99% (tests/test_roughplastic_host.py,
   DESIGN.md 2); a warning says when they are used.

The bytes are handed to the library unchanged (mtsgpu_bsdf_desc.rtrans_data);
the library parses, checks and reduces them as RoughPlastic::configure does.
"""
import os
import warnings

from . import PKG_DIR

NAMES = {'beckmann': 'beckmann', 'ggx': 'ggx', 'phong': 'phong', 'as': 'phong'}
GENERATED_DIR = os.path.join(PKG_DIR, '_build', 'microfacet')
_cache = {}
_warned = set()


def search_dirs(extra=None):
    dirs = [d for d in (extra or []) if d]
    env = os.environ.get('MTSGPU_MICROFACET_DIR')
    if env:
        dirs.append(env)
    root = os.environ.get('MITSUBA_DIR')
    if root:
        dirs.append(os.path.join(root, 'data', 'microfacet'))
    return dirs


def table_path(distribution, extra_dirs=None):
    name = NAMES[distribution.lower()] + '.dat'
    for d in search_dirs(extra_dirs):
        for cand in (os.path.join(d, name), os.path.join(d, 'data', 'microfacet', name)):
            if os.path.isfile(cand):
                return cand
    gen = os.path.join(GENERATED_DIR, name)
    if os.path.isfile(gen):
        if name not in _warned:
            _warned.add(name)
            warnings.warn('roughplastic: using the generated table %s (tools/rtrans_nd.c); point '
                          'MTSGPU_MICROFACET_DIR at Mitsuba\'s data/microfacet for the reference\'s own' % gen)
        return gen
    raise FileNotFoundError('roughplastic: no rough transmittance table data/microfacet/%s (set '
                            'MTSGPU_MICROFACET_DIR, or run __graft_entry__.build() to generate one)' % name)


def table_bytes(distribution, extra_dirs=None):
    """The file's bytes (cached per path)."""
    path = table_path(distribution, extra_dirs)
    data = _cache.get(path)
    if data is None:
        with open(path, 'rb') as fh:
            data = fh.read()
        _cache[path] = data
    return data
