"""Import helper: the package directory is `mitsuba0.6_amd/` (a dot in the name),
so it is loaded by path and registered as `mitsuba_amd`."""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))


def mitsuba_amd():
    if 'mitsuba_amd' in sys.modules:
        return sys.modules['mitsuba_amd']
    pkg_dir = os.path.join(REPO, 'mitsuba0.6_amd')
    spec = importlib.util.spec_from_file_location('mitsuba_amd', os.path.join(pkg_dir, '__init__.py'),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules['mitsuba_amd'] = mod
    spec.loader.exec_module(mod)
    return mod
