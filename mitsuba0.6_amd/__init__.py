"""mitsuba0.6_amd -- MI355X-native drop-in for Mitsuba 0.6's `path` integrator.

The hot path (MIPathTracer::Li and the renderBlock loop around it,
src/integrators/path/path.cpp:119-294, src/librender/integrator.cpp:140-188)
runs as hand-written HIP kernels for gfx950 inside libmtsgpu.so, behind the
C-ABI declared in include/mtsgpu.h.  This package is the host-side mirror of
the reference's plugin interface: scene model (scene.py), synthetic configs
(scenes.py) and the `PathTracer` integrator (integrator.py).

The directory name contains a dot, so import it through
`mitsuba0.6_amd/__init__.py` by path (see tests/conftest.py) as `mitsuba_amd`.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
DATA_DIR = os.path.join(PKG_DIR, 'data')
LIB_PATH = os.path.join(PKG_DIR, '_build', 'libmtsgpu.so')
SOBOL_PARAMS = os.path.join(DATA_DIR, 'sobol_joe_kuo_1024.txt')

from . import abi  # noqa: E402
from .scene import (BSDF, DirectIntegrator, Emitter, Mesh, PathIntegrator, Scene, Sensor,  # noqa: E402
                    VolpathIntegrator, film_border, look_at)
from .film import HDRFilm, MFilm  # noqa: E402
from .transform import Transform  # noqa: E402
from .xmlscene import load_scene, save_scene  # noqa: E402

__all__ = ['abi', 'BSDF', 'DirectIntegrator', 'Emitter', 'Mesh', 'PathIntegrator', 'Scene', 'Sensor',
           'VolpathIntegrator', 'HDRFilm', 'MFilm',
           'film_border', 'look_at', 'Transform', 'load_scene', 'save_scene', 'PKG_DIR', 'LIB_PATH',
           'SOBOL_PARAMS']
