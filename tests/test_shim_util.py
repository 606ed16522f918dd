"""integration/gpupath_util.h: the Mitsuba-free parts of the plugin shim,
compiled here with g++ (the shim itself needs boost, absent from this image).

- gpupath_probe_uv: the surface positions at which the shim evaluates a BSDF
  that the scene file does not hold, to refuse a textured one.  Checked
  against the checkerboard texture (src/textures/checkerboard.cpp:66-74 after
  Texture2D's uv transform, src/librender/texture.cpp:81-95) over a sweep of
  scales and offsets: every checkerboard the probe must catch shows both
  colours.  The round-4 two-point probe missed the default checkerboard.
- gpupath_loader_params: the loader's $parameters from the integrator's
  'parameters' property or from `mitsuba -D name=value` arguments
  (src/mitsuba/mitsuba.cpp:168-173).
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, 'integration', 'gpupath_util.h')

HARNESS = r'''
#include <cstdio>
#include <cstring>
#include <iostream>
#include "gpupath_util.h"
int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "probe")) {
        std::vector<std::pair<float, float> > uv = gpupath_probe_uv();
        for (size_t k = 0; k < uv.size(); ++k) printf("%.9g %.9g\n", uv[k].first, uv[k].second);
        return 0;
    }
    /* params <has_property> <property> then the cmdline on stdin */
    std::string cmd((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
    std::vector<std::string> n, v;
    std::string bad;
    bool known = true;
    const bool ok = gpupath_loader_params(argv[2][0] == '1', argv[3], cmd, n, v, bad, &known);
    if (!ok) { printf("BAD %s\n", bad.c_str()); return 0; }
    if (!known) { printf("UNKNOWN\n"); return 0; }
    for (size_t k = 0; k < n.size(); ++k) printf("%s|%s\n", n[k].c_str(), v[k].c_str());
    return 0;
}
'''


@pytest.fixture(scope='module')
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp('shimutil')
    src = d / 'h.cpp'
    src.write_text(HARNESS)
    exe = d / 'h'
    subprocess.run(['g++', '-std=c++11', '-Wall', '-Werror', '-I', os.path.dirname(HDR), '-o', str(exe), str(src)],
                   check=True)
    return str(exe)


def _probe(harness):
    out = subprocess.run([harness, 'probe'], check=True, capture_output=True, text=True).stdout
    return np.array([[float(x) for x in l.split()] for l in out.splitlines()], dtype=np.float32)


def _checker(uv, us, vs, uo, vo):
    """checkerboard.cpp:66-74: x = 2*modulo((int)(u*2), 2) - 1 (C truncation, non-negative modulo),
    colour 0 iff x*y == 1, on u = uv.x*uscale + uoffset (texture.cpp:81-95), in float."""
    u = (uv[:, 0] * np.float32(us) + np.float32(uo)).astype(np.float32)
    v = (uv[:, 1] * np.float32(vs) + np.float32(vo)).astype(np.float32)
    xi = np.trunc(u * np.float32(2)).astype(np.int64) % 2
    yi = np.trunc(v * np.float32(2)).astype(np.int64) % 2
    return np.where((2 * xi - 1) * (2 * yi - 1) == 1, 0, 1)


def test_round4_probe_aliases():
    old = np.array([[0.173, 0.291], [0.618, 0.854]], dtype=np.float32)
    c = _checker(old, 1, 1, 0, 0)
    assert c[0] == c[1] == 0        # both color0: the round-4 shim took the texture for a constant


def test_probe_sees_both_colours(harness):
    uv = _probe(harness)
    assert len(uv) == 16 * 16 + 64
    rng = np.random.default_rng(5)
    scales = [1 / 8, 1 / 4, 1 / 3, 0.5, 1, 1.5, 2, 3, 4, 6.5, 8]
    missed = []
    for us in scales:
        for vs in scales:
            for uo, vo in [(0, 0), (0.1, 0), (0, -0.7), (0.25, 0.25)] + [tuple(rng.uniform(-3, 3, 2)) for _ in range(8)]:
                if len(set(_checker(uv, us, vs, uo, vo))) < 2:
                    missed.append((us, vs, uo, vo))
    assert not missed, missed[:10]


@pytest.mark.parametrize('prop,cmd,want', [
    (None, ['mitsuba', '-D', 'a=1', '-Db=0.5,0.2', '-o', 'x.exr', 'scene.xml'], ['a|1', 'b|0.5,0.2']),
    (None, ['mitsuba', 'scene.xml'], []),
    (None, ['mitsuba', '--', '-Dx=1'], []),
    ('a=1;b=2;', ['mitsuba', '-Dc=3'], ['a|1', 'b|2']),          # the property wins over argv
    (None, ['mitsuba', '-Dnoequals'], ['BAD noequals']),
    (None, ['mitsuba', '-Da='], ['BAD a=']),
    ('x=1=2', [], ['BAD x=1=2']),
    # tokenize(optarg, "=") drops empty tokens (mitsuba.cpp:169-172)
    (None, ['/opt/mitsuba/bin/mitsuba', '-Da==b', '-D', '=c=d'], ['a|b', 'c|d']),
    ('x==1;=y=2', [], ['x|1', 'y|2']),
    # -D arguments of another program are not the loader's (mtssrv, mtsgui, python)
    (None, ['python3', 'render.py', '-Da=1'], ['UNKNOWN']),
    (None, ['mtssrv', '-Da=1'], ['UNKNOWN']),
    ('a=1', ['python3', '-Db=2'], ['a|1']),
])
def test_loader_params(harness, prop, cmd, want):
    out = subprocess.run([harness, 'params', '1' if prop is not None else '0', prop or ''],
                         input='\0'.join(cmd) + '\0', check=True, capture_output=True, text=True).stdout
    assert out.splitlines() == want
