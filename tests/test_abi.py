"""The C-ABI boundary without a GPU: libmtsgpu.so loads, exports every entry
point include/mtsgpu.h declares, its structs have the layout the Python mirror
(abi.py) assumes, and calls fail cleanly (no device -> MTSGPU_ENODEV)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from mitsuba_amd import abi, integrator

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, 'include', 'mtsgpu.h')


def _declared():
    src = open(HDR).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mtsgpu_\w+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    L = integrator.load_library()
    names = _declared()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(integrator.EXPORTS) <= set(names)
    assert L.mtsgpu_abi_version() == abi.ABI_VERSION == 8


STRUCTS = {'mtsgpu_bsdf_desc': abi.BsdfDesc, 'mtsgpu_emitter_desc': abi.EmitterDesc,
           'mtsgpu_mesh_desc': abi.MeshDesc, 'mtsgpu_sensor_desc': abi.SensorDesc,
           'mtsgpu_scene_desc': abi.SceneDesc, 'mtsgpu_render_params': abi.RenderParams,
           'mtsgpu_stats': abi.Stats, 'mtsgpu_develop_params': abi.DevelopParams,
           'mtsgpu_texture_desc': abi.TextureDesc, 'mtsgpu_xml_node': abi.XmlNode, 'mtsgpu_xml_prop': abi.XmlProp}


def test_struct_layout_matches_python_mirror(tmp_path):
    """sizeof/offsetof from the C compiler == ctypes layout of abi.py."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HDR, 'int main(void) {']
    for cname, py in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    lines.append('return 0; }')
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-o', str(exe), str(src)], check=True)
    out = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines())
    for cname, py in STRUCTS.items():
        assert int(out[cname]) == C.sizeof(py), cname
        for f in py._fields_:
            assert int(out['%s.%s' % (cname, f[0])]) == getattr(py, f[0]).offset, (cname, f[0])


def test_film_border_matches_reference_rule():
    """ReconstructionFilter::m_borderSize = ceil(radius - 0.5) (rfilter.cpp:50)."""
    L = integrator.load_library()
    assert L.mtsgpu_film_border(abi.RFILTER_BOX, C.c_float(0.5)) == 1   # radius 0.5 + 1e-5
    assert L.mtsgpu_film_border(abi.RFILTER_GAUSSIAN, C.c_float(0.5)) == 2  # radius 4 * stddev
    assert L.mtsgpu_film_border(7, C.c_float(0.5)) == abi.EINVAL


def test_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip('a GPU is present')
    L = integrator.load_library()
    h = C.c_void_p()
    rc = L.mtsgpu_create(0, C.byref(h))
    assert rc == abi.ENODEV and not h.value
    assert L.mtsgpu_last_error(None)
    with pytest.raises(integrator.NativeUnavailable):
        integrator.Context()


def test_null_arguments_are_rejected():
    L = integrator.load_library()
    assert L.mtsgpu_create(0, None) == abi.EINVAL
    assert L.mtsgpu_upload_scene(None, None) == abi.EINVAL
    assert L.mtsgpu_render(None, None, None, None, None) == abi.EINVAL
