"""mtsgpu_xml_bsdf: the BSDF subtree reader the plugin shim uses for nested
(twosided) and textured BSDFs, which are private children inside Mitsuba
(src/bsdfs/twosided.cpp:198-210) but readable from the scene's source file
(Scene::getSourceFile, include/mitsuba/render/scene.h:1107).

Bar: the tree the C reader returns for a BSDF id carries exactly what the
library's own XML loader (xmlscene.py) reads for that BSDF -- the element tree
is rebuilt from the returned nodes and properties, converted by the loader's
make_bsdf, and its mtsgpu_bsdf_desc (nested ones included) equals the one the
loader makes from the file itself, byte for byte.  No GPU."""
import ctypes as C
import xml.etree.ElementTree as ET

import pytest

from mitsuba_amd import abi, integrator
from mitsuba_amd.xmlscene import XMLSceneLoader

SCENE = '''<?xml version="1.0" encoding="utf-8"?>
<!-- nested and textured BSDFs, by reference and inline -->
<scene version="0.6.0">
    <default name="rough" value="0.25"/>
    <default name="tint" value="0.8, 0.3, 0.2"/>
    <texture type="checkerboard" id="checks">
        <rgb name="color0" value="0.7, 0.7, 0.65"/>
        <rgb name="color1" value="$tint"/>
        <float name="uscale" value="6"/>
        <float name="vscale" value="4"/>
        <float name="uoffset" value="0.1"/>
    </texture>
    <bsdf type="roughconductor" id="copper">
        <string name="distribution" value="ggx"/>
        <float name="alpha" value="$rough"/>
        <string name="material" value="Cu"/>
    </bsdf>
    <bsdf type="twosided" id="twocopper">
        <ref id="copper"/>
    </bsdf>
    <bsdf type="twosided" id="frontback">
        <bsdf type="diffuse">
            <ref name="reflectance" id="checks"/>
        </bsdf>
        <bsdf type='roughplastic'>
            <string name="distribution" value="beckmann"/>
            <texture type="checkerboard" name="alpha">
                <float name="color0" value="0.05"/>
                <float name="color1" value="0.3"/>
                <float name="uvscale" value="3"/>
            </texture>
            <srgb name="diffuseReflectance" value="#4080c0"/>
            <boolean name="nonlinear" value="true"/>
        </bsdf>
    </bsdf>
    <bsdf type="diffuse" id="texdiffuse">
        <texture type="checkerboard" name="reflectance">
            <rgb name="color0" value="0.1 0.2 0.3"/>
        </texture>
    </bsdf>
    <bsdf type="plastic" id="amp&amp;quote">
        <float name="intIOR" value="1.6"/>
        <spectrum name="diffuseReflectance" value="0.4"/>
    </bsdf>
</scene>
'''

IDS = ['copper', 'twocopper', 'frontback', 'texdiffuse', 'amp&quote']


@pytest.fixture(scope='module')
def scene_file(tmp_path_factory):
    p = tmp_path_factory.mktemp('xml') / 'scene.xml'
    p.write_text(SCENE)
    return str(p)


def _read(path, bsdf_id, node_cap=16, prop_cap=64):
    L = integrator.load_library()
    nodes, props = (abi.XmlNode * max(1, node_cap))(), (abi.XmlProp * max(1, prop_cap))()
    nn, np_ = C.c_int(), C.c_int()
    err = C.create_string_buffer(512)
    rc = L.mtsgpu_xml_bsdf(path.encode(), bsdf_id.encode(), nodes, node_cap, props, prop_cap, C.byref(nn),
                           C.byref(np_), err, 512)
    return rc, list(nodes[:nn.value]) if rc == abi.OK else None, list(props[:np_.value]) if rc == abi.OK else None, \
        (nn.value, np_.value), err.value.decode()


def _rebuild(nodes, props):
    """The element tree the shim would rebuild (here as XML for xmlscene's parser)."""
    els = []
    for k, n in enumerate(nodes):
        tag = 'bsdf' if n.kind == abi.XML_BSDF else 'texture'
        e = ET.Element(tag, {'type': n.plugin.decode()})
        if n.name:
            e.set('name', n.name.decode())
        for p in props[n.first_prop:n.first_prop + n.num_props]:
            a = {'value': p.value.decode()}
            if p.name:
                a['name'] = p.name.decode()
            ET.SubElement(e, p.tag.decode(), a)
        if n.parent >= 0:
            els[n.parent].append(e)
        else:
            assert k == 0
        els.append(e)
    return els[0]


def _desc_bytes(b):
    d = b.to_desc()
    raw = bytes(C.string_at(C.addressof(d), C.sizeof(d)))
    # the rtrans pointer differs per descriptor; compare the table bytes instead
    off = abi.BsdfDesc.rtrans_data.offset
    tail = C.string_at(d.rtrans_data, d.rtrans_bytes) if d.rtrans_bytes else b''
    nested = [_desc_bytes(x) for x in getattr(b, 'nested', [])]
    return raw[:off] + raw[off + 8:], tail, nested


@pytest.mark.parametrize('bsdf_id', IDS)
def test_reader_tree_equals_loader(scene_file, bsdf_id):
    rc, nodes, props, _, err = _read(scene_file, bsdf_id)
    assert rc == abi.OK, err
    assert nodes[0].id.decode() == bsdf_id and nodes[0].parent == -1
    ref = XMLSceneLoader(scene_file, {})
    root = ET.parse(scene_file).getroot()
    ref._expand(root)
    for el in root:
        if el.tag in ('bsdf', 'texture'):
            ref.parse_object(el)
    want = ref.make_bsdf(ref.named[bsdf_id])
    ld = XMLSceneLoader(scene_file, {})
    got = ld.make_bsdf(ld.parse_object(_rebuild(nodes, props)))
    assert _desc_bytes(got) == _desc_bytes(want)


def test_tree_shape(scene_file):
    rc, nodes, props, _, _ = _read(scene_file, 'frontback')
    assert rc == abi.OK
    assert [(n.kind, n.plugin, n.name, n.parent) for n in nodes] == [
        (abi.XML_BSDF, b'twosided', b'', -1), (abi.XML_BSDF, b'diffuse', b'', 0),
        (abi.XML_TEXTURE, b'checkerboard', b'reflectance', 1), (abi.XML_BSDF, b'roughplastic', b'', 0),
        (abi.XML_TEXTURE, b'checkerboard', b'alpha', 3)]
    assert nodes[2].id == b'checks'       # resolved through <ref>
    c1 = [p for p in props[nodes[2].first_prop:nodes[2].first_prop + nodes[2].num_props] if p.name == b'color1']
    assert c1[0].value == b'0.8, 0.3, 0.2'   # $tint from <default>


def test_errors_and_capacity(scene_file, tmp_path):
    rc, _, _, _, err = _read(scene_file, 'nosuch')
    assert rc == abi.EINVAL and 'nosuch' in err
    rc, _, _, counts, err = _read(scene_file, 'frontback', node_cap=2, prop_cap=64)
    assert rc == abi.ENOMEM and counts[0] == 5
    bad = tmp_path / 'bad.xml'
    bad.write_text('<scene><bsdf type="diffuse" id="a"><float name="x" value="1"></bsdf></scene>')
    rc, _, _, _, err = _read(str(bad), 'a')
    assert rc == abi.EINVAL and 'mismatched' in err
    undef = tmp_path / 'undef.xml'
    undef.write_text('<scene><bsdf type="roughconductor" id="a"><float name="alpha" value="$nope"/></bsdf></scene>')
    rc, _, _, _, err = _read(str(undef), 'a')
    assert rc == abi.EINVAL and '$nope' in err
    cyc = tmp_path / 'cyc.xml'
    cyc.write_text('<scene><bsdf type="twosided" id="a"><ref id="a"/></bsdf></scene>')
    rc, _, _, _, err = _read(str(cyc), 'a')
    assert rc == abi.EINVAL and 'deeply' in err
    rc, _, _, _, err = _read(str(tmp_path / 'missing.xml'), 'a')
    assert rc == abi.EINVAL and 'cannot read' in err
