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


def _read(path, bsdf_id, node_cap=16, prop_cap=64, params=None, lookup=None):
    """mtsgpu_xml_bsdf (no params, by id) or mtsgpu_xml_bsdf_ex (params dict and/or lookup given)."""
    L = integrator.load_library()
    nodes, props = (abi.XmlNode * max(1, node_cap))(), (abi.XmlProp * max(1, prop_cap))()
    nn, np_ = C.c_int(), C.c_int()
    err = C.create_string_buffer(512)
    if params is None and lookup is None:
        rc = L.mtsgpu_xml_bsdf(path.encode(), bsdf_id.encode(), nodes, node_cap, props, prop_cap, C.byref(nn),
                               C.byref(np_), err, 512)
    else:
        params = params or {}
        names = (C.c_char_p * max(1, len(params)))(*[k.encode() for k in params])
        values = (C.c_char_p * max(1, len(params)))(*[v.encode() for v in params.values()])
        rc = L.mtsgpu_xml_bsdf_ex(path.encode(), bsdf_id.encode(), abi.XML_BY_ID if lookup is None else lookup,
                                  names, values, len(params), nodes, node_cap, props, prop_cap, C.byref(nn),
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
    assert rc == abi.ENOENT and 'nosuch' in err
    rc, _, _, _, err = _read(scene_file, 'checks')          # a texture, not a BSDF
    assert rc == abi.EINVAL and '<texture>' in err
    rc, _, _, counts, err = _read(scene_file, 'frontback', node_cap=2, prop_cap=64)
    assert rc == abi.ENOMEM and counts[0] == 5
    bad = tmp_path / 'bad.xml'
    bad.write_text('<scene><bsdf type="diffuse" id="a"><float name="x" value="1"></bsdf></scene>')
    rc, _, _, _, err = _read(str(bad), 'a')
    assert rc == abi.EINVAL and 'mismatched' in err
    undef = tmp_path / 'undef.xml'
    undef.write_text('<scene><bsdf type="roughconductor" id="a"><float name="alpha" value="$nope"/></bsdf></scene>')
    rc, _, _, _, err = _read(str(undef), 'a')
    assert rc == abi.EINVAL and '$nope' in err and 'undefined parameter' in err
    cyc = tmp_path / 'cyc.xml'
    cyc.write_text('<scene><bsdf type="twosided" id="a"><ref id="a"/></bsdf></scene>')
    rc, _, _, _, err = _read(str(cyc), 'a')
    assert rc == abi.EINVAL and 'deeply' in err
    rc, _, _, _, err = _read(str(tmp_path / 'missing.xml'), 'a')
    assert rc == abi.EINVAL and 'cannot read' in err


# ---- the shim's routing -------------------------------------------

DEFAULT_CHECKER = '''<?xml version="1.0"?>
<scene version="0.6.0">
    <bsdf type="roughplastic" id="rp">
        <string name="distribution" value="ggx"/>
        <texture type="checkerboard" name="alpha">
            <float name="color0" value="0.05"/>
            <float name="color1" value="0.3"/>
        </texture>
        <texture type="checkerboard" name="diffuseReflectance"/>
    </bsdf>
    <shape type="obj" id="blob">
        <string name="filename" value="blob.obj"/>
        <bsdf type="diffuse">
            <texture type="checkerboard" name="reflectance"/>
        </bsdf>
    </shape>
    <shape type="obj" id="byref">
        <string name="filename" value="blob.obj"/>
        <ref id="rp"/>
    </shape>
    <shape type="obj" id="bare">
        <string name="filename" value="blob.obj"/>
    </shape>
    <emitter type="constant" id="sky"/>
</scene>
'''


def _checker(uv, uscale=1.0, vscale=1.0, uoffset=0.0, voffset=0.0):
    """checkerboard.cpp:66-74 after Texture2D's uv transform (texture.cpp:81-95): 0 = color0, 1 = color1.
    (int) truncates toward zero; math::modulo is the non-negative remainder."""
    u, v = uv[0] * uscale + uoffset, uv[1] * vscale + voffset
    x = 2 * (int(u * 2) % 2) - 1
    y = 2 * (int(v * 2) % 2) - 1
    return 0 if x * y == 1 else 1


def test_default_checkerboard_reads_as_textures(tmp_path):
    """A roughplastic with default-uvscale checkerboard alpha and diffuseReflectance: the file route
    returns both textures (the round-4 shim took such a BSDF for constant and rendered the defaults)."""
    p = tmp_path / 'checker.xml'
    p.write_text(DEFAULT_CHECKER)
    rc, nodes, props, _, err = _read(str(p), 'rp')
    assert rc == abi.OK, err
    assert [(n.kind, n.plugin, n.name) for n in nodes] == [
        (abi.XML_BSDF, b'roughplastic', b''), (abi.XML_TEXTURE, b'checkerboard', b'alpha'),
        (abi.XML_TEXTURE, b'checkerboard', b'diffuseReflectance')]
    ld = XMLSceneLoader(str(p), {})
    d = ld.make_bsdf(ld.parse_object(_rebuild(nodes, props))).to_desc()
    assert d.alpha_tex.type == abi.TEX_CHECKERBOARD and d.reflectance_tex.type == abi.TEX_CHECKERBOARD
    assert (d.alpha_tex.uscale, d.alpha_tex.vscale, d.alpha_tex.uoffset) == (1.0, 1.0, 0.0)
    # an inline BSDF has no id of its own: the shim finds it through its shape's id
    rc, nodes, _, _, err = _read(str(p), 'blob', lookup=abi.XML_BY_SHAPE)
    assert rc == abi.OK, err
    assert [(n.plugin, n.name) for n in nodes] == [(b'diffuse', b''), (b'checkerboard', b'reflectance')]
    rc, nodes, _, _, err = _read(str(p), 'byref', lookup=abi.XML_BY_SHAPE)
    assert rc == abi.OK and nodes[0].id == b'rp', err
    rc, _, _, _, err = _read(str(p), 'bare', lookup=abi.XML_BY_SHAPE)
    assert rc == abi.ENOENT and 'no <bsdf>' in err          # the shape's default diffuse
    rc, _, _, _, err = _read(str(p), 'nosuch', lookup=abi.XML_BY_SHAPE)
    assert rc == abi.ENOENT
    rc, _, _, _, err = _read(str(p), 'sky', lookup=abi.XML_BY_SHAPE)
    assert rc == abi.EINVAL and '<emitter>' in err
    rc, _, _, _, err = _read(str(p), 'blob')                 # by id, a shape is not a BSDF
    assert rc == abi.EINVAL and 'not a <bsdf>' in err


def test_old_probe_aliases_on_default_checkerboard():
    """Why the shim no longer trusts a probe for BSDFs the file holds: the round-4 probe points
    (0.173, 0.291) and (0.618, 0.854) fall in cells (0,0) and (1,1) of the default checkerboard,
    both color0, so a textured BSDF looked constant."""
    old = [(0.173, 0.291), (0.618, 0.854)]
    assert _checker(old[0]) == _checker(old[1]) == 0


def test_params_take_precedence_over_defaults(tmp_path):
    """scenehandler.cpp:208-220 / 684-687: the loader's parameters win over <default>; every attribute
    is substituted (ids in <ref> included), by substring, longest name first; flags tell the source."""
    p = tmp_path / 'params.xml'
    p.write_text('''<scene version="0.6.0">
        <default name="a" value="0.25"/>
        <default name="which" value="one"/>
        <bsdf type="roughconductor" id="one"><float name="alpha" value="$a"/></bsdf>
        <bsdf type="roughconductor" id="two"><float name="alpha" value="0.5"/></bsdf>
        <bsdf type="TwoSided" id="ts"><ref id="$which"/></bsdf>
        <bsdf type="roughconductor" id="sub"><float name="alpha" value="$ab"/>
            <string name="distribution" value="$a$which"/><float name="extEta" value="1.0"/></bsdf>
    </scene>''')
    rc, nodes, props, _, err = _read(str(p), 'one', params={})
    assert rc == abi.OK and props[0].value == b'0.25'
    assert props[0].flags == abi.XML_PROP_PARAM | abi.XML_PROP_DEFAULT
    rc, nodes, props, _, err = _read(str(p), 'one', params={'a': '0.125'})
    assert rc == abi.OK and props[0].value == b'0.125' and props[0].flags == abi.XML_PROP_PARAM
    rc, nodes, props, _, err = _read(str(p), 'ts', params={'which': 'two'})
    assert rc == abi.OK, err
    assert nodes[0].plugin == b'twosided'                    # type is lower-cased (:275)
    assert nodes[1].id == b'two' and props[nodes[1].first_prop].value == b'0.5'
    rc, nodes, props, _, err = _read(str(p), 'sub', params={'ab': '0.75'})
    assert rc == abi.OK, err
    got = {q.name: (q.value, q.flags) for q in props}
    assert got[b'alpha'] == (b'0.75', abi.XML_PROP_PARAM)   # $ab before $a (reverse name order)
    assert got[b'distribution'] == (b'0.25one', abi.XML_PROP_PARAM | abi.XML_PROP_DEFAULT)
    assert got[b'extEta'] == (b'1.0', 0)


def test_ids_alias_include_and_duplicates(tmp_path):
    inc = tmp_path / 'sub' / 'mats.xml'
    inc.parent.mkdir()
    inc.write_text('<scene version="0.6.0"><bsdf type="diffuse" id="inc"><rgb name="reflectance" value="$r"/></bsdf>'
                   '</scene>')
    p = tmp_path / 'main.xml'
    p.write_text('''<scene version="0.6.0">
        <default name="r" value="0.1, 0.2, 0.3"/>
        <include filename="sub/mats.xml"/>
        <alias id="inc" as="again"/>
        <bsdf type="twosided" id="ts"><ref id="again"/></bsdf>
    </scene>''')
    rc, nodes, props, _, err = _read(str(p), 'ts')
    assert rc == abi.OK, err
    assert nodes[1].id == b'inc' and props[0].value == b'0.1, 0.2, 0.3'
    rc, nodes, props, _, err = _read(str(p), 'again')
    assert rc == abi.OK and nodes[0].plugin == b'diffuse'
    dup = tmp_path / 'dup.xml'
    dup.write_text('<scene version="0.6.0"><bsdf type="diffuse" id="x"/><texture type="checkerboard" id="x"/>'
                   '<bsdf type="twosided" id="y"><ref id="x"/></bsdf></scene>')
    rc, _, _, _, err = _read(str(dup), 'y')
    assert rc == abi.EINVAL and "Duplicate ID 'x'" in err
    dup2 = tmp_path / 'dup2.xml'
    dup2.write_text('<scene version="0.6.0"><bsdf type="diffuse" id="x"/><bsdf type="diffuse" id="z"/>'
                    '<alias id="z" as="x"/></scene>')
    rc, _, _, _, err = _read(str(dup2), 'x')
    assert rc == abi.EINVAL and 'Duplicate ID' in err
    noinc = tmp_path / 'noinc.xml'
    noinc.write_text('<scene version="0.6.0"><include filename="missing.xml"/><bsdf type="diffuse" id="a"/></scene>')
    rc, _, _, _, err = _read(str(noinc), 'a')
    assert rc == abi.EINVAL and 'missing.xml' in err


# ---- unsupported property forms, <include> parameter scope, one parse per scene -----

def test_unsupported_property_forms_are_flagged(tmp_path):
    """<spectrum filename=...>, sampled spectra and <blackbody> are not turned into values
    here: the element comes back flagged MTSGPU_XML_PROP_UNSUPPORTED with its attributes,
    and the shim takes the loader's parsed value from the plugin's own Properties."""
    p = tmp_path / 'spd.xml'
    p.write_text('''<scene version="0.6.0">
        <bsdf type="roughconductor" id="c">
            <string name="distribution" value="ggx"/>
            <spectrum name="eta" filename="data/ior/Cu.eta.spd"/>
            <spectrum name="k" value="400:0.1, 500:0.2"/>
            <blackbody name="specularReflectance" temperature="5000K" scale="0.5"/>
            <float name="alpha" value="0.2"/>
        </bsdf></scene>''')
    rc, nodes, props, _, err = _read(str(p), 'c')
    assert rc == abi.OK, err
    got = {q.name.decode(): (q.tag.decode(), q.value.decode(), q.flags) for q in props}
    U = abi.XML_PROP_UNSUPPORTED
    assert got['eta'] == ('spectrum', 'filename=data/ior/Cu.eta.spd', U)
    assert got['k'][2] & U and got['k'][1] == '400:0.1, 500:0.2'
    assert got['specularReflectance'] == ('blackbody', 'temperature=5000K scale=0.5', U)
    assert got['alpha'] == ('float', '0.2', 0) and got['distribution'][2] == 0


def test_include_gets_a_copy_of_the_parameters(tmp_path):
    """SceneHandler(m_params, ...) for an <include> (scenehandler.cpp:670): the included
    file sees the including file's parameters, but its own <default> does not reach the
    including file, whose later <default> of the same name then applies."""
    sub = tmp_path / 'sub'
    sub.mkdir()
    (sub / 'inc.xml').write_text('''<scene version="0.6.0"><default name="a" value="0.9"/>
        <bsdf type="roughconductor" id="inner"><float name="alpha" value="$a"/>
        <string name="material" value="$m"/></bsdf><include filename="leaf.xml"/></scene>''')
    # the FileResolver has the main scene's directory first: leaf.xml resolves there, not in sub/
    (tmp_path / 'leaf.xml').write_text('<scene version="0.6.0"><bsdf type="diffuse" id="leaf"/></scene>')
    p = tmp_path / 'main.xml'
    p.write_text('''<scene version="0.6.0"><default name="m" value="Au"/>
        <include filename="sub/inc.xml"/>
        <default name="a" value="0.3"/>
        <bsdf type="roughconductor" id="outer"><float name="alpha" value="$a"/></bsdf></scene>''')
    rc, _, props, _, err = _read(str(p), 'inner')
    assert rc == abi.OK, err
    assert {q.name: q.value for q in props} == {b'alpha': b'0.9', b'material': b'Au'}
    rc, _, props, _, err = _read(str(p), 'outer')
    assert rc == abi.OK and props[0].value == b'0.3', err
    rc, nodes, _, _, err = _read(str(p), 'leaf')
    assert rc == abi.OK and nodes[0].plugin == b'diffuse', err


def test_large_scene_parsed_once(tmp_path):
    """An exported scene with thousands of shapes: a parse is linear in the file size and is
    reused for every BSDF of the scene while the file is unchanged."""
    import time
    n = 4000
    parts = ['<scene version="0.6.0">']
    for k in range(n):
        parts.append('<bsdf type="diffuse" id="b%d"><rgb name="reflectance" value="%g, 0.5, 0.5"/></bsdf>' % (k, k / n))
        parts.append('<shape type="obj" id="s%d"><string name="filename" value="m%d.obj"/><ref id="b%d"/></shape>'
                     % (k, k, k))
    parts.append('</scene>')
    p = tmp_path / 'big.xml'
    p.write_text('\n'.join(parts))
    t0 = time.perf_counter()
    for k in range(0, n, 10):
        rc, nodes, props, _, err = _read(str(p), 's%d' % k, lookup=abi.XML_BY_SHAPE)
        assert rc == abi.OK and props[0].value.decode().startswith('%g' % (k / n)), err
    assert time.perf_counter() - t0 < 10.0
    # a changed file is read again
    time.sleep(0.01)
    p.write_text('\n'.join(parts).replace('id="b0"><rgb name="reflectance" value="0,', 'id="b0"><rgb name="reflectance" value="0.25,'))
    rc, _, props, _, err = _read(str(p), 'b0')
    assert rc == abi.OK and props[0].value.startswith(b'0.25'), err
