"""hdrfilm output (film.py) without a GPU: the constructor's property handling
(hdrfilm.cpp:205-360), the develop restatement's known answers
(fmtconv.cpp:955-1030), and PFM / RGBE / OpenEXR writers against their readers
and against the formats' published layouts.

The OpenEXR container bytes are checked against the file format's published
layout (magic, attribute list, offset table, ZIP predictor); no OpenEXR
library is importable here, so byte-level interchange with libIlmImf is
parity unpinned.  Pixel values are pinned through the develop parity test
(tests/test_gpu_film.py)."""
import struct
import zlib

import numpy as np
import pytest

from mitsuba_amd import film as F
from mitsuba_amd import xmlscene
from oracle.film_oracle import develop_ref

f32 = np.float32


def test_hdrfilm_defaults_and_overrides():
    h = F.HDRFilm()
    assert (h.fileFormat, h.pixel_format, h.componentFormat, h.banner) == ('openexr', 'rgb', 'float16', True)
    assert h.channel_names == ['R', 'G', 'B'] and not h.hasAlpha
    # RGBE forces rgb/float32, PFM forces float32 and rgb unless luminance (hdrfilm.cpp:314-338)
    h = F.HDRFilm(fileFormat='rgbe', pixelFormat='rgba', componentFormat='float16')
    assert (h.pixel_format, h.componentFormat, h.hasAlpha) == ('rgb', 'float32', False)
    h = F.HDRFilm(fileFormat='PFM', pixelFormat='xyza')
    assert (h.pixel_format, h.componentFormat) == ('rgb', 'float32')
    assert F.HDRFilm(fileFormat='pfm', pixelFormat='luminance').pixel_format == 'luminance'
    h = F.HDRFilm(pixelFormat='luminanceAlpha', channelNames='beauty')
    assert h.channel_names == ['beauty.Y', 'beauty.A'] and h.hasAlpha
    assert F.HDRFilm(pixelFormat='XYZA').channel_names == ['X', 'Y', 'Z', 'A']


@pytest.mark.parametrize('kw,msg', [
    (dict(fileFormat='png'), 'fileFormat'),
    (dict(pixelFormat=''), 'At least one pixel format'),
    (dict(pixelFormat='rgb', channelNames='a,b'), 'Number of channel names'),
    (dict(pixelFormat='rgb,luminance', channelNames='a,b', fileFormat='pfm'), 'multi-channel'),
    (dict(pixelFormat='spectrum'), 'spectral image'),
    (dict(pixelFormat='hsv'), 'pixelFormat'),
    (dict(componentFormat='uint8'), 'componentFormat'),
])
def test_hdrfilm_errors(kw, msg):
    with pytest.raises(ValueError, match=msg):
        F.HDRFilm(**kw)


def test_output_path_extension():
    """hdrfilm.cpp:508-519: a wrong extension is replaced, case-insensitively kept."""
    assert F.HDRFilm().output_path('/tmp/a.png') == '/tmp/a.exr'
    assert F.HDRFilm().output_path('/tmp/a.EXR') == '/tmp/a.EXR'
    assert F.HDRFilm(fileFormat='rgbe').output_path('/tmp/a') == '/tmp/a.rgbe'
    assert F.HDRFilm(fileFormat='pfm').output_path('/tmp/a.exr') == '/tmp/a.pfm'


def _film(rng, h=6, w=7, b=1):
    film = rng.random((h + 2 * b, w + 2 * b, 5), dtype=np.float32) * f32(3)
    film[..., 3] = np.minimum(film[..., 3], film[..., 4])
    film[b + 1, b + 2, :] = 0                       # weight 0 -> 0 (invWeight = weight)
    film[b, b, :3] = f32(7e4)                       # overflows half -> inf
    film[b, b, 4] = f32(1)
    film[b + 2, b, :3] = f32(3e-7)                  # half subnormal
    film[b + 2, b, 4] = f32(1)
    return film


def test_develop_ref_known_answers():
    film = np.zeros((3, 3, 5), f32)
    film[1, 1] = (1.5, 3.0, 0.75, 0.6, 3.0)
    out = develop_ref(film, 1, 'rgba', 'float32')
    inv = f32(1) / f32(3)
    np.testing.assert_array_equal(out[0, 0], [f32(1.5) * inv, f32(3.0) * inv, f32(0.75) * inv, f32(0.6) * inv])
    assert develop_ref(film, 1, 'rgb', 'float16').dtype == np.float16
    lum = develop_ref(film, 1, 'luminance', 'float32')[0, 0, 0]
    expect = ((f32(1.5) * f32(0.212671) + f32(3.0) * f32(0.715160)) + f32(0.75) * f32(0.072169)) * inv
    assert lum == f32(expect)
    u = develop_ref(film, 1, 'rgb', 'uint32')[0, 0]
    assert u[0] == 1 << 31 and u[1] == 0   # 0.5 * 2^32 + 0.5 -> 2^31 (fits), 1.0 -> 2^32 wraps to 0 (x86 cast)
    film[1, 1, :3] = (0.25, 1.0, -1.0)
    film[1, 1, 4] = 1.0
    u = develop_ref(film, 1, 'rgb', 'uint32')[0, 0]
    assert u.tolist() == [1 << 30, 0, 0]


def test_pfm_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.random((5, 9, 3), dtype=np.float32)
    p = str(tmp_path / 'a.pfm')
    F.write_pfm(p, img)
    raw = open(p, 'rb').read()
    assert raw.startswith(b'PF\n9 5\n-1\n')
    # bottom-up rows (bitmap.cpp:3834-3835)
    assert np.frombuffer(raw[len(b'PF\n9 5\n-1\n'):], '<f4', 27).tolist() == img[4].reshape(-1).tolist()
    np.testing.assert_array_equal(F.read_pfm(p), img)
    F.write_pfm(p, img[:, :, :1])
    assert open(p, 'rb').read(2) == b'Pf'
    with pytest.raises(ValueError):
        F.write_pfm(p, img.astype(np.float16))


def test_rgbe_known_answers():
    px = F.rgbe_from_float(np.array([[1.0, 0.5, 0.25], [0.0, 0.0, 0.0], [3.0, 0.0, 1e-33]], f32))
    assert px[0].tolist() == [128, 64, 32, 129]
    assert px[1].tolist() == [0, 0, 0, 0]
    assert px[2].tolist() == [192, 0, 0, 130]          # frexp(3) = 0.75 * 2^2
    np.testing.assert_array_equal(F.rgbe_to_float(px[:1]), [[1.0, 0.5, 0.25]])


def test_rgbe_rle_round_trip(tmp_path):
    rng = np.random.default_rng(2)
    img = rng.random((4, 40, 3), dtype=np.float32) * f32(10)
    img[1, 5:30] = f32(2.0)                            # long runs
    img[2, :, 1] = 0
    p = str(tmp_path / 'a.rgbe')
    F.write_rgbe(p, img)
    back = F.read_rgbe(p)
    np.testing.assert_array_equal(back, F.rgbe_to_float(F.rgbe_from_float(img)))
    assert np.max(np.abs(back - img) / np.maximum(img.max(axis=-1, keepdims=True), 1e-6)) < 1 / 128
    small = img[:, :5]                                 # w < 8: flat pixels
    F.write_rgbe(p, small)
    np.testing.assert_array_equal(F.read_rgbe(p), F.rgbe_to_float(F.rgbe_from_float(small)))


def test_rle_encoder_matches_walter_layout():
    data = bytes([7] * 10 + [1, 2, 3] + [9] * 2 + [4])
    enc = F._rle_bytes(data)
    assert enc == bytes([128 + 10, 7, 6, 1, 2, 3, 9, 9, 4])


@pytest.mark.parametrize('dtype', [np.float16, np.float32, np.uint32])
@pytest.mark.parametrize('compression', ['zip', 'none', 'zips'])
def test_exr_round_trip(tmp_path, dtype, compression):
    rng = np.random.default_rng(3)
    img = (rng.random((37, 21, 4)) * 100).astype(dtype)
    img[3:9, 2:12] = 0                                 # compressible area
    p = str(tmp_path / 'a.exr')
    F.write_exr(p, img, ['R', 'G', 'B', 'A'], compression=compression)
    planes, attrs = F.read_exr(p)
    assert sorted(planes) == ['A', 'B', 'G', 'R']
    for i, c in enumerate('RGBA'):
        assert planes[c].dtype == np.dtype(dtype)
        np.testing.assert_array_equal(planes[c], img[:, :, i])
    assert attrs['lineOrder'][1] == b'\0'
    assert struct.unpack('<4i', attrs['dataWindow'][1]) == (0, 0, 20, 36)


def test_exr_layout():
    """Scanline single-part file: magic 20000630, version 2, name-sorted chlist,
    ZIP blocks of 16 lines with (y, size) chunk headers at the offsets."""
    import tempfile
    img = np.arange(2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3)
    with tempfile.NamedTemporaryFile(suffix='.exr') as fh:
        F.write_exr(fh.name, img, ['R', 'G', 'B'], compression='none')
        raw = open(fh.name, 'rb').read()
    assert struct.unpack_from('<ii', raw) == (20000630, 2)
    attrs, pos = F.read_exr_header(raw)
    chl = attrs['channels'][1]
    assert chl.split(b'\0')[0] == b'B'                # B, G, R order
    assert attrs['compression'] == ('compression', b'\0')
    off = struct.unpack_from('<2Q', raw, pos)
    y, size = struct.unpack_from('<ii', raw, off[1])
    assert (y, size) == (1, 36)
    assert np.frombuffer(raw, '<f4', 3, off[1] + 8).tolist() == img[1, :, 2].tolist()   # B of row 1


def test_exr_zip_predictor_and_rle_decode():
    raw = bytes(range(10)) + bytes([200] * 7)
    comp = F._zip_encode(raw)
    t = np.frombuffer(zlib.decompress(comp), np.uint8)
    inter = np.concatenate([np.frombuffer(raw, np.uint8)[0::2], np.frombuffer(raw, np.uint8)[1::2]])
    assert t[0] == inter[0] and all(int(t[i]) == (int(inter[i]) - int(inter[i - 1]) + 128) % 256
                                    for i in range(1, t.size))
    assert F._zip_decode(comp, len(raw)) == raw
    # RLE: encode the predicted stream by hand (run of 3 x 'a' -> count 2; 2 literals -> -2)
    pred = bytearray(t.tobytes())
    rle = bytes([256 - len(pred)]) + bytes(pred) if len(pred) <= 127 else None
    assert F._rle_decode(rle, len(raw)) == raw


def test_load_bitmap_detects_formats(tmp_path):
    rng = np.random.default_rng(4)
    img = rng.random((8, 16, 3), dtype=np.float32)
    F.write_pfm(str(tmp_path / 'e.pfm'), img)
    F.write_exr(str(tmp_path / 'e.exr'), img.astype(np.float16), ['R', 'G', 'B'])
    F.write_exr(str(tmp_path / 'y.exr'), img[:, :, :1], ['Y'])
    F.write_rgbe(str(tmp_path / 'e.hdr'), img)
    np.testing.assert_array_equal(F.load_bitmap(str(tmp_path / 'e.pfm')), img)
    np.testing.assert_array_equal(F.load_bitmap(str(tmp_path / 'e.exr')), img.astype(np.float16).astype(f32))
    np.testing.assert_array_equal(F.load_bitmap(str(tmp_path / 'y.exr')), np.repeat(img[:, :, :1], 3, 2))
    np.testing.assert_array_equal(F.load_bitmap(str(tmp_path / 'e.hdr')),
                                  F.rgbe_to_float(F.rgbe_from_float(img)))


def test_xml_film_properties(tmp_path):
    (tmp_path / 's.xml').write_text('''<scene version="0.6.0">
      <integrator type="path"/>
      <sensor type="perspective"><float name="fov" value="40"/>
        <sampler type="sobol"><integer name="sampleCount" value="4"/></sampler>
        <film type="hdrfilm"><integer name="width" value="32"/><integer name="height" value="24"/>
          <string name="pixelFormat" value="xyza"/><string name="componentFormat" value="float32"/>
          <boolean name="banner" value="false"/></film></sensor>
      <shape type="cube"/></scene>''')
    sc, it = xmlscene.load_scene(str(tmp_path / 's.xml'))
    assert it.film.pixel_format == 'xyza' and it.film.componentFormat == 'float32' and not it.film.banner
    assert it.hasAlpha
    xmlscene.save_scene(sc, it, str(tmp_path / 'out'))
    sc2, it2 = xmlscene.load_scene(str(tmp_path / 'out' / 'scene.xml'))
    assert (it2.film.pixel_format, it2.film.componentFormat, it2.film.banner) == ('xyza', 'float32', False)
    bad = (tmp_path / 's.xml').read_text().replace('xyza', 'spectrum')
    (tmp_path / 'b.xml').write_text(bad)
    with pytest.raises(xmlscene.SceneError, match='spectral'):
        xmlscene.load_scene(str(tmp_path / 'b.xml'))


# --- mfilm (src/films/mfilm.cpp) ---------------------------------------------
_MF_IMG = np.array([[[1, 4], [0.5, 0], [1e-5, 7]], [[2.25, 8], [123456, 9], [-3, 10]]], np.float32)   # (2, 3, 2)


def test_mfilm_matlab_text():
    """mfilm.cpp:278-318: `var = [` rows `, `-separated, `;\\n\\t` between rows,
    `];\\n` at the end, later channels as `\\nvar(:, :, c) = [`; %.{digits}g values."""
    t = F.mfilm_text(_MF_IMG[:, :, :1], 'matlab')
    assert t == 'data = [1, 0.5, 1e-05;\n\t2.25, 1.235e+05, -3];\n'
    t = F.mfilm_text(_MF_IMG, 'matlab', digits=2, variable='img')
    assert t == ('img = [1, 0.5, 1e-05;\n\t2.2, 1.2e+05, -3];\n'
                 '\nimg(:, :, 2) = [4, 0, 7;\n\t8, 9, 10];\n')


def test_mfilm_mathematica_text():
    """mfilm.cpp:285-330: nested braces, `Transpose[..., {3,1,2}]` for several
    channels, and the `*^` exponent notation."""
    t = F.mfilm_text(_MF_IMG[:, :, :1], 'mathematica')
    assert t == 'data = {{1, 0.5, 1*^-05},\n\t{2.25, 1.235*^+05, -3}};\n'
    t = F.mfilm_text(_MF_IMG, 'mathematica')
    assert t == ('data = Transpose[{{{1, 0.5, 1*^-05},\n\t{2.25, 1.235*^+05, -3}},\n\n\t{{'
                 '4, 0, 7},\n\t{8, 9, 10}}}, {3,1,2}];\n')


def test_mfilm_npy_header_is_cnpy():
    """cnpy::create_npy_header (cnpy.h:207-236): dict padded to 10 + len = 0 mod 16,
    a full extra 16 spaces when already aligned, and the array reads back."""
    h = F.npy_header((24, 32, 3))
    d = "{'descr': '<f4', 'fortran_order': False, 'shape': (24, 32, 3), }"
    assert h == b'\x93NUMPY\x01\x00' + struct.pack('<H', 70) + (d + ' ' * 5 + '\n').encode()
    h = F.npy_header((10000, 1000, 10))          # 10 + 70 already aligned -> 16 more
    assert len(h) == 10 + 86 and h.endswith(b' ' * 15 + b'\n')
    assert F.npy_header((5,))[10:].startswith(b"{'descr': '<f4', 'fortran_order': False, 'shape': (5,), }")


def test_mfilm_write_and_properties(tmp_path):
    mf = F.MFilm(fileFormat='numpy', pixelFormat='rgba')
    assert mf.hasAlpha and mf.componentFormat == 'float32' and mf.channel_names == ['R', 'G', 'B', 'A']
    img = np.random.default_rng(3).random((5, 7, 4), dtype=np.float32)
    p = mf.write(str(tmp_path / 'out.exr'), img)
    assert p.endswith('out.npy')
    assert np.array_equal(np.load(p), img)
    lum = F.MFilm(fileFormat='numpy')            # one channel -> 2D array (mfilm.cpp:343-344)
    p = lum.write(str(tmp_path / 'y.NPY'), img[:, :, :1])
    assert p.endswith('y.NPY') and np.load(p).shape == (5, 7)
    m = F.MFilm()
    assert (m.fileFormat, m.pixel_format, m.digits, m.variable) == ('matlab', 'luminance', 4, 'data')
    assert m.write(str(tmp_path / 'a.txt'), img[:, :, :1]).endswith('a.m')
    assert F.MFilm(fileFormat='mathematica').output_path('x.M') == 'x.M'
    with pytest.raises(ValueError, match='fileFormat'):
        F.MFilm(fileFormat='csv')
    with pytest.raises(ValueError, match='spectral'):
        F.MFilm(pixelFormat='spectrumAlpha')
    with pytest.raises(ValueError, match='pixelFormat'):
        F.MFilm(pixelFormat='bgr')


def test_xml_mfilm(tmp_path):
    """<film type="mfilm">: 1x1 default size (film.cpp:27-33), box filter by
    default (mfilm.cpp:156-165), its own properties, and a save/load round trip."""
    (tmp_path / 's.xml').write_text('''<scene version="0.6.0">
      <integrator type="path"/>
      <sensor type="perspective"><float name="fov" value="40"/>
        <sampler type="sobol"><integer name="sampleCount" value="4"/></sampler>
        <film type="mfilm"><string name="fileFormat" value="numpy"/><string name="pixelFormat" value="rgb"/>
          <integer name="digits" value="6"/><string name="variable" value="img"/></film></sensor>
      <shape type="cube"/></scene>''')
    sc, it = xmlscene.load_scene(str(tmp_path / 's.xml'))
    assert (sc.sensor.width, sc.sensor.height) == (1, 1)
    assert (it.rfilter, it.rfilterParam) == ('box', 0.5)
    assert isinstance(it.film, F.MFilm) and (it.film.fileFormat, it.film.pixel_format) == ('numpy', 'rgb')
    assert (it.film.digits, it.film.variable) == (6, 'img') and not it.hasAlpha
    xmlscene.save_scene(sc, it, str(tmp_path / 'out'))
    sc2, it2 = xmlscene.load_scene(str(tmp_path / 'out' / 'scene.xml'))
    assert isinstance(it2.film, F.MFilm)
    assert (it2.film.fileFormat, it2.film.pixel_format, it2.film.digits, it2.film.variable) == ('numpy', 'rgb', 6,
                                                                                                'img')
    bad = (tmp_path / 's.xml').read_text().replace('<film type="mfilm">',
                                                   '<film type="mfilm"><integer name="cropWidth" value="2"/>')
    (tmp_path / 'b.xml').write_text(bad)
    with pytest.raises(xmlscene.SceneError, match='crop window'):
        xmlscene.load_scene(str(tmp_path / 'b.xml'))
