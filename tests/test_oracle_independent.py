"""The `independent` sampler (src/samplers/independent.cpp) in the oracle.

The reference draws every value from one SFMT19937 generator per worker
thread, so which value a sample gets depends on the block schedule: its
renders are not reproducible across thread counts.  Here each
(pixel, sample) owns a counter-based stream (include/mtsgpu.h,
MTSGPU_SAMPLER_INDEPENDENT).  Parity with the reference is statistical and
these tests pin it that way: the stream (restated below in numpy) is uniform
on [0, 1) with Random::nextFloat's 2^-23 grid (random.cpp:630-639), and the
image it renders agrees with the Sobol render within Monte-Carlo error.  The
GPU reproduces the oracle bit for bit (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from mitsuba_amd import scenes, xmlscene
from mitsuba_amd.scene import DirectIntegrator, PathIntegrator

M64 = (1 << 64) - 1


def _mix64(z):
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _key(px, py, frame):
    return _mix64(((px << 48) | (py << 32) | frame) ^ 0x6A09E667F3BCC909)


def _value(key, dim):
    u = _mix64((key + (dim + 1) * 0x9E3779B97F4A7C15) & M64) & 0xFFFFFFFF
    return np.float32(np.uint32((u >> 9) | 0x3F800000).view(np.float32) - np.float32(1))


def test_independent_pixel_jitter_is_the_stream(oracle):
    """renderBlock's samplePos = offset + next2D() (integrator.cpp:175-178) takes
    dims 0 and 1 of the sample's stream."""
    sc, _ = scenes.build('C1', width=8, height=6, spp=4)
    it = PathIntegrator(sampleCount=4, rfilter='box', sampler='independent')
    _, smp, _ = oracle.render(sc, it, samples=True)
    for pi in range(0, 48, 5):
        px, py = pi % 8, pi // 8
        for j in range(4):
            rec = smp[pi * 4 + j]
            k = _key(px, py, j)
            assert rec[4] == np.float32(np.float32(px) + _value(k, 0))
            assert rec[5] == np.float32(np.float32(py) + _value(k, 1))


def test_independent_stream_uniform():
    """Uniform on [0, 1) on the 2^-23 grid; no correlation between dims or samples."""
    from scipy import stats
    keys = [_key(x, y, j) for x in range(16) for y in range(16) for j in range(8)]
    v = np.array([[_value(k, d) for d in range(4)] for k in keys], np.float64)
    assert v.min() >= 0 and v.max() < 1
    assert np.all(np.float32(v * 2 ** 23) == np.round(v * 2 ** 23))
    for d in range(4):
        assert stats.kstest(v[:, d], 'uniform').pvalue > 1e-3
    c = np.corrcoef(v.T)
    assert np.all(np.abs(c[np.triu_indices(4, 1)]) < 0.05)
    assert abs(np.corrcoef(v[:-1, 0], v[1:, 0])[0, 1]) < 0.05


@pytest.mark.parametrize('integ', ['path', 'direct'])
def test_independent_render_matches_sobol_statistically(oracle, integ):
    """Same scene, same spp: the independent and Sobol images estimate the same
    radiance; their per-pixel difference is Monte-Carlo noise only."""
    sc, _ = scenes.build('C1', width=24, height=24, spp=64, materials='rough')
    mk = (lambda s: PathIntegrator(sampleCount=64, rfilter='box', sampler=s)) if integ == 'path' else \
        (lambda s: DirectIntegrator(sampleCount=64, rfilter='box', sampler=s, emitterSamples=2, bsdfSamples=2))
    _, s_i, _ = oracle.render(sc, mk('independent'), samples=True, threads=8)
    _, s_s, _ = oracle.render(sc, mk('sobol'), samples=True, threads=8)
    # per-pixel means and standard errors of both estimates from their own samples
    Li, Ls = s_i[:, :3].reshape(24 * 24, 64, 3), s_s[:, :3].reshape(24 * 24, 64, 3)
    se = np.sqrt(Li.var(axis=1) / 64 + Ls.var(axis=1) / 64)
    z = (Li.mean(axis=1) - Ls.mean(axis=1)) / np.maximum(se, 1e-3)
    assert np.mean(np.abs(z) < 4) > 0.99
    gi, gs = Li.reshape(-1, 3), Ls.reshape(-1, 3)
    assert np.all(np.abs(gi.mean(0) - gs.mean(0)) < 4 * np.sqrt((gi.var(0) + gs.var(0)) / len(gi)))


def test_xml_independent_sampler(tmp_path):
    """No <sampler>: independent with 4 spp (sensor.cpp:92-97); explicit
    <sampler type="independent">; save/load round trip."""
    body = '''<scene version="0.6.0"><integrator type="path"/>
      <sensor type="perspective"><float name="fov" value="40"/>%s
        <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
      <shape type="cube"/></scene>'''
    (tmp_path / 'a.xml').write_text(body % '')
    _, it = xmlscene.load_scene(str(tmp_path / 'a.xml'))
    assert (it.sampler, it.sampleCount) == ('independent', 4)
    (tmp_path / 'b.xml').write_text(body % '<sampler type="independent"><integer name="sampleCount" value="16"/>'
                                          '</sampler>')
    sc, it = xmlscene.load_scene(str(tmp_path / 'b.xml'))
    assert (it.sampler, it.sampleCount) == ('independent', 16)
    xmlscene.save_scene(sc, it, str(tmp_path / 'out'))
    _, it2 = xmlscene.load_scene(str(tmp_path / 'out' / 'scene.xml'))
    assert (it2.sampler, it2.sampleCount) == ('independent', 16)
    (tmp_path / 'c.xml').write_text(body % '<sampler type="halton"/>')
    with pytest.raises(NotImplementedError, match='halton'):
        xmlscene.load_scene(str(tmp_path / 'c.xml'))
    with pytest.raises(ValueError, match='sampler'):
        PathIntegrator(sampler='stratified')
