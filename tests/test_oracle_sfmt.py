"""SFMT19937 and the reference's render order in the oracle.

* The generator is pinned by the reference's own known-answer vector:
  Random(4321)::nextULong, src/tests/test_random.cpp:433-508
  (tests/golden/sfmt19937_kat.json, extracted by make_sfmt_golden.py).
* The replay order -- BlockedImageProcess's spiral over 32x32 blocks
  (imageproc.cpp:28-80) and HilbertCurve2D<uint8_t> within each block
  (sfcurve.h) -- is checked against an independent Python restatement.
* The replay samplers ('independent-sfmt': the one-worker stream of
  `mitsuba -p 1`; 'independent-sfmt-blocks': one clone per block) are
  deterministic and estimate the same image as sobol within Monte-Carlo error."""
import json
import math
import os

import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.scene import PathIntegrator

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden', 'sfmt19937_kat.json')


def test_sfmt_known_answer(oracle):
    kat = json.load(open(GOLDEN))
    ref = np.array([int(v, 16) for v in kat['next_ulong']], np.uint64)
    assert kat['seed'] == 4321 and ref.size == 192
    got = oracle.sfmt_u64(kat['seed'], ref.size)
    assert np.array_equal(got, ref)


def test_sfmt_crosses_state_refills(oracle):
    """Several gen_rand_all refills (312 outputs each): the stream stays a valid
    uniform 64-bit sequence (bit balance) and differs between seeds."""
    a = oracle.sfmt_u64(5489, 4000)
    b = oracle.sfmt_u64(5490, 4000)
    assert not np.array_equal(a, b)
    bits = np.unpackbits(a.view(np.uint8)).mean()
    assert abs(bits - 0.5) < 0.01


def _spiral(nbx, nby):
    """BlockedImageProcess::generateWork (imageproc.cpp:43-80)."""
    cx, cy, d, left, steps = nbx // 2, nby // 2, 0, 1, 1
    out = []
    for k in range(nbx * nby):
        out.append((cx, cy))
        if k + 1 == nbx * nby:
            break
        while True:
            if d == 0:
                cx += 1
            elif d == 1:
                cy += 1
            elif d == 2:
                cx -= 1
            else:
                cy -= 1
            left -= 1
            if left == 0:
                d = (d + 1) % 4
                if d in (0, 2):
                    steps += 1
                left = steps
            if 0 <= cx < nbx and 0 <= cy < nby:
                break
    return out


def _hilbert(w, h):
    """HilbertCurve2D<uint8_t>::initialize / generate (sfcurve.h), uint8 wrap-around."""
    order = math.ceil(np.float32(1.0 / np.float32(math.log(2.0))) * np.float32(math.log(float(max(w, h)))))
    pos = [0, 0]
    pts = []

    def move(d):
        if d == 0:
            pos[1] = (pos[1] - 1) & 255
        elif d == 1:
            pos[0] = (pos[0] + 1) & 255
        elif d == 2:
            pos[1] = (pos[1] + 1) & 255
        else:
            pos[0] = (pos[0] - 1) & 255

    def gen(o, front, right, back, left):
        if o == 0:
            if pos[0] < w and pos[1] < h:
                pts.append(tuple(pos))
            return
        gen(o - 1, left, back, right, front)
        move(right)
        gen(o - 1, front, right, back, left)
        move(back)
        gen(o - 1, front, right, back, left)
        move(left)
        gen(o - 1, right, front, left, back)

    gen(order, 0, 1, 2, 3)
    return pts


@pytest.mark.parametrize('size', [(64, 48), (100, 37), (33, 95), (1280, 720)])
def test_render_order_matches_restatement(oracle, size):
    W, H = size
    pts, bs = oracle.render_order(W, H)
    nbx, nby = -(-W // 32), -(-H // 32)
    exp = []
    starts = [0]
    for bx, by in _spiral(nbx, nby):
        bw, bh = min(32, W - bx * 32), min(32, H - by * 32)
        exp += [(bx * 32 + x, by * 32 + y) for x, y in _hilbert(bw, bh)]
        starts.append(len(exp))
    assert np.array_equal(pts, np.array(exp, np.int32))
    assert np.array_equal(bs, np.array(starts, np.int32))
    # every pixel of the crop exactly once
    assert len({tuple(p) for p in pts.tolist()}) == W * H


def test_hilbert_full_block_is_a_path(oracle):
    pts, bs = oracle.render_order(32, 32)
    d = np.abs(np.diff(pts, axis=0)).sum(1)
    assert np.all(d == 1)   # consecutive Hilbert points are 4-neighbours


def test_sfmt_replay_deterministic_and_unbiased(oracle):
    sc, _ = scenes.build('C1', width=48, height=40, spp=8, materials='rough')
    imgs = {}
    for name in ('independent-sfmt', 'independent-sfmt-blocks', 'sobol'):
        it = PathIntegrator(sampleCount=8, rfilter='box', sampler=name)
        f1, s1, st = oracle.render(sc, it, samples=True, threads=8)
        if name != 'sobol':
            f2, s2, _ = oracle.render(sc, it, samples=True, threads=3)
            assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32)), name   # thread-count independent
        assert st['samples'] == 48 * 40 * 8
        imgs[name] = s1[:, :3].astype(np.float64)
    # the two SFMT variants share no draws after the first block, but estimate the same image
    for name in ('independent-sfmt', 'independent-sfmt-blocks'):
        m, ms = imgs[name].mean(0), imgs['sobol'].mean(0)
        err = imgs[name].std(0) / math.sqrt(imgs[name].shape[0])
        assert np.all(np.abs(m - ms) < 5 * err + 1e-6), (name, m, ms, err)
    # the replay streams are not the counter-based ones
    it = PathIntegrator(sampleCount=8, rfilter='box', sampler='independent')
    _, si, _ = oracle.render(sc, it, samples=True, threads=8)
    it = PathIntegrator(sampleCount=8, rfilter='box', sampler='independent-sfmt')
    _, sr, _ = oracle.render(sc, it, samples=True, threads=8)
    assert not np.array_equal(si[:, 4:6], sr[:, 4:6])


def _next_float(u64):
    """Random::nextFloat (random.cpp:630-639) of one nextULong output."""
    b = ((np.uint32(u64 & np.uint64(0xFFFFFFFF)) >> np.uint32(9)) | np.uint32(0x3f800000))
    return np.float32(np.array([b], np.uint32).view(np.float32)[0] - np.float32(1.0))


@pytest.mark.parametrize('sampler,block', [('independent-sfmt', 0), ('independent-sfmt-blocks', 0),
                                           ('independent-sfmt-blocks', 3)])
def test_sfmt_replay_block_head_is_the_clone_head(oracle, sampler, block):
    """The first pixel of a block takes its worker clone's next two nextFloat draws
    as its image-plane offset (integrator.cpp:170-176): for the one-worker replay
    and block 0 the first clone's stream head, for block k of the per-block
    replay the (k+1)-th clone's."""
    sc, _ = scenes.build('C1', width=96, height=64, spp=1)
    it = PathIntegrator(sampleCount=1, rfilter='box', sampler=sampler)
    _, smp, _ = oracle.render(sc, it, samples=True, threads=4)
    pts, bs = oracle.render_order(96, 64)
    x0, y0 = pts[bs[block]]
    rec = smp[y0 * 96 + x0]
    head = oracle.sfmt_u64(5489, 2, clone=block + 1)
    assert rec[4] == np.float32(x0) + _next_float(head[0])
    assert rec[5] == np.float32(y0) + _next_float(head[1])


def test_replay_rejects_row_shards_and_arrays(oracle):
    from mitsuba_amd.scene import DirectIntegrator
    sc, _ = scenes.build('C1', width=32, height=32, spp=2)
    it = PathIntegrator(sampleCount=2, rfilter='box', sampler='independent-sfmt')
    with pytest.raises(RuntimeError):
        oracle.render(sc, it, row=(8, 2, 0))
    d = DirectIntegrator(sampleCount=2, rfilter='box', sampler='independent-sfmt', emitterSamples=2)
    with pytest.raises(RuntimeError):
        oracle.render(sc, d)
