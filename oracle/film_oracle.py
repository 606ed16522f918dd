"""TEST INFRASTRUCTURE: CPU restatement of HDRFilm::develop's conversion.

Only tests/ use this (the product develop is libmtsgpu's film_kernel.hip).
Follows Bitmap::convert -> FormatConverterImpl for a SpectrumAlphaWeight
source (src/libcore/fmtconv.cpp:955-1030) and convertScalar
(fmtconv.cpp:1137-1160), in float32 with the reference's operation order;
numpy float32 arithmetic is IEEE single precision without contraction.
"""
import numpy as np

f32 = np.float32
PIX = {'luminance': 0, 'luminancealpha': 1, 'rgb': 2, 'rgba': 3, 'xyz': 4, 'xyza': 5}


def _conv(v, comp, mult=f32(1)):
    v = (np.asarray(v, f32) * f32(mult)).astype(f32)
    if comp == 'float16':
        return v.astype(np.float16)                       # half(float): round to nearest even
    if comp == 'float32':
        return v
    m = f32(4294967295.0)                                 # (Float) numeric_limits<uint32_t>::max()
    r = (v * m).astype(f32) + f32(0.5)
    r = np.where(f32(0) < r, r, f32(0)).astype(f32)       # std::max((Float) 0, r)
    r = np.where(r < m, r, m).astype(f32)                 # std::min(max, r)
    return (r.astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)   # x86-64 cvttss2si (64-bit), low word


def develop_ref(film, border, pixel_format='rgb', component_format='float16', multiplier=1.0):
    """(H+2b, W+2b, 5) {R,G,B,alpha,weight} -> (H, W, C)."""
    with np.errstate(over='ignore', invalid='ignore', divide='ignore'):
        return _develop(film, border, pixel_format, component_format, multiplier)


def _develop(film, border, pixel_format, component_format, multiplier):
    b = int(border)
    f = np.asarray(film, f32)[b:film.shape[0] - b, b:film.shape[1] - b]
    s0, s1, s2, alpha, w = (f[..., i] for i in range(5))
    with np.errstate(divide='ignore', invalid='ignore'):
        inv = np.where(w != 0, f32(1) / w, w).astype(f32)
    mult = f32(multiplier)
    fmt = pixel_format.lower()
    out = []
    if fmt in ('luminance', 'luminancealpha'):
        lum = ((s0 * f32(0.212671)).astype(f32) + (s1 * f32(0.715160)).astype(f32)).astype(f32) \
            + (s2 * f32(0.072169)).astype(f32)
        out.append(_conv((lum.astype(f32) * inv).astype(f32), component_format, mult))
    elif fmt in ('rgb', 'rgba'):
        for s in (s0, s1, s2):
            out.append(_conv((s * inv).astype(f32), component_format, mult))
    elif fmt in ('xyz', 'xyza'):
        r, g, bb = (((s * inv).astype(f32) * mult).astype(f32) for s in (s0, s1, s2))
        for c0, c1, c2 in ((0.412453, 0.357580, 0.180423), (0.212671, 0.715160, 0.072169),
                           (0.019334, 0.119193, 0.950227)):
            v = ((r * f32(c0)).astype(f32) + (g * f32(c1)).astype(f32)).astype(f32) + (bb * f32(c2)).astype(f32)
            out.append(_conv(v.astype(f32), component_format))
    else:
        raise ValueError(pixel_format)
    if fmt in ('luminancealpha', 'rgba', 'xyza'):
        out.append(_conv((alpha * inv).astype(f32), component_format))
    return np.stack(out, -1)
