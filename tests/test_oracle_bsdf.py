"""Oracle BSDFs against the reference's own acceptance criteria
(src/tests/test_chisquare.cpp:94-215): sample() weights consistent with
eval()/pdf() (relative/absolute error 1e-2 in single precision, :33-37), and a
chi-square goodness-of-fit of sampled directions against the integrated pdf
(significance 0.25% per test, :27-31)."""
import ctypes as C
import os

import numpy as np
import pytest
from scipy import stats

from mitsuba_amd.scene import BSDF, Checkerboard

# roughplastic reads data/microfacet/<distribution>.dat: the reference's own
# files when this container has them, else the in-tree generated tables
REF_MICROFACET = '/root/reference/data/microfacet'
RT_DIR = REF_MICROFACET if os.path.isdir(REF_MICROFACET) else None

ERROR_REQ = 1e-2
CASES = {
    'diffuse': BSDF('diffuse', reflectance=(0.5, 0.6, 0.7)),
    'rc_beckmann': BSDF('roughconductor', distribution='beckmann', alpha=0.3, eta=(0.2, 0.9, 1.1), k=(3.9, 2.4, 2.1)),
    'rc_ggx': BSDF('roughconductor', distribution='ggx', alpha=0.2, eta=(0.2, 0.9, 1.1), k=(3.9, 2.4, 2.1)),
    'rc_ggx_all': BSDF('roughconductor', distribution='ggx', alpha=0.4, sampleVisible=False, material='none'),
    'rc_phong': BSDF('roughconductor', distribution='phong', alpha=0.3, material='none'),
    'rc_ggx_aniso': BSDF('roughconductor', distribution='ggx', alphaU=0.1, alphaV=0.4, material='none'),
    'rd_beckmann': BSDF('roughdielectric', distribution='beckmann', alpha=0.3, intIOR=1.5),
    'rd_ggx': BSDF('roughdielectric', distribution='ggx', alpha=0.2, intIOR=1.33),
    'rd_ggx_all': BSDF('roughdielectric', distribution='ggx', alpha=0.5, sampleVisible=False, intIOR=1.5),
    # data/tests/test_bsdf.xml:131-136: roughplastic, beckmann, alpha .7
    'rp_beckmann': BSDF('roughplastic', distribution='beckmann', alpha=0.7, rtransDir=RT_DIR),
    'rp_ggx': BSDF('roughplastic', distribution='ggx', alpha=0.2, diffuseReflectance=(0.2, 0.5, 0.8),
                   rtransDir=RT_DIR),
    'rp_phong_nonlinear': BSDF('roughplastic', distribution='phong', alpha=0.3, nonlinear=True, rtransDir=RT_DIR),
    'rp_ggx_all_tex': BSDF('roughplastic', distribution='ggx', sampleVisible=False, rtransDir=RT_DIR,
                           alpha=Checkerboard(color0=0.25, color1=0.05)),   # uv (0,0) -> color0
    # smooth plastic: the diffuse lobe is checked here, its delta coating in test_oracle_smooth.py
    'plastic': BSDF('plastic', diffuseReflectance=(0.3, 0.5, 0.7)),
    'plastic_nonlinear': BSDF('plastic', intIOR=1.6, nonlinear=True, diffuseReflectance=(0.8, 0.4, 0.1)),
}
DELTA = 0x20 | 0x40   # EDeltaReflection | EDeltaTransmission: no density w.r.t. solid angle


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def _sample(L, d, wi, u):
    wo, w, pdf, eta = (C.c_float * 3)(), (C.c_float * 3)(), C.c_float(), C.c_float()
    t = L.oracle_bsdf_sample(C.byref(d), _f3(wi), _f3(u), wo, w, C.byref(pdf), C.byref(eta), 0)
    return np.array(wo[:], np.float32), np.array(w[:], np.float32), pdf.value, t


def _eval(L, d, wi, wo):
    v, pdf = (C.c_float * 3)(), C.c_float()
    L.oracle_bsdf_eval(C.byref(d), _f3(wi), _f3(wo), v, C.byref(pdf), 0)
    return np.array(v[:], np.float32), pdf.value


def _wi(cos_theta, phi=0.3):
    s = np.sqrt(max(0.0, 1 - cos_theta * cos_theta))
    return np.array([s * np.cos(phi), s * np.sin(phi), cos_theta], np.float32)


@pytest.mark.parametrize('name', sorted(CASES))
def test_sample_weight_matches_eval_over_pdf(oracle, name):
    L = oracle.lib()
    d = CASES[name].to_desc()
    rng = np.random.default_rng(7)
    cosines = [0.9, 0.5, 0.15] + ([-0.6] if name.startswith('rd') else [])
    checked = 0
    for ct in cosines:
        wi = _wi(ct)
        for _ in range(400):
            u = rng.random(3).astype(np.float32)
            wo, w, pdf, t = _sample(L, d, wi, u)
            if not np.any(w) or t & DELTA:
                continue
            f, p = _eval(L, d, wi, wo)
            assert p > 0 and np.isfinite(w).all()
            manual = f / np.float32(p)
            for a, c in zip(w, manual):
                mn, err = min(a, c), abs(a - c)
                bad = (err > ERROR_REQ) if mn < ERROR_REQ else (err / mn > ERROR_REQ)
                assert not bad, (name, ct, u, w, manual)
            checked += 1
    assert checked > 300


def _chi2(L, d, wi, n=40000, nt=16, nphi=32, seed=3, both=False, k=8):
    rng = np.random.default_rng(seed)
    lo = -1.0 if both else 0.0
    obs = np.zeros((nt, nphi))
    for _ in range(n):
        wo, w, pdf, t = _sample(L, d, wi, rng.random(3).astype(np.float32))
        if not np.any(w) or t & DELTA:
            continue
        ct = float(np.clip(wo[2], -1, 1))
        ph = float(np.arctan2(wo[1], wo[0])) % (2 * np.pi)
        i = min(nt - 1, int((ct - lo) / (1 - lo) * nt))
        j = min(nphi - 1, int(ph / (2 * np.pi) * nphi))
        if ct >= lo:
            obs[i, j] += 1
    exp = np.zeros_like(obs)
    for i in range(nt):
        for j in range(nphi):
            acc = 0.0
            for a in range(k):
                ct = lo + (i + (a + 0.5) / k) * (1 - lo) / nt
                st = np.sqrt(max(0.0, 1 - ct * ct))
                for b in range(k):
                    ph = (j + (b + 0.5) / k) * 2 * np.pi / nphi
                    f, p = _eval(L, d, wi, np.array([st * np.cos(ph), st * np.sin(ph), ct], np.float32))
                    # roughdielectric's pdf() (roughdielectric.cpp:350-430) omits eval()'s side tests
                    # (:296-300), so it also covers directions sample() never produces: integrate
                    # the density over the directions eval() accepts
                    acc += p if np.any(f) else 0.0
            exp[i, j] = acc / (k * k) * ((1 - lo) / nt) * (2 * np.pi / nphi) * n
    # pool cells with small expectation (chisquare.cpp pools below 5)
    o, e = obs.ravel(), exp.ravel()
    order = np.argsort(e)
    po, pe, acc_o, acc_e = [], [], 0.0, 0.0
    for idx in order:
        acc_o += o[idx]
        acc_e += e[idx]
        if acc_e >= 5:
            po.append(acc_o); pe.append(acc_e); acc_o = acc_e = 0.0
    if acc_e > 0 and pe:
        po[-1] += acc_o; pe[-1] += acc_e
    po, pe = np.array(po), np.array(pe)
    pe *= po.sum() / pe.sum()   # compare shapes (samples rejected below the horizon are not binned)
    chi2 = float(((po - pe) ** 2 / pe).sum())
    return stats.chi2.sf(chi2, len(po) - 1), obs.sum() / n


@pytest.mark.parametrize('name', ['diffuse', 'rc_beckmann', 'rc_ggx', 'rc_ggx_all', 'rc_ggx_aniso', 'rd_ggx',
                                  'rp_beckmann', 'rp_ggx', 'rp_phong_nonlinear', 'rp_ggx_all_tex', 'plastic'])
def test_chi_square_goodness_of_fit(oracle, name):
    L = oracle.lib()
    d = CASES[name].to_desc()
    p, frac = _chi2(L, d, _wi(0.7), n=20000, both=name.startswith('rd'))
    assert p > 0.0025, (name, p)
    assert frac > (0.3 if name == 'plastic' else 0.5)
