"""Oracle delta BSDFs (conductor, dielectric, plastic's coating) and the
quadrature behind plastic, checked against closed forms evaluated in float64.

* fresnelDiffuseReflectance (util.cpp:814-860) = the hemispherical average
  2 * int_0^1 F(cos) cos dcos, computed here with scipy's adaptive quadrature;
  the reference's own fast fits (util.cpp:822-853, quoted accurate to 0.1-0.6%)
  bound it independently.
* sample(): the mirror / Snell directions, pdf and weights of
  conductor.cpp:269-283, dielectric.cpp:277-333 and plastic.cpp:356-420.
"""
import ctypes as C

import numpy as np
import pytest
from scipy import integrate

from mitsuba_amd.scene import BSDF

E_DELTA_REFL, E_DELTA_TRANS, E_DIFF_REFL = 0x20, 0x40, 0x02


def _fresnel(cos_i, eta):
    """fresnelDielectricExt in float64 (util.cpp:651-677)."""
    if eta == 1:
        return 0.0, -cos_i
    scale = 1 / eta if cos_i > 0 else eta
    ct2 = 1 - (1 - cos_i * cos_i) * scale * scale
    if ct2 <= 0:
        return 1.0, 0.0
    ci, ct = abs(cos_i), np.sqrt(ct2)
    rs = (ci - eta * ct) / (ci + eta * ct)
    rp = (eta * ci - ct) / (eta * ci + ct)
    return 0.5 * (rs * rs + rp * rp), (-ct if cos_i > 0 else ct)


def _fast_fdr(eta):   # util.cpp:822-853
    if eta < 1:
        return -1.4399 * eta * eta + 0.7099 * eta + 0.6681 + 0.0636 / eta
    ie = 1 / eta
    return 0.919317 - 3.4793 * ie + 6.75335 * ie ** 2 - 7.80989 * ie ** 3 + 4.98554 * ie ** 4 - 1.36881 * ie ** 5


@pytest.mark.parametrize('eta', [1.49, 1 / 1.49, 1.5, 1 / 1.5, 1.33, 2.0, 1 / 1.6])
def test_fresnel_diffuse_reflectance(oracle, eta):
    L = oracle.lib()
    got = L.oracle_fresnel_diffuse_reflectance(eta)
    # int_0^1 F(sqrt(xi)) dxi, with the total-internal-reflection kink as a breakpoint
    pts = [1 - eta ** 2] if eta < 1 else None
    exact = integrate.quad(lambda xi: _fresnel(np.sqrt(xi), eta)[0], 0, 1, points=pts, epsabs=1e-12, limit=200)[0]
    assert abs(got - exact) <= 5e-5 * exact, (eta, got, exact)   # relError 1e-5, float arithmetic
    assert abs(got - _fast_fdr(eta)) <= 0.01 * exact, (eta, got, _fast_fdr(eta))


def _sample(L, b, wi, u):
    d = b.to_desc()
    f3 = C.c_float * 3
    wo, w, pdf, eta = f3(), f3(), C.c_float(), C.c_float()
    t = L.oracle_bsdf_sample(C.byref(d), f3(*wi), f3(*u), wo, w, C.byref(pdf), C.byref(eta), 0)
    return np.array(wo[:]), np.array(w[:]), pdf.value, eta.value, t


def _wi(ct, phi=0.7):
    s = np.sqrt(1 - ct * ct)
    return [s * np.cos(phi), s * np.sin(phi), ct]


def _conductor_f(ct, eta, k):
    """fresnelConductorExact in float64 (util.cpp:739-761)."""
    ct2 = ct * ct
    st2 = 1 - ct2
    t1 = eta * eta - k * k - st2
    a2pb2 = np.sqrt(t1 * t1 + 4 * k * k * eta * eta)
    a = np.sqrt(0.5 * (a2pb2 + t1))
    term1, term2 = a2pb2 + ct2, 2 * a * ct
    rs2 = (term1 - term2) / (term1 + term2)
    term3, term4 = a2pb2 * ct2 + st2 * st2, term2 * st2
    rp2 = rs2 * (term3 - term4) / (term3 + term4)
    return 0.5 * (rp2 + rs2)


def test_conductor_mirror(oracle):
    L = oracle.lib()
    eta, k = np.array([0.2, 0.9, 1.1]), np.array([3.9, 2.4, 2.1])
    b = BSDF('conductor', material=None, eta=tuple(eta), k=tuple(k), specularReflectance=(0.9, 0.8, 0.7))
    for ct in (0.95, 0.5, 0.1):
        wi = _wi(ct)
        wo, w, pdf, e, t = _sample(L, b, wi, (0.3, 0.6, 0.0))
        assert t == E_DELTA_REFL and pdf == 1.0 and e == 1.0
        np.testing.assert_allclose(wo, [-wi[0], -wi[1], wi[2]], rtol=0, atol=1e-7)
        np.testing.assert_allclose(w, np.array([0.9, 0.8, 0.7]) * _conductor_f(ct, eta / 1.000277, k / 1.000277),
                                   rtol=2e-5)
    assert _sample(L, b, _wi(0.5) * np.array([1, 1, -1]), (0.3, 0.6, 0))[4] == 0   # below the surface


@pytest.mark.parametrize('ct', [0.9, 0.4, -0.3, -0.9])
def test_dielectric_snell(oracle, ct):
    L = oracle.lib()
    eta = 1.5 / 1.000277
    b = BSDF('dielectric', intIOR=1.5, specularTransmittance=(0.9, 0.8, 0.7))
    wi = _wi(ct)
    F, ctt = _fresnel(ct, eta)
    # sample.x <= F: reflection with pdf F and weight specularReflectance
    if F > 1e-3:
        wo, w, pdf, e, t = _sample(L, b, wi, (F * 0.5, 0.5, 0))
        assert t == E_DELTA_REFL and e == 1.0
        np.testing.assert_allclose(pdf, F, rtol=1e-5)
        np.testing.assert_allclose(w, [1, 1, 1], rtol=0)
        np.testing.assert_allclose(wo, [-wi[0], -wi[1], wi[2]], atol=1e-7)
    if F < 1:
        wo, w, pdf, e, t = _sample(L, b, wi, ((1 + F) * 0.5, 0.5, 0))
        assert t == E_DELTA_TRANS
        np.testing.assert_allclose(pdf, 1 - F, rtol=1e-5)
        np.testing.assert_allclose(wo[2], ctt, rtol=1e-5)
        # Snell: sin_t = sin_i / eta_rel, tangential direction reversed
        eta_rel = eta if ct > 0 else 1 / eta
        np.testing.assert_allclose(wo[:2], -np.array(wi[:2]) / eta_rel, rtol=1e-5)
        np.testing.assert_allclose(np.linalg.norm(wo), 1.0, rtol=1e-5)
        np.testing.assert_allclose(e, eta if ctt < 0 else 1 / eta, rtol=1e-6)
        factor = 1 / eta if ctt < 0 else eta                       # radiance scaling (dielectric.cpp:303-307)
        np.testing.assert_allclose(w, np.array([0.9, 0.8, 0.7]) * factor * factor, rtol=1e-5)


def test_dielectric_total_internal_reflection(oracle):
    L = oracle.lib()
    b = BSDF('dielectric', intIOR=1.5)
    wi = _wi(-0.2)                                  # inside, beyond the critical angle
    for x in (0.01, 0.99):
        wo, w, pdf, e, t = _sample(L, b, wi, (x, 0.5, 0))
        assert t == E_DELTA_REFL and pdf == 1.0


def test_plastic_lobe_choice(oracle):
    L = oracle.lib()
    dr, sr = np.array([0.3, 0.5, 0.7]), np.array([1.0, 1.0, 1.0])
    b = BSDF('plastic', diffuseReflectance=tuple(dr))
    eta = 1.49 / 1.000277
    lum = lambda s: s[0] * 0.212671 + s[1] * 0.715160 + s[2] * 0.072169
    sw = lum(sr) / (lum(dr) + lum(sr))
    for ct in (0.9, 0.3):
        wi = _wi(ct)
        Fi = _fresnel(ct, eta)[0]
        ps = Fi * sw / (Fi * sw + (1 - Fi) * (1 - sw))
        wo, w, pdf, e, t = _sample(L, b, wi, (ps * 0.5, 0.5, 0))
        assert t == E_DELTA_REFL
        np.testing.assert_allclose(pdf, ps, rtol=1e-5)
        np.testing.assert_allclose(w, sr * Fi / ps, rtol=1e-5)
        np.testing.assert_allclose(wo, [-wi[0], -wi[1], wi[2]], atol=1e-7)
        wo, w, pdf, e, t = _sample(L, b, wi, ((1 + ps) * 0.5, 0.25, 0))
        assert t == E_DIFF_REFL and wo[2] > 0
        np.testing.assert_allclose(pdf, (1 - ps) * wo[2] / np.pi, rtol=1e-5)
    assert _sample(L, b, _wi(-0.5), (0.5, 0.5, 0))[4] == 0
