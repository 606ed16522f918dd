"""Named conductor IORs (roughconductor `material`, roughconductor.cpp:172-190)."""
import numpy as np
import pytest

from mitsuba_amd.conductors import conductor_rgb, materials
from mitsuba_amd.scene import BSDF


def test_table_covers_reference_materials():
    names = materials()
    assert len(names) >= 70 and {'Cu', 'Au', 'Ag', 'Al', 'Cr', 'W'} <= set(names)
    for n in names:
        eta, k = conductor_rgb(n)
        assert np.all(np.isfinite(eta)) and np.all(np.isfinite(k)), n


def test_copper_is_plausible():
    """RGB Cu as commonly quoted for RGB renderers (within a few percent: the
    reference integrates its own .spd tables against CIE 1931)."""
    eta, k = conductor_rgb('Cu')
    np.testing.assert_allclose(eta, (0.2004, 0.9240, 1.1022), rtol=0.05)
    np.testing.assert_allclose(k, (3.9129, 2.4528, 2.1422), rtol=0.05)
    # values are exact float32
    assert all(float(np.float32(v)) == v for v in eta + k)


def test_material_defaults_and_overrides():
    d = BSDF('roughconductor').to_desc()                 # default material = Cu
    eta, k = conductor_rgb('Cu')
    np.testing.assert_array_equal(list(d.eta), np.float32(eta))
    np.testing.assert_array_equal(list(d.k), np.float32(k))
    d = BSDF('roughconductor', material='none').to_desc()
    assert list(d.eta) == [0, 0, 0] and list(d.k) == [1, 1, 1]
    d = BSDF('roughconductor', material='Au', eta=(1.0, 2.0, 3.0)).to_desc()   # explicit eta wins, k from Au
    assert list(d.eta) == [1, 2, 3]
    np.testing.assert_array_equal(list(d.k), np.float32(conductor_rgb('Au')[1]))
    with pytest.raises(ValueError):
        BSDF('roughconductor', material='Unobtainium').to_desc()
