"""The plugin shim (integration/gpupath.cpp) dispatches on class-name and
plugin-name string literals.  It cannot be compiled here (boost is absent), so
this test checks every such literal against what the reference registers:

- a literal compared with ``getClass()->getName()`` (or a variable holding it)
  must name a concrete class the reference declares with
  ``MTS_IMPLEMENT_CLASS[_S](Name, false, Parent)`` -- an abstract class such as
  ``PerspectiveCamera`` (``src/librender/sensor.cpp:319``) is never the runtime
  class of a plugin object, so comparing against it rejects every object;
- ``MTS_CLASS(X)`` must name a registered class;
- plugin names (``getPluginName()``, the CPU integrator behind ``Li``) must be
  plugins the reference builds (``src/**/<name>.cpp``).

Needs ``/root/reference`` (the CPU container); skipped elsewhere.
"""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = '/root/reference'
SHIM = os.path.join(REPO, 'integration', 'gpupath.cpp')

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, 'src')),
                                reason='reference sources not present')


def _registry():
    """{class name: abstract?} from every MTS_IMPLEMENT_CLASS[_S] in the reference."""
    reg = {}
    pat = re.compile(r'MTS_IMPLEMENT_CLASS(?:_S)?\(\s*(\w+)\s*,\s*(true|false)\s*,')
    for root in ('src', 'include'):
        for dp, _, fns in os.walk(os.path.join(REF, root)):
            for fn in fns:
                if not fn.endswith(('.cpp', '.h', '.inl')):
                    continue
                with open(os.path.join(dp, fn), errors='replace') as f:
                    for m in pat.finditer(f.read()):
                        reg[m.group(1)] = reg.get(m.group(1), True) and m.group(2) == 'true'
    return reg


def _plugins():
    names = set()
    for dp, _, fns in os.walk(os.path.join(REF, 'src')):
        for fn in fns:
            if fn.endswith('.cpp'):
                names.add(fn[:-4])
    return names


def _shim():
    with open(SHIM) as f:
        src = f.read()
    # drop comments so prose does not count as code
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return re.sub(r'//[^\n]*', '', src)


def _class_name_vars(src):
    """Variables initialised from getClass()->getName()."""
    return set(re.findall(r'std::string\s+(\w+)\s*=\s*[\w>.()-]*getClass\(\)->getName\(\)', src))


def _compared_literals(src, lhs_pattern):
    out = []
    for m in re.finditer(r'(?:' + lhs_pattern + r')\s*(?:==|!=)\s*"([^"]*)"', src):
        out.append(m.group(1))
    return out


def test_class_name_literals_are_concrete_reference_classes():
    src = _shim()
    reg = _registry()
    assert reg.get('PerspectiveCamera') is True            # abstract (sensor.cpp:319)
    assert reg.get('PerspectiveCameraImpl') is False       # the 'perspective' plugin (perspective.cpp:474)
    vars_ = _class_name_vars(src)
    assert {'cls', 'smpName', 'rfName'} <= vars_, vars_
    lits = _compared_literals(src, r'getClass\(\)->getName\(\)|\b(?:' + '|'.join(sorted(vars_)) + r')\b')
    assert len(lits) >= 10, lits
    bad = [n for n in lits if reg.get(n) is not False]
    assert not bad, 'literals naming no concrete reference class: %s' % bad


def test_mts_class_arguments_are_registered():
    src = _shim()
    reg = _registry()
    names = re.findall(r'MTS_CLASS\((\w+)\)', src)
    assert 'PerspectiveCamera' in names
    assert all(n in reg for n in names), [n for n in names if n not in reg]


def test_plugin_name_literals_are_reference_plugins():
    src = _shim()
    plugins = _plugins()
    lits = _compared_literals(src, r'\bname\b|getPluginName\(\)|std::string\(n\.plugin\)')
    assert {'diffuse', 'roughconductor', 'roughdielectric', 'roughplastic', 'twosided', 'checkerboard'} <= set(lits)
    cpu = re.search(r'cpuPluginName\(\)\s*\{(.*?)\}', src, flags=re.S).group(1)
    lits += re.findall(r'"(\w+)"', cpu)
    bad = [n for n in lits if n not in plugins]
    assert not bad, 'plugin names the reference does not build: %s' % bad


def test_detector_would_catch_the_abstract_sensor_name():
    """The round-2 shim compared the sensor against "PerspectiveCamera"."""
    reg = _registry()
    old = 'if (sensor->getClass()->getName() != "PerspectiveCamera")'
    lits = _compared_literals(old, r'getClass\(\)->getName\(\)')
    assert lits == ['PerspectiveCamera'] and reg[lits[0]] is not False
