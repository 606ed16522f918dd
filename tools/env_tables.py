"""Fetch environment-emitter tables from the product library (host configure,
no GPU) or from the oracle, for CPU-side comparison (tests/test_host_configure.py)."""
import ctypes as C

import numpy as np


def env_tables(fn, scene):
    d = scene.desc()
    env = next(e for e in scene.emitters if e.type == 'envmap')
    h, w = env.bitmap.shape[:2]
    params = np.zeros(64, np.float32)
    rc = fn(C.byref(d), params.ctypes.data_as(C.POINTER(C.c_float)), None, 0, None, None, None)
    if rc != 0:
        raise RuntimeError('env tables rc=%d' % rc)
    total = int(params[11])
    tex = np.zeros(4 * total, np.uint16)
    rows = np.zeros(h + 1, np.float32)
    cols = np.zeros(h * (w + 1), np.float32)
    wts = np.zeros(h, np.float32)
    f = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    rc = fn(C.byref(d), f(params), tex.ctypes.data_as(C.POINTER(C.c_uint16)), tex.size, f(rows), f(cols), f(wts))
    if rc != 0:
        raise RuntimeError('env tables rc=%d' % rc)
    return params, tex, rows, cols, wts


def bind(lib, name):
    fn = getattr(lib, name)
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_uint16), C.c_size_t,
                   C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    return fn
