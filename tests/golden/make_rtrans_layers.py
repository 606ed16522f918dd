#!/usr/bin/env python3
"""Generates tests/golden/rtrans_c5_ggx_layers.npz: the eta layers of the
reference's data/microfacet/ggx.dat that C5's roughplastic reads.

RoughPlastic::configure reduces the 3D (eta, alpha, theta) rough-transmittance
table to 2D at its relative IOR (roughplastic.cpp:281-293: setEta(eta) on the
external table, setEta(1/eta) on the internal one).  setEta
(rtrans.h:291-330) evaluates evalCubicInterp3D (spline.cpp:379-450) at the
warped eta, whose stencil touches only the four eta layers knot-1 .. knot+2
(every other layer has weight 0); 1/eta < 1 selects the file's second block
with the same knot.  The fixture keeps those layers (two extra on each side),
for both blocks, with the file header: C5's eta = polypropylene / air
(1.49 / 1.000277, roughplastic.cpp:198-203, the IOR table of ior.h).

The file is read in place from /root/reference (nothing else is copied); the
fixture is data: the table values of the rows listed in `rows`.  Usage:
    python tests/golden/make_rtrans_layers.py [/root/reference/data/microfacet/ggx.dat]
"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/data/microfacet/ggx.dat'
ETA = np.float32(np.float32(1.49) / np.float32(1.000277))     # C5: intIOR polypropylene, extIOR air
HEADER = 57                                                     # 'MTS_TRANSMITTANCE', 3 x u64, 4 x f32


def layer_rows(n_eta, eta_min, eta_max, eta, pad=2):
    """File rows (0 .. 2 n_eta - 1) setEta(eta) and setEta(1/eta) read, widened by `pad`."""
    w = ((float(eta) - eta_min) / (eta_max - eta_min)) ** 0.25
    knot = min(int(w * (n_eta - 1)), n_eta - 2)
    lo, hi = max(knot - 1 - pad, 0), min(knot + 2 + pad, n_eta - 1)
    rows = list(range(lo, hi + 1))
    return rows + [n_eta + r for r in rows]


def main():
    raw = open(SRC, 'rb').read()
    assert raw[:17] == b'MTS_TRANSMITTANCE'
    n_eta, n_alpha, n_theta = struct.unpack_from('<QQQ', raw, 17)
    eta_min, eta_max, _, _ = struct.unpack_from('<4f', raw, 41)
    data = np.frombuffer(raw, '<f4', offset=HEADER).reshape(2 * n_eta, n_alpha, n_theta + 1)
    rows = np.array(layer_rows(n_eta, eta_min, eta_max, ETA), np.int32)
    out = os.path.join(HERE, 'rtrans_c5_ggx_layers.npz')
    np.savez_compressed(out, header=np.frombuffer(raw[:HEADER], np.uint8), rows=rows,
                        layers=np.ascontiguousarray(data[rows]), eta=np.float32(ETA))
    print('%s: rows %s, %d bytes' % (out, rows.tolist(), os.path.getsize(out)))


if __name__ == '__main__':
    main()
