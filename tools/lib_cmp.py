#!/usr/bin/env python3
"""Bit-for-bit comparison of two tools/lib_dump.py outputs; exits 1 on any
difference.  python tools/lib_cmp.py a.npz b.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = 0
for k in a.files:
    x, y = a[k], b[k]
    diff = x.view(np.uint8).reshape(x.shape[0], -1) != y.view(np.uint8).reshape(y.shape[0], -1)
    rows = int(diff.any(axis=1).sum())
    print("%s: %d of %d chains differ" % (k, rows, x.shape[0]))
    bad += rows
sys.exit(1 if bad else 0)
