"""Bit-compare two float32 .npy images: python tools/cmp_npy.py A.npy B.npy"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
same = a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
print(f"{sys.argv[1]} vs {sys.argv[2]}: bit-equal {same}")
sys.exit(0 if same else 1)
