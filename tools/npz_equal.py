"""Bitwise comparison of two .npz files (the A/B scripts' outputs): prints
whether every array is equal and the first keys that differ; exit 0 either way."""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
diff = [k for k in a.files if k not in b.files or not np.array_equal(a[k], b[k], equal_nan=True)]
print("bitwise equal:", not diff, len(a.files), diff[:4])
