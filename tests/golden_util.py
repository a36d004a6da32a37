"""Restatement of the two input/sampling helpers of tests/golden/make_golden.py (importing
that script would install its scandir stand-in), for fixtures that store seeds and sampled
entries instead of whole tensors."""
import zlib

import numpy as np


def sampled(name, a, n=8192):
    a = np.asarray(a, np.float32).reshape(-1)
    if a.size <= n:
        return a
    idx = np.random.default_rng(zlib.crc32(name.encode())).choice(a.size, n, replace=False)
    return a[np.sort(idx)]


def seeded(seed, shape):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)
