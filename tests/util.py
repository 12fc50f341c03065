import hashlib

import numpy as np


def sha1(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def assert_close_normwise(got, ref, tol=1e-5, what=""):
    """Parity gate of north_star / SURVEY §8d: max|got-ref| <= tol * max|ref| per tensor."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    scale = np.abs(ref).max() if ref.size else 0.0
    err = np.abs(got - ref).max() if ref.size else 0.0
    assert err <= tol * max(scale, 1e-30), f"{what}: max|d|={err:.3e} > {tol}*{scale:.3e}"
