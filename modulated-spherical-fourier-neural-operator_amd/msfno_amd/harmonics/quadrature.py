"""Quadrature rules on [a, b] — mirror of ``torch_harmonics.quadrature`` (the
reference calls ``legendre_gauss_weights(H, -1, 1)`` at MSFNO/Models/losses.py:90,129).
Computed natively (fp64, libmsfno ``msfno_quadrature``)."""
from __future__ import annotations

import numpy as np

from .. import _native as N


def _rule(n: int, grid: str, a: float, b: float):
    x = np.zeros(n, dtype=np.float64)
    w = np.zeros(n, dtype=np.float64)
    N.check(N.lib().msfno_quadrature(n, N.GRID[grid], x.ctypes.data, w.ctypes.data), "quadrature")
    x = (b - a) * 0.5 * x + (b + a) * 0.5
    w = w * (b - a) * 0.5
    return x, w


def legendre_gauss_weights(n: int, a: float = -1.0, b: float = 1.0):
    return _rule(n, "legendre-gauss", a, b)


def clenshaw_curtiss_weights(n: int, a: float = -1.0, b: float = 1.0):
    return _rule(n, "equiangular", a, b)
