"""The BASELINE.json workloads, forward and adjoint, written out by hand (ORACLE — test-only).

Each adjoint follows the TF-MAD rule of the reference (``_autodiff.py:104-109``):
for ``out[c] = Σ_k w_k · u[c + o_k]`` the adjoint is the *flipped* gather
``diffu[c] = Σ_k w_k · diffout[c − o_k]``; reads outside the domain are 0
(``boundary_handling='zeros'``, ``transformations.py:12-36``). The README op's
adjoint is the derivative by hand (``docs/index.rst:77-78``). None of this uses
the package's symbolic AD core, so these functions cross-check the whole chain
(AD → lowering → HIP kernel).
"""
import itertools

import numpy as np

__all__ = ['linear_stencil', 'taps_diffusion_7pt', 'taps_laplace_5pt', 'taps_27pt', 'taps_asym_7pt',
           'readme_forward', 'readme_backward', 'DIFFUSION_ALPHA', 'flip']

DIFFUSION_ALPHA = 0.1


def linear_stencil(u, taps):
    """``out[c] = Σ w · u[c + o]`` with zero padding; float64 result."""
    u = np.asarray(u, dtype=np.float64)
    r = max(max(abs(o) for o in off) for off in taps)
    p = np.pad(u, r)
    out = np.zeros_like(u)
    for off, w in taps.items():
        sl = tuple(slice(r + o, r + o + n) for o, n in zip(off, u.shape))
        out += w * p[sl]
    return out


def flip(taps):
    return {tuple(-o for o in off): w for off, w in taps.items()}


def taps_diffusion_7pt(alpha=DIFFUSION_ALPHA):
    """``out = u + α(Σ₆ u[nb] − 6u)``."""
    taps = {(0, 0, 0): 1.0 - 6.0 * alpha}
    for d in range(3):
        for s in (-1, 1):
            off = [0, 0, 0]
            off[d] = s
            taps[tuple(off)] = alpha
    return taps


def taps_laplace_5pt():
    """``out = u[1,0]+u[-1,0]+u[0,1]+u[0,-1]−4u``."""
    return {(1, 0): 1.0, (-1, 0): 1.0, (0, 1): 1.0, (0, -1): 1.0, (0, 0): -4.0}


def taps_27pt():
    """27 distinct, asymmetric constant weights over {-1,0,1}³."""
    return {off: (i - 13.3) / 50.0 for i, off in enumerate(itertools.product((-1, 0, 1), repeat=3))}


def taps_asym_7pt():
    """An asymmetric 7-point stencil: a transposition bug in the adjoint cannot hide in it."""
    return {(0, 0, 0): 0.5, (1, 0, 0): 0.11, (-1, 0, 0): -0.23, (0, 1, 0): 0.37, (0, -1, 0): 0.05,
            (0, 0, 1): -0.41, (0, 0, -1): 0.29}


def readme_forward(x, y):
    """``z = x·log(x·y)`` (README.rst:52-68)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    return x * np.log(x * y)


def readme_backward(x, y, diffz):
    """``diffx = diffz·(log(x·y) + 1)``, ``diffy = diffz·x/y`` (docs/index.rst:77-78)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    dz = np.asarray(diffz, np.float64)
    return dz * (np.log(x * y) + 1.0), dz * x / y
