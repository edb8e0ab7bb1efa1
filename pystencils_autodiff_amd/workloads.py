"""The BASELINE.json workloads as assignment collections (built with the public API).

Used by ``bench.py``, ``__graft_entry__`` and the tests; mirrors how a user of
the reference would write these stencils (``README.rst:52-68``,
``tests/test_tfmad.py:186-231``).
"""
import itertools

import sympy as sp

from . import ps

__all__ = ['diffusion_7pt', 'laplace_5pt', 'stencil_27pt', 'readme_op', 'asym_7pt', 'vector_laplace_7pt',
           'varcoef_diffusion_7pt',
           'WEIGHTS_27PT', 'ALPHA']

ALPHA = 0.1
WEIGHTS_27PT = [(i - 13.3) / 50.0 for i in range(27)]


def _fields(names, dtype, ndim, shape):
    spec = f"{names}: {dtype}[{','.join(str(s) for s in shape)}]" if shape else f"{names}: {dtype}[{ndim}d]"
    return ps.fields(spec)


def diffusion_7pt(shape=None, dtype='float32', alpha=ALPHA):
    """3-D 7-point diffusion ``out = u + α(Σ₆ u[nb] − 6u)`` (BASELINE configs 3 and 4)."""
    u, out = _fields('u, out', dtype, 3, shape)
    nb = [u[1, 0, 0], u[-1, 0, 0], u[0, 1, 0], u[0, -1, 0], u[0, 0, 1], u[0, 0, -1]]
    return ps.AssignmentCollection({out.center: u.center + alpha * (sp.Add(*nb) - 6 * u.center)})


def laplace_5pt(shape=None, dtype='float32'):
    """2-D 5-point Laplacian ``u[1,0]+u[-1,0]+u[0,1]+u[0,-1]−4u`` (BASELINE config 2)."""
    u, out = _fields('u, out', dtype, 2, shape)
    return ps.AssignmentCollection({out.center: u[1, 0] + u[-1, 0] + u[0, 1] + u[0, -1] - 4 * u.center})


def stencil_27pt(shape=None, dtype='float16', weights=WEIGHTS_27PT):
    """3-D 27-point anisotropic stencil with 27 distinct constant weights (BASELINE config 5)."""
    u, out = _fields('u, out', dtype, 3, shape)
    offs = list(itertools.product((-1, 0, 1), repeat=3))
    return ps.AssignmentCollection({out.center: sp.Add(*[sp.Float(w) * u[o] for w, o in zip(weights, offs)])})


def asym_7pt(shape=None, dtype='float32'):
    """Asymmetric 7-point stencil (detects un-flipped adjoint offsets)."""
    u, out = _fields('u, out', dtype, 3, shape)
    taps = {(0, 0, 0): 0.5, (1, 0, 0): 0.11, (-1, 0, 0): -0.23, (0, 1, 0): 0.37, (0, -1, 0): 0.05,
            (0, 0, 1): -0.41, (0, 0, -1): 0.29}
    return ps.AssignmentCollection({out.center: sp.Add(*[sp.Float(w) * u[o] for o, w in taps.items()])})


def readme_op(shape=(20, 30), dtype='float32'):
    """``z = x·log(x·y)`` (README.rst:52-68, BASELINE config 1)."""
    z, y, x = _fields('z, y, x', dtype, 2, shape)
    return ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(x[0, 0] * y[0, 0])})


def vector_laplace_7pt(shape=None, dtype='float32', ncomp=3, layout='numpy'):
    """Component-wise 3-D 7-point Laplacian of a vector field ``u(c)`` (index dimension; components
    fastest in memory, or slowest with ``layout='fzyx'``) — the vector-field row of SURVEY.md §8(f)
    (``_autodiff.py:125-152``)."""
    spec = f"u({ncomp}), out({ncomp}): {dtype}[{','.join(str(v) for v in shape)}]" if shape else \
        f"u({ncomp}), out({ncomp}): {dtype}[3d]"
    u, out = ps.fields(spec, layout=layout)
    nb = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
    return ps.AssignmentCollection({out.center(c): sp.Add(*[u[o](c) for o in nb]) - 6 * u.center(c)
                                    for c in range(ncomp)})


def varcoef_diffusion_7pt(shape=None, dtype='float32', alpha=ALPHA):
    """3-D 7-point diffusion with a conductivity field ``k`` (face value = mean of the two cells):
    ``out = u + α Σ₆ ½(k + k[nb])(u[nb] − u)`` — the learn-the-coefficient problem of differentiable PDE
    solvers; its adjoint has two outputs (``diffu``, ``diffk``) from three inputs."""
    u, k, out = _fields('u, k, out', dtype, 3, shape)
    nb = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
    half = sp.Rational(1, 2)
    return ps.AssignmentCollection({out.center: u.center + alpha * sp.Add(
        *[half * (k.center + k[o]) * (u[o] - u.center) for o in nb])})
