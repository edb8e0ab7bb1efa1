"""pystencils_autodiff_amd — MI355X-native forward/adjoint stencil operators.

Drop-in for the hot path of ``pystencils_autodiff`` (reference
``src/pystencils_autodiff/__init__.py:1-27``): the same API names —
``AutoDiffOp``, ``create_backward_assignments``, ``AdjointField``,
``DiffModes``, ``AutoDiffBoundaryHandling``, ``get_jacobian_of_assignments``,
``AutoDiffAstPair`` — with ``AutoDiffOp.create_tensorflow_op(backend='torch_native')``
returning a ``torch.autograd.Function`` whose forward and TF-MAD adjoint
kernels are HIP kernels emitted for gfx950 and compiled with hiprtc.

``pystencils_autodiff_amd.ps`` is the pystencils-compatible symbolic
front-end (``Field``, ``fields``, ``Assignment``, ``AssignmentCollection``, ``fd``).
"""
import sys

from . import backends, ps  # noqa: F401
from ._adjoint_field import AdjointField
from .autodiff import (
    AutoDiffAstPair, AutoDiffBoundaryHandling, AutoDiffOp, DiffModes, create_backward_assignments,
    get_jacobian_of_assignments)
from .printing import show_code

__version__ = '0.1.0'

__all__ = ['backends', 'ps', 'AdjointField', 'get_jacobian_of_assignments', 'create_backward_assignments',
           'AutoDiffOp', 'AutoDiffAstPair', 'DiffModes', 'AutoDiffBoundaryHandling', 'show_code']

# like the reference (``__init__.py:26-27``), make ``ps.autodiff`` resolve to this package
ps.autodiff = sys.modules[__name__]
