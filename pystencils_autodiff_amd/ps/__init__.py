"""A minimal pystencils-compatible symbolic front-end.

The reference (``pystencils_autodiff``) is an add-on to pystencils, which is
an external dependency that is neither vendored in the reference nor
installable here. This sub-package restates exactly the
symbolic objects the autodiff hot path consumes — ``Field`` / ``Field.Access``,
``Assignment`` / ``AssignmentCollection``, ``fields()``, the ``fd`` module's
``Diff`` + ``Discretization2ndOrder`` and sympy CSE — so user code written
against ``import pystencils as ps`` runs unchanged with
``import pystencils_autodiff_amd.ps as ps``.

Kernel generation (pystencils ``create_kernel`` / ``generate_c`` / the CUDA
backend) is NOT restated here: that is what ``pystencils_autodiff_amd.backends``
replaces with the MI355X HIP emitter.
"""
from . import fd, simp
from .assignment import Assignment, AssignmentCollection
from .data_types import BasicType, create_type
from .field import (
    Field, FieldShapeSymbol, FieldStrideSymbol, FieldType, direction_string_to_offset, fields,
    offset_to_direction_string)

__all__ = ['Field', 'FieldType', 'fields', 'Assignment', 'AssignmentCollection', 'fd', 'simp',
           'BasicType', 'create_type', 'FieldShapeSymbol', 'FieldStrideSymbol',
           'offset_to_direction_string', 'direction_string_to_offset', 'x_vector']


def x_vector(ndim):
    """Symbols ``ctr_0 .. ctr_{ndim-1}`` for the current cell's coordinates."""
    import sympy as sp
    return sp.Matrix([sp.Symbol(f"ctr_{i}", integer=True) for i in range(ndim)])
