"""Symbolic boundary handling.

``add_fixed_constant_boundary_handling`` restates ``transformations.py:12-36``
of the reference: every relative (non-absolute) field access on a right-hand
side becomes ``ConditionalFieldAccess(a, OR_d(ctr_d + off_d < 0 or >= shape_d))``
so that out-of-domain reads yield 0 ("zeros" boundary handling); a collection
whose accesses all sit at offset 0 is returned unchanged; CSE is applied when
``with_cse`` is truthy.

The MI355X kernels do not evaluate these predicates per access: the lowering
(``backends/kernel_ir.py``) turns the whole collection into a zero-filled
halo load, which yields the same operand values (exactly 0 outside the
domain) for every cell.
"""
import itertools

import sympy as sp

from .ps import Assignment, AssignmentCollection, Field, x_vector
from .ps.conditional import ConditionalFieldAccess
from .ps.simp import sympy_cse

__all__ = ['add_fixed_constant_boundary_handling']


def _out_of_bounds(position, shape):
    return sp.Or(*[sp.Or(p < 0, p >= s) for p, s in zip(position, shape)])


def add_fixed_constant_boundary_handling(assignments, with_cse=True):
    if not isinstance(assignments, AssignmentCollection):
        assignments = AssignmentCollection(list(assignments), [])
    accesses = set(itertools.chain.from_iterable(a.atoms(Field.Access) for a in assignments.all_assignments))
    if all(all(o == 0 for o in a.offsets) for a in accesses):
        return assignments
    shape = next(iter(accesses)).field.spatial_shape
    ctr = x_vector(len(shape))

    def guard(a):
        pos = sp.Matrix(a.offsets) + ctr
        return ConditionalFieldAccess(a, _out_of_bounds(list(pos), shape))

    guarded = [Assignment(a.lhs, a.rhs.xreplace({acc: guard(acc) for acc in a.rhs.atoms(Field.Access)
                                                   if not acc.is_absolute_access}))
               for a in assignments.all_assignments]
    n_sub = len(assignments.subexpressions)
    result = AssignmentCollection(guarded[n_sub:], guarded[:n_sub])
    return sympy_cse(result) if with_cse else result
