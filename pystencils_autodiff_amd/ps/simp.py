"""Common-subexpression elimination on assignment lists.

Restates pystencils ``simp.sympy_cse`` / ``sympy_cse_on_assignment_list``
([ext]; called from ``_autodiff.py:160,415`` and ``transformations.py:33``):
``sympy.cse`` over all right-hand sides, new subexpressions named ``xi_<n>``
(skipping names already in use), topologically ordered.
"""
import sympy as sp
from sympy.simplify.cse_main import reps_toposort

from .assignment import Assignment, AssignmentCollection

__all__ = ['sympy_cse', 'sympy_cse_on_assignment_list']


def _symbol_gen(used):
    names = {str(s) for s in used}
    i = 0
    while True:
        name = f"xi_{i}"
        i += 1
        if name not in names:
            yield sp.Symbol(name)


def sympy_cse(ac, **kwargs):
    assignments = ac.all_assignments
    used = set()
    for a in assignments:
        used |= a.rhs.free_symbols
        used.add(a.lhs)
    gen = ac.subexpression_symbol_generator or _symbol_gen(used)
    replacements, new_rhs = sp.cse([a.rhs for a in assignments], symbols=gen, **kwargs)
    new_eqs = [Assignment(a.lhs, r) for a, r in zip(assignments, new_rhs)]
    n_sub = len(ac.subexpressions)
    modified_sub = new_eqs[:n_sub]
    modified_main = new_eqs[n_sub:]
    pairs = [[s, e] for s, e in replacements] + [[a.lhs, a.rhs] for a in modified_sub]
    ordered = reps_toposort(pairs)
    new_sub = [Assignment(a[0], a[1]) for a in ordered]
    return ac.copy(modified_main, new_sub)


def sympy_cse_on_assignment_list(assignments):
    ac = AssignmentCollection([], list(assignments))
    return sympy_cse(ac).all_assignments
