"""Assignments and assignment collections.

Restates pystencils' ``Assignment`` / ``AssignmentCollection`` ([ext]
``pystencils/assignment.py``, ``simp/assignment_collection.py``) as far as the
autodiff path uses them (``_autodiff.py:35-50,156-168,242-244,271-294``):
main assignments (lhs is a ``Field.Access``) plus subexpressions (lhs is a
plain symbol), ``free_fields`` / ``bound_fields``, ``new_without_subexpressions``
and the ``Subexpressions:/Main Assignments:`` string form the reference's doc
tests print (``docs/index.rst:71-78``).
"""
import itertools

import sympy as sp

from .field import Field

__all__ = ['Assignment', 'AssignmentCollection']


class Assignment:
    """``lhs ← rhs``; ``lhs`` is a ``Field.Access`` or a ``sympy.Symbol``."""

    __slots__ = ('lhs', 'rhs')

    def __init__(self, lhs, rhs):
        self.lhs = lhs
        self.rhs = sp.sympify(rhs)

    @property
    def args(self):
        return (self.lhs, self.rhs)

    @property
    def free_symbols(self):
        return self.rhs.free_symbols

    def atoms(self, *types):
        return self.lhs.atoms(*types) | self.rhs.atoms(*types)

    def subs(self, *args, **kwargs):
        return Assignment(self.lhs, self.rhs.subs(*args, **kwargs))

    def __iter__(self):
        return iter((self.lhs, self.rhs))

    def __eq__(self, other):
        return isinstance(other, Assignment) and self.lhs == other.lhs and self.rhs == other.rhs

    def __hash__(self):
        return hash((self.lhs, self.rhs))

    def __str__(self):
        return f"{self.lhs} ← {self.rhs}"

    def __repr__(self):
        return str(self)


def _as_assignments(items):
    if items is None:
        return []
    if isinstance(items, dict):
        return [Assignment(k, v) for k, v in items.items()]
    out = []
    for a in items:
        if isinstance(a, Assignment):
            out.append(a)
        elif isinstance(a, sp.Eq):
            out.append(Assignment(a.lhs, a.rhs))
        elif isinstance(a, (tuple, list)) and len(a) == 2:
            out.append(Assignment(a[0], a[1]))
        elif hasattr(a, 'lhs') and hasattr(a, 'rhs'):
            out.append(Assignment(a.lhs, a.rhs))
        else:
            raise TypeError(f"not an assignment: {a!r}")
    return out


class AssignmentCollection:
    """Ordered main assignments + subexpressions."""

    def __init__(self, main_assignments, subexpressions=(), simplification_hints=None,
                 subexpression_symbol_generator=None):
        if isinstance(main_assignments, AssignmentCollection):
            subexpressions = list(main_assignments.subexpressions) + list(_as_assignments(subexpressions))
            main_assignments = main_assignments.main_assignments
        # kept as given (pystencils does the same); the autodiff layer splits plain-symbol lhs
        # into subexpressions itself (``_autodiff.py:242-244``)
        self.main_assignments = _as_assignments(main_assignments)
        self.subexpressions = _as_assignments(subexpressions)
        self.simplification_hints = dict(simplification_hints or {})
        self.subexpression_symbol_generator = subexpression_symbol_generator

    # -- views ----------------------------------------------------------------------------------
    @property
    def all_assignments(self):
        return list(self.subexpressions) + list(self.main_assignments)

    def __iter__(self):
        return iter(self.all_assignments)

    def __len__(self):
        return len(self.all_assignments)

    def __getitem__(self, i):
        return self.all_assignments[i]

    @property
    def rhs_symbols(self):
        out = set()
        for a in self.all_assignments:
            out |= a.rhs.free_symbols
        return out

    @property
    def free_symbols(self):
        """Symbols used on a rhs and not defined by any assignment of the collection."""
        return self.rhs_symbols - self.bound_symbols

    @property
    def bound_symbols(self):
        return {a.lhs for a in self.all_assignments}

    @property
    def free_fields(self):
        return {s.field for s in self.free_symbols if isinstance(s, Field.Access)}

    @property
    def bound_fields(self):
        return {a.lhs.field for a in self.main_assignments if isinstance(a.lhs, Field.Access)}

    @property
    def main_assignments_dict(self):
        return {a.lhs: a.rhs for a in self.main_assignments}

    @property
    def subexpressions_dict(self):
        return {a.lhs: a.rhs for a in self.subexpressions}

    def atoms(self, *types):
        out = set()
        for a in self.all_assignments:
            out |= a.atoms(*types)
        return out

    # -- transformations ------------------------------------------------------------------------
    def new_with_substitutions(self, substitutions):
        return AssignmentCollection([a.subs(substitutions) for a in self.main_assignments],
                                    [a.subs(substitutions) for a in self.subexpressions])

    def new_without_subexpressions(self, subexpressions_to_keep=()):
        keep = set(subexpressions_to_keep)
        subs = {}
        kept = []
        for a in self.subexpressions:
            rhs = a.rhs.xreplace(subs) if subs else a.rhs
            if a.lhs in keep:
                kept.append(Assignment(a.lhs, rhs))
            else:
                subs[a.lhs] = rhs
        main = [Assignment(a.lhs, a.rhs.xreplace(subs) if subs else a.rhs) for a in self.main_assignments]
        return AssignmentCollection(main, kept)

    def copy(self, main_assignments=None, subexpressions=None):
        return AssignmentCollection(list(self.main_assignments if main_assignments is None else main_assignments),
                                    list(self.subexpressions if subexpressions is None else subexpressions),
                                    self.simplification_hints)

    # -- comparison / printing -----------------------------------------------------------------
    def __eq__(self, other):
        if not isinstance(other, AssignmentCollection):
            return False
        return set(self.all_assignments) == set(other.all_assignments)

    def __hash__(self):
        return hash(frozenset(self.all_assignments))

    def __str__(self):
        result = "Subexpressions:\n"
        for eq in self.subexpressions:
            result += f"\t{eq}\n"
        result += "Main Assignments:\n"
        for eq in self.main_assignments:
            result += f"\t{eq}\n"
        return result

    def __repr__(self):
        return f"AssignmentCollection: {', '.join(str(a.lhs) for a in self.main_assignments)} <- " \
               f"f({', '.join(str(s) for s in sorted(self.free_symbols, key=str))})"


def iterate_accesses(assignments):
    """All ``Field.Access`` atoms of a list of assignments (lhs and rhs)."""
    return set(itertools.chain.from_iterable(a.atoms(Field.Access) for a in assignments))
