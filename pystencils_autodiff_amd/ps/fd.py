"""Finite-difference derivatives and their 2nd-order central discretisation.

Restates the subset of pystencils ``fd`` ([ext] ``pystencils/fd/derivative.py``
``Diff`` and ``fd/finitedifferences.py`` ``Discretization2ndOrder`` /
``fd_stencils_standard``) that the reference's tests use to build stencils
(``tests/test_tfmad.py:16-18,105-108,196-198``):

* 1st derivative along ``d``: ``(f[+e_d] - f[-e_d]) / (2 dx)``
* 2nd derivative along ``d``: ``(f[-e_d] - 2 f + f[+e_d]) / dx**2``
* mixed ``d1 != d2``: ``sum_{o1,o2=±1} o1 o2 f[o1 e_d1 + o2 e_d2] / (4 dx**2)``
"""
import sympy as sp

from .field import Field

__all__ = ['Diff', 'Discretization2ndOrder', 'fd_stencils_standard', 'diff_args']


class Diff(sp.Expr):
    """Unevaluated spatial derivative ``∂ arg / ∂ x_target``."""

    is_commutative = True
    is_number = False

    def __new__(cls, argument, target=-1, superscript=-1):
        if isinstance(argument, Field):
            argument = argument.center
        if argument == 0:
            return sp.Rational(0, 1)
        return sp.Expr.__new__(cls, sp.sympify(argument), sp.sympify(target), sp.sympify(superscript))

    @property
    def arg(self):
        return self.args[0]

    @property
    def target(self):
        return int(self.args[1])

    @property
    def superscript(self):
        return int(self.args[2])

    def _sympystr(self, printer):
        return f"D({printer.doprint(self.arg)})"


def diff_args(expr):
    """``Diff(Diff(f, 0), 1)`` -> ``(f, 0, 1)`` (innermost argument, then targets outside-in)."""
    targets = []
    while isinstance(expr, Diff):
        targets.append(expr.target)
        expr = expr.arg
    return (expr, *reversed(targets))


def fd_stencils_standard(indices, dx, fa):
    order = len(indices)
    if order == 1:
        idx = indices[0]
        return (fa.neighbor(idx, 1) - fa.neighbor(idx, -1)) / (2 * dx)
    if order == 2:
        if indices[0] == indices[1]:
            return (-2 * fa + fa.neighbor(indices[0], -1) + fa.neighbor(indices[0], +1)) / (dx ** 2)
        offsets = [(1, 1), (-1, 1), (1, -1), (-1, -1)]
        return sum(o1 * o2 * fa.neighbor(indices[0], o1).neighbor(indices[1], o2)
                   for o1, o2 in offsets) / (4 * dx ** 2)
    raise NotImplementedError('only derivatives up to order two are discretised')


class Discretization2ndOrder:
    """Replaces every ``Diff`` in an expression by its central 2nd-order stencil."""

    def __init__(self, dx=sp.Symbol('dx'), dt=sp.Symbol('dt'), discretization_stencil_func=fd_stencils_standard):
        self.dx = dx
        self.dt = dt
        self.spatial_stencil = discretization_stencil_func

    def _discretize_spatial(self, e):
        if isinstance(e, Diff):
            arg, *indices = diff_args(e)
            if not isinstance(arg, Field.Access):
                raise ValueError('Only derivatives with field or field accesses as arguments can be discretized')
            return self.spatial_stencil(indices, self.dx, arg)
        if not e.args or isinstance(e, Field.Access):
            return e
        return e.func(*[self._discretize_spatial(a) for a in e.args])

    def __call__(self, expr):
        if isinstance(expr, (list, tuple)):
            return [self(e) for e in expr]
        from .assignment import Assignment, AssignmentCollection
        if isinstance(expr, Assignment):
            return Assignment(expr.lhs, self(expr.rhs))
        if isinstance(expr, AssignmentCollection):
            return AssignmentCollection([self(a) for a in expr.main_assignments],
                                        [self(a) for a in expr.subexpressions])
        return self._discretize_spatial(sp.sympify(expr))
