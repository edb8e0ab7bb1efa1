"""``ConditionalFieldAccess``: a field read that yields a constant outside the domain.

pystencils' ``astnodes.ConditionalFieldAccess`` ([ext]) as used by the
reference's ``transformations.add_fixed_constant_boundary_handling``
(``transformations.py:8,26-30``). The kernel lowering
(``backends/kernel_ir.py``) recognises it and realises it as a zero-filled
halo load instead of a per-access predicate.
"""
import sympy as sp

__all__ = ['ConditionalFieldAccess']


class ConditionalFieldAccess(sp.Function):
    """``ConditionalFieldAccess(access, out_of_bounds_condition, out_of_bounds_value=0)``."""

    nargs = (2, 3)

    @classmethod
    def eval(cls, *args):
        return None

    @property
    def access(self):
        return self.args[0]

    @property
    def outofbounds_condition(self):
        return self.args[1]

    @property
    def outofbounds_value(self):
        return self.args[2] if len(self.args) > 2 else sp.Integer(0)

    def _eval_derivative(self, s):
        # differentiate the guarded access; the guard is piecewise constant
        d = sp.diff(self.access, s)
        return sp.Piecewise((0, self.outofbounds_condition), (d, True)) if d != 0 else sp.Integer(0)

    def _sympystr(self, printer):
        return (f"(({printer.doprint(self.outofbounds_condition)}) ? "
                f"({printer.doprint(self.outofbounds_value)}) : ({printer.doprint(self.access)}))")
