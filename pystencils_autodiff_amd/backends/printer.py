"""SymPy → C/HIP expression printing for the kernel emitters.

Plays the role of pystencils' ``CBackend`` / ``CustomSympyPrinter`` ([ext],
used by the reference through ``printer.py:69-86``) for right-hand sides:

* field accesses and subexpression symbols print as local variable names;
* small integer powers print as products (pystencils does the same), ``x**-1``
  as ``1/x``, ``x**(1/2)`` as ``sqrt(x)``;
* literals are printed in the kernel's compute type (``0.1f`` for float,
  17 significant digits for double), math functions with the type's spelling
  (``logf`` / ``log``);
* ``Piecewise`` prints as nested ternaries, relations / boolean ops as C.
"""
import sympy as sp
from sympy.printing.c import C99CodePrinter

__all__ = ['KernelExprPrinter']

_FLOAT_FUNCS = {
    'exp': 'expf', 'log': 'logf', 'sin': 'sinf', 'cos': 'cosf', 'tan': 'tanf', 'asin': 'asinf',
    'acos': 'acosf', 'atan': 'atanf', 'atan2': 'atan2f', 'sinh': 'sinhf', 'cosh': 'coshf', 'tanh': 'tanhf',
    'asinh': 'asinhf', 'acosh': 'acoshf', 'atanh': 'atanhf', 'sqrt': 'sqrtf', 'Abs': 'fabsf', 'floor': 'floorf',
    'ceiling': 'ceilf', 'erf': 'erff', 'erfc': 'erfcf', 'gamma': 'tgammaf', 'loggamma': 'lgammaf',
    'cbrt': 'cbrtf', 'Min': 'fminf', 'Max': 'fmaxf', 'pow': 'powf',
}
_DOUBLE_FUNCS = {k: v[:-1] for k, v in _FLOAT_FUNCS.items()}   # every float spelling ends in 'f'


class KernelExprPrinter(C99CodePrinter):
    """Prints one right-hand side in compute type ``ctype`` ('float' or 'double')."""

    def __init__(self, ctype='float', symbol_names=None):
        super().__init__({'strict': False})
        assert ctype in ('float', 'double')
        self.ctype = ctype
        self.symbol_names = symbol_names or {}
        self.funcs = _FLOAT_FUNCS if ctype == 'float' else _DOUBLE_FUNCS

    # -- atoms ----------------------------------------------------------------------------------
    def _print_Symbol(self, expr):
        if expr in self.symbol_names:
            return self.symbol_names[expr]
        return super()._print_Symbol(expr)

    def _literal(self, value):
        v = float(value)
        if v != v or v in (float('inf'), float('-inf')):
            raise ValueError(f"non-finite literal {value} in kernel expression")
        if self.ctype == 'float':
            s = repr(float(v))
            if 'e' not in s and '.' not in s:
                s += '.0'
            return f"{s}f"
        s = repr(float(v))
        if 'e' not in s and '.' not in s:
            s += '.0'
        return s

    def _print_Float(self, expr):
        return self._literal(expr)

    def _print_Rational(self, expr):
        return self._literal(sp.Float(expr, 20))

    def _print_Integer(self, expr):
        return self._literal(int(expr))

    def _print_Zero(self, expr):
        return self._literal(0)

    def _print_One(self, expr):
        return self._literal(1)

    def _print_NegativeOne(self, expr):
        return self._literal(-1)

    def _print_Half(self, expr):
        return self._literal(0.5)

    def _print_Pi(self, expr):
        return self._literal(sp.pi.evalf(20))

    def _print_Exp1(self, expr):
        return self._literal(sp.E.evalf(20))

    def _print_BooleanTrue(self, expr):
        return 'true'

    def _print_BooleanFalse(self, expr):
        return 'false'

    # -- operators ------------------------------------------------------------------------------
    def _print_Pow(self, expr):
        base, e = expr.base, expr.exp
        if e.is_Integer and 0 < int(e) < 8:
            b = self.parenthesize(base, 100)
            return '(' + '*'.join([b] * int(e)) + ')'
        if e.is_Integer and -8 < int(e) < 0:
            b = self.parenthesize(base, 100)
            return f"({self._literal(1)}/(" + '*'.join([b] * (-int(e))) + '))'
        if e == sp.Rational(1, 2):
            return f"{self.funcs['sqrt']}({self._print(base)})"
        if e == sp.Rational(-1, 2):
            return f"({self._literal(1)}/{self.funcs['sqrt']}({self._print(base)}))"
        if e == sp.Rational(1, 3):
            return f"{self.funcs['cbrt']}({self._print(base)})"
        return f"{self.funcs['pow']}({self._print(base)}, {self._print(e)})"

    def _print_Mul(self, expr):
        # keep a leading -1 as a negation so "-x" stays one instruction
        c, rest = expr.as_coeff_Mul()
        if c == -1:
            return '-' + self.parenthesize(rest, 50)
        return super()._print_Mul(expr)

    def _print_Function(self, expr):
        name = type(expr).__name__
        if name in self.funcs:
            args = ', '.join(self._print(a) for a in expr.args)
            if name in ('Min', 'Max') and len(expr.args) > 2:
                head, *tail = expr.args
                inner = type(expr)(*tail)
                return f"{self.funcs[name]}({self._print(head)}, {self._print(inner)})"
            return f"{self.funcs[name]}({args})"
        if name == 'ConditionalFieldAccess':
            return (f"(({self._print(expr.args[1])}) ? ({self._print(expr.args[2] if len(expr.args) > 2 else 0)})"
                    f" : ({self._print(expr.args[0])}))")
        if name == 'cast_func':
            return self._print(expr.args[0])
        raise NotImplementedError(f"function '{name}' is not supported in stencil kernels")

    _print_exp = _print_Function
    _print_log = _print_Function
    _print_sin = _print_Function
    _print_cos = _print_Function
    _print_tan = _print_Function
    _print_sinh = _print_Function
    _print_cosh = _print_Function
    _print_tanh = _print_Function
    _print_asin = _print_Function
    _print_acos = _print_Function
    _print_atan = _print_Function
    _print_atan2 = _print_Function
    _print_Abs = _print_Function
    _print_floor = _print_Function
    _print_ceiling = _print_Function
    _print_erf = _print_Function
    _print_Min = _print_Function
    _print_Max = _print_Function
    _print_sqrt = _print_Function

    def _print_Piecewise(self, expr):
        if expr.args[-1].cond != True:  # noqa: E712 - sympy boolean
            raise ValueError('Piecewise without a default branch cannot be printed')
        out = self._print(expr.args[-1].expr)
        for e, c in reversed(expr.args[:-1]):
            out = f"(({self._print(c)}) ? ({self._print(e)}) : ({out}))"
        return out

    def _print_Relational(self, expr):
        op = {'==': '==', '!=': '!=', '<': '<', '<=': '<=', '>': '>', '>=': '>='}[expr.rel_op]
        return f"({self._print(expr.lhs)} {op} {self._print(expr.rhs)})"

    def _print_And(self, expr):
        return '(' + ' && '.join(self._print(a) for a in expr.args) + ')'

    def _print_Or(self, expr):
        return '(' + ' || '.join(self._print(a) for a in expr.args) + ')'

    def _print_Not(self, expr):
        return f"(!{self._print(expr.args[0])})"

    def doprint_expr(self, expr):
        return self._print(sp.sympify(expr))
