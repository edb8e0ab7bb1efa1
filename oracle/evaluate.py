"""float64 NumPy evaluation of stencil assignment collections (ORACLE — test-only).

Semantics restated from the reference:

* ``boundary_handling='zeros'``: ``add_fixed_constant_boundary_handling``
  (``transformations.py:12-36``) guards every relative access with
  ``ConditionalFieldAccess(a, out_of_bounds)`` and the kernel is built with
  ``ghost_layers=0`` (``_autodiff.py:482-484,497-499,514-516,531-533``): every
  cell is written; a read outside the domain is 0.
* ``boundary_handling=None``: ``ghost_layers=None`` → pystencils iterates the
  interior ``[g, N-g)`` of every axis with ``g`` the largest ``|offset|`` of any
  access; the border keeps the zeros the op allocated
  (``backends/_torch_native.py:61-73,107-112``).
* Statements run in order (subexpressions, then main assignments); free
  non-field symbols are scalar parameters.

Independent of ``pystencils_autodiff_amd.backends``: accesses are found by
walking the SymPy trees, shifted views come from a zero-padded copy, and the
right-hand sides are evaluated with ``sympy.lambdify`` on float64 arrays.
"""
import numpy as np
import sympy as sp

__all__ = ['evaluate', 'accesses_of']


def _is_access(s):
    return hasattr(s, 'field') and hasattr(s, 'offsets') and isinstance(s, sp.Symbol)


def _strip(expr):
    return expr.replace(lambda e: type(e).__name__ == 'ConditionalFieldAccess', lambda e: e.args[0])


def accesses_of(assignments):
    out = set()
    for a in assignments:
        for s in _strip(a.rhs).free_symbols:
            if _is_access(s):
                out.add(s)
        if _is_access(a.lhs):
            out.add(a.lhs)
    return out


def evaluate(collection, arrays, scalars=None, boundary_handling='zeros', outputs=None):
    """Evaluate ``collection`` on ``arrays`` ({field name: ndarray}); returns {output name: float64 ndarray}.

    ``outputs`` may give initial contents of written fields (default zeros) — used for
    accumulating (time-constant) adjoints.
    """
    scalars = dict(scalars or {})
    subs = list(collection.subexpressions)
    mains = list(collection.main_assignments)
    ordered = [(a.lhs, _strip(a.rhs)) for a in subs + mains]
    accs = accesses_of(subs + mains)
    ndim = next(iter(accs)).field.spatial_dimensions
    written = {}
    for lhs, _ in ordered:
        if _is_access(lhs):
            written[lhs.field.name] = lhs.field
    ref_name = sorted(written)[0]
    shape = None
    for name, arr in arrays.items():
        shape = np.shape(arr)[:ndim]
        break
    if shape is None:
        shape = tuple(int(s) for s in written[ref_name].spatial_shape)
    g_max = max([max([abs(int(o)) for o in a.offsets] + [0]) for a in accs] + [0])
    zeros = boundary_handling is not None and str(getattr(boundary_handling, 'value', boundary_handling)) \
        in ('zeros', 'valid')
    if any(type(e).__name__ == 'ConditionalFieldAccess' for a in subs + mains for e in sp.preorder_traversal(a.rhs)):
        zeros = True
    pad = g_max
    padded = {}

    def view(field, offsets, index):
        name = field.name
        if name not in padded:
            if name in arrays:
                base = np.asarray(arrays[name], dtype=np.float64)
            elif outputs is not None and name in outputs:
                base = np.asarray(outputs[name], dtype=np.float64)
            else:
                base = np.zeros(tuple(shape) + tuple(int(s) for s in field.index_shape))
            widths = [(pad, pad)] * ndim + [(0, 0)] * (base.ndim - ndim)
            padded[name] = np.pad(base, widths)
        p = padded[name]
        sl = tuple(slice(pad + int(o), pad + int(o) + n) for o, n in zip(offsets, shape))
        v = p[sl]
        for i in index:
            v = v[..., int(i)]
        return v

    g = 0 if zeros else g_max
    interior = tuple(slice(g, max(g, n - g)) for n in shape)
    env = {}
    results = {}
    for name, f in written.items():
        init = outputs.get(name) if outputs is not None and name in outputs else None
        results[name] = np.array(init, dtype=np.float64) if init is not None else \
            np.zeros(tuple(shape) + tuple(int(s) for s in f.index_shape))
    for lhs, rhs in ordered:
        syms = sorted(rhs.free_symbols, key=str)
        vals = []
        for s in syms:
            if _is_access(s):
                vals.append(view(s.field, s.offsets, s.index))
            elif s in env:
                vals.append(env[s])
            elif s.name in scalars:
                vals.append(np.float64(scalars[s.name]))
            else:
                raise KeyError(f"no value for symbol {s}")
        fn = sp.lambdify(syms, rhs, modules='numpy', dummify=True)
        val = np.broadcast_to(np.asarray(fn(*vals), dtype=np.float64), tuple(shape)).copy()
        if _is_access(lhs):
            if any(int(o) != 0 for o in lhs.offsets):
                raise NotImplementedError('oracle: writes at non-zero offsets')
            tgt = results[lhs.field.name]
            for i in lhs.index:
                tgt = tgt[..., int(i)]
            tgt[interior] = val[interior]
        else:
            env[lhs] = val
    return results
