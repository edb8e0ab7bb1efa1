import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running')


def golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture
def load_golden():
    return golden


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


def assert_close_rel(actual, expected, rtol, what=''):
    """|actual - expected| <= rtol * max|expected| (SURVEY.md §7 tolerance form)."""
    actual = np.asarray(actual, dtype=np.float64)
    expected = np.asarray(expected, dtype=np.float64)
    assert actual.shape == expected.shape, f"{what}: shape {actual.shape} != {expected.shape}"
    scale = max(float(np.max(np.abs(expected))) if expected.size else 0.0, 1e-30)
    err = float(np.max(np.abs(actual - expected))) if expected.size else 0.0
    assert err <= rtol * scale, f"{what}: max abs err {err:.3e} > {rtol:.1e} * {scale:.3e}"


F32_EPS = 2.0 ** -24           # unit roundoff of fp32 (round to nearest)


def fp16_ulp(x):
    """Spacing of fp16 at |x| (subnormal spacing 2^-24 near zero)."""
    return np.spacing(np.abs(np.asarray(x, dtype=np.float64)).astype(np.float16)).astype(np.float64)


def assert_cells(actual, ref, absterms, nterms, storage, what='', rtol=1e-6, slack=4.0):
    """Element-wise parity of one output against the float64 oracle, cell by cell:

        |gpu − ref| ≤ rtol·|ref| + (nterms + 2)·2⁻²⁴·slack·Σ|terms|   [+ ½ ulp₁₆(|ref| + that) for fp16 storage]

    ``rtol`` is the north star's 1e-6 relative; the second term is the fp32 arithmetic of the kernel (a sum of
    ``nterms`` products with fp32-rounded weights, standard forward-error bound γₙ·Σ|terms|, ``slack`` for the
    unfolded intermediates a kernel may form); fp16 storage adds the final rounding of the fp32 result to fp16
    — i.e. the stored value is within half an fp16 ulp of the fp32 result, which is within the accumulation
    bound of the exact one. ``absterms`` = Σ|w·u| per cell (the same stencil with |w| on |u|)."""
    actual = np.asarray(actual, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    absterms = np.asarray(absterms, dtype=np.float64)
    assert actual.shape == ref.shape == absterms.shape, f'{what}: shapes {actual.shape} {ref.shape} {absterms.shape}'
    acc = (nterms + 2) * F32_EPS * slack * absterms
    bound = rtol * np.abs(ref) + acc
    if np.dtype(storage) == np.float16:
        bound = bound + 0.5 * fp16_ulp(np.abs(ref) + acc)
    err = np.abs(actual - ref)
    bad = err > bound
    if bad.any():
        i = np.unravel_index(int(np.argmax(np.where(bad, err / np.maximum(bound, 1e-300), 0))), err.shape)
        raise AssertionError(f'{what}: {int(bad.sum())} of {bad.size} cells outside the element-wise bound; worst at '
                             f'{i}: gpu {actual[i]!r} ref {ref[i]!r} err {err[i]:.3e} bound {bound[i]:.3e} '
                             f'(Σ|terms| {absterms[i]:.3e})')


def _degree(rest):
    """Degree of a monomial of field accesses (positive integer powers), or None for anything else."""
    import sympy as sp

    from pystencils_autodiff_amd import ps
    deg = 0
    for f in sp.Mul.make_args(rest):
        b, e = f.as_base_exp()
        if not isinstance(b, ps.Field.Access) or not (e.is_Integer and int(e) > 0):
            return None
        deg += int(e)
    return deg


def abs_poly(collection, max_degree=1):
    """(collection, degree): every main assignment's right-hand side (subexpressions substituted) replaced by
    Σ|c|·monomial over its polynomial expansion — evaluated on |inputs| it gives Σ|terms| per cell — and the highest
    monomial degree. None if a right-hand side is not a polynomial of degree <= ``max_degree`` in the field accesses
    with numeric coefficients (functions, divisions by accesses, symbolic parameters)."""
    import sympy as sp

    from pystencils_autodiff_amd import ps
    flat = collection.new_without_subexpressions()
    mains, top = [], 0
    for a in flat.main_assignments:
        new = 0
        for t in sp.Add.make_args(sp.expand(a.rhs)):
            c, rest = t.as_coeff_Mul()
            d = _degree(rest)
            if d is None or d > max_degree or not c.is_number:
                return None
            top = max(top, d)
            new += abs(float(c)) * rest
        mains.append(ps.Assignment(a.lhs, new))
    return ps.AssignmentCollection(mains), top


def abs_linear(collection):
    """``abs_poly`` of a linear collection (Σ|c|·access per main assignment), None if one is not linear."""
    r = abs_poly(collection)
    return r[0] if r is not None else None


def abs_terms(collection, inputs, boundary_handling='zeros'):
    """{output name: Σ|terms| per cell} for a linear collection on ``inputs`` ({name: array})."""
    from oracle import evaluate as OE
    ac = abs_linear(collection)
    assert ac is not None, 'abs_terms needs a linear stencil'
    return OE.evaluate(ac, {n: np.abs(np.asarray(a, dtype=np.float64)) for n, a in inputs.items()},
                       boundary_handling=boundary_handling)


def assert_cells_linear(actual, ref, collection, inputs, boundary_handling, storage, what=''):
    """``assert_cells`` for a polynomial ``collection`` (Σ|terms| of its expansion from the inputs, its term count;
    products of d accesses round d − 1 more times: ``slack`` 4·d); one with functions of the accesses keeps the
    caller's field-scaled check only. Returns whether the element-wise check ran."""
    from oracle import evaluate as OE
    pr = abs_poly(collection, max_degree=4)
    if pr is None:
        return False
    ac, deg = pr
    absr = OE.evaluate(ac, {n: np.abs(np.asarray(a, dtype=np.float64)) for n, a in inputs.items()},
                       boundary_handling=boundary_handling)
    nt = max(len(__import__('sympy').Add.make_args(a.rhs)) for a in ac.main_assignments)
    for name, r in (ref.items() if isinstance(ref, dict) else [(None, ref)]):
        a = actual[name] if isinstance(actual, dict) else actual
        n = name if name is not None else next(iter(absr))
        assert_cells(a, r, absr[n], nt, storage, f'{what} {n}', slack=4.0 * max(1, deg))
    return True


def n_terms(collection):
    """Most terms in one main assignment's linear expansion (the products the kernel sums per cell)."""
    ac = abs_linear(collection)
    import sympy as sp
    return max(len(sp.Add.make_args(a.rhs)) for a in ac.main_assignments)
