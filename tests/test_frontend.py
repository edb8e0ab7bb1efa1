"""The pystencils-compatible symbolic front-end (names, parsing, printing)."""
import numpy as np
import pytest
import sympy as sp

from pystencils_autodiff_amd import ps


def test_fields_parsing_fixed_and_generic():
    a, b, out = ps.fields("a, b, out: float64[5,7]")
    assert a.shape == (5, 7) and a.strides == (7, 1) and a.dtype.numpy_dtype == np.float64
    assert a.spatial_dimensions == 2 and a.index_dimensions == 0 and a.has_fixed_shape
    z, y, x = ps.fields("z, y, x: [20,40]")          # default dtype double
    assert z.dtype.numpy_dtype == np.float64 and z.shape == (20, 40)
    u = ps.fields("u: float32[3d]")
    assert u.spatial_dimensions == 3 and not u.has_fixed_shape
    assert u.dtype.numpy_dtype == np.float32
    f = ps.fields("f(2): [2D]")
    assert f.index_dimensions == 1 and f.index_shape == (2,)
    h = ps.fields("h: float16[8,8,8]")
    assert h.dtype.numpy_dtype == np.float16


def test_fields_from_arrays():
    arr = np.zeros((6, 7), np.float32)
    x = ps.fields(x=arr)
    assert x.shape == (6, 7) and x.strides == (7, 1) and x.dtype.numpy_dtype == np.float32
    torch = pytest.importorskip('torch')
    t = torch.zeros(20, 10)
    y = ps.fields(y=t)
    assert y.shape == (20, 10) and y.dtype.numpy_dtype == np.float32


def test_access_names_and_str():
    x, y = ps.fields("x, y: [2d]")
    assert x.center.name == 'x_C'
    assert x[1, 0].name == 'x_E' and x[-1, 0].name == 'x_W'
    assert x[0, 1].name == 'x_N' and x[0, -1].name == 'x_S'
    assert x[1, -1].name == 'x_SE'
    assert x[2, 0].name == 'x_2E'
    u = ps.fields("u: [3d]")
    assert u[0, 0, 1].name == 'u_T' and u[0, 0, -1].name == 'u_B'
    assert str(x[0, 0]) == 'x[0,0]'
    assert str(x[1, -1]) == 'x[1,-1]'
    # accesses are sympy symbols; equal by field + offset
    assert x[1, 0] == x.neighbor(0, 1) and x[1, 0] != y[1, 0]
    assert sp.diff(x[1, 0] ** 2, x[1, 0]) == 2 * x[1, 0]


def test_vector_field_access():
    f = ps.fields("f(2): [2D]")
    assert f.center(1).index == (1,)
    assert f.center.at_index(0).index == (0,)
    with pytest.raises(ValueError):
        f.center(0, 1)


def test_assignment_collection_printing_and_sets():
    z, y, x = ps.fields("z, y, x: [20,30]")
    ac = ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(x[0, 0] * y[0, 0])})
    # README.rst / docs/index.rst:44-48 output
    assert str(ac) == "Subexpressions:\nMain Assignments:\n\tz[0,0] ← x_C*log(x_C*y_C)\n"
    assert ac.free_fields == {x, y} and ac.bound_fields == {z}
    assert ac.free_symbols == {x.center, y.center}


def test_new_without_subexpressions():
    u, out = ps.fields("u, out: [2d]")
    s = sp.Symbol('s')
    ac = ps.AssignmentCollection([ps.Assignment(out.center, 2 * s)], [ps.Assignment(s, u[1, 0] + u[-1, 0])])
    flat = ac.new_without_subexpressions()
    assert flat.subexpressions == [] and flat.main_assignments[0].rhs == 2 * (u[1, 0] + u[-1, 0])


def test_fd_discretization_matches_pystencils_rule():
    a = ps.fields("a: [2d]")
    d = ps.fd.Discretization2ndOrder(dx=1)
    assert sp.simplify(d(ps.fd.Diff(a, 0)) - (a[1, 0] - a[-1, 0]) / 2) == 0
    assert sp.simplify(d(ps.fd.Diff(ps.fd.Diff(a, 1), 1)) - (a[0, 1] - 2 * a.center + a[0, -1])) == 0
    mixed = d(ps.fd.Diff(ps.fd.Diff(a, 0), 1))
    assert sp.simplify(mixed - (a[1, 1] - a[-1, 1] - a[1, -1] + a[-1, -1]) / 4) == 0


def test_direction_strings_roundtrip():
    for off in [(1, 0, 0), (0, -1, 0), (0, 0, 2), (1, -1, 1), (0, 0, 0)]:
        s = ps.offset_to_direction_string(off)
        assert ps.direction_string_to_offset(s, 3) == off


def test_unsupported_layout_raises():
    """Fortran-ordered spatial axes are not handled; 'fzyx' is (tests/test_fzyx.py)."""
    with pytest.raises(NotImplementedError):
        ps.fields("a: double[3,4]", layout='reverse_numpy')
    assert ps.fields("a: double[3,4]", layout='fzyx').strides == (4, 1)
