"""Symbolic AD core vs the reference's own known-answer tests.

Mirrors tests/test_autodiff.py, tests/test_tfmad.py (symbolic parts) and the
docs/index.rst doctest of the reference.
"""
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from pystencils_autodiff_amd import DiffModes, ps


def _readme():
    z, y, x = ps.fields("z, y, x: [20,30]")
    return z, y, x, ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(x[0, 0] * y[0, 0])})


def test_jacobian_kat():
    # reference tests/test_autodiff.py:16-21 and :38-46
    z, y, x = ps.fields("z, y, x: [2d]")
    fa = ps.AssignmentCollection([ps.Assignment(z[0, 0], x[0, 0] * sp.log(x[0, 0] * y[0, 0]))], [])
    jac = pa.get_jacobian_of_assignments(fa, [x[0, 0], y[0, 0]])
    assert jac.shape == (len(fa.bound_symbols), len(fa.free_symbols))
    assert repr(jac) == 'Matrix([[log(x_C*y_C) + 1, x_C/y_C]])'
    raw = [ps.Assignment(z[0, 0], x[0, 0] * sp.log(x[0, 0] * y[0, 0]))]
    jac = pa.get_jacobian_of_assignments(raw, [x[0, 0], y[0, 0]])
    assert jac.shape == (1, 2) and repr(jac) == 'Matrix([[log(x_C*y_C) + 1, x_C/y_C]])'


def test_diff_modes_agree_on_pointwise_and_double_application():
    # reference tests/test_autodiff.py:23-33
    z, y, x = ps.fields("z, y, x: [2d]")
    fa = ps.AssignmentCollection([ps.Assignment(z[0, 0], x[0, 0] * sp.log(x[0, 0] * y[0, 0]))], [])
    for mode in DiffModes:
        pa.create_backward_assignments(fa, diff_mode=mode)
        pa.create_backward_assignments(pa.create_backward_assignments(fa), diff_mode=mode)
    r1 = pa.create_backward_assignments(fa, diff_mode=DiffModes.TRANSPOSED)
    r2 = pa.create_backward_assignments(fa, diff_mode=DiffModes.TF_MAD)
    assert r1 == r2


def test_docs_backward_kat():
    # reference docs/index.rst:56-78 (doctest) and README.rst:80-86
    _, _, _, fa = _readme()
    b = pa.create_backward_assignments(fa)
    b.main_assignments = sorted(b.main_assignments, key=lambda a: str(a))
    assert str(b) == ("Subexpressions:\nMain Assignments:\n"
                      "\t\\hat{x}[0,0] ← diffz_C*(log(x_C*y_C) + 1)\n"
                      "\t\\hat{y}[0,0] ← diffz_C*x_C/y_C\n")


def test_field_orders_and_adjoint_fields():
    z, y, x, fa = _readme()
    op = pa.AutoDiffOp(fa)
    assert [f.name for f in op.forward_input_fields] == ['x', 'y']
    assert [f.name for f in op.forward_output_fields] == ['z']
    assert [f.name for f in op.backward_input_fields] == ['diffz', 'x', 'y']
    assert [f.name for f in op.backward_output_fields] == ['diffx', 'diffy']
    dx = op.backward_output_fields[0]
    assert isinstance(dx, pa.AdjointField) and dx.corresponding_forward_field == x
    assert dx.shape == x.shape and dx.strides == x.strides and dx.dtype == x.dtype
    assert dx.latex_name == r'\hat{x}'


def test_tfmad_flips_offsets():
    # reference tests/test_tfmad.py:12-28 stencil: out = D0 f - D1 f
    f, out = ps.fields("f, out: double[2D]")
    disc = ps.fd.Discretization2ndOrder(dx=1)(ps.fd.Diff(f, 0) - ps.fd.Diff(f, 1))
    ac = ps.AssignmentCollection([ps.Assignment(out.center(), disc)], [])
    back = pa.create_backward_assignments(ac, diff_mode='transposed-forward')
    (a,) = back.main_assignments
    diffout = a.rhs.free_symbols
    d = ps.fields("diffout: double[2D]")
    # forward f[1,0]/2 -> adjoint diffout[-1,0]/2 ; forward -f[0,1]/2 -> adjoint -diffout[0,-1]/2
    expect = d[-1, 0] / 2 - d[1, 0] / 2 - d[0, -1] / 2 + d[0, 1] / 2
    assert sp.simplify(a.rhs - expect) == 0, (a.rhs, diffout)
    assert str(a.lhs) == r'\hat{f}[0,0]'


def test_tfmad_two_stencils_orders():
    # reference tests/test_tfmad.py:31-53
    a, b, out = ps.fields("a, b, out: double[2D]")
    cont = ps.fd.Diff(a, 0) - ps.fd.Diff(a, 1) - ps.fd.Diff(b, 0) + ps.fd.Diff(b, 1)
    ac = ps.AssignmentCollection([ps.Assignment(out.center(), ps.fd.Discretization2ndOrder(dx=1)(cont))], [])
    op = pa.AutoDiffOp(ac, diff_mode='transposed-forward')
    assert [f.name for f in op.forward_input_fields] == ['a', 'b']
    assert [f.name for f in op.backward_output_fields] == ['diffa', 'diffb']
    assert 'Forward:' in repr(op) and 'Backward:' in repr(op)


def test_three_outputs_unshifted_partial_quirk():
    # reference tests/test_tfmad.py:242-248; TF-MAD evaluates d exp(b[-1,0]) at the forward cell
    a, b, o1, o2, o3 = ps.fields("a, b, out1, out2, out3: float64[21,13]")
    ac = ps.AssignmentCollection({o1.center: a.center + b.center, o2.center: a.center - b.center,
                                  o3.center: sp.exp(b[-1, 0])})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    rhs = {str(x.lhs): x.rhs for x in op.backward_assignments.main_assignments}
    d1, d2, d3 = ps.fields("diffout1, diffout2, diffout3: float64[21,13]")
    assert sp.simplify(rhs[r'\hat{a}[0,0]'] - (d1.center + d2.center)) == 0
    assert sp.simplify(rhs[r'\hat{b}[0,0]'] - (d1.center - d2.center + d3[1, 0] * sp.exp(b[-1, 0]))) == 0


def test_time_constant_accumulates():
    u, out = ps.fields("u, out: double[2D]")
    ac = ps.AssignmentCollection({out.center: 2 * u[1, 0]})
    op = pa.AutoDiffOp(ac, time_constant_fields=[u])
    (a,) = op.backward_assignments.main_assignments
    du = a.lhs.field
    assert sp.simplify(a.rhs - (du.center + 2 * ps.fields("diffout: double[2D]")[-1, 0])) == 0


def test_constant_fields_get_no_adjoint():
    u, w, out = ps.fields("u, w, out: double[2D]")
    ac = ps.AssignmentCollection({out.center: w.center * u[1, 0]})
    op = pa.AutoDiffOp(ac, constant_fields=[w])
    assert [f.name for f in op.backward_output_fields] == ['diffu']
    op2 = pa.AutoDiffOp(ac, constant_fields=['w'])
    assert [f.name for f in op2.backward_output_fields] == ['diffu']


def test_valid_boundary_raises_like_reference():
    _, _, _, fa = _readme()
    with pytest.raises(NotImplementedError):
        pa.AutoDiffOp(fa, boundary_handling='valid')


def test_cse_subexpressions():
    u, out = ps.fields("u, out: double[2D]")
    e = sp.exp(u[1, 0] + u[-1, 0])
    ac = ps.AssignmentCollection({out.center: e * e + sp.sin(u[1, 0] + u[-1, 0])})
    back = pa.create_backward_assignments(ac)
    assert back.subexpressions, 'CSE should extract the shared exp/sum terms'
    assert pa.autodiff.has_exclusive_writes(back)


def test_transposed_mode_rejects_stencils():
    u, out = ps.fields("u, out: double[2D]")
    ac = ps.AssignmentCollection({out.center: u[1, 0] + u[-1, 0]})
    with pytest.raises(AssertionError):
        pa.AutoDiffOp(ac, diff_mode='transposed')


def test_boundary_transformation_wraps_accesses():
    from pystencils_autodiff_amd.ps.conditional import ConditionalFieldAccess
    from pystencils_autodiff_amd.transformations import add_fixed_constant_boundary_handling
    x, y = ps.fields("x, y: float64[2d]")
    ac = ps.AssignmentCollection({y.center: (x[0, 0] + x[1, 0] + x[0, 1] + x[1, 1]) / 4})
    bh = add_fixed_constant_boundary_handling(ac)
    assert any(isinstance(e, ConditionalFieldAccess) for a in bh.all_assignments for e in sp.preorder_traversal(a.rhs))
    pointwise = ps.AssignmentCollection({y.center: 2 * x.center})
    assert add_fixed_constant_boundary_handling(pointwise) is pointwise


def test_reproducible_code_generation():
    # reference tests/backends/test_torch_native_compilation.py:214-244
    from sympy.core.cache import clear_cache
    first = None
    for _ in range(4):
        _, _, _, fa = _readme()
        op = pa.AutoDiffOp(fa)
        code = op.forward_ast_gpu.compile().code + op.backward_ast_gpu.compile().code
        clear_cache()
        first = first or code
        assert code == first


def test_op_pickle_roundtrip():
    import pickle
    u, out = ps.fields("u, out: float32[3d]")
    op = pa.AutoDiffOp(ps.AssignmentCollection({out.center: u[1, 0, 0] - 2 * u[0, -1, 0]}), boundary_handling='zeros',
                       op_name='pickled')
    op2 = pickle.loads(pickle.dumps(op))
    assert str(op2.forward_assignments) == str(op.forward_assignments)
    assert str(op2.backward_assignments) == str(op.backward_assignments)
    assert op2.boundary_handling == op.boundary_handling and op2.op_name == 'pickled'
    assert [f.name for f in op2.backward_output_fields] == ['diffu']
