"""``create_tensorflow_op(backend='torch_native', use_cuda=False)`` — the reference's CPU path.

Mirrors tests/test_tfmad.py:186-285 (with_cuda=False) and
tests/backends/test_torch_native_compilation.py:47-80,153-211 of the reference.
"""
import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from tests.conftest import assert_close_rel, golden

torch = pytest.importorskip('torch')


@pytest.mark.parametrize('with_offsets', (False, True))
def test_tfmad_gradient_check_torch_native_cpu(with_offsets):
    a, b, out = ps.fields("a, b, out: float64[5,7]")
    if with_offsets:
        cont = 2 * ps.fd.Diff(a, 0) - 1.5 * ps.fd.Diff(a, 1) - ps.fd.Diff(b, 0) + 3 * ps.fd.Diff(b, 1)
        asg = ps.Assignment(out.center(), ps.fd.Discretization2ndOrder(dx=1)(cont) + 1.2 * a.center())
    else:
        asg = ps.Assignment(out.center(), 1.2 * a.center + 0.1 * b.center)
    op = pa.AutoDiffOp(ps.AssignmentCollection([asg], []), boundary_handling='zeros', diff_mode='transposed-forward')
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    d = {a: torch.zeros(*a.shape, dtype=torch.float64, requires_grad=True),
         b: torch.zeros(*b.shape, dtype=torch.float64, requires_grad=True)}
    assert torch.autograd.gradcheck(fn.apply, tuple(d[f] for f in op.forward_input_fields), atol=1e-4)


def test_tfmad_gradient_check_two_outputs_cpu():
    a, b, o1, o2, o3 = ps.fields("a, b, out1, out2, out3: float64[21,13]")
    ac = ps.AssignmentCollection({o1.center: a.center + b.center, o2.center: a.center - b.center,
                                  o3.center: sp.exp(b[-1, 0])})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros', diff_mode='transposed-forward')
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    at = torch.zeros(*a.shape, dtype=torch.float64, requires_grad=True)
    bt = torch.zeros(*b.shape, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(fn.apply, (at, bt), atol=1e-4)


def test_op_attributes_and_call():
    z, y, x = ps.fields("z, y, x: float64[20,40]")
    a = sp.Symbol('a')
    op = pa.AutoDiffOp(ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(a * x[0, 0] * y[0, 0])}))
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    for attr in ('class_kwargs', 'kernel', 'ast', 'parameters', 'forward_parameters', 'forward_ast',
                 'backward_ast', 'num_regs', 'code'):
        assert hasattr(fn, attr), attr
    assert [p.symbol.name for p in fn.forward_parameters] == ['x', 'y']
    fn.class_kwargs['a'] = 5.0
    rng = np.random.default_rng(0)
    xv = torch.from_numpy(rng.uniform(0.5, 1.5, (20, 40))).requires_grad_(True)
    yv = torch.from_numpy(rng.uniform(0.5, 1.5, (20, 40))).requires_grad_(True)
    zt = fn.call(x=xv, y=yv)
    assert isinstance(zt, torch.Tensor)
    ref = xv.detach().numpy() * np.log(5.0 * xv.detach().numpy() * yv.detach().numpy())
    assert np.allclose(zt.detach().numpy(), ref, atol=1e-12)
    tup = fn.apply(xv, yv)
    assert isinstance(tup, tuple) and len(tup) == 1
    tup[0].sum().backward()
    assert np.allclose(xv.grad.numpy(), np.log(5.0 * xv.detach().numpy() * yv.detach().numpy()) + 1)


def test_execute_kernel_directly_like_reference():
    # reference tests/backends/test_torch_native_compilation.py:153-211
    z, y, x = ps.fields("z, y, x: [20,40]")
    a = sp.Symbol('a')
    fa = ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(a * x[0, 0] * y[0, 0])})
    op = pa.AutoDiffOp(fa)
    k = op.forward_ast_cpu
    rng = np.random.default_rng(1)
    xv, yv = rng.random((20, 40)), rng.random((20, 40))
    zv = np.zeros((20, 40))
    k(x=xv, y=yv, z=zv, a=5.)
    assert np.allclose(zv[1:-1, 1:-1], (xv * np.log(5 * xv * yv))[1:-1, 1:-1], atol=1e-6)
    assert 'call_' + k.function_name in [w.function_name for w in
                                          op.create_tensorflow_op(use_cuda=False, backend='torch_native').ast.kernel_wrappers]


@pytest.mark.parametrize('case,builder,bh', [
    ('diffusion7_f32_32cube', W.diffusion_7pt, 'zeros'),
    ('asym7_f32_16cube', W.asym_7pt, 'zeros'),
    ('laplace5_f32_64x64_none', W.laplace_5pt, None),
    ('stencil27_f16_16cube', W.stencil_27pt, 'zeros'),
])
def test_cpu_op_vs_golden(case, builder, bh):
    g = golden(case)
    op = pa.AutoDiffOp(builder(), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    u = torch.from_numpy(g['u']).requires_grad_(True)
    (out,) = fn.apply(u)
    out.backward(torch.from_numpy(g['diffout']))
    tol = 1e-3 if g['u'].dtype == np.float16 else 1e-6
    assert_close_rel(out.detach().numpy(), g['out'], tol, 'out')
    assert_close_rel(u.grad.numpy(), g['diffu'], tol, 'diffu')


def test_time_constant_accumulation_cpu():
    u, out = ps.fields("u, out: float64[6,7]")
    ac = ps.AssignmentCollection({out.center: 2 * u[1, 0] + u.center ** 2})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros', time_constant_fields=[u])
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    rng = np.random.default_rng(0)
    uv = torch.from_numpy(rng.uniform(-1, 1, (6, 7))).requires_grad_(True)
    assert torch.autograd.gradcheck(fn.apply, (uv,), atol=1e-8)
    ref = OE.evaluate(op.backward_assignments, {'u': uv.detach().numpy(), 'diffout': np.ones((6, 7))},
                      boundary_handling='zeros')['diffu']
    (o,) = fn.apply(uv)
    g, = torch.autograd.grad(o, uv, torch.ones(6, 7, dtype=torch.float64))
    assert_close_rel(g.numpy(), ref, 1e-12)


def test_openmp_kernel_matches_serial():
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros', cpu_openmp=True)
    op2 = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    rng = np.random.default_rng(0)
    u = rng.uniform(0, 1, (12, 13, 14)).astype(np.float32)
    o1, o2 = np.zeros_like(u), np.zeros_like(u)
    op.forward_ast_cpu(u=u, out=o1)
    op2.forward_ast_cpu(u=u, out=o2)
    assert '#pragma omp' in op.forward_ast_cpu.compile().code
    assert np.array_equal(o1, o2)


def test_strided_inputs_generic_cpu():
    op = pa.AutoDiffOp(W.laplace_5pt(), boundary_handling='zeros')
    rng = np.random.default_rng(0)
    big = rng.uniform(0, 1, (20, 30))
    u = big[::2, 1::3]                                  # non-contiguous view
    out = np.zeros(u.shape)
    op64 = pa.AutoDiffOp(W.laplace_5pt(dtype='float64'), boundary_handling='zeros')
    op64.forward_ast_cpu(u=u, out=out)
    ref = OE.evaluate(op64.forward_assignments, {'u': np.ascontiguousarray(u)}, boundary_handling='zeros')['out']
    assert_close_rel(out, ref, 1e-14)
    del op


def test_readme_op_cpu_backend_fp32_golden():
    """BASELINE config 1: README op z = x*log(x*y) on [20,30] fp32, CPU backend, forward+backward."""
    g = golden('readme_f32_20x30')
    op = pa.AutoDiffOp(W.readme_op())
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    x = torch.from_numpy(g['x']).requires_grad_(True)
    y = torch.from_numpy(g['y']).requires_grad_(True)
    (z,) = fn.apply(x, y)
    z.backward(torch.from_numpy(g['diffz']))
    assert_close_rel(z.detach().numpy(), g['z'], 1e-6, 'z')
    assert_close_rel(x.grad.numpy(), g['diffx'], 1e-6, 'diffx')
    assert_close_rel(y.grad.numpy(), g['diffy'], 1e-6, 'diffy')
    # the reference interior-only semantics: boundary_handling=None and offset-free -> every cell written
    assert op.forward_ast_cpu.ir.ghost_layers == 0


@pytest.mark.parametrize('radius', (1, 2, 3))
def test_fixed_constant_bh_one_sided_box_cpu(radius):
    """tests/test_fixed_constant_bh.py:22-48 of the reference on the CPU backend, checked against the oracle."""
    import itertools
    x, y = ps.fields("x, y: float64[2d]")
    offs = list(itertools.product(range(radius + 1), repeat=2))
    ac = ps.AssignmentCollection({y.center: sp.Add(*[x[o] for o in offs]) / len(offs)})
    xv = np.random.default_rng(radius).random((20, 30))
    for bh in ('zeros', None):
        op = pa.AutoDiffOp(ac, boundary_handling=bh)
        fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
        (out,) = fn.apply(torch.from_numpy(xv))
        ref = OE.evaluate(op.forward_assignments, {'x': xv}, boundary_handling=bh)['y']
        assert_close_rel(out.numpy(), ref, 1e-12, f'{bh}')


def test_tfmad_two_outputs_vector_field_cpu():
    """tests/test_tfmad.py:353-401 of the reference (curl into a vector field) on the CPU backend, with the
    symbolic adjoint checked term by term and the dot-product identity."""
    inp = ps.Field.create_fixed_size(field_name='curl_input', shape=(20, 30), index_dimensions=0)
    u = ps.Field.create_fixed_size(field_name='curl', shape=(20, 30, 2), index_dimensions=1)
    disc = ps.fd.Discretization2ndOrder(dx=1)
    ac = ps.AssignmentCollection([ps.Assignment(u.center(0), disc(ps.fd.Diff(inp, 0))),
                                  ps.Assignment(u.center(1), disc(ps.fd.Diff(inp, 1)))], [])
    op = pa.AutoDiffOp(ac, diff_mode='transposed-forward', boundary_handling='zeros')
    (bw,) = op.backward_assignments.main_assignments
    dc = op.backward_output_fields[0]
    assert bw.lhs == dc.center
    g_ = [f for f in op.backward_input_fields if f.name == 'diffcurl'][0]
    expected = sp.Rational(1, 2) * (g_[-1, 0](0) - g_[1, 0](0) + g_[0, -1](1) - g_[0, 1](1))
    assert sp.simplify(sp.expand(bw.rhs) - sp.expand(expected)) == 0
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    rng = np.random.default_rng(4)
    x = torch.from_numpy(rng.uniform(-1, 1, (20, 30))).requires_grad_(True)
    g = torch.from_numpy(rng.uniform(-1, 1, (20, 30, 2)))
    (c,) = fn.apply(x)
    c.backward(g)
    cg = float((c.detach() * g).sum())
    assert abs(cg - float((x.detach() * x.grad).sum())) < 1e-10 * float((c.detach() * g).abs().sum())
    ref = OE.evaluate(op.forward_assignments, {'curl_input': x.detach().numpy()}, boundary_handling='zeros')['curl']
    assert_close_rel(c.detach().numpy(), ref, 1e-12, 'curl')


def test_vector_field_partial_writes_and_variable_shapes_cpu():
    """Outputs whose components are not all written keep zero-initialised components (the reference
    allocates every output with torch.zeros, _torch_native.py:64,108); variable-size vector outputs get the
    input's spatial extent plus their own index shape. The vector-field TF-MAD branch stores only the last
    component's adjoint (_autodiff.py:138-152), reproduced on purpose."""
    op = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling='zeros')
    (bw,) = op.backward_assignments.main_assignments
    assert bw.lhs.index == (2,)
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    rng = np.random.default_rng(2)
    u = torch.from_numpy(rng.uniform(-1, 1, (5, 6, 7, 3)).astype(np.float32)).requires_grad_(True)
    g = torch.from_numpy(rng.uniform(-1, 1, (5, 6, 7, 3)).astype(np.float32))
    (o,) = fn.apply(u)
    o.backward(g)
    ref = OE.evaluate(op.forward_assignments, {'u': u.detach().numpy()}, boundary_handling='zeros')['out']
    assert_close_rel(o.detach().numpy(), ref, 1e-6, 'vector laplacian')
    assert torch.count_nonzero(u.grad[..., :2]) == 0
    refb = OE.evaluate(op.backward_assignments, {'diffout': g.numpy()}, boundary_handling='zeros')['diffu']
    assert_close_rel(u.grad.numpy(), refb, 1e-6, 'quirky adjoint')
    # curl with variable-size fields: output (20, 30, 2) from a (20, 30) input
    inp, cu = ps.fields("curl_input, curl(2): float64[2d]")
    disc = ps.fd.Discretization2ndOrder(dx=1)
    ac = ps.AssignmentCollection([ps.Assignment(cu.center(0), disc(ps.fd.Diff(inp, 0))),
                                  ps.Assignment(cu.center(1), disc(ps.fd.Diff(inp, 1)))], [])
    op2 = pa.AutoDiffOp(ac, diff_mode='transposed-forward', boundary_handling='zeros')
    fn2 = op2.create_tensorflow_op(use_cuda=False, backend='torch_native')
    x = torch.from_numpy(rng.uniform(-1, 1, (20, 30))).requires_grad_(True)
    (c,) = fn2.apply(x)
    assert tuple(c.shape) == (20, 30, 2)
    c.backward(torch.ones_like(c))
    assert tuple(x.grad.shape) == (20, 30)


def test_tfmad_gradient_check_torch_backend():
    """tests/test_tfmad.py:100-131 of the reference: backend='torch' with an input-field -> tensor dict,
    gradcheck of the returned Function (here the native Function on the dict tensors' device)."""
    a, b, out = ps.fields("a, b, out: float64[5,7]")
    cont = 2 * ps.fd.Diff(a, 0) - 1.5 * ps.fd.Diff(a, 1) - ps.fd.Diff(b, 0) + 3 * ps.fd.Diff(b, 1)
    assignment = ps.Assignment(out.center(), ps.fd.Discretization2ndOrder(dx=1)(cont) + 1.2 * a.center)
    # boundary 'zeros' (the reference test leaves boundary_handling=None, whose interior-only adjoint is not
    # the forward's transpose at the border, so its gradcheck cannot pass; the torch_native twin uses 'zeros')
    op = pa.AutoDiffOp(ps.AssignmentCollection([assignment], []), diff_mode='transposed-forward',
                       boundary_handling='zeros')
    at = torch.zeros(*a.shape, dtype=torch.float64, requires_grad=True)
    bt = torch.zeros(*b.shape, dtype=torch.float64, requires_grad=True)
    fn = op.create_tensorflow_op({a: at, b: bt}, backend='torch')
    assert torch.autograd.gradcheck(fn.apply, [at, bt])
    with pytest.raises(NotImplementedError):
        op.create_tensorflow_op({a: at, b: bt}, forward_loop=lambda **kw: None, backend='torch')


def test_create_forward_backward_kernel_like_reference():
    """AutoDiffOp.create_forward_kernel / create_backward_kernel (_autodiff.py:592-598): pystencils'
    create_kernel defaults (interior only), ghost_layers=0 -> every cell with zero-padded reads."""
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    rng = np.random.default_rng(3)
    u = rng.uniform(-1, 1, (6, 7, 8)).astype(np.float32)
    for gl, bh in ((None, None), (0, 'zeros')):
        k = op.create_forward_kernel(ghost_layers=gl) if gl is not None else op.create_forward_kernel()
        out = np.zeros_like(u)
        k(u=u, out=out)
        ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=bh)['out']
        assert_close_rel(out, ref, 1e-6, f'forward ghost_layers={gl}')
    kb = op.create_backward_kernel('cpu', ghost_layers=0)
    du = np.zeros_like(u)
    kb(diffout=u, diffu=du)
    assert_close_rel(du, OE.evaluate(op.backward_assignments, {'diffout': u}, boundary_handling='zeros')['diffu'],
                     1e-6, 'backward')


@pytest.mark.parametrize('target', ['cpu', pytest.param('gpu', marks=pytest.mark.gpu)])
@pytest.mark.parametrize('islice', [(slice(1, -1), slice(2, 5)), (slice(0, 3), 4, slice(None)), (-1,),
                                    (slice(2, 2),), (slice(0, None, 2),), (slice(1, -1, 3), slice(None), slice(7, 0, 1)),
                                    (slice(None, None, 2), 3, slice(1, None, 3)), (slice(5, 6, 4), slice(0, 7, 5))])
def test_create_kernel_iteration_slice(target, islice):
    """create_forward_kernel(iteration_slice=...) like pystencils' create_kernel: only the cells of the slice are
    written (absolute coordinates, ghost layers ignored, strided slices: every step-th cell from the start), the rest
    keeps its contents; reads that leave the domain read zeros. CPU (C) and GPU (the one-thread-per-cell HIP
    schedule)."""
    from pystencils_autodiff_amd.lbm import make_slice  # noqa: F401 (the same make_slice surface)
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    rng = np.random.default_rng(9)
    u = rng.uniform(-1, 1, (6, 7, 8)).astype(np.float32)
    k = op.create_forward_kernel(target, iteration_slice=islice)
    ref_full = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out']
    expect = np.full_like(u, 7.0)
    sl = tuple(it if isinstance(it, slice) else slice(it, it + 1 if it != -1 else None) for it in islice)
    expect[sl] = ref_full[sl]
    if target == 'cpu':
        out = np.full_like(u, 7.0)
        k(u=u, out=out)
    else:
        import torch
        ot = torch.full(u.shape, 7.0, device='cuda')
        k(u=torch.from_numpy(u).cuda(), out=ot)
        torch.cuda.synchronize()
        out = ot.cpu().numpy()
        assert k.last_variant[0] == 'generic'
    assert np.array_equal(out == 7.0, expect == 7.0) or np.allclose(out, expect, atol=1e-6)
    assert_close_rel(out, expect, 1e-6, f'slice {islice}')
    with pytest.raises(NotImplementedError):
        op.create_forward_kernel(target, iteration_slice=(slice(None, None, -1),))


@pytest.mark.parametrize('gl', [1, 2, [(1, 2), 3, (2, 1)], [1, 1, (1, 1)]])
def test_create_kernel_explicit_ghost_layers(gl):
    """create_forward_kernel(ghost_layers=k | per-axis (lower, upper)) like pystencils: the kernel writes
    [lower, N - upper) per axis and leaves the rest. The same k >= the stencil radius on every side is the
    interior-only kernel (no iteration slice: on the GPU the tuned schedules); other layers take the
    iteration-slice kernel."""
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    u = np.random.default_rng(4).uniform(-1, 1, (7, 8, 9)).astype(np.float32)
    k = op.create_forward_kernel('cpu', ghost_layers=gl)
    uniform = isinstance(gl, int) or gl == [1, 1, (1, 1)]
    assert (k.ir.islice is None) == uniform, k.ir.islice
    kg = op.create_forward_kernel('gpu', ghost_layers=gl)
    assert (kg.ir.islice is None) == uniform and (not uniform or kg.ir.ghost_layers == (gl if isinstance(gl, int) else 1))
    out = np.full_like(u, 5.0)
    k(u=u, out=out)
    gls = [(gl, gl)] * 3 if isinstance(gl, int) else [(g, g) if isinstance(g, int) else g for g in gl]
    sl = tuple(slice(lo, n - hi) for (lo, hi), n in zip(gls, u.shape))
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out']
    expect = np.full_like(u, 5.0)
    expect[sl] = ref[sl]
    assert_close_rel(out, expect, 1e-6, f'ghost_layers={gl}')


@pytest.mark.parametrize('bmin', [0, 1 << 30])
@pytest.mark.parametrize('builder', [W.asym_7pt, W.stencil_27pt])
def test_interior_only_border_allocation(monkeypatch, bmin, builder):
    """boundary_handling=None (the reference default): outputs are torch.empty + zeroed border slabs
    (BORDER_ZERO_MIN=0) or one memset; uninitialised memory is poisoned with NaN so a missed border
    cell shows up."""
    from pystencils_autodiff_amd.backends import _torch_native as TN
    monkeypatch.setattr(TN, 'BORDER_ZERO_MIN', bmin)
    empty = torch.empty
    monkeypatch.setattr(torch, 'empty', lambda *a, **k: empty(*a, **k).fill_(float('nan')))
    op = pa.AutoDiffOp(builder(), boundary_handling=None)
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    rng = np.random.default_rng(4)
    dt = np.float16 if builder is W.stencil_27pt else np.float32
    u = rng.uniform(-1, 1, (7, 9, 12)).astype(dt)
    d = rng.uniform(-1, 1, (7, 9, 12)).astype(dt)
    uu = torch.from_numpy(u).requires_grad_(True)
    (o,) = fn.apply(uu)
    o.backward(torch.from_numpy(d))
    tol = 1e-3 if dt == np.float16 else 1e-6
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=None)['out']
    refb = OE.evaluate(op.backward_assignments, {'diffout': d}, boundary_handling=None)['diffu']
    assert_close_rel(o.detach().numpy(), ref, tol, 'out')
    assert_close_rel(uu.grad.numpy(), refb, tol, 'diffu')
