"""GPU parity: HIP kernels (through the C ABI) vs the oracle on the same inputs.

Tolerances (north_star: 1e-6 relative for fp32):
  fp32: |gpu - ref| <= 1e-6 * max|ref|, ref = float64 evaluation of the same inputs
  fp64: 1e-12 relative
  fp16 storage (27-point): output rounded to fp16 -> 1e-3 relative (no fp16 path in the reference)
  element-wise (``assert_cells``, the golden linear stencils, the 512³ C-oracle run and the full-size sampled planes):
  |gpu - ref| <= 1e-6·|ref| + (n+2)·2^-24·4·Σ|terms| per cell, + half an fp16 ulp for fp16 storage
"""
import itertools

import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from oracle import stencils as S
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from tests.conftest import abs_terms, assert_cells, assert_cells_linear, assert_close_rel, golden, n_terms

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

TOL = {np.float32: 1e-6, np.float64: 1e-12, np.float16: 1e-3}


def _op(ac, bh='zeros', **kw):
    op = pa.AutoDiffOp(ac, boundary_handling=bh, **kw)
    return op, op.create_tensorflow_op(use_cuda=True, backend='torch_native')


def _run(fn, inputs, grads):
    ins = [torch.from_numpy(np.ascontiguousarray(a)).cuda().requires_grad_(True) for a in inputs]
    outs = fn.apply(*ins)
    torch.autograd.backward(list(outs), [torch.from_numpy(np.ascontiguousarray(g)).cuda() for g in grads])
    torch.cuda.synchronize()
    return [o.detach().cpu().numpy() for o in outs], [i.grad.cpu().numpy() if i.grad is not None else None
                                                      for i in ins]


@pytest.mark.parametrize('case,builder,bh', [
    ('diffusion7_f32_32cube', lambda: W.diffusion_7pt(), 'zeros'),
    ('asym7_f32_16cube', lambda: W.asym_7pt(), 'zeros'),
    ('laplace5_f32_64x64_zeros', lambda: W.laplace_5pt(), 'zeros'),
    ('laplace5_f32_64x64_none', lambda: W.laplace_5pt(), None),
    ('stencil27_f16_16cube', lambda: W.stencil_27pt(), 'zeros'),
])
def test_golden_linear_stencils(case, builder, bh):
    g = golden(case)
    op, fn = _op(builder(), bh)
    (out,), (du,) = _run(fn, [g['u']], [g['diffout']])
    tol = TOL[g['u'].dtype.type]
    assert_close_rel(out, g['out'], tol, f'{case} forward')
    assert_close_rel(du, g['diffu'], tol, f'{case} adjoint')
    # and cell by cell: 1e-6 relative + the fp32 arithmetic bound (+ half an fp16 ulp for fp16 storage)
    st = g['u'].dtype
    assert_cells(out, g['out'], abs_terms(op.forward_assignments, {'u': g['u']}, bh)['out'],
                 n_terms(op.forward_assignments), st, f'{case} forward cells')
    assert_cells(du, g['diffu'], abs_terms(op.backward_assignments, {'diffout': g['diffout']}, bh)['diffu'],
                 n_terms(op.backward_assignments), st, f'{case} adjoint cells')
    k = op.forward_ast_gpu.compile()
    assert k.last_variant[0] == 'march'


def test_golden_readme_op():
    g = golden('readme_f32_20x30')
    op, fn = _op(W.readme_op(), None)
    (z,), (dx, dy) = _run(fn, [g['x'], g['y']], [g['diffz']])
    assert_close_rel(z, g['z'], 1e-6, 'z')
    assert_close_rel(dx, g['diffx'], 1e-6, 'diffx')
    assert_close_rel(dy, g['diffy'], 1e-6, 'diffy')
    assert op.forward_ast_gpu.compile().last_variant[0] == 'pointwise'


def test_golden_tfmad_2d_f64():
    g = golden('tfmad2d_f64_5x7')
    a, b, out = ps.fields("a, b, out: float64[5,7]")
    cont = 2 * ps.fd.Diff(a, 0) - 1.5 * ps.fd.Diff(a, 1) - ps.fd.Diff(b, 0) + 3 * ps.fd.Diff(b, 1)
    ac = ps.AssignmentCollection([ps.Assignment(out.center(), ps.fd.Discretization2ndOrder(dx=1)(cont)
                                                + 1.2 * a.center())], [])
    _, fn = _op(ac)
    (o,), (da, db) = _run(fn, [g['a'], g['b']], [g['diffout']])
    assert_close_rel(o, g['out'], 1e-12, 'out')
    assert_close_rel(da, g['diffa'], 1e-12, 'diffa')
    assert_close_rel(db, g['diffb'], 1e-12, 'diffb')


def test_golden_three_outputs_f64():
    g = golden('three_outputs_f64_21x13')
    a, b, o1, o2, o3 = ps.fields("a, b, out1, out2, out3: float64[21,13]")
    ac = ps.AssignmentCollection({o1.center: a.center + b.center, o2.center: a.center - b.center,
                                  o3.center: sp.exp(b[-1, 0])})
    _, fn = _op(ac)
    outs, (da, db) = _run(fn, [g['a'], g['b']], [g['diffout1'], g['diffout2'], g['diffout3']])
    for got, name in zip(outs, ('out1', 'out2', 'out3')):
        assert_close_rel(got, g[name], 1e-12, name)
    assert_close_rel(da, g['diffa'], 1e-12, 'diffa')
    assert_close_rel(db, g['diffb'], 1e-12, 'diffb')


@pytest.mark.parametrize('with_offsets', (False, True))
def test_gradcheck_torch_native_gpu(with_offsets):
    # reference tests/test_tfmad.py:186-231 with with_cuda=True
    a, b, out = ps.fields("a, b, out: float64[5,7]")
    if with_offsets:
        cont = 2 * ps.fd.Diff(a, 0) - 1.5 * ps.fd.Diff(a, 1) - ps.fd.Diff(b, 0) + 3 * ps.fd.Diff(b, 1)
        asg = ps.Assignment(out.center(), ps.fd.Discretization2ndOrder(dx=1)(cont) + 1.2 * a.center())
    else:
        asg = ps.Assignment(out.center(), 1.2 * a.center + 0.1 * b.center)
    op = pa.AutoDiffOp(ps.AssignmentCollection([asg], []), boundary_handling='zeros',
                       diff_mode='transposed-forward')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    at = torch.zeros(*a.shape, dtype=torch.float64, requires_grad=True).cuda()
    bt = torch.zeros(*b.shape, dtype=torch.float64, requires_grad=True).cuda()
    assert torch.autograd.gradcheck(fn.apply, (at, bt), atol=1e-4, raise_exception=True)
    at = torch.rand(*a.shape, dtype=torch.float64).cuda().requires_grad_(True)
    bt = torch.rand(*b.shape, dtype=torch.float64).cuda().requires_grad_(True)
    assert torch.autograd.gradcheck(fn.apply, (at, bt), atol=1e-6, raise_exception=True)


def test_gradcheck_two_outputs_gpu():
    # reference tests/test_tfmad.py:234-285 with with_cuda=True
    a, b, o1, o2, o3 = ps.fields("a, b, out1, out2, out3: float64[21,13]")
    ac = ps.AssignmentCollection({o1.center: a.center + b.center, o2.center: a.center - b.center,
                                  o3.center: sp.exp(b[-1, 0])})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros', diff_mode='transposed-forward')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    at = torch.zeros(*a.shape, dtype=torch.float64).cuda().requires_grad_(True)
    bt = torch.zeros(*b.shape, dtype=torch.float64).cuda().requires_grad_(True)
    assert torch.autograd.gradcheck(fn.apply, (at, bt), atol=1e-4, raise_exception=True)


def _random_op_case(shape, dtype, bh, taps_per_field=2, seed=0, nonlinear=False):
    """A random multi-field stencil, evaluated through every schedule vs the numpy oracle."""
    rng = np.random.default_rng(seed)
    nd = len(shape)
    tname = {np.float32: 'float32', np.float64: 'float64'}[dtype]
    a, b, out = ps.fields(f"a, b, out: {tname}[{nd}d]")
    offs = [o for o in itertools.product((-1, 0, 1), repeat=nd)]
    rhs = 0
    for f in (a, b):
        for k in rng.choice(len(offs), taps_per_field, replace=False):
            rhs += sp.Float(round(float(rng.uniform(-1, 1)), 3)) * f[offs[k]]
    if nonlinear:
        rhs += sp.Float(0.25) * sp.sin(a.center) * b[offs[rng.integers(len(offs))]]
    return ps.AssignmentCollection({out.center: rhs})


@pytest.mark.parametrize('shape', [(17, 33, 45), (9, 20, 128), (5, 7, 3), (64, 3, 70), (40, 37), (3, 260)])
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_schedules_vs_oracle(shape, bh, dtype):
    ac = _random_op_case(shape, dtype, bh, seed=sum(shape), nonlinear=True)
    op = pa.AutoDiffOp(ac, boundary_handling=bh)
    rng = np.random.default_rng(1)
    a = rng.uniform(-1, 1, shape).astype(dtype)
    b = rng.uniform(-1, 1, shape).astype(dtype)
    d = rng.uniform(-1, 1, shape).astype(dtype)
    ref = OE.evaluate(op.forward_assignments, {'a': a, 'b': b}, boundary_handling=bh)['out']
    refb = OE.evaluate(op.backward_assignments, {'a': a, 'b': b, 'diffout': d}, boundary_handling=bh)
    fk = op.forward_ast_gpu.compile()
    bk = op.backward_ast_gpu.compile()
    ta, tb, td = (torch.from_numpy(x).cuda() for x in (a, b, d))
    for sched in ('march', 'generic'):
        out = torch.zeros(shape, dtype=ta.dtype, device='cuda')
        fk(a=ta, b=tb, out=out, force_schedule=sched)
        da = torch.zeros_like(out)
        db = torch.zeros_like(out)
        bk(a=ta, b=tb, diffout=td, diffa=da, diffb=db, force_schedule=sched)
        torch.cuda.synchronize()
        tol = TOL[dtype]
        assert_close_rel(out.cpu().numpy(), ref, tol, f'{sched} forward')
        assert_close_rel(da.cpu().numpy(), refb['diffa'], tol, f'{sched} diffa')
        assert_close_rel(db.cpu().numpy(), refb['diffb'], tol, f'{sched} diffb')


def test_march_unaligned_variant():
    """X not a multiple of the vector width and a base pointer one element off: the LDS-DMA ring still takes
    16-byte pieces (element-aligned) and zero-fills past each row end (XM)."""
    ac = W.asym_7pt()
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    rng = np.random.default_rng(3)
    u = rng.uniform(0, 1, (8, 9, 31)).astype(np.float32)
    buf = torch.zeros(u.size + 1, device='cuda')
    tu = buf[1:].view(u.shape)
    tu.copy_(torch.from_numpy(u))
    out = torch.zeros(u.shape, device='cuda')
    k(u=tu, out=out)
    torch.cuda.synchronize()
    assert k.last_variant[1].XM and k.last_variant[1].WS
    assert_close_rel(out.cpu().numpy(), S.linear_stencil(u, S.taps_asym_7pt()), 1e-6)


def test_march_halo_planes_equal_full_domain():
    """Two z-slabs with halo planes from their neighbour == one full-domain launch (bitwise)."""
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    g = torch.Generator().manual_seed(0)
    u = torch.rand((24, 20, 64), generator=g).cuda()
    full = torch.empty_like(u)
    k(u=u, out=full)
    lo, hi = u[:10].contiguous(), u[10:].contiguous()
    out_lo, out_hi = torch.empty_like(lo), torch.empty_like(hi)
    k(u=lo, out=out_lo, halos={'u': (None, hi[:1].contiguous())})
    k(u=hi, out=out_hi, halos={'u': (lo[-1:].contiguous(), None)})
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([out_lo, out_hi]), full)


@pytest.mark.parametrize('builder', [W.asym_7pt, lambda: W.stencil_27pt(dtype='float32')], ids=['asym7', '27pt'])
def test_split_launches_interior_then_two_faces(builder):
    """The z-slab launch pattern: interior planes first, then both faces in ONE two-range launch
    (chunk stride = the gap) with halo planes == one full-domain launch, bitwise."""
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    g = torch.Generator().manual_seed(3)
    u = torch.rand((30, 21, 64), generator=g).cuda()
    full = torch.empty_like(u)
    k(u=u, out=full)
    parts = [(0, 11), (11, 19), (19, 30)]
    outs = []
    for i, (a, b) in enumerate(parts):
        sl = u[a:b].contiguous()
        out = torch.full_like(sl, float('nan'))
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < 30 else None
        k(u=sl, out=out, z_range=(1, b - a - 1))
        k(u=sl, out=out, halos={'u': (lo, hi)}, z_range=((0, 1), (b - a - 1, b - a)))
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
    with pytest.raises(ValueError):
        k(u=u, out=full, z_range=((0, 2), (1, 3)))


def test_adjoint_dot_product_identity_large():
    """<A u, d> == <u, A^T d> for the forward / backward kernels at 256^3 (size-independent property)."""
    op, fn = _op(W.asym_7pt())
    g = torch.Generator().manual_seed(0)
    n = 256
    u = torch.rand((n, n, n), generator=g, dtype=torch.float32).cuda().requires_grad_(True)
    d = (torch.rand((n, n, n), generator=g, dtype=torch.float32) * 2 - 1).cuda()
    (out,) = fn.apply(u)
    out.backward(d)
    lhs = torch.sum(out.double() * d.double()).item()
    rhs = torch.sum(u.detach().double() * u.grad.double()).item()
    assert abs(lhs - rhs) <= 1e-5 * max(abs(lhs), 1.0), (lhs, rhs)


def test_diffusion_512_vs_c_oracle():
    """BASELINE config 3 size: forward + adjoint vs the C restatement of the reference CPU kernel."""
    from oracle import cref
    lib = cref.load()
    op, fn = _op(W.diffusion_7pt())
    g = torch.Generator().manual_seed(0)
    n = 512
    u = torch.rand((n, n, n), generator=g, dtype=torch.float32)
    d = torch.rand((n, n, n), generator=g, dtype=torch.float32) * 2 - 1
    uc = u.cuda().requires_grad_(True)
    (out,) = fn.apply(uc)
    out.backward(d.cuda())
    ref_out = lib.diffusion7_f32(u.numpy(), W.ALPHA)
    ref_du = lib.diffusion7_f32(d.numpy(), W.ALPHA)
    # fp32 C reference vs fp32 GPU: both round; compare at 2 ulp of the field scale
    assert_close_rel(out.detach().cpu().numpy(), ref_out, 1e-6, 'out 512^3')
    assert_close_rel(uc.grad.cpu().numpy(), ref_du, 1e-6, 'diffu 512^3')
    # cell by cell: each side within the fp32 arithmetic bound of the exact value, so within twice it of each other
    taps = S.taps_diffusion_7pt()
    absw = {o: abs(w) for o, w in taps.items()}
    assert_cells(out.detach().cpu().numpy(), ref_out, S.linear_stencil(np.abs(u.numpy()), absw), 7, np.float32,
                 'out 512^3 cells', slack=8.0)
    assert_cells(uc.grad.cpu().numpy(), ref_du, S.linear_stencil(np.abs(d.numpy()), absw), 7, np.float32,
                 'diffu 512^3 cells', slack=8.0)


def test_vector_field_generic_schedule():
    f, out = ps.fields("f(2), out: float64[12,10]")
    ac = ps.AssignmentCollection({out.center: f.center(0) * f[1, 0](1) - f[0, -1](0)})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    rng = np.random.default_rng(0)
    fa = rng.uniform(-1, 1, (12, 10, 2))
    ref = OE.evaluate(op.forward_assignments, {'f': fa}, boundary_handling='zeros')['out']
    for sched in (None, 'generic'):        # the default (2-D view: everything on the centre plane -> zsum)
        o = torch.zeros((12, 10), dtype=torch.float64, device='cuda')
        k(f=torch.from_numpy(fa).cuda(), out=o, force_schedule=sched)
        assert k.last_variant[0] == (sched or 'march')
        assert_close_rel(o.cpu().numpy(), ref, 1e-12)


@pytest.mark.parametrize('params', [
    dict(CX=4, NR=8, NT_STORE=True), dict(CX=1, NR=1), dict(CX=2, WX=2, NR=3),
    dict(CX=4, NR=8, ZC=5), dict(CX=1, WX=4, NR=2, ZC=3),
    dict(CX=2, NR=3, NW=1, ZC=4), dict(CX=1, WX=2, NW=2, NR=2),
])
@pytest.mark.parametrize('builder', [W.diffusion_7pt, W.asym_7pt, W.stencil_27pt])
def test_march_tunings_vs_oracle(params, builder):
    """Every tile shape / ring kind gives the oracle's result (ragged tiles, short chunks)."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    is16 = builder is W.stencil_27pt
    dt = np.float16 if is16 else np.float32
    shape = (13, 37, 70) if not is16 else (11, 21, 72)
    rng = np.random.default_rng(5)
    u = rng.uniform(0, 1, shape).astype(dt)
    d = rng.uniform(-1, 1, shape).astype(dt)
    for which, ac, ins, outname in (('f', op.forward_assignments, {'u': u}, 'out'),
                                    ('b', op.backward_assignments, {'diffout': d}, 'diffu')):
        k = StencilKernel(ac, boundary_handling='zeros', function_name=f'tn_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')[outname]
        out = torch.zeros(shape, dtype=torch.float16 if is16 else torch.float32, device='cuda')
        k(**{n: torch.from_numpy(v).cuda() for n, v in ins.items()}, **{outname: out})
        torch.cuda.synchronize()
        assert k.last_variant[0] == 'march'
        assert_close_rel(out.cpu().numpy(), ref, 1e-3 if is16 else 1e-6, f'{params} {which}')
        assert_cells_linear(out.cpu().numpy(), ref, ac, ins, 'zeros', dt, f'{params} {which}')


@pytest.mark.parametrize('params', [dict(VIEW2D='yx'), dict(VIEW2D='zy'), dict(VIEW2D='yx', CX=1, NR=3),
                                    dict(VIEW2D='zy', CX=2, WX=4, NR=1, ZC=7)])
@pytest.mark.parametrize('bh', ['zeros', None])
def test_march_2d_views_vs_oracle(params, bh):
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    u, out = ps.fields("u, out: float32[2d]")
    ac = ps.AssignmentCollection({out.center: 0.3 * u[1, 0] - 0.7 * u[-1, 0] + 0.2 * u[0, 1] + 0.9 * u[0, -1]
                                  - 1.1 * u[1, 1] + u.center})
    rng = np.random.default_rng(2)
    uv = rng.uniform(-1, 1, (45, 300)).astype(np.float32)
    ref = OE.evaluate(ac, {'u': uv}, boundary_handling=bh)['out']
    k = StencilKernel(ac, boundary_handling=bh, function_name='v2d', target='gpu', gpu_indexing_params=params).compile()
    o = torch.zeros(uv.shape, device='cuda')
    k(u=torch.from_numpy(uv).cuda(), out=o)
    torch.cuda.synchronize()
    assert k.last_variant[0] == 'march' and k.last_variant[1].VIEW2D == params['VIEW2D']
    assert_close_rel(o.cpu().numpy(), ref, 1e-6)


def _zsum_cases():
    u, v, out = ps.fields("u, v, out: float32[3d]")
    mixed = ps.AssignmentCollection({out.center: 0.3 * u[1, 1, -1] - 0.2 * u[-1, 0, 1] + 0.5 * u[0, 1, 0]
                                     + sp.sin(u.center) * v.center + 0.1 * v.center})
    return [('27pt', W.stencil_27pt), ('7pt', W.diffusion_7pt), ('asym', W.asym_7pt), ('mixed', lambda: mixed)]


@pytest.mark.parametrize('params', [dict(ZSUM=True), dict(ZSUM=True, CX=1, NR=3, ZC=5),
                                    dict(ZSUM=True, CX=4, NR=8, NT_STORE=True), dict(ZSUM=True, WX=2, CX=2, NR=2),
                                    dict(ZSUM=True, PK=True, CX=2, NR=3, ZC=7),
                                    dict(ZSUM=True, PK=True, AR=True, CX=2, NR=3, ZC=7),
                                    dict(ZSUM=True, PK=True, AR=True, WX=2, CX=4, NR=2, ZC=4),
                                    dict(ZSUM=True, WS=False, NW=1, CX=2, NR=3, ZC=5),
                                    dict(ZSUM=True, WS=False, NW=2, WX=2, PK=True, AR=True, CX=2, NR=2, ZC=6)])
@pytest.mark.parametrize('case', _zsum_cases(), ids=lambda c: c[0])
@pytest.mark.parametrize('bh', ['zeros', None])
def test_zsum_schedule_vs_oracle(params, case, bh):
    """z-partial-sum schedule: forward and adjoint of linear (and linear+centre-nonlinear) stencils."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    name, builder = case
    op = pa.AutoDiffOp(builder(), boundary_handling=bh)
    is16 = name == '27pt'
    dt = np.float16 if is16 else np.float32
    shape = (12, 35, 70)
    rng = np.random.default_rng(7)
    arrays = {f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.forward_input_fields}
    arrays.update({f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.backward_input_fields
                   if f.name not in arrays})
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(ac, boundary_handling=bh, function_name=f'zs_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ir = k.ir
        ins = {f.name: arrays[f.name] for f in ir.fields_read}
        ref = OE.evaluate(ac, ins, boundary_handling=bh)
        outs = {f.name: torch.zeros(shape, dtype=torch.float16 if is16 else torch.float32, device='cuda')
                for f in ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        assert k.last_variant[0] == 'march' and k.last_variant[1].ZSUM
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], 1e-3 if is16 else 1e-6, f'{name} {which} {n}')
        assert_cells_linear({n: t.cpu().numpy() for n, t in outs.items()}, ref, ac, ins, bh, dt, f'{name} {which}')


@pytest.mark.parametrize('params', [dict(ZSUM=True, CX=1, NR=2, ZC=4), dict(ZSUM=True, CX=2, NR=2, PK=True),
                                    dict(ZSUM=True, CX=2, WX=2, NR=4, PK=True, AR=True),
                                    dict(ZSUM=True, CX=2, WX=2, NR=1, PK=True, ZC=3),
                                    dict(ZSUM=False, CX=1, NR=2)])
@pytest.mark.parametrize('case', _zsum_cases(), ids=lambda c: c[0])
def test_interior_tiles_vs_oracle(params, case):
    """Shapes with interior tiles AND edge tiles, odd extents in y."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    name, builder = case
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    is16 = name == '27pt'
    dt = np.float16 if is16 else np.float32
    shape = (7, 29, 520)
    rng = np.random.default_rng(11)
    arrays = {f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.forward_input_fields}
    arrays.update({f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.backward_input_fields
                   if f.name not in arrays})
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(ac, boundary_handling='zeros', function_name=f'it_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')
        outs = {f.name: torch.full(shape, float('nan'), dtype=torch.float16 if is16 else torch.float32, device='cuda')
                for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        assert k.last_variant[0] == 'march'
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], 1e-3 if is16 else 1e-6, f'{name} {which} {n} {params}')
        assert_cells_linear({n: t.cpu().numpy() for n, t in outs.items()}, ref, ac, ins, 'zeros', dt,
                            f'{name} {which} {params}')


def test_zsum_halo_planes_equal_full_domain():
    op = pa.AutoDiffOp(W.stencil_27pt(dtype='float32'), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    assert k.primary_variant()[1].ZSUM
    g = torch.Generator().manual_seed(0)
    u = torch.rand((20, 24, 64), generator=g).cuda()
    full = torch.empty_like(u)
    k(u=u, out=full)
    lo, hi = u[:9].contiguous(), u[9:].contiguous()
    out_lo, out_hi = torch.empty_like(lo), torch.empty_like(hi)
    k(u=lo, out=out_lo, halos={'u': (None, hi[:1].contiguous())})
    k(u=hi, out=out_hi, halos={'u': (lo[-1:].contiguous(), None)})
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([out_lo, out_hi]), full)


def test_hip_graph_capture_of_op():
    """The op's launches are capturable: forward in a torch.cuda.graph, fwd+bwd via make_graphed_callables."""
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    shape = (16, 40, 64)
    g = torch.Generator().manual_seed(0)
    static_u = torch.rand(shape, generator=g).cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn.apply(static_u)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        (static_out,) = fn.apply(static_u)
    new_u = torch.rand(shape, generator=g)
    static_u.copy_(new_u.cuda())
    graph.replay()
    torch.cuda.synchronize()
    assert_close_rel(static_out.cpu().numpy(), S.linear_stencil(new_u.numpy(), S.taps_asym_7pt()), 1e-6, 'graph fwd')

    class M(torch.nn.Module):
        def forward(self, u):
            return fn.apply(u)[0]

    m = torch.cuda.make_graphed_callables(M(), (torch.rand(shape, device='cuda', requires_grad=True),))
    u = torch.rand(shape, generator=g).cuda().requires_grad_(True)
    d = torch.rand(shape, generator=g) * 2 - 1
    out = m(u)
    out.backward(d.cuda())
    torch.cuda.synchronize()
    taps = S.taps_asym_7pt()
    assert_close_rel(out.detach().cpu().numpy(), S.linear_stencil(u.detach().cpu().numpy(), taps), 1e-6, 'graphed out')
    assert_close_rel(u.grad.cpu().numpy(), S.linear_stencil(d.numpy(), S.flip(taps)), 1e-6, 'graphed grad')


def test_scalar_parameter_op_gpu():
    z, y, x = ps.fields("z, y, x: float32[20,40]")
    a = sp.Symbol('a')
    op = pa.AutoDiffOp(ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(a * x[0, 0] * y[0, 0])}))
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(0)
    xv = torch.from_numpy(rng.uniform(0.5, 1.5, (20, 40)).astype(np.float32)).cuda().requires_grad_(True)
    yv = torch.from_numpy(rng.uniform(0.5, 1.5, (20, 40)).astype(np.float32)).cuda().requires_grad_(True)
    with pytest.raises(TypeError, match='class_kwargs'):
        fn.apply(xv, yv)
    fn.class_kwargs['a'] = 5.0
    zt = fn.call(x=xv, y=yv)
    zt.sum().backward()
    xn, yn = xv.detach().cpu().numpy().astype(np.float64), yv.detach().cpu().numpy().astype(np.float64)
    assert_close_rel(zt.detach().cpu().numpy(), xn * np.log(5 * xn * yn), 1e-6)
    assert_close_rel(xv.grad.cpu().numpy(), np.log(5 * xn * yn) + 1, 1e-6)
    assert_close_rel(yv.grad.cpu().numpy(), xn / yn, 1e-6)


def _radius2_cases():
    u, out = ps.fields("u, out: float32[3d]")
    star = 0
    w = [-1 / 12, 4 / 3, -5 / 2, 4 / 3, -1 / 12]                 # 4th-order Laplacian, radius 2
    for d in range(3):
        for k, o in enumerate(range(-2, 3)):
            off = [0, 0, 0]
            off[d] = o
            star += sp.Float(w[k]) * u[tuple(off)]
    asym = 0.3 * u[2, -1, 0] - 0.7 * u[-2, 1, 1] + 0.11 * u[0, 2, -2] + 0.5 * u.center - 0.2 * u[1, 0, 2]
    nonlin = sp.exp(0.1 * u[-2, 0, 0]) * u[0, 1, 0] + 0.3 * u[2, 0, 0]
    return [('star4', ps.AssignmentCollection({out.center: star})),
            ('asym2', ps.AssignmentCollection({out.center: asym})),
            ('nonlin2', ps.AssignmentCollection({out.center: nonlin}))]


@pytest.mark.parametrize('case', _radius2_cases(), ids=lambda c: c[0])
@pytest.mark.parametrize('params', [dict(), dict(ZSUM=False), dict(CX=1, NR=3, ZC=7), dict(ZSUM=False, CX=2, NR=2)])
@pytest.mark.parametrize('bh', ['zeros', None])
def test_radius2_stencils_vs_oracle(case, params, bh):
    from pystencils_autodiff_amd.backends.hip_emitter import zsum_plan
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    name, ac = case
    op = pa.AutoDiffOp(ac, boundary_handling=bh)
    shape = (14, 23, 70)
    rng = np.random.default_rng(11)
    arrays = {'u': rng.uniform(-1, 1, shape).astype(np.float32),
              'diffout': rng.uniform(-1, 1, shape).astype(np.float32)}
    for which, a in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(a, boundary_handling=bh, function_name=f'r2_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(a, ins, boundary_handling=bh)
        outs = {f.name: torch.zeros(shape, device='cuda') for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(v).cuda() for n, v in ins.items()}, **outs)
        torch.cuda.synchronize()
        assert k.last_variant[0] == 'march'
        if params.get('ZSUM', True) is not False and zsum_plan(k.ir, k.last_variant[1]) is None:
            assert not k.last_variant[1].ZSUM
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], 1e-6, f'{name} {which} {n}')


def _ws_cases():
    u, v, out = ps.fields("u, v, out: float32[3d]")
    mixed = ps.AssignmentCollection({out.center: 0.3 * u[1, 1, -1] - 0.2 * u[-1, 0, 1] + 0.5 * u[0, 1, 0]
                                     + sp.sin(u.center) * v.center + 0.1 * v[0, 0, 1]})
    two = ps.AssignmentCollection({out.center: 0.3 * u[1, 0, 0] - 0.2 * v[-1, 0, 1] + 0.5 * u[0, -1, 0]
                                   + 0.25 * v[0, 1, 0] - u.center})
    return [('7pt', W.diffusion_7pt, np.float32), ('asym', W.asym_7pt, np.float32),
            ('27pt_f32', lambda: W.stencil_27pt(dtype='float32'), np.float32), ('mixed', lambda: mixed, np.float32),
            ('two_fields', lambda: two, np.float32), ('7pt_f64', lambda: W.diffusion_7pt(dtype='float64'), np.float64),
            ('27pt_f16', W.stencil_27pt, np.float16), ('asym_f16', lambda: W.asym_7pt(dtype='float16'), np.float16)]


@pytest.mark.parametrize('params', [dict(ZSUM=True, WS=True), dict(ZSUM=True, WS=True, D=1, CX=1, NR=3, ZC=5),
                                    dict(ZSUM=True, WS=True, D=2, CX=2, WX=2, NR=2, ZC=4),
                                    dict(ZSUM=True, WS=True, D=4, CX=4, NR=4, ZC=6),
                                    dict(ZSUM=True, WS=True, PK=True, CX=2, NR=3, ZC=7),
                                    dict(ZSUM=True, WS=True, D=3, CX=2, NR=8, ZC=64),
                                    dict(ZSUM=True, WS=True, PK=True, AR=True, CX=2, WX=2, NR=4, ZC=5),
                                    dict(ZSUM=True, WS=True, CX=4, NR=2, D=2, ZC=5),
                                    dict(ZSUM=True, WS=True, CX=8, NR=1, D=3, ZC=4),
                                    dict(ZSUM=True, WS=True, CX=4, WX=2, NR=3, D=4),
                                    dict(ZSUM=True, WS=True, CX=4, NR=3, D=1)])
@pytest.mark.parametrize('shape', [(12, 35, 72), (7, 29, 520), (4, 5, 8), (9, 3, 264)])
@pytest.mark.parametrize('case', _ws_cases(), ids=lambda c: c[0])
def test_ws_loader_schedule_vs_oracle(params, shape, case):
    """Warp-specialised zsum: LDS-DMA loader wave, counted vmcnt ring, hardware zero fill at the
    domain edge (out-of-range pieces, absent halo planes) — forward and adjoint vs the oracle."""
    from pystencils_autodiff_amd.backends.hip_emitter import ws_geometry
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    name, builder, dt = case
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    rng = np.random.default_rng(sum(shape))
    arrays = {f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.forward_input_fields}
    arrays.update({f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.backward_input_fields
                   if f.name not in arrays})
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(ac, boundary_handling='zeros', function_name=f'ws_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')
        outs = {f.name: torch.full(shape, float('nan'), dtype=getattr(torch, np.dtype(dt).name), device='cuda')
                for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        cfg = k.last_variant[1]
        assert k.last_variant[0] == 'march' and cfg.ZSUM
        if not (params.get('PK') and dt == np.float64) and shape[-1] % (16 // np.dtype(dt).itemsize) == 0 and \
                (dt != np.float16 or cfg.CX % 4 == 0):
            assert ws_geometry(k.ir, cfg) is not None, cfg
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], TOL[dt], f'{name} {which} {n} {params}')
        if dt != np.float64:
            assert_cells_linear({n: t.cpu().numpy() for n, t in outs.items()}, ref, ac, ins, 'zeros', dt,
                                f'{name} {which} {params}')


def test_ws_tilings_bitwise_same_process():
    """The warp-specialised zsum ring (LDS-DMA loader wave, consumer plane barrier ``WS_CONSUMER_BARRIER``): ring
    depths and chunk lengths change which slot holds a plane and when the loader refills it, not the FMA chain of a
    cell — so every such variant, each launched three times in one process, gives bitwise the same 7-point fp32
    forward and adjoint. A consumer read sunk below the next plane barrier (the band kernel's round-4 race) would
    show here as run-to-run or variant-to-variant differences. Another tile shape is other code (the compiler
    contracts the taps differently: 67 025 of 3.4 M cells differ in the last bit, deterministically,
    gpurun_out r05_tests1.log): it is repeated for determinism and checked element-wise against the oracle, as is
    the first variant."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    shape = (70, 96, 512)
    g = torch.Generator().manual_seed(5)
    u = (torch.rand(shape, generator=g) * 2 - 1).cuda()
    variants = (dict(), dict(ZSUM=True, WS=True, D=2), dict(ZSUM=True, WS=True, D=3, ZMIN=8, ZMAX=8),
                dict(ZSUM=True, WS=True, D=4, ZMIN=33, ZMAX=33), dict(ZSUM=True, WS=True, D=1, ZMIN=16, ZMAX=16))
    other_tile = dict(ZSUM=True, WS=True, CX=4, NR=8, D=2)
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        res = []
        for params in variants + (other_tile,):
            k = StencilKernel(ac, boundary_handling='zeros', function_name=f'wsb_{which}', target='gpu',
                              gpu_indexing_params=params).compile()
            for rep in range(3):
                out = torch.full(shape, float('nan'), device='cuda')
                (fin,) = k.ir.fields_read
                k(**{fin.name: u}, **{f.name: out for f in k.ir.fields_written})
                cfg = k.last_variant[1]
                assert cfg.WS and cfg.ZSUM and not cfg.BAND, cfg
                res.append((params, rep, out))
        torch.cuda.synchronize()
        ins = {fin.name: u.cpu().numpy()}
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')
        (name, r64), = ref.items()
        for first in (res[0], res[-3]):
            assert_close_rel(first[2].cpu().numpy(), r64, TOL[np.float32], f'ws {which} {first[0]}')
            assert assert_cells_linear({name: first[2].cpu().numpy()}, ref, ac, ins, 'zeros', np.float32,
                                       f'ws {which} {first[0]}')
        bad = [f'{p} run {rep}: {int((o != res[0][2]).sum())} cells differ' for p, rep, o in res[1:-3]
               if not torch.equal(o, res[0][2])]
        bad += [f'{p} run {rep} vs run 0: {int((o != res[-3][2]).sum())} cells differ' for p, rep, o in res[-2:]
                if not torch.equal(o, res[-3][2])]
        assert not bad, f'{which}: ' + '; '.join(bad)


@pytest.mark.parametrize('case', [
    ('7pt_f32', W.diffusion_7pt, np.float32, (9, 37, 262), 'xm'), ('7pt_f32', W.diffusion_7pt, np.float32, (6, 20, 261), 'xm'),
    ('7pt_f32', W.diffusion_7pt, np.float32, (13, 45, 255), 'xm'), ('asym_f32', W.asym_7pt, np.float32, (11, 29, 134), 'xm'),
    ('27pt_f32', lambda: W.stencil_27pt(dtype='float32'), np.float32, (9, 23, 259), 'xm'),
    ('27pt_f16', W.stencil_27pt, np.float16, (7, 33, 260), 'xm'), ('27pt_f16', W.stencil_27pt, np.float16, (5, 19, 258), 'xm'),
    ('27pt_f16', W.stencil_27pt, np.float16, (6, 17, 131), 'xo'), ('27pt_f16', W.stencil_27pt, np.float16, (7, 20, 255), 'xo'),
    ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16'), np.float16, (8, 41, 132), 'xm'),
    ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16'), np.float16, (9, 70, 262), 'xm'),
    ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16'), np.float16, (5, 23, 133), 'xo'),
    ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16'), np.float16, (9, 33, 257), 'xo'),
    ('7pt_f64', lambda: W.diffusion_7pt(dtype='float64'), np.float64, (6, 17, 65), 'xm'),
    ('5pt_f32', W.laplace_5pt, np.float32, (130, 262), 2), ('5pt_f32', W.laplace_5pt, np.float32, (67, 129), 'generic')],
    ids=lambda c: f'{c[0]}_{"x".join(map(str, c[3]))}')
def test_row_pitch_vector_width_vs_oracle(case):
    """Rows whose byte pitch is not a multiple of 16: with a dword-aligned pitch (fp32 / fp64, fp16 with X even)
    the LDS-DMA ring keeps 16-byte pieces and zero-fills past each row end (XM); odd fp16 rows (every other row
    starts on a half dword) stay on the half-precision ring, loaded one element early and shifted back in LDS
    (XO); 2-D scalar rows take the generic schedule — forward and adjoint of the op's kernels vs the float64
    oracle, NaN-poisoned outputs."""
    name, builder, dt, shape, expect = case
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    rng = np.random.default_rng(sum(shape) + 3)
    arrays = {f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.forward_input_fields}
    arrays.update({f.name: rng.uniform(-1, 1, shape).astype(dt) for f in op.backward_input_fields
                   if f.name not in arrays})
    for which, ac, k in (('f', op.forward_assignments, op.forward_ast_gpu.compile()),
                         ('b', op.backward_assignments, op.backward_ast_gpu.compile())):
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')
        outs = {f.name: torch.full(shape, float('nan'), dtype=getattr(torch, np.dtype(dt).name), device='cuda')
                for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        if expect == 'generic':
            assert k.last_variant[0] == 'generic', k.last_variant
        elif expect == 'xm':            # the LDS-DMA ring with dword-aligned pieces
            assert k.last_variant[0] == 'march' and k.last_variant[1].WS and k.last_variant[1].XM, k.last_variant
        elif expect == 'xo':            # the half ring with rows on half dwords shifted in LDS
            assert k.last_variant[0] == 'march' and k.last_variant[1].WS and k.last_variant[1].XO, k.last_variant
        else:
            assert k.last_variant[0] == 'march' and k.last_variant[1].VE == expect, k.last_variant
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], TOL[dt], f'{name} {which} {n} {shape}')
        if dt != np.float64:
            assert_cells_linear({n: t.cpu().numpy() for n, t in outs.items()}, ref, ac, ins, 'zeros', dt,
                                f'{name} {which} {shape}')


@pytest.mark.parametrize('case', [('27pt_f16', W.stencil_27pt, np.float16, (6, 20, 136)),
                                  ('7pt_f32', W.diffusion_7pt, np.float32, (5, 18, 132))], ids=lambda c: c[0])
def test_one_kernel_alternating_pointer_alignment(case):
    """ONE compiled kernel called with views at element offsets whose byte alignment is 16 (not 32), then 2 or 4,
    then 16 again, then 64: each call must take a plan for its own alignment class (a 16-byte LDS-DMA plan
    reused for a 2-byte-aligned view returns wrong data) — outputs vs the float64 oracle."""
    name, builder, dt, shape = case
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    es = np.dtype(dt).itemsize
    n = int(np.prod(shape))
    tdt = getattr(torch, np.dtype(dt).name)
    rng = np.random.default_rng(11)
    for off_bytes in (16, 2 if es == 2 else 4, 16, 64, 8):
        u = rng.uniform(-1, 1, shape).astype(dt)
        ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out']
        base = torch.empty(n + 64, dtype=tdt, device='cuda')
        ebase = (-base.data_ptr() % 256) // es            # elements to a 256-byte boundary
        tu = base[ebase + off_bytes // es: ebase + off_bytes // es + n].view(shape)
        tu.copy_(torch.from_numpy(u))
        assert tu.data_ptr() % 256 == off_bytes % 256
        out = torch.full(shape, float('nan'), dtype=tdt, device='cuda')
        k(u=tu, out=out)
        torch.cuda.synchronize()
        assert_close_rel(out.cpu().numpy(), ref, TOL[dt], f'{name} offset {off_bytes} B')
        assert_cells_linear(out.cpu().numpy(), ref, op.forward_assignments, {'u': u}, 'zeros', dt, f'offset {off_bytes}')


@pytest.mark.parametrize('shape', [(10, 70, 264), (33, 97, 520), (130, 64, 256)])
@pytest.mark.parametrize('builder', [lambda: W.asym_7pt(dtype='float16'), lambda: W.diffusion_7pt(dtype='float16')],
                         ids=['asym_f16', '7pt_f16'])
def test_ws_fp16_star_default_tiles_vs_oracle(builder, shape):
    """fp16 star stencils at their defaults: half-precision ring with 256×32 tiles (NR=8) and WS chunks down to
    8 planes (the chunk model picks them for small domains) — forward and adjoint vs the float64 oracle."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    rng = np.random.default_rng(sum(shape) + 1)
    arrays = {f.name: rng.uniform(-1, 1, shape).astype(np.float16) for f in op.forward_input_fields}
    arrays.update({f.name: rng.uniform(-1, 1, shape).astype(np.float16) for f in op.backward_input_fields
                   if f.name not in arrays})
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(ac, boundary_handling='zeros', function_name=f'f16s_{which}', target='gpu').compile()
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(ac, ins, boundary_handling='zeros')
        outs = {f.name: torch.full(shape, float('nan'), dtype=torch.float16, device='cuda') for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        kind, cfg = k.last_variant[0], k.last_variant[1]
        assert kind == 'march' and cfg.WS and cfg.NR == 8 and cfg.CX == 4, cfg
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], TOL[np.float16], f'{which} {n} {shape}')
        assert_cells_linear({n: t.cpu().numpy() for n, t in outs.items()}, ref, ac, ins, 'zeros', np.float16,
                            f'{which} {shape}')


@pytest.mark.parametrize('params', [dict(), dict(ZSUM=True, WS=True, D=2, CX=1, NR=2, ZC=3),
                                    dict(ZSUM=True, WS=True, D=4, CX=2, NR=4)])
def test_ws_halos_and_two_range_launches(params):
    """z-slab launch pattern through the LDS-DMA loader: halo planes read in place by the DMA,
    interior planes first, both faces in one two-range launch == one full-domain launch, bitwise."""
    from pystencils_autodiff_amd.backends.hip_emitter import ws_geometry
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros')
    k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='wsh', target='gpu',
                      gpu_indexing_params=params).compile()
    g = torch.Generator().manual_seed(5)
    u = torch.rand((30, 21, 136), generator=g).cuda()
    full = torch.empty_like(u)
    k(u=u, out=full)
    assert ws_geometry(k.ir, k.last_variant[1]) is not None
    parts = [(0, 11), (11, 19), (19, 30)]
    outs = []
    for a, b in parts:
        sl = u[a:b].contiguous()
        out = torch.full_like(sl, float('nan'))
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < 30 else None
        k(u=sl, out=out, z_range=(1, b - a - 1))
        k(u=sl, out=out, halos={'u': (lo, hi)}, z_range=((0, 1), (b - a - 1, b - a)))
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
    ref = S.linear_stencil(u.cpu().numpy(), S.taps_asym_7pt())
    assert_close_rel(full.cpu().numpy(), ref, 1e-6)


@pytest.mark.parametrize('dtype,X', [(torch.float32, 134), (torch.float32, 133), (torch.float64, 67),
                                     (torch.float16, 262), (torch.float16, 263)])
@pytest.mark.parametrize('bh', ['zeros', None])
def test_xm_rows_halos_two_range_and_interior_only(dtype, X, bh):
    """Rows whose pitch is not a multiple of 16 bytes on the LDS-DMA ring (XM): z-slab launch pattern (halo
    planes read in place, interior planes then both faces in one two-range launch) == one full-domain launch,
    bitwise; ``None`` boundary handling (interior-only writes) too; vs the float64 oracle."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    dts = {torch.float32: 'float32', torch.float64: 'float64', torch.float16: 'float16'}[dtype]
    op = pa.AutoDiffOp(W.asym_7pt(dtype=dts), boundary_handling=bh)
    k = StencilKernel(op.forward_assignments, boundary_handling=bh, function_name='xmh', target='gpu').compile()
    g = torch.Generator().manual_seed(X)
    u = torch.rand((30, 21, X), generator=g).to(dtype).cuda()
    full = torch.zeros_like(u)
    k(u=u, out=full)
    assert k.last_variant[1].WS and k.last_variant[1].XM, k.last_variant
    assert bool(k.last_variant[1].XO) == (X % 2 == 1 and dtype == torch.float16), k.last_variant
    kz = None if bh == 'zeros' else (1, 29)
    parts = [(0, 11), (11, 19), (19, 30)]
    outs = []
    from pystencils_autodiff_amd.zslab import ZSlabOp
    for a, b in parts:
        sl = u[a:b].contiguous()
        out = torch.zeros_like(sl)
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < 30 else None
        zl = None if kz is None else (max(0, kz[0] - a), min(b - a, kz[1] - a))
        inner, faces = ZSlabOp._launches(b - a, 1, zl or (0, b - a))     # the z-slab sweep's launch split
        if inner:
            k(u=sl, out=out, z_range=inner, z_limits=zl)
        ZSlabOp._launch_faces(k, {'u': (lo, hi)}, faces, zl, {'u': sl, 'out': out})
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
    ref = OE.evaluate(op.forward_assignments, {'u': u.double().cpu().numpy()}, boundary_handling=bh)['out']
    tol = TOL[{torch.float32: np.float32, torch.float64: np.float64, torch.float16: np.float16}[dtype]]
    assert_close_rel(full.double().cpu().numpy(), ref, tol)


@pytest.mark.parametrize('radius', (1, 2, 3))
@pytest.mark.parametrize('ndim', (2, 3))
def test_fixed_constant_bh_one_sided_box(radius, ndim):
    """Mirror of the reference's tests/test_fixed_constant_bh.py:22-48: a one-sided box mean filter
    (offsets 0..r per axis) with 'zeros' boundary handling (ghost_layers=0) and without (interior
    only), float64 — forward and adjoint through the drop-in op vs the oracle; both agree inside."""
    x, y = ps.fields(f"x, y: float64[{ndim}d]")
    offs = list(itertools.product(range(radius + 1), repeat=ndim))
    ac = ps.AssignmentCollection({y.center: sp.Add(*[x[o] for o in offs]) / len(offs)})
    shape = (20, 30, 40)[:ndim]
    rng = np.random.default_rng(radius)
    xv = rng.random(shape)
    dv = rng.uniform(-1, 1, shape)
    res = {}
    for bh in ('zeros', None):
        op, fn = _op(ac, bh)
        (out,), (dx,) = _run(fn, [xv], [dv])
        ref = OE.evaluate(op.forward_assignments, {'x': xv}, boundary_handling=bh)['y']
        refb = OE.evaluate(op.backward_assignments, {'diffy': dv}, boundary_handling=bh)['diffx']
        assert_close_rel(out, ref, 1e-12, f'{bh} forward')
        assert_close_rel(dx, refb, 1e-12, f'{bh} adjoint')
        res[bh] = out
    inner = tuple(slice(radius, s - radius) for s in shape)
    np.testing.assert_allclose(res['zeros'][inner], res[None][inner], rtol=0, atol=1e-12)


@pytest.mark.parametrize('shape', [(1, 1, 1), (1, 5, 8), (3, 1, 16), (2, 3, 1), (5, 2, 4), (0, 4, 8), (4, 0, 8), (4, 4, 0)])
@pytest.mark.parametrize('case', [('7pt', W.diffusion_7pt, np.float32), ('asym', W.asym_7pt, np.float32),
                                  ('27pt', W.stencil_27pt, np.float16)], ids=lambda c: c[0])
def test_degenerate_and_empty_shapes(shape, case):
    """Single-cell / single-plane / single-row fields (every tap but the centre reads zeros) and empty
    fields through the drop-in op, forward and adjoint, vs the oracle."""
    name, builder, dt = case
    op, fn = _op(builder())
    rng = np.random.default_rng(sum(shape) + 1)
    u = rng.uniform(-1, 1, shape).astype(dt)
    d = rng.uniform(-1, 1, shape).astype(dt)
    (out,), (du,) = _run(fn, [u], [d])
    assert out.shape == shape and du.shape == shape
    if 0 in shape:
        return
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out']
    refb = OE.evaluate(op.backward_assignments, {'diffout': d}, boundary_handling='zeros')['diffu']
    tol = TOL[dt]
    assert_close_rel(out, ref, tol, f'{name} forward {shape}')
    assert_close_rel(du, refb, tol, f'{name} adjoint {shape}')
    assert_cells_linear(out, ref, op.forward_assignments, {'u': u}, 'zeros', dt, f'{name} forward {shape}')
    assert_cells_linear(du, refb, op.backward_assignments, {'diffout': d}, 'zeros', dt, f'{name} adjoint {shape}')


def _curl_op(bh):
    """tests/test_tfmad.py:353-401 of the reference: the curl of a scalar field into a 2-component vector
    field (fixed-size [20, 30] / [20, 30, 2]), diff_mode='transposed-forward'."""
    inp = ps.Field.create_fixed_size(field_name='curl_input', shape=(20, 30), index_dimensions=0)
    u = ps.Field.create_fixed_size(field_name='curl', shape=(20, 30, 2), index_dimensions=1)
    disc = ps.fd.Discretization2ndOrder(dx=1)
    ac = ps.AssignmentCollection([ps.Assignment(u.center(0), disc(ps.fd.Diff(inp, 0))),
                                  ps.Assignment(u.center(1), disc(ps.fd.Diff(inp, 1)))], [])
    return pa.AutoDiffOp(ac, diff_mode='transposed-forward', boundary_handling=bh)


@pytest.mark.parametrize('bh', ['zeros', None])
def test_tfmad_two_outputs_vector_field_gpu(bh):
    op = _curl_op(bh)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(4)
    x = rng.uniform(-1, 1, (20, 30))
    g = rng.uniform(-1, 1, (20, 30, 2))
    (c,), (dx,) = _run(fn, [x], [g])
    ref = OE.evaluate(op.forward_assignments, {'curl_input': x}, boundary_handling=bh)['curl']
    refb = OE.evaluate(op.backward_assignments, {'diffcurl': g}, boundary_handling=bh)['diffcurl_input']
    assert_close_rel(c, ref, 1e-12, 'curl')
    assert_close_rel(dx, refb, 1e-12, 'diffcurl_input')
    # the adjoint is the transpose of the forward: <A x, g> == <x, A^T g> ('zeros' only: the interior-only
    # variant leaves border cells untouched, which is not a linear map's transpose)
    if bh == 'zeros':
        assert abs(float(np.sum(c * g)) - float(np.sum(x * dx))) < 1e-10 * float(np.sum(np.abs(c * g)))


def test_vector_field_partial_writes_and_variable_shapes_gpu():
    """GPU twin of test_cpu_backend.test_vector_field_partial_writes_and_variable_shapes_cpu."""
    op, fn = _op(W.vector_laplace_7pt())
    rng = np.random.default_rng(2)
    u = rng.uniform(-1, 1, (5, 6, 7, 3)).astype(np.float32)
    g = rng.uniform(-1, 1, (5, 6, 7, 3)).astype(np.float32)
    (o,), (du,) = _run(fn, [u], [g])
    assert_close_rel(o, OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out'], 1e-6, 'fwd')
    assert np.count_nonzero(du[..., :2]) == 0
    refb = OE.evaluate(op.backward_assignments, {'diffout': g}, boundary_handling='zeros')['diffu']
    assert_close_rel(du, refb, 1e-6, 'quirky adjoint')
    inp, cu = ps.fields("curl_input, curl(2): float64[2d]")
    disc = ps.fd.Discretization2ndOrder(dx=1)
    ac = ps.AssignmentCollection([ps.Assignment(cu.center(0), disc(ps.fd.Diff(inp, 0))),
                                  ps.Assignment(cu.center(1), disc(ps.fd.Diff(inp, 1)))], [])
    op2 = pa.AutoDiffOp(ac, diff_mode='transposed-forward', boundary_handling='zeros')
    fn2 = op2.create_tensorflow_op(use_cuda=True, backend='torch_native')
    x = rng.uniform(-1, 1, (20, 30))
    (c,), (dx,) = _run(fn2, [x], [np.ones((20, 30, 2))])
    assert c.shape == (20, 30, 2) and dx.shape == (20, 30)
    assert_close_rel(c, OE.evaluate(op2.forward_assignments, {'curl_input': x}, boundary_handling='zeros')['curl'],
                     1e-12, 'curl')


def _vector_cases():
    u, v, out = ps.fields("u(3), v, out(2): float32[3d]")
    mix = ps.AssignmentCollection({out.center(0): 0.3 * u[1, 0, 0](1) - 0.2 * u[0, -1, 1](2) + 0.5 * u.center(0)
                                   + sp.sin(v.center) * u.center(1),
                                   out.center(1): 0.7 * u[-1, 1, 0](0) + 0.1 * u[0, 0, -1](2) - v.center})
    w, o2 = ps.fields("w(2), o2(2): float64[3d]")
    d64 = ps.AssignmentCollection({o2.center(c): w[1, 0, 0](c) + w[0, 0, -1](1 - c) - 2.5 * w.center(c)
                                   for c in range(2)})
    q, o3 = ps.fields("q(4), o3(4): float32[2d]")
    two_d = ps.AssignmentCollection({o3.center(c): q[1, 0](c) - q[0, -1]((c + 1) % 4) + 0.25 * q.center(c)
                                     for c in range(4)})
    return [('veclap3', W.vector_laplace_7pt, np.float32), ('mixed', lambda: mix, np.float32),
            ('f64_2comp', lambda: d64, np.float64), ('2d_4comp', lambda: two_d, np.float32)]


@pytest.mark.parametrize('params', [dict(), dict(ZSUM=True, WS=False, CX=1, NR=3, ZC=5),
                                    dict(ZSUM=True, WS=True, D=2, CX=2, NR=2, ZC=4),
                                    dict(ZSUM=True, WS=False, CX=2, WX=2, NR=2, PK=True)])
@pytest.mark.parametrize('case', _vector_cases(), ids=lambda c: c[0])
def test_vector_fields_zsum_vs_oracle(params, case):
    """Vector fields (components fastest in memory) through the zsum schedule: the plane image holds
    the interleaved components, taps and stores carry the component offset — forward and the TF-MAD
    adjoint vs the oracle, ragged shapes with interior and edge tiles."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    name, builder, dt = case
    ac = builder()
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    is2d = name.startswith('2d')
    spatial = (37, 72) if is2d else (6, 13, 136)
    rng = np.random.default_rng(len(name))

    def arr(f):
        return rng.uniform(-1, 1, spatial + tuple(int(n) for n in f.index_shape)).astype(dt)
    arrays = {f.name: arr(f) for f in list(op.forward_input_fields) + list(op.backward_input_fields)}
    for which, a in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = StencilKernel(a, boundary_handling='zeros', function_name=f'vz_{which}', target='gpu',
                          gpu_indexing_params=params).compile()
        ins = {f.name: arrays[f.name] for f in k.ir.fields_read}
        ref = OE.evaluate(a, ins, boundary_handling='zeros')
        outs = {f.name: torch.full(spatial + tuple(int(n) for n in f.index_shape), float('nan'),
                                   dtype=getattr(torch, np.dtype(dt).name), device='cuda') for f in k.ir.fields_written}
        for n, t in outs.items():          # components a kernel does not write stay as allocated (zeros here)
            t.zero_()
        k(**{n: torch.from_numpy(v).cuda() for n, v in ins.items()}, **outs)
        torch.cuda.synchronize()
        if k.ir.stencil_fields:
            assert k.last_variant[0] == 'march' and k.last_variant[1].ZSUM, k.last_variant
        for n, t in outs.items():
            assert_close_rel(t.cpu().numpy(), ref[n], TOL[dt], f'{name} {which} {n} {params}')


def test_vector_field_halos_and_two_range_launches():
    """z-slab launch pattern for a vector field: halo planes carry all components."""
    op = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    g = torch.Generator().manual_seed(9)
    u = torch.rand((20, 11, 72, 3), generator=g).cuda()
    full = torch.empty_like(u)
    k(u=u, out=full)
    assert k.last_variant[0] == 'march'
    outs = []
    for a, b in [(0, 7), (7, 13), (13, 20)]:
        sl = u[a:b].contiguous()
        out = torch.full_like(sl, float('nan'))
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < 20 else None
        k(u=sl, out=out, z_range=(1, b - a - 1))
        k(u=sl, out=out, halos={'u': (lo, hi)}, z_range=((0, 1), (b - a - 1, b - a)))
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)


@pytest.mark.parametrize('shape', [(100, 40, 384), (37, 24, 640), (130, 17, 768)])
def test_ws_residency_chunking_shapes_vs_oracle(shape):
    """Default 7-point op at x extents that trigger half-width WS tiles / residency-aware chunk counts."""
    g = np.random.default_rng(sum(shape))
    u = g.uniform(0, 1, shape).astype(np.float32)
    d = g.uniform(-1, 1, shape).astype(np.float32)
    op, fn = _op(W.asym_7pt())
    (out,), (du,) = _run(fn, [u], [d])
    taps = S.taps_asym_7pt()
    assert_close_rel(out, S.linear_stencil(u, taps), 1e-6, 'out')
    assert_close_rel(du, S.linear_stencil(d, S.flip(taps)), 1e-6, 'diffu')
    assert op.forward_ast_gpu.compile().last_variant[1].WS


@pytest.mark.parametrize('bmin', [0, 1 << 30])
@pytest.mark.parametrize('builder,shape', [(W.asym_7pt, (20, 33, 70)), (W.stencil_27pt, (9, 24, 80)),
                                           (W.laplace_5pt, (40, 70)), (W.asym_7pt, (6, 9, 300)),
                                           (W.vector_laplace_7pt, (7, 10, 40, 3))])
@pytest.mark.parametrize('native', [False, True])
def test_interior_only_border_allocation_gpu(monkeypatch, bmin, builder, shape, native):
    """boundary_handling=None: torch.empty outputs with zeroed border slabs (or one memset) on the GPU;
    uninitialised memory poisoned with NaN. ``native``: through the C++ autograd node (which allocates
    small interior-only outputs with one memset, ``_NativePath``), its uninitialised outputs poisoned too."""
    from pystencils_autodiff_amd.backends import _torch_native as TN
    monkeypatch.setattr(TN, 'BORDER_KERNEL', bmin == 0)
    empty = torch.empty
    monkeypatch.setattr(torch, 'empty', lambda *a, **k: empty(*a, **k).fill_(float('nan')))
    m = TN.native_module()
    if not native:
        monkeypatch.setattr(TN, '_native', False)
    g = np.random.default_rng(6)
    dt = np.float16 if builder is W.stencil_27pt else np.float32
    u = g.uniform(-1, 1, shape).astype(dt)
    d = g.uniform(-1, 1, shape).astype(dt)
    m.set_debug_poison(native)
    try:
        op, fn = _op(builder(), None)
        (out,), (du,) = _run(fn, [u], [d])
    finally:
        m.set_debug_poison(False)
    tol = 1e-3 if dt == np.float16 else 1e-6
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=None)['out']
    refb = OE.evaluate(op.backward_assignments, {'diffout': d}, boundary_handling=None)['diffu']
    assert_close_rel(out, ref, tol, 'out')
    assert_close_rel(du, refb, tol, 'diffu')
    assert_cells_linear(out, ref, op.forward_assignments, {'u': u}, None, dt, 'out')
    assert_cells_linear(du, refb, op.backward_assignments, {'diffout': d}, None, dt, 'diffu')
    if bmin == 0 and not native:
        v = op.forward_ast_gpu.compile().last_variant[1]
        assert v.XB or not v.ZSUM              # zsum launches store the x ends themselves


@pytest.mark.parametrize('builder,n,tol', [(W.diffusion_7pt, 1024, 1e-6), (W.stencil_27pt, 768, 1e-3)])
def test_full_size_properties(builder, n, tol):
    """BASELINE full sizes (1024³ fp32 7-point, 768³ fp16 27-point) through the op: sampled planes (both
    domain faces, the middle, chunk edges) vs the oracle evaluated on the 3-plane neighbourhood,
    the adjoint dot-product identity <A u, d> = <u, Aᵀ d>, and linearity A(u + 2v) = Au + 2Av."""
    op, fn = _op(builder())
    dt = torch.float16 if builder is W.stencil_27pt else torch.float32
    taps = S.taps_27pt() if builder is W.stencil_27pt else S.taps_diffusion_7pt()
    g = torch.Generator(device='cuda').manual_seed(7)
    u = torch.rand((n, n, n), generator=g, device='cuda').to(dt).requires_grad_(True)
    d = (torch.rand((n, n, n), generator=g, device='cuda') * 2 - 1).to(dt)
    (out,) = fn.apply(u)
    out.backward(d)
    torch.cuda.synchronize()
    for z in (0, 1, n // 2, 127, 128, n - 2, n - 1):
        lo, hi = max(0, z - 1), min(n, z + 2)
        uu = u.detach()[lo:hi].cpu().numpy()
        dd = d[lo:hi].cpu().numpy()
        ref_o = S.linear_stencil(uu, taps)[z - lo]
        ref_g = S.linear_stencil(dd, S.flip(taps))[z - lo]
        assert_close_rel(out.detach()[z].cpu().numpy(), ref_o, tol, f'out plane {z}')
        assert_close_rel(u.grad[z].cpu().numpy(), ref_g, tol, f'diffu plane {z}')
        # cell by cell (1e-6 relative + fp32 arithmetic bound; fp16 storage: + half an fp16 ulp)
        absw = {o: abs(w) for o, w in taps.items()}
        st = np.float16 if dt == torch.float16 else np.float32
        assert_cells(out.detach()[z].cpu().numpy(), ref_o, S.linear_stencil(np.abs(uu), absw)[z - lo], len(taps), st,
                     f'out plane {z} cells')
        assert_cells(u.grad[z].cpu().numpy(), ref_g, S.linear_stencil(np.abs(dd), S.flip(absw))[z - lo], len(taps), st,
                     f'diffu plane {z} cells')
    lhs = torch.sum(out.detach().double() * d.double()).item()
    rhs = torch.sum(u.detach().double() * u.grad.double()).item()
    assert abs(lhs - rhs) <= (1e-5 if dt == torch.float32 else 2e-3) * max(abs(lhs), 1.0), (lhs, rhs)
    if dt == torch.float32:
        v = torch.rand((n, n, n), generator=g, device='cuda')
        with torch.no_grad():
            (a1,) = fn.apply(u.detach())
            (a2,) = fn.apply(v)
            (a3,) = fn.apply(u.detach() + 2 * v)
            err = (a3 - (a1 + 2 * a2)).abs().max().item()
        assert err <= 4e-6 * a3.abs().max().item(), err


def test_full_size_2d_and_readme_op():
    """BASELINE config 2 at full size (4096² 5-point, every cell vs the oracle, field-scaled AND element-wise) and
    the README op at 16384² (sampled rows vs the closed-form forward / adjoint, field-scaled and per cell: the fp32
    evaluation of ``x·log(x·y)`` and its adjoint bounded by a few ulps of each cell's own terms)."""
    op, fn = _op(W.laplace_5pt())
    g = np.random.default_rng(3)
    u = g.uniform(0, 1, (4096, 4096)).astype(np.float32)
    d = g.uniform(-1, 1, (4096, 4096)).astype(np.float32)
    (out,), (du,) = _run(fn, [u], [d])
    ref_o, ref_d = S.linear_stencil(u, S.taps_laplace_5pt()), S.linear_stencil(d, S.flip(S.taps_laplace_5pt()))
    assert_close_rel(out, ref_o, 1e-6, 'laplace 4096² out')
    assert_close_rel(du, ref_d, 1e-6, 'laplace 4096² diffu')
    absu = S.linear_stencil(np.abs(u), {o: abs(w) for o, w in S.taps_laplace_5pt().items()})
    absd = S.linear_stencil(np.abs(d), {o: abs(w) for o, w in S.flip(S.taps_laplace_5pt()).items()})
    assert_cells(out, ref_o, absu, 5, np.float32, 'laplace 4096² out')
    assert_cells(du, ref_d, absd, 5, np.float32, 'laplace 4096² diffu')
    op, fn = _op(W.readme_op(shape=None), None)
    n = 16384
    gt = torch.Generator(device='cuda').manual_seed(5)
    x = (torch.rand((n, n), generator=gt, device='cuda') + 0.5).requires_grad_(True)
    y = (torch.rand((n, n), generator=gt, device='cuda') + 0.5).requires_grad_(True)
    dz = torch.rand((n, n), generator=gt, device='cuda') * 2 - 1
    (z,) = fn.apply(x, y)
    z.backward(dz)
    for r in (0, 1, n // 2, n - 1):
        xr, yr, dr = (t.detach()[r].cpu().numpy() for t in (x, y, dz))
        z_ref = S.readme_forward(xr, yr)
        assert_close_rel(z.detach()[r].cpu().numpy(), z_ref, 1e-6, f'z row {r}')
        dx_ref, dy_ref = S.readme_backward(xr, yr, dr)
        assert_close_rel(x.grad[r].cpu().numpy(), dx_ref, 1e-6, f'diffx row {r}')
        assert_close_rel(y.grad[r].cpu().numpy(), dy_ref, 1e-6, f'diffy row {r}')
        # per cell: the rounding of x·y, log and the products, each a few ulps of the cell's own magnitudes
        x64, y64, d64 = (np.asarray(a, np.float64) for a in (xr, yr, dr))
        lg = np.abs(np.log(x64 * y64))
        assert_cells(z.detach()[r].cpu().numpy(), z_ref, np.abs(x64) * (lg + 1) + np.abs(z_ref), 2, np.float32,
                     f'z row {r}')
        assert_cells(x.grad[r].cpu().numpy(), dx_ref, np.abs(d64) * (lg + 2), 2, np.float32, f'diffx row {r}')
        assert_cells(y.grad[r].cpu().numpy(), dy_ref, 3 * np.abs(dy_ref), 2, np.float32, f'diffy row {r}')
