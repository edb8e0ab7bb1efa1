"""Variable-coefficient diffusion ``out = u + α Σ₆ ½(k + k[nb])(u[nb] − u)`` (``workloads.varcoef_diffusion_7pt``):
a bilinear stencil of two input fields whose TF-MAD adjoint has two outputs from three inputs.

The reference's TF-MAD (``_autodiff.py:101-106``) multiplies ``∂rhs/∂u[o]`` — evaluated at the OUTPUT cell —
by ``diffout[−o]``; the true reverse-mode gradient evaluates that derivative at the cell ``−o``. The two agree for
stencils whose derivatives do not vary in space (every linear stencil, or this one with a uniform ``k``), and
differ here otherwise: a user of the reference gets the TF-MAD adjoint, so that is what the drop-in computes and
what parity is checked against — the numpy oracle evaluating the op's TF-MAD assignments, cell by cell with
|got − ref| ≤ 1e-6·|ref| + 32·2⁻²⁴·Σ|terms| for fp32 (Σ|terms| = every expanded product made non-negative, on
|inputs|), 1e-12 for fp64. The forward is also checked against torch float64, and the adjoint against torch
float64 autograd where the two semantics coincide (uniform ``k``, cells away from the zero border)."""
import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from tests.conftest import fp16_ulp

torch = pytest.importorskip('torch')

NB = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
_OPS = {}


def _op(dts='float32'):
    if dts not in _OPS:
        _OPS[dts] = pa.AutoDiffOp(W.varcoef_diffusion_7pt(dtype=dts), boundary_handling='zeros')
    return _OPS[dts]


def _shift(t, o):
    """t[x + o] with zeros outside the box."""
    p = torch.nn.functional.pad(t, (1, 1, 1, 1, 1, 1))
    s = t.shape
    return p[1 + o[0]:1 + o[0] + s[0], 1 + o[1]:1 + o[1] + s[1], 1 + o[2]:1 + o[2] + s[2]]


def torch_varcoef(u, k, alpha=W.ALPHA):
    acc = 0
    for o in NB:
        acc = acc + 0.5 * (k + _shift(k, o)) * (_shift(u, o) - u)
    return u + alpha * acc


def _abs_terms(collection):
    """The collection with every expanded product's coefficient made non-negative: on |inputs| it gives
    Σ|terms| per cell."""
    flat = collection.new_without_subexpressions()
    mains = []
    for a in flat.main_assignments:
        new = 0
        for t in sp.Add.make_args(sp.expand(a.rhs)):
            c, rest = t.as_coeff_Mul()
            new += abs(float(c)) * rest
        mains.append(ps.Assignment(a.lhs, new))
    return ps.AssignmentCollection(mains)


def oracle(op, u, k, d):
    """({out, diffu, diffk} of the op's TF-MAD assignments, same keys: Σ|terms|), float64 numpy."""
    arrs = {'u': u, 'k': k}
    absd = {'u': np.abs(u), 'k': np.abs(k), 'diffout': np.abs(d)}
    ref = {**OE.evaluate(op.forward_assignments, arrs, boundary_handling='zeros'),
           **OE.evaluate(op.backward_assignments, {**arrs, 'diffout': d}, boundary_handling='zeros')}
    ab = {**OE.evaluate(_abs_terms(op.forward_assignments), absd, boundary_handling='zeros'),
          **OE.evaluate(_abs_terms(op.backward_assignments), absd, boundary_handling='zeros')}
    return ref, ab


def check(got, ref, absterms, fp64, what, fp16=False):
    """fp16 storage: the fp32 bound plus half an fp16 ulp of the stored result (conftest.assert_cells' form)."""
    got = got.detach().double().cpu().numpy() if hasattr(got, 'detach') else np.asarray(got, np.float64)
    bound = 1e-12 * (np.abs(ref) + absterms) if fp64 else 1e-6 * np.abs(ref) + 32 * 2.0 ** -24 * absterms
    if fp16:
        bound = bound + 0.5 * fp16_ulp(np.abs(ref) + bound)
    err = np.abs(got - ref)
    bad = err > bound
    assert not bad.any(), f'{what}: {int(bad.sum())} of {bad.size} cells outside the bound, worst err {err.max():.3e}'


def _inputs(shape, dtype, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    u = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1).to(dtype)
    k = (torch.rand(shape, generator=g, dtype=torch.float64) + 0.1).to(dtype)
    d = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1).to(dtype)
    return [x.to(device) for x in (u, k, d)]


def _apply(op, u, k, d, device):
    assert [f.name for f in op.forward_input_fields] == ['k', 'u']
    fn = op.create_tensorflow_op(use_cuda=device == 'cuda', backend='torch_native')
    kk, uu = k.clone().requires_grad_(True), u.clone().requires_grad_(True)
    out = fn.apply(kk, uu)
    out = out[0] if isinstance(out, (tuple, list)) else out
    out.backward(d)
    return out, uu.grad, kk.grad


def _run(shape, dtype, device, seed=0):
    fp64, fp16 = dtype == torch.float64, dtype == torch.float16
    op = _op({torch.float64: 'float64', torch.float16: 'float16'}.get(dtype, 'float32'))
    u, k, d = _inputs(shape, dtype, device, seed)
    out, gu, gk = _apply(op, u, k, d, device)
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], fp64, 'out', fp16)
    check(gu, ref['diffu'], ab['diffu'], fp64, 'diffu', fp16)
    check(gk, ref['diffk'], ab['diffk'], fp64, 'diffk', fp16)
    # the forward against an independent restatement
    ro = torch_varcoef(u.double().cpu(), k.double().cpu()).numpy()
    check(out, ro, ab['out'], fp64, 'out vs torch', fp16)


def test_varcoef_cpu_backend_vs_oracle():
    _run((6, 9, 11), torch.float64, 'cpu')
    _run((5, 8, 13), torch.float32, 'cpu', seed=1)


def test_polynomial_cell_bound_engages_on_varcoef():
    """``conftest.assert_cells_linear`` takes polynomial (not only linear) collections: the varcoef forward and its
    TF-MAD adjoint (products of two taps) are checked cell by cell with Σ|terms| of their expansion — here on the C
    kernels (fp32 arithmetic); the GPU tests call the same helper. A stencil with a function of its taps still returns
    False (the caller's field-scaled check only)."""
    from tests.conftest import abs_poly, assert_cells_linear
    op = _op('float32')
    u, k, d = _inputs((9, 14, 20), torch.float32, 'cpu', seed=21)
    out, gu, gk = _apply(op, u, k, d, 'cpu')
    arr = {'u': u.double().numpy(), 'k': k.double().numpy(), 'diffout': d.double().numpy()}
    ref = {**OE.evaluate(op.forward_assignments, arr, boundary_handling='zeros'),
           **OE.evaluate(op.backward_assignments, arr, boundary_handling='zeros')}
    assert abs_poly(op.forward_assignments, 4)[1] == 2 and abs_poly(op.backward_assignments, 4)[1] == 2
    assert assert_cells_linear({'out': out.detach().numpy()}, {'out': ref['out']}, op.forward_assignments,
                               {'u': arr['u'], 'k': arr['k']}, 'zeros', np.float32, 'fwd')
    assert assert_cells_linear({'diffu': gu.numpy(), 'diffk': gk.numpy()},
                               {'diffu': ref['diffu'], 'diffk': ref['diffk']}, op.backward_assignments, arr, 'zeros',
                               np.float32, 'bwd')
    a, b = ps.fields('a, b: float32[3d]')
    assert abs_poly(ps.AssignmentCollection({b.center: sp.sin(a[1, 0, 0]) * a[0, 0, -1]}), 4) is None


def test_varcoef_tfmad_is_reverse_mode_for_uniform_k():
    """With a uniform conductivity the TF-MAD ``diffu`` is the true gradient away from the zero border (where
    ``k[nb]`` reads 0 and the derivative varies in space); with a varying one it is not, and ``diffk`` (whose
    derivatives ``½α(u[nb] − u)`` vary with ``u``) never is — the reference's semantics, ``_autodiff.py:101-106``."""
    op = _op('float64')
    shape = (8, 9, 10)
    u, k, d = _inputs(shape, torch.float64, 'cpu', seed=2)
    for uniform in (True, False):
        kk = torch.full(shape, 0.7, dtype=torch.float64) if uniform else k
        _, gu, gk = _apply(op, u, kk, d, 'cpu')
        u64, k64 = u.clone().requires_grad_(True), kk.clone().requires_grad_(True)
        tu, tk = torch.autograd.grad(torch_varcoef(u64, k64), (u64, k64), d)
        inner = (slice(2, -2),) * 3
        assert torch.allclose(gu[inner], tu[inner], rtol=1e-12, atol=1e-12) == uniform
        assert not torch.allclose(gk[inner], tk[inner], rtol=1e-6, atol=1e-6)


def test_ws_fallback_config_drops_eight_waves():
    """Planes beyond the loader's 32-bit offsets take the register-prefetch form of the same schedule; an NW=8
    override (LDS-DMA ring only) falls back to four waves instead of raising (geometry only, no GPU)."""
    from pystencils_autodiff_amd.backends.hip_emitter import MarchConfig
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel, ws_fallback_config
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = _op('float32')
    k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='vcfb', target='gpu',
                      gpu_indexing_params=dict(WS=1, NW=8, CX=2, WX=2, NR=1, D=2))
    cfg = HipStencilKernel(k)._march_cfg(4, (64, 64, 256))
    assert cfg.WS and cfg.NW == 8 and not cfg.ZSUM
    fb = ws_fallback_config(cfg)
    assert not fb.WS and fb.NW == 4 and fb.WX == 2 and (fb.CX, fb.NR) == (cfg.CX, cfg.NR)
    four = ws_fallback_config(MarchConfig(**{**cfg.__dict__, 'NW': 4, 'WX': 1}))
    assert not four.WS and four.NW == 4 and four.WX == 1


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(17, 33, 45), (9, 20, 128), (5, 7, 3), (40, 64, 256), (33, 50, 130)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.float64, torch.float16], ids=['f32', 'f64', 'f16'])
def test_varcoef_gpu_vs_oracle(shape, dtype):
    _run(shape, dtype, 'cuda')


@pytest.mark.gpu
@pytest.mark.parametrize('sched', ['march', 'generic'])
def test_varcoef_schedules_gpu(sched):
    """Each schedule the kernels can take, forced, on an unaligned box."""
    op = _op()
    shape = (21, 34, 67)
    u, k, d = _inputs(shape, torch.float32, 'cuda', seed=3)
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    out = torch.zeros_like(u)
    fk(u=u, k=k, out=out, force_schedule=sched)
    du, dk = torch.zeros_like(u), torch.zeros_like(u)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk, force_schedule=sched)
    torch.cuda.synchronize()
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], False, f'{sched} out')
    check(du, ref['diffu'], ab['diffu'], False, f'{sched} diffu')
    check(dk, ref['diffk'], ab['diffk'], False, f'{sched} diffk')


@pytest.mark.gpu
def test_varcoef_full_size_gpu():
    """160³ fp32 on the default schedule, every cell against the oracle."""
    _run((160, 160, 160), torch.float32, 'cuda', seed=5)


@pytest.mark.gpu
@pytest.mark.parametrize('params', [dict(WS=1, NW=8, CX=4, NR=1, D=2), dict(WS=1, NW=8, CX=2, NR=2, D=3),
                                    dict(WS=1, CX=2, NR=2, D=1), dict(WS=1, CX=1, WX=4, NR=4, D=2),
                                    dict(WS=0, CX=2, NR=2), dict(WS=0, PD=2, CX=2, NR=2),
                                    dict(WS=0, PD=2, CX=4, NR=1, PR=1)], ids=str)
def test_varcoef_ring_tilings_gpu(params):
    """The plane ring's tilings (8 compute waves, ring depths, register-prefetch form) on a box of ragged tiles and
    chunks, every cell against the oracle."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = _op()
    shape = (19, 37, 200)
    u, k, d = _inputs(shape, torch.float32, 'cuda', seed=7)
    fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='vct_f', target='gpu',
                       gpu_indexing_params=params).compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='vct_b', target='gpu',
                       gpu_indexing_params=params).compile()
    out, du, dk = (torch.zeros_like(u) for _ in range(3))
    fk(u=u, k=k, out=out)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
    torch.cuda.synchronize()
    assert fk.last_variant[1].WS == bool(params['WS']) and bk.last_variant[1].WS == bool(params['WS'])
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], False, f'{params} out')
    check(du, ref['diffu'], ab['diffu'], False, f'{params} diffu')
    check(dk, ref['diffk'], ab['diffk'], False, f'{params} diffk')


@pytest.mark.gpu
@pytest.mark.parametrize('params,dts', [(None, 'float32'), (dict(WS=0), 'float32'), (None, 'float16'),
                                        (dict(WS=0, PR=0), 'float16')],
                         ids=['ring_dma', 'ring_registers', 'ring_dma_f16_pairs', 'ring_registers_f16'])
def test_varcoef_slab_halos_and_two_range_launches_gpu(params, dts):
    """The z-slab launch pattern on the plane ring, forward and adjoint: halo planes of every stencil field read in
    place, interior planes first, both faces in one two-range launch == one full-domain launch, bitwise (fp16: the
    LDS-DMA ring of fp16 images with cell-pair taps, and the register ring)."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = _op(dts)
    tdt = torch.float16 if dts == 'float16' else torch.float32
    kf = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='vch_f', target='gpu',
                       gpu_indexing_params=params).compile()
    kb = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='vch_b', target='gpu',
                       gpu_indexing_params=params).compile()
    Z = 30
    u, k, d = _inputs((Z, 21, 136), tdt, 'cuda', seed=11)
    full = torch.empty_like(u)
    kf(u=u, k=k, out=full)
    fdu, fdk = torch.empty_like(u), torch.empty_like(u)
    kb(u=u, k=k, diffout=d, diffu=fdu, diffk=fdk)
    assert kf.last_variant[1].WS == (params is None) and kb.last_variant[1].WS == (params is None)
    assert kf.last_variant[1].PR == (dts == 'float16' and params is None)
    outs, dus, dks = [], [], []
    for a, b in [(0, 11), (11, 19), (19, Z)]:
        sl = {n: t[a:b].contiguous() for n, t in (('u', u), ('k', k), ('diffout', d))}
        halo = {n: (t[a - 1:a].contiguous() if a > 0 else None, t[b:b + 1].contiguous() if b < Z else None)
                for n, t in (('u', u), ('k', k), ('diffout', d))}
        out, du, dk = (torch.full_like(sl['u'], float('nan')) for _ in range(3))
        kf(u=sl['u'], k=sl['k'], out=out, z_range=(1, b - a - 1))
        kf(u=sl['u'], k=sl['k'], out=out, halos={'u': halo['u'], 'k': halo['k']},
           z_range=((0, 1), (b - a - 1, b - a)))
        kb(**sl, diffu=du, diffk=dk, z_range=(1, b - a - 1))
        kb(**sl, diffu=du, diffk=dk, halos=halo, z_range=((0, 1), (b - a - 1, b - a)))
        outs.append(out)
        dus.append(du)
        dks.append(dk)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
    assert torch.equal(torch.cat(dus), fdu)
    assert torch.equal(torch.cat(dks), fdk)
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(full, ref['out'], ab['out'], False, 'out', dts == 'float16')
    check(fdu, ref['diffu'], ab['diffu'], False, 'diffu', dts == 'float16')
    check(fdk, ref['diffk'], ab['diffk'], False, 'diffk', dts == 'float16')


@pytest.mark.gpu
@pytest.mark.parametrize('params', [None, dict(WS=0), dict(WS=1, NW=8, CX=2, NR=2, D=2)], ids=['dma', 'registers', 'dma8'])
@pytest.mark.parametrize('dtype', ['float32', 'float64'])
def test_plane_ring_radius2_full_ring_fields_gpu(params, dtype):
    """Nonlinear stencil of radius 2 whose fields are read off-centre BEHIND the centre plane (full rings of
    2·RZ + 1 + D slots, no register queue), two outputs, on unaligned tiles — forward and TF-MAD adjoint against the
    oracle evaluating the op's own assignments."""
    import sympy as sp
    from pystencils_autodiff_amd import ps
    from pystencils_autodiff_amd.backends.hip_emitter import march_geometry
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    a, b, o1, o2 = ps.fields(f'a, b, o1, o2: {dtype}[3d]')
    ac = ps.AssignmentCollection({
        o1.center: a[0, 0, 2] * b[0, 0, -2] + sp.sin(a[-2, 1, 0]) * b.center + 0.5 * a[1, -1, -1] * a[-1, 2, 0],
        o2.center: b[2, 0, 1] * b[-1, -2, 0] - a[0, 1, 0] * b[-2, 0, 0]})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    shape = (23, 35, 140)
    g = torch.Generator().manual_seed(9)
    tdt = torch.float32 if dtype == 'float32' else torch.float64
    A, Bf, D1, D2 = (torch.rand(shape, generator=g, dtype=torch.float64).mul(2).sub(1).to(tdt).cuda() for _ in range(4))
    fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='r2_f', target='gpu',
                       gpu_indexing_params=params).compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='r2_b', target='gpu',
                       gpu_indexing_params=params).compile()
    O1, O2, DA, DB = (torch.zeros_like(A) for _ in range(4))
    fk(a=A, b=Bf, o1=O1, o2=O2)
    bk(a=A, b=Bf, diffo1=D1, diffo2=D2, diffa=DA, diffb=DB)
    torch.cuda.synchronize()
    cfg = fk.last_variant[1]
    assert fk.last_variant[0] == 'march' and not cfg.ZSUM and cfg.WS == (params is None or bool(params['WS']))
    assert march_geometry(fk.ir, cfg)['RZ'] == 2 and not march_geometry(fk.ir, cfg)['lite']
    arr = {n: t.double().cpu().numpy() for n, t in (('a', A), ('b', Bf))}
    ref = {**OE.evaluate(op.forward_assignments, arr, boundary_handling='zeros'),
           **OE.evaluate(op.backward_assignments, {**arr, 'diffo1': D1.double().cpu().numpy(),
                                                   'diffo2': D2.double().cpu().numpy()}, boundary_handling='zeros')}
    tol = 1e-5 if dtype == 'float32' else 1e-12
    for name, got in (('o1', O1), ('o2', O2), ('diffa', DA), ('diffb', DB)):
        np.testing.assert_allclose(got.double().cpu().numpy(), ref[name], rtol=tol, atol=tol * 4, err_msg=name)


def _varcoef2d(dts):
    u, k, out = ps.fields(f'u, k, out: {dts}[2d]')
    nb = [(1, 0), (-1, 0), (0, 1), (0, -1)]
    return ps.AssignmentCollection({out.center: u.center + 0.1 * sp.Add(
        *[sp.Rational(1, 2) * (k.center + k[o]) * (u[o] - u.center) for o in nb])})


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
@pytest.mark.parametrize('shape', [(100, 300), (37, 129), (5, 3), (64, 256)], ids=str)
def test_varcoef_2d_gpu_vs_oracle(dts, shape):
    """2-D variable-coefficient diffusion (nonlinear 5-point; the register ring on 128×8 tiles, one tile per
    workgroup) through the drop-in Function, forward and TF-MAD adjoint vs the oracle, cell by cell."""
    op = pa.AutoDiffOp(_varcoef2d(dts), boundary_handling='zeros')
    tdt = torch.float16 if dts == 'float16' else torch.float32
    u, k, d = _inputs(shape, tdt, 'cuda', seed=23)
    out, gu, gk = _apply(op, u, k, d, 'cuda')
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    for kk in (fk, bk):
        if shape[1] * (2 if dts == 'float16' else 4) % 16 == 0:      # rows of whole 16-byte vectors: the ring
            assert kk.last_variant[0] == 'march' and (kk.last_variant[1].CX, kk.last_variant[1].NR) in ((2, 2), (1, 2))
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], False, f'{shape} out', dts == 'float16')
    check(gu, ref['diffu'], ab['diffu'], False, f'{shape} diffu', dts == 'float16')
    check(gk, ref['diffk'], ab['diffk'], False, f'{shape} diffk', dts == 'float16')


def test_2d_row_ring_selection_and_overrides():
    """Schedule selection (no GPU): nonlinear 2-D stencils on long rows take the row ring (``VIEW2D='zy'``, LDS-DMA
    loader, fp16 as cell pairs), short rows the (1, Y, X) tiles; a tile or ``VIEW2D='yx'`` override falls back to the
    (1, Y, X) form (vector fields: its zsum plane) instead of a ring configuration it cannot take; every emitted source
    compiles for gfx950."""
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    u2, o2 = ps.fields('u(2), o(2): float16[2d]')
    E2, M2 = [(1, 0), (0, 1)], [(-1, 0), (0, -1)]
    adv = ps.AssignmentCollection({o2.center(c): u2.center(c) - 0.05 * sp.Add(
        *[u2.center(d) * (u2[E2[d]](c) - u2[M2[d]](c)) / 2 for d in range(2)]) for c in range(2)})
    for ac, ve, vec in ((_varcoef2d('float32'), 4, False), (_varcoef2d('float16'), 8, False), (adv, 8, True)):
        op = pa.AutoDiffOp(ac, boundary_handling='zeros')
        for params in (None, {'VIEW2D': 'yx'}, {'CX': 2, 'NR': 2}):
            hk = HipStencilKernel(StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='r2',
                                                target='gpu', gpu_indexing_params=params))
            for shape in ((4096, 4096), (64, 256)):
                c = hk._march_cfg(ve, shape)
                ring = params is None and shape[1] >= 512
                assert (c.VIEW2D == 'zy' and c.WS) == ring, (params, shape, c)
                assert bool(c.PR) == (ring and ve == 8), (params, shape, c)
                if vec and not ring:
                    assert c.ZSUM, (params, shape, c)
                v = ('march', c)
                assert len(rt.compile_hip(hk.source(v)[0], HipStencilKernel.options(v))) > 0


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16', 'float64'])
@pytest.mark.parametrize('shape', [(40, 1024), (23, 1160), (3, 2048), (130, 520)], ids=str)
def test_varcoef_2d_row_ring_gpu(dts, shape):
    """2-D nonlinear stencils on long rows march along axis 0 (``VIEW2D='zy'``: rows are the planes of the LDS-DMA
    ring; fp16 as x-adjacent cell pairs): forward and adjoint through the drop-in Function vs the oracle, cell by cell,
    on whole and ragged tiles and fewer rows than a chunk; then the z-slab launch pattern (interior rows, then both
    faces reading halo rows in place) bitwise equal to one full launch."""
    from pystencils_autodiff_amd.zslab import ZSlabOp
    op = pa.AutoDiffOp(_varcoef2d(dts), boundary_handling='zeros')
    tdt = getattr(torch, dts)
    fp64 = dts == 'float64'
    u, k, d = _inputs(shape, tdt, 'cuda', seed=31)
    out, gu, gk = _apply(op, u, k, d, 'cuda')
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    row_ring = shape[1] >= (1024 if fp64 else 512)      # (fp64: 1024-cell strips)
    for kk in (fk, bk):
        c = kk.last_variant[1]
        assert kk.last_variant[0] == 'march' and (c.VIEW2D == 'zy' and c.WS) == row_ring, kk.last_variant
        assert bool(c.PR) == (row_ring and dts == 'float16'), kk.last_variant
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], fp64, f'{shape} out', dts == 'float16')
    check(gu, ref['diffu'], ab['diffu'], fp64, f'{shape} diffu', dts == 'float16')
    check(gk, ref['diffk'], ab['diffk'], fp64, f'{shape} diffk', dts == 'float16')
    if shape[0] < 8 or not row_ring:
        return
    full = torch.zeros_like(u)
    fk(u=u, k=k, out=full)
    outs, Z = [], shape[0]
    cuts = [0, Z // 3, 2 * Z // 3, Z]
    for a, b in zip(cuts, cuts[1:]):
        sl = {n: t[a:b].contiguous() for n, t in (('u', u), ('k', k))}
        o = torch.zeros_like(sl['u'])
        halos = {n: (t[a - 1:a].contiguous() if a > 0 else None, t[b:b + 1].contiguous() if b < Z else None)
                 for n, t in (('u', u), ('k', k))}
        inner, faces = ZSlabOp._launches(b - a, 1, (0, b - a))
        if inner:
            fk(u=sl['u'], k=sl['k'], out=o, z_range=inner)
        ZSlabOp._launch_faces(fk, halos, faces, None, {**sl, 'out': o})
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
@pytest.mark.parametrize('mode', ['none', 'time_constant'])
def test_varcoef_2d_row_ring_none_mode_and_time_constant_gpu(mode, dts):
    """The 2-D row ring (``VIEW2D='zy'``) under ``boundary_handling=None`` (NaN-poisoned border rows and columns left
    untouched) and with a time-constant conductivity (``diffk`` accumulated), vs the oracle."""
    f16 = dts == 'float16'
    tdt = torch.float16 if f16 else torch.float32
    bh = None if mode == 'none' else 'zeros'
    ac = _varcoef2d(dts)
    kfield = next(f for f in ac.free_symbols if hasattr(f, 'field') and f.field.name == 'k').field
    op = pa.AutoDiffOp(ac, boundary_handling=bh, time_constant_fields=[kfield] if mode == 'time_constant' else None)
    shape = (45, 1032)
    u, k, d = _inputs(shape, tdt, 'cuda', seed=37)
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    fill = float('nan') if mode == 'none' else 0.0
    out, du = torch.full_like(u, fill), torch.full_like(u, fill)
    dk = torch.full_like(u, fill) if mode == 'none' else torch.rand(shape, device='cuda').to(tdt)
    dk0 = dk.clone()
    fk(u=u, k=k, out=out)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
    torch.cuda.synchronize()
    for kk in (fk, bk):
        assert kk.last_variant[1].VIEW2D == 'zy' and kk.last_variant[1].WS, kk.last_variant
    arr = {n: t.double().cpu().numpy() for n, t in (('u', u), ('k', k))}
    ref = OE.evaluate(op.forward_assignments, arr, boundary_handling=bh)
    refb = OE.evaluate(op.backward_assignments, {**arr, 'diffout': d.double().cpu().numpy()}, boundary_handling=bh,
                       outputs={'diffk': dk0.double().cpu().numpy()} if mode == 'time_constant' else None)
    inner = (slice(1, -1),) * 2 if mode == 'none' else (slice(None),) * 2
    for got, name, r in ((out, 'out', ref), (du, 'diffu', refb), (dk, 'diffk', refb)):
        g_ = got.double().cpu().numpy()
        tol = 2e-3 if f16 else 1e-5
        np.testing.assert_allclose(g_[inner], r[name][inner], rtol=tol, atol=tol, err_msg=f'{mode} {name}')
        if mode == 'none':
            border = np.ones(shape, bool)
            border[inner] = False
            assert np.isnan(g_[border]).all(), f'{name}: a border cell was written'


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
@pytest.mark.parametrize('shape', [(64, 256), (37, 136), (9, 520)], ids=str)
def test_varcoef_2d_pairs_gpu(dts, shape):
    """The packed-pair form (``PR=1``) on a 2-D field (one (1, Y, X) plane on the register ring), forward and adjoint
    kernels vs the oracle, cell by cell."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(_varcoef2d(dts), boundary_handling='zeros')
    tdt = torch.float16 if dts == 'float16' else torch.float32
    u, k, d = _inputs(shape, tdt, 'cuda', seed=29)
    fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='v2p_f', target='gpu',
                       gpu_indexing_params=dict(PR=1)).compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='v2p_b', target='gpu',
                       gpu_indexing_params=dict(PR=1)).compile()
    out, du, dk = (torch.full_like(u, float('nan')) for _ in range(3))
    fk(u=u, k=k, out=out)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
    torch.cuda.synchronize()
    for kk in (fk, bk):
        assert kk.last_variant[0] == 'march' and kk.last_variant[1].PR
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], False, f'{shape} out', dts == 'float16')
    check(du, ref['diffu'], ab['diffu'], False, f'{shape} diffu', dts == 'float16')
    check(dk, ref['diffk'], ab['diffk'], False, f'{shape} diffk', dts == 'float16')


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(23, 35, 140), (9, 20, 131)], ids=str)
def test_fp16_nonlinear_functions_register_ring_gpu(shape):
    """fp16 storage with a function of the taps (no packed-pair form: ``pair_ok`` is False) keeps the register ring on
    128×8 tiles (the fp16 LDS-DMA ring needs the pair form) — the radius-2 collection of
    ``test_plane_ring_radius2_full_ring_fields_gpu`` in fp16, forward and adjoint vs the oracle on the fp16-rounded
    inputs (bound: fp16 rounding of outputs of magnitude <= a few units)."""
    import sympy as sp
    from pystencils_autodiff_amd import ps
    from pystencils_autodiff_amd.backends.hip_emitter import pair_ok
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    a, b, o1, o2 = ps.fields('a, b, o1, o2: float16[3d]')
    ac = ps.AssignmentCollection({
        o1.center: a[0, 0, 2] * b[0, 0, -2] + sp.sin(a[-2, 1, 0]) * b.center + 0.5 * a[1, -1, -1] * a[-1, 2, 0],
        o2.center: b[2, 0, 1] * b[-1, -2, 0] - a[0, 1, 0] * b[-2, 0, 0]})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    g = torch.Generator().manual_seed(31)
    A, Bf, D1, D2 = (torch.rand(shape, generator=g, dtype=torch.float64).mul(2).sub(1).half().cuda() for _ in range(4))
    fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='h16_f', target='gpu').compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='h16_b', target='gpu').compile()
    O1, O2, DA, DB = (torch.zeros_like(A) for _ in range(4))
    fk(a=A, b=Bf, o1=O1, o2=O2)
    bk(a=A, b=Bf, diffo1=D1, diffo2=D2, diffa=DA, diffb=DB)
    torch.cuda.synchronize()
    for k in (fk, bk):
        assert not pair_ok(k.ir) and k.last_variant[0] == 'march'
        assert not k.last_variant[1].WS and not k.last_variant[1].PR and not k.last_variant[1].ZSUM
    arr = {n: t.double().cpu().numpy() for n, t in (('a', A), ('b', Bf))}
    ref = {**OE.evaluate(op.forward_assignments, arr, boundary_handling='zeros'),
           **OE.evaluate(op.backward_assignments, {**arr, 'diffo1': D1.double().cpu().numpy(),
                                                   'diffo2': D2.double().cpu().numpy()}, boundary_handling='zeros')}
    for name, got in (('o1', O1), ('o2', O2), ('diffa', DA), ('diffb', DB)):
        r = ref[name]
        bound = 2.0 ** -10 * np.abs(r) + 2e-3
        err = np.abs(got.double().cpu().numpy() - r)
        assert (err <= bound).all(), f'{name}: worst {err.max():.3e}'


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['none', 'time_constant'])
def test_varcoef_ring_none_mode_and_time_constant_gpu(mode):
    """The plane ring under ``boundary_handling=None`` (interior cells only, the border untouched) and with a
    time-constant conductivity (``diffk`` accumulated: read-modify-write of the adjoint, ``_autodiff.py:110-113``),
    every cell against the oracle; NaN-poisoned outputs show any write outside the written box."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    ac = W.varcoef_diffusion_7pt()
    bh = None if mode == 'none' else 'zeros'
    kfield = next(f for f in ac.free_symbols if hasattr(f, 'field') and f.field.name == 'k').field
    op = pa.AutoDiffOp(ac, boundary_handling=bh, time_constant_fields=[kfield] if mode == 'time_constant' else None)
    shape = (19, 37, 136)
    u, k, d = _inputs(shape, torch.float32, 'cuda', seed=13)
    fk = StencilKernel(op.forward_assignments, boundary_handling=bh, function_name='vn_f', target='gpu').compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling=bh, function_name='vn_b', target='gpu').compile()
    fill = float('nan') if mode == 'none' else 0.0
    out = torch.full_like(u, fill)
    du = torch.full_like(u, fill)
    dk = torch.full_like(u, fill) if mode == 'none' else torch.rand(shape, device='cuda')
    dk0 = dk.clone()
    fk(u=u, k=k, out=out)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
    torch.cuda.synchronize()
    assert fk.last_variant[1].WS and not fk.last_variant[1].ZSUM
    arr = {n: t.double().cpu().numpy() for n, t in (('u', u), ('k', k))}
    ref = OE.evaluate(op.forward_assignments, arr, boundary_handling=bh)
    refb = OE.evaluate(op.backward_assignments, {**arr, 'diffout': d.double().cpu().numpy()}, boundary_handling=bh,
                       outputs={'diffk': dk0.double().cpu().numpy()} if mode == 'time_constant' else None)
    if mode == 'none':
        inner = (slice(1, -1),) * 3
        for got, name, r in ((out, 'out', ref), (du, 'diffu', refb), (dk, 'diffk', refb)):
            g_ = got.double().cpu().numpy()
            np.testing.assert_allclose(g_[inner], r[name][inner], rtol=1e-5, atol=1e-5, err_msg=name)
            border = np.ones(shape, bool)
            border[inner] = False
            assert np.isnan(g_[border]).all(), f'{name}: a border cell was written'
    else:
        np.testing.assert_allclose(out.double().cpu().numpy(), ref['out'], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(du.double().cpu().numpy(), refb['diffu'], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(dk.double().cpu().numpy(), refb['diffk'], rtol=1e-5, atol=1e-5)


PAIR_PARAMS = [dict(PR=1), dict(PR=1, WS=0), dict(PR=1, WS=0, CX=2, NR=4), dict(PR=1, WS=1, NW=8, CX=2, NR=2, D=2),
               dict(PR=1, SFAST=0), dict(PR=1, WS=1, CX=4, NR=2, D=2), dict(PR=1, WS=1, CX=2, NR=2, D=3)]


@pytest.mark.gpu
@pytest.mark.parametrize('params', PAIR_PARAMS, ids=str)
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16], ids=['f32', 'f16'])
@pytest.mark.parametrize('shape', [(19, 37, 200), (17, 33, 45), (9, 20, 129), (6, 5, 3), (12, 40, 256)], ids=str)
def test_varcoef_pairs_gpu(params, dtype, shape):
    """Packed cell pairs (``PR``: lanes own x-adjacent cells, f32x2 arithmetic, pair stores where aligned) on the plane
    ring — LDS-DMA and register forms, fp32 and fp16 storage — on ragged tiles and odd rows (pairs straddling the
    box edge, rows whose pairs start on odd cells), every cell against the oracle's element-wise bound."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    fp16 = dtype == torch.float16
    op = _op('float16' if fp16 else 'float32')
    u, k, d = _inputs(shape, dtype, 'cuda', seed=17)
    fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='vcp_f', target='gpu',
                       gpu_indexing_params=params).compile()
    bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='vcp_b', target='gpu',
                       gpu_indexing_params=params).compile()
    out, du, dk = (torch.full_like(u, float('nan')) for _ in range(3))
    fk(u=u, k=k, out=out)
    bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
    torch.cuda.synchronize()
    for kk in (fk, bk):
        assert kk.last_variant[0] == 'march' and kk.last_variant[1].PR and not kk.last_variant[1].ZSUM
    ref, ab = oracle(op, *(x.double().cpu().numpy() for x in (u, k, d)))
    check(out, ref['out'], ab['out'], False, f'{params} out', fp16)
    check(du, ref['diffu'], ab['diffu'], False, f'{params} diffu', fp16)
    check(dk, ref['diffk'], ab['diffk'], False, f'{params} diffk', fp16)


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
@pytest.mark.parametrize('mode', ['none', 'time_constant'])
def test_varcoef_pairs_none_mode_and_time_constant_gpu(mode, dts):
    """Packed pairs under ``boundary_handling=None`` (NaN-poisoned border untouched: pairs straddling the written box
    store one cell) and with a time-constant conductivity (``diffk`` read back pairwise and accumulated), on a row of
    odd length (fp32) / of whole 16-byte pieces (fp16: the LDS-DMA ring of fp16 images) and of odd length (fp16: the
    register ring)."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    ac = W.varcoef_diffusion_7pt(dtype=dts)
    f16 = dts == 'float16'
    tdt = torch.float16 if f16 else torch.float32
    bh = None if mode == 'none' else 'zeros'
    kfield = next(f for f in ac.free_symbols if hasattr(f, 'field') and f.field.name == 'k').field
    op = pa.AutoDiffOp(ac, boundary_handling=bh, time_constant_fields=[kfield] if mode == 'time_constant' else None)
    for shape, params in (((19, 37, 137), dict(PR=1)), ((19, 37, 137), dict(PR=1, WS=0)), ((19, 37, 136), dict(PR=1))):
        u, k, d = _inputs(shape, tdt, 'cuda', seed=19)
        fk = StencilKernel(op.forward_assignments, boundary_handling=bh, function_name='vpn_f', target='gpu',
                           gpu_indexing_params=params).compile()
        bk = StencilKernel(op.backward_assignments, boundary_handling=bh, function_name='vpn_b', target='gpu',
                           gpu_indexing_params=params).compile()
        fill = float('nan') if mode == 'none' else 0.0
        out, du = torch.full_like(u, fill), torch.full_like(u, fill)
        dk = torch.full_like(u, fill) if mode == 'none' else torch.rand(shape, device='cuda').to(tdt)
        dk0 = dk.clone()
        fk(u=u, k=k, out=out)
        bk(u=u, k=k, diffout=d, diffu=du, diffk=dk)
        torch.cuda.synchronize()
        assert fk.last_variant[1].PR and bk.last_variant[1].PR
        arr = {n: t.double().cpu().numpy() for n, t in (('u', u), ('k', k))}
        ref = OE.evaluate(op.forward_assignments, arr, boundary_handling=bh)
        refb = OE.evaluate(op.backward_assignments, {**arr, 'diffout': d.double().cpu().numpy()}, boundary_handling=bh,
                           outputs={'diffk': dk0.double().cpu().numpy()} if mode == 'time_constant' else None)
        inner = (slice(1, -1),) * 3 if mode == 'none' else (slice(None),) * 3
        for got, name, r in ((out, 'out', ref), (du, 'diffu', refb), (dk, 'diffk', refb)):
            g_ = got.double().cpu().numpy()
            tol = 2e-3 if f16 else 1e-5
            np.testing.assert_allclose(g_[inner], r[name][inner], rtol=tol, atol=tol, err_msg=f'{shape} {params} {name}')
            if mode == 'none':
                border = np.ones(shape, bool)
                border[inner] = False
                assert np.isnan(g_[border]).all(), f'{params} {name}: a border cell was written'


def test_pair_form_eligibility():
    """``PR`` takes fp32 arithmetic of +, ×, integer powers on scalar fields; functions raise (no GPU needed)."""
    import sympy as sp
    from pystencils_autodiff_amd.backends.hip_emitter import pair_ok
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    for dts, ok in (('float32', True), ('float16', True), ('float64', False)):
        k = StencilKernel(_op(dts).backward_assignments, boundary_handling='zeros', function_name='pe', target='gpu')
        assert pair_ok(HipStencilKernel(k).ir) == ok
    a, b = ps.fields('a, b: float32[3d]')
    op = pa.AutoDiffOp(ps.AssignmentCollection({b.center: sp.sin(a[1, 0, 0]) * a[0, 0, -1]}), boundary_handling='zeros')
    k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='pe2', target='gpu',
                      gpu_indexing_params=dict(PR=1))
    hk = HipStencilKernel(k)
    assert not pair_ok(hk.ir)
    with pytest.raises(ValueError, match='PR=1'):
        hk.source(('march', hk._march_cfg(4, (16, 16, 256))))


# ------------------------------------------------------------------------------------------------------------------
# nonlinear stencils on vector fields (index dimension, components fastest): the LDS-DMA plane ring with the
# components interleaved in each plane image (as the zsum schedule keeps them) — reference vector-field TF-MAD branch
# _autodiff.py:125-152 (only the last component's adjoint assignment is kept), tests/test_tfmad.py:381-401
E3 = [(1, 0, 0), (0, 1, 0), (0, 0, 1)]
M3 = [(-1, 0, 0), (0, -1, 0), (0, 0, -1)]


def _advection(dts='float32', C=3):
    """``out(c) = u(c) − α Σ_d u(d)·(u[+e_d](c) − u[−e_d](c))/2`` (scripts/probes/vector_nonlinear.py)."""
    u, out = ps.fields(f'u({C}), out({C}): {dts}[3d]')
    return ps.AssignmentCollection({out.center(c): u.center(c) - 0.05 * sp.Add(
        *[u.center(d % C) * (u[E3[d]](c) - u[M3[d]](c)) / 2 for d in range(3)]) for c in range(C)})


def _adv_oracle(op, bh, un, dn):
    """(out, diffu) of the op's assignments and their Σ|terms|, float64 numpy, fields [Z, Y, X, C]."""
    ref = {**OE.evaluate(op.forward_assignments, {'u': un}, boundary_handling=bh),
           **OE.evaluate(op.backward_assignments, {'u': un, 'diffout': dn}, boundary_handling=bh)}
    ab = {**OE.evaluate(_abs_terms(op.forward_assignments), {'u': np.abs(un)}, boundary_handling=bh),
          **OE.evaluate(_abs_terms(op.backward_assignments), {'u': np.abs(un), 'diffout': np.abs(dn)},
                        boundary_handling=bh)}
    return ref, ab


def test_vector_nonlinear_takes_the_plane_ring():
    """Schedule selection (no GPU): the advection forward and its TF-MAD adjoint are not linear off the centre plane,
    so not zsum; they take the LDS-DMA plane ring with interleaved components (they took one thread per cell before
    round 6), and the emitted sources compile for gfx950."""
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    for dts, ve in (('float32', 4), ('float16', 8)):
        op = pa.AutoDiffOp(_advection(dts), boundary_handling='zeros')
        assert [str(a.lhs) for a in op.backward_assignments.main_assignments] == ['\\hat{u}[0,0,0,2]']   # the quirk
        for asg in (op.forward_assignments, op.backward_assignments):
            hk = HipStencilKernel(StencilKernel(asg, boundary_handling='zeros', function_name='advr', target='gpu'))
            assert hk.schedule() == 'march'
            cfg = hk._march_cfg(ve, (64, 64, 256))
            assert cfg.WS and not cfg.ZSUM, cfg
            if dts == 'float16':          # fp16 images in the ring: 128×8 tiles of x-adjacent cell pairs
                assert (cfg.CX, cfg.NR, cfg.NW, cfg.PR) == (2, 2, 4 if asg is op.forward_assignments else 8, 1), cfg
            src = hk.source(('march', cfg))[0]
            assert 'LDS-DMA loader wave' in src and len(rt.compile_hip(src)) > 0


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(17, 33, 45), (9, 20, 128), (40, 64, 256), (5, 7, 3), (33, 50, 130),
                                   (21, 30, 132), (70, 9, 264)])
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('dts', ['float32', 'float16'])
def test_vector_advection_ring_gpu_vs_oracle(shape, bh, dts):
    """The advection op through the drop-in Function on the vector plane ring, forward and TF-MAD adjoint vs the
    float64 oracle, cell by cell (``check``: 1e-6·|ref| + 32·2⁻²⁴·Σ|terms|, plus half an fp16 ulp of the stored
    result for fp16 fields), both boundary modes; the adjoint's first two components are the zeros of the
    reference's last-component quirk (``_autodiff.py:138-152``). fp16 fields: the ring holds fp16 plane images, lanes
    own x-adjacent cell pairs evaluated as packed fp32 (``PR``), 128×8 tiles, eight compute waves for the adjoint."""
    op = pa.AutoDiffOp(_advection(dts), boundary_handling=bh)
    tdt = getattr(torch, dts)
    g = torch.Generator().manual_seed(sum(shape))
    u = (torch.rand(shape + (3,), generator=g, dtype=torch.float64) * 2 - 1).to(tdt)
    d = (torch.rand(shape + (3,), generator=g, dtype=torch.float64) * 2 - 1).to(tdt)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    uu = u.cuda().requires_grad_(True)
    (out,) = fn.apply(uu)
    out.backward(d.cuda())
    torch.cuda.synchronize()
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    for k in (fk, bk):
        if (shape[2] * 3 * tdt.itemsize) % 16 == 0:   # rows of whole 16-byte pieces (the others: one thread per cell)
            assert k.last_variant[0] == 'march' and k.last_variant[1].WS and not k.last_variant[1].ZSUM, k.last_variant
            if dts == 'float16':
                assert k.last_variant[1].PR and k.last_variant[1].NW == (8 if k is bk else 4), k.last_variant
    ref, ab = _adv_oracle(op, bh, u.double().numpy(), d.double().numpy())
    half = dts == 'float16'
    check(out, ref['out'], ab['out'], False, f'{shape} {bh} {dts} out', fp16=half)
    check(uu.grad, ref['diffu'], ab['diffu'], False, f'{shape} {bh} {dts} diffu', fp16=half)
    assert not uu.grad[..., :2].any()


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
@pytest.mark.parametrize('shape', [(40, 1024), (17, 600), (9, 100)], ids=str)
def test_vector_advection_2d_gpu_vs_oracle(shape, dts):
    """2-D advection on u(2) (components interleaved): on rows of >= 512 cells the 2-D row ring (``VIEW2D='zy'``, the
    LDS-DMA ring with rows as planes), shorter rows the (1, Y, X) zsum plane or one thread per cell — forward and
    TF-MAD adjoint vs the float64 oracle, cell by cell, with the reference's last-component quirk
    (``_autodiff.py:138-152``)."""
    u, out = ps.fields(f'u(2), out(2): {dts}[2d]')
    E2, M2 = [(1, 0), (0, 1)], [(-1, 0), (0, -1)]
    ac = ps.AssignmentCollection({out.center(c): u.center(c) - 0.05 * sp.Add(
        *[u.center(d) * (u[E2[d]](c) - u[M2[d]](c)) / 2 for d in range(2)]) for c in range(2)})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    tdt = getattr(torch, dts)
    g = torch.Generator().manual_seed(sum(shape))
    uu0 = (torch.rand(shape + (2,), generator=g, dtype=torch.float64) * 2 - 1).to(tdt)
    d = (torch.rand(shape + (2,), generator=g, dtype=torch.float64) * 2 - 1).to(tdt)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    uu = uu0.cuda().requires_grad_(True)
    (o,) = fn.apply(uu)
    o.backward(d.cuda())
    torch.cuda.synchronize()
    for k in (op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()):
        if shape[1] >= 512:             # (fp16: as x-adjacent cell pairs)
            assert k.last_variant[0] == 'march' and k.last_variant[1].VIEW2D == 'zy' and k.last_variant[1].WS, \
                k.last_variant
            assert k.last_variant[1].PR == int(dts == 'float16'), k.last_variant
        else:                             # (the (1, Y, X) zsum plane or one thread per cell)
            assert not (k.last_variant[0] == 'march' and k.last_variant[1].WS), k.last_variant
    ref, ab = _adv_oracle(op, 'zeros', uu0.double().numpy(), d.double().numpy())
    half = dts == 'float16'
    check(o, ref['out'], ab['out'], False, f'{shape} {dts} out', fp16=half)
    check(uu.grad, ref['diffu'], ab['diffu'], False, f'{shape} {dts} diffu', fp16=half)
    assert not uu.grad[..., :1].any()


@pytest.mark.gpu
@pytest.mark.parametrize('dts', ['float32', 'float16'])
def test_vector_advection_ring_tilings_and_slab_gpu(dts):
    """Other ring tilings of the vector advection (8 compute waves, depth 1 and 3) and the z-slab launch pattern
    (interior z range, then both faces in one launch reading halo planes in place) bitwise equal to one full launch;
    fp32 and fp16 fields."""
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    from pystencils_autodiff_amd.zslab import ZSlabOp
    op = pa.AutoDiffOp(_advection(dts), boundary_handling='zeros')
    shape = (23, 37, 200)
    g = torch.Generator().manual_seed(4)
    u = (torch.rand(shape + (3,), generator=g) * 2 - 1).to(getattr(torch, dts)).cuda()
    ref, ab = _adv_oracle(op, 'zeros', u.double().cpu().numpy(), np.zeros(shape + (3,)))
    for params in (dict(WS=1, NW=8, CX=2, NR=1, D=2), dict(WS=1, CX=1, NR=4, D=1), dict(WS=1, CX=2, NR=2, D=3),
                   dict(WS=1, CX=4, NR=2, PR=1), dict(WS=1, CX=2, NR=2, PR=0)):    # cell pairs on and off
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='advt', target='gpu',
                          gpu_indexing_params=params).compile()
        out = torch.full_like(u, float('nan'))
        k(u=u, out=out)
        torch.cuda.synchronize()
        assert k.last_variant[1].WS and not k.last_variant[1].ZSUM
        # (fp16: the default pair form, which yields to an odd CX)
        assert k.last_variant[1].PR == params.get('PR', int(dts == 'float16' and params['CX'] % 2 == 0)), params
        check(out, ref['out'], ab['out'], False, f'{params} {dts} out', fp16=dts == 'float16')
    k = op.forward_ast_gpu.compile()
    full = torch.zeros_like(u)
    k(u=u, out=full)
    outs = []
    for a, b in [(0, 9), (9, 16), (16, 23)]:
        sl = u[a:b].contiguous()
        o = torch.zeros_like(sl)
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < shape[0] else None
        inner, faces = ZSlabOp._launches(b - a, 1, (0, b - a))
        if inner:
            k(u=sl, out=o, z_range=inner)
        ZSlabOp._launch_faces(k, {'u': (lo, hi)}, faces, None, {'u': sl, 'out': o})
        assert k.last_variant[1].WS and not k.last_variant[1].ZSUM
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
