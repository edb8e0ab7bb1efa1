"""GPU parity for the SURVEY.md §8(f) rows beyond the headline sweep, through the HIP path vs the oracle.

* f1 ``time_constant_fields`` (``_autodiff.py:110-113``): the adjoint of a time-constant field is
  ``diffF = diffF + Σ …`` — read-modify-write of the output in place. Through the op it starts from the
  reference's ``torch.zeros`` gradient (``_torch_native.py:107-112``); a direct kernel call accumulates
  onto whatever the caller passes (pre-seeded here). Every stencil schedule: WS (LDS-DMA loader), zsum
  register-prefetch, the packed 27-point zsum, the LDS ring (``march``) and ``generic``.
* f4 ``diff_mode='transposed'`` (``_autodiff.py:354-437``): on pointwise ops it equals TF-MAD
  (``tests/test_autodiff.py:29-33``); with a shifted read its adjoint writes at an offset (exclusive
  writes, so the reference allows it) — the ``generic`` schedule's guarded offset stores.
* z-slab RCCL sweep with a backward whose z radius exceeds the forward's (receive buffers per radius).

Tolerances as in ``test_gpu_parity.py``: fp32 1e-6 · max|ref|, fp64 1e-12, fp16 storage 1e-3.
"""
import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from tests.conftest import assert_close_rel, golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

TOL = {np.float32: 1e-6, np.float64: 1e-12, np.float16: 1e-3}


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


# --- f1: time-constant accumulation ---------------------------------------------------------------------

TC_CASES = [
    # (id, builder, dtype, shape, tuning, expected schedule (ZSUM, WS) or kind)
    ('ws_7pt', lambda: W.asym_7pt(), np.float32, (20, 24, 136), {}, ('march', True, True)),
    ('zsum_7pt', lambda: W.asym_7pt(), np.float32, (20, 24, 136), {'WS': False}, ('march', True, False)),
    ('zsum_27pt_f16', lambda: W.stencil_27pt(), np.float16, (18, 20, 140), {}, ('march', True, False)),
    ('ring_2d', lambda: W.laplace_5pt(), np.float32, (40, 72), {}, ('march', None, None)),
    ('generic_7pt', lambda: W.asym_7pt(), np.float32, (11, 13, 17), {'force': 'generic'}, ('generic',)),
]


def _tc_op(builder, bh, tuning):
    ac = builder()
    u = [f for f in ac.free_fields if f.name == 'u'][0] if hasattr(ac, 'free_fields') else None
    kw = {k: v for k, v in tuning.items() if k != 'force'}
    op = pa.AutoDiffOp(ac, boundary_handling=bh, time_constant_fields=[u],
                       **({'gpu_indexing_params': kw} if kw else {}))
    return op


@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('case,builder,dtype,shape,tuning,expect', TC_CASES, ids=[c[0] for c in TC_CASES])
def test_time_constant_accumulation_direct_kernel(case, builder, dtype, shape, tuning, expect, bh):
    """``diffu += Σ ∂f/∂u · diffout[-o]`` onto a pre-seeded ``diffu`` (direct kernel call, no memset)."""
    op = _tc_op(builder, bh, tuning)
    bwd = op.backward_assignments
    assert any(str(a.rhs).count('diffu') for a in bwd.main_assignments), 'adjoint must read diffu (+=)'
    rng = np.random.default_rng(11)
    d = rng.uniform(-1, 1, shape).astype(dtype)
    seed = rng.uniform(-2, 2, shape).astype(dtype)
    k = op.backward_ast_gpu.compile()
    tdu = _dev(seed)
    k(diffout=_dev(d), diffu=tdu, force_schedule=tuning.get('force'))
    torch.cuda.synchronize()
    ref = OE.evaluate(bwd, {'diffout': d}, boundary_handling=bh, outputs={'diffu': seed.astype(np.float64)})
    assert_close_rel(tdu.cpu().numpy(), ref['diffu'], TOL[dtype], f'{case} accumulated diffu')
    got = k.last_variant
    assert got[0] == expect[0], got
    if expect[0] == 'march' and expect[1] is not None:
        assert bool(got[1].ZSUM) == expect[1] and bool(getattr(got[1], 'WS', False)) == expect[2], got[1]


@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('case,builder,dtype,shape,tuning,expect', TC_CASES[:4], ids=[c[0] for c in TC_CASES[:4]])
def test_time_constant_through_op(case, builder, dtype, shape, tuning, expect, bh):
    """Through ``Op.apply`` + ``backward``: the accumulated adjoint starts from the reference's zeros."""
    op = _tc_op(builder, bh, tuning)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(12)
    u = rng.uniform(0, 1, shape).astype(dtype)
    d = rng.uniform(-1, 1, shape).astype(dtype)
    tu = _dev(u).requires_grad_(True)
    (out,) = fn.apply(tu)
    out.backward(_dev(d))
    torch.cuda.synchronize()
    ref_out = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=bh)['out']
    ref_du = OE.evaluate(op.backward_assignments, {'diffout': d}, boundary_handling=bh)['diffu']
    assert_close_rel(out.detach().cpu().numpy(), ref_out, TOL[dtype], f'{case} out')
    assert_close_rel(tu.grad.cpu().numpy(), ref_du, TOL[dtype], f'{case} diffu')
    # twice in a row: the second call must not see the first call's accumulation
    tu.grad = None
    (out,) = fn.apply(tu)
    out.backward(_dev(d))
    torch.cuda.synchronize()
    assert_close_rel(tu.grad.cpu().numpy(), ref_du, TOL[dtype], f'{case} diffu (2nd call)')


def test_time_constant_two_outputs_accumulate_per_assignment():
    """Two forward assignments reading the time-constant field: ``_autodiff.py:110-113`` accumulates one
    ``diffu = diffu + …`` per assignment — after CSE a single assignment summing both contributions."""
    u, a, b = ps.fields('u, a, b: float32[3d]')
    ac = ps.AssignmentCollection([ps.Assignment(a.center, 2 * u[1, 0, 0] - u[0, -1, 0]),
                                  ps.Assignment(b.center, u[0, 0, 1] * 0.5 + u.center)], [])
    op = pa.AutoDiffOp(ac, boundary_handling='zeros', time_constant_fields=[u])
    shape = (9, 12, 70)
    rng = np.random.default_rng(3)
    da = rng.uniform(-1, 1, shape).astype(np.float32)
    db = rng.uniform(-1, 1, shape).astype(np.float32)
    seed = rng.uniform(-1, 1, shape).astype(np.float32)
    k = op.backward_ast_gpu.compile()
    tdu = _dev(seed)
    k(diffa=_dev(da), diffb=_dev(db), diffu=tdu)
    torch.cuda.synchronize()
    ref = OE.evaluate(op.backward_assignments, {'diffa': da, 'diffb': db}, boundary_handling='zeros',
                      outputs={'diffu': seed.astype(np.float64)})
    assert_close_rel(tdu.cpu().numpy(), ref['diffu'], 1e-6, 'diffu')


# --- f4: transposed mode ----------------------------------------------------------------------------------

@pytest.mark.parametrize('bh', [None, 'zeros'])
def test_transposed_pointwise_equals_tfmad_gpu(bh):
    """README op ``z = x·log(x·y)`` in ``diff_mode='transposed'`` through HIP: equal to the TF-MAD op and
    to the golden vectors (``tests/test_autodiff.py:29-33``: both modes agree on pointwise ops)."""
    g = golden('readme_f32_20x30')
    res = {}
    for mode in ('transposed', 'transposed-forward'):
        op = pa.AutoDiffOp(W.readme_op(), boundary_handling=bh, diff_mode=mode)
        fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
        x, y = _dev(g['x']).requires_grad_(True), _dev(g['y']).requires_grad_(True)
        # transposed mode keeps the reference's unsorted field order (_autodiff.py:427-437): feed by name
        order = {'x': x, 'y': y}
        (z,) = fn.apply(*[order[f.name] for f in op.forward_input_fields])
        z.backward(_dev(g['diffz']))
        torch.cuda.synchronize()
        res[mode] = (z.detach().cpu().numpy(), x.grad.cpu().numpy(), y.grad.cpu().numpy())
        assert op.backward_ast_gpu.compile().last_variant[0] == 'pointwise'
    for i, name in enumerate(('z', 'diffx', 'diffy')):
        assert_close_rel(res['transposed'][i], g[name], 1e-6, f'transposed {name}')
        assert_close_rel(res['transposed'][i], res['transposed-forward'][i], 1e-6, f'modes agree on {name}')


@pytest.mark.parametrize('shape', [(37, 45), (5, 300)])
def test_transposed_shifted_read_writes_at_offset_gpu(shape):
    """``out[0,0] = u[1,0]²``: the transposed adjoint is ``diffu[1,0] = 2·u[1,0]·diffout[0,0]`` — one
    exclusive write at an offset. Interior-only (``boundary_handling=None``, g = 1): cells c of
    ``[1, N-1)²`` write ``diffu[c + (1,0)]``; everything else keeps the zeros of the allocation."""
    u, out = ps.fields('u, out: float32[2d]')
    ac = ps.AssignmentCollection([ps.Assignment(out.center, u[1, 0] ** 2)], [])
    op = pa.AutoDiffOp(ac, diff_mode='transposed')
    (bw,) = op.backward_assignments.main_assignments
    assert tuple(bw.lhs.offsets) == (1, 0)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(4)
    un = rng.uniform(0.5, 1.5, shape).astype(np.float32)
    dn = rng.uniform(-1, 1, shape).astype(np.float32)
    tu = _dev(un).requires_grad_(True)
    (o,) = fn.apply(tu)
    o.backward(_dev(dn))
    torch.cuda.synchronize()
    u64, d64 = un.astype(np.float64), dn.astype(np.float64)
    ref_o = np.zeros(shape)
    ref_o[1:-1, 1:-1] = u64[2:, 1:-1] ** 2
    ref_du = np.zeros(shape)
    ref_du[2:, 1:-1] = 2 * u64[2:, 1:-1] * d64[1:-1, 1:-1]
    assert_close_rel(o.detach().cpu().numpy(), ref_o, 1e-6, 'out')
    assert_close_rel(tu.grad.cpu().numpy(), ref_du, 1e-6, 'diffu (offset writes)')
    assert op.backward_ast_gpu.compile().last_variant[0] == 'generic'


def test_transposed_stencil_rejected_like_reference():
    """Stencils have non-exclusive transposed writes: the reference asserts (``_autodiff.py:425-426``)."""
    with pytest.raises(AssertionError):
        pa.AutoDiffOp(W.diffusion_7pt(), diff_mode='transposed')


# --- z-slab: receive buffers per radius -----------------------------------------------------------------

def test_zslab_rccl_loopback_backward_radius_larger_than_forward():
    """A user-given backward reading ``u`` at z radius 2 after a radius-1 forward: the RCCL face exchange
    keeps one receive buffer per (field, radius), so the backward gets 2 halo planes of ``u``, not the
    forward's 1 (periodic z through the loopback communicator)."""
    from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp
    fwd = W.diffusion_7pt()
    u, out = sorted(fwd.free_fields, key=str)[0], sorted(fwd.bound_fields, key=str)[0]
    du, dout = ps.fields('diffu, diffout: float32[3d]')
    bwd = ps.AssignmentCollection([ps.Assignment(du.center, dout.center + 0.25 * dout[1, 0, 0] + 0.5 * u[2, 0, 0]
                                                 - 0.125 * u[-2, 0, -1])], [])
    op = pa.AutoDiffOp(fwd, boundary_handling='zeros', backward_assignments=bwd)
    shape = (9, 20, 72)
    rng = np.random.default_rng(8)
    un = rng.uniform(0, 1, shape).astype(np.float32)
    dn = rng.uniform(-1, 1, shape).astype(np.float32)
    z = ZSlabOp(op, use_cuda=True)
    z._halo = RcclHalo(loopback=True)
    try:
        tu, td = _dev(un), _dev(dn)
        to, tdu = torch.empty_like(tu), torch.empty_like(tu)
        z.warm_exchange(u=tu, diffout=td)
        z.fwd(u=tu, out=to)
        z.bwd(u=tu, diffout=td, diffu=tdu)
        torch.cuda.synchronize()

        def periodic(ac, arrays, r, name):
            ext = {k: np.concatenate([a[-r:], a, a[:r]]).astype(np.float64) for k, a in arrays.items()}
            return OE.evaluate(ac, ext, boundary_handling='zeros')[name][r:-r]
        assert_close_rel(to.cpu().numpy(), periodic(fwd, {'u': un}, 1, 'out'), 1e-6, 'out')
        assert_close_rel(tdu.cpu().numpy(), periodic(bwd, {'u': un, 'diffout': dn}, 2, 'diffu'), 1e-6, 'diffu')
        radii = sorted(k[2] for k in z._bufs if k[0] == 'rccl' and k[1] == 'u')
        assert radii == [1, 2], radii
    finally:
        z.close()
    assert out is not None and sp is not None
