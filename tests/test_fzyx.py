"""``layout='fzyx'`` fields (reference ``tests/test_tfmad.py:299``, ``lbm/_autodiff_lbstep.py:73-74``).

Scalar fzyx fields are C-ordered memory; vector fzyx fields store each component as its own C-ordered
spatial array (SoA). On the GPU every component becomes a scalar field of the kernel
(``kernel_ir.split_soa``), so the stencil schedules run on it unchanged; the CPU C kernels take the
strides as they are.
"""
import numpy as np
import pytest

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from tests.conftest import assert_close_rel

torch = pytest.importorskip('torch')


def test_fzyx_field_strides():
    u, out = ps.fields("u(3), out(3): float32[4,5,6]", layout='fzyx')
    assert u.strides == (30, 6, 1, 120) and u.is_soa and u.memory_layout == 'fzyx'
    s = ps.fields("s: float32[4,5,6]", layout='fzyx')
    assert s.strides == (30, 6, 1) and not s.is_soa           # scalar fzyx == C order
    a = ps.fields("a(3): float32[4,5,6]")
    assert a.strides == (90, 18, 3, 1) and not a.is_soa
    assert a != ps.Field.create_fixed_size('a', (4, 5, 6, 3), index_dimensions=1, dtype='float32', layout='fzyx')
    g = ps.fields("g(9): float64[2d]", layout='soa')
    assert g.is_soa and pa.AdjointField(g).is_soa
    t = torch.empty(9, 5, 6).permute(1, 2, 0)
    assert ps.Field.create_from_numpy_array('t', t, index_dimensions=1).is_soa
    with pytest.raises(NotImplementedError):
        ps.fields("f: float32[4,5]", layout='reverse_numpy')


def test_split_soa_ir():
    from pystencils_autodiff_amd.backends.kernel_ir import split_soa
    op = pa.AutoDiffOp(W.vector_laplace_7pt(layout='fzyx'), boundary_handling='zeros')
    ir, comps = split_soa(op.forward_ast_gpu.ir)
    assert [f.name for f in ir.fields] == ['out__c0', 'out__c1', 'out__c2', 'u__c0', 'u__c1', 'u__c2']
    assert not ir.has_index_dims and len(ir.stores) == 3 and len(ir.reads) == 21
    assert [c.name for c, _ in comps['u']] == ['u__c0', 'u__c1', 'u__c2']
    aos = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling='zeros')
    assert split_soa(aos.forward_ast_gpu.ir)[1] == {}


@pytest.mark.parametrize('bh', ['zeros', None])
def test_fzyx_vector_op_cpu_matches_aos(bh):
    """The CPU op on fzyx vector fields: same values as the C-order op, outputs and gradients in fzyx."""
    shape = (6, 7, 8)
    fn = pa.AutoDiffOp(W.vector_laplace_7pt(layout='fzyx'), boundary_handling=bh).create_tensorflow_op(
        use_cuda=False, backend='torch_native')
    fa = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling=bh).create_tensorflow_op(
        use_cuda=False, backend='torch_native')
    g = torch.Generator().manual_seed(3)
    x = torch.rand(shape + (3,), generator=g, dtype=torch.float32)
    d = torch.rand(shape + (3,), generator=g, dtype=torch.float32)
    xs, xa = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    (o,), (oa,) = fn.apply(xs), fa.apply(xa)
    assert o.stride() == (56, 8, 1, 336)
    assert torch.equal(o, oa)
    o.backward(d)
    oa.backward(d)
    assert torch.equal(xs.grad, xa.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('shape', [(6, 13, 136), (9, 40, 64)])
def test_fzyx_vector_laplacian_gpu(bh, shape):
    """fzyx vector Laplacian through the HIP op: per-component zsum launches, forward and adjoint vs the
    oracle, results in fzyx order, identical to the C-order op."""
    op = pa.AutoDiffOp(W.vector_laplace_7pt(layout='fzyx'), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    fa = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling=bh).create_tensorflow_op(
        use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(5)
    u = rng.uniform(-1, 1, shape + (3,)).astype(np.float32)
    d = rng.uniform(-1, 1, shape + (3,)).astype(np.float32)
    xs = torch.from_numpy(u).cuda().requires_grad_(True)
    xa = torch.from_numpy(u).cuda().requires_grad_(True)
    (o,), (oa,) = fn.apply(xs), fa.apply(xa)
    o.backward(torch.from_numpy(d).cuda())
    oa.backward(torch.from_numpy(d).cuda())
    torch.cuda.synchronize()
    k = op.forward_ast_gpu.compile()
    assert k.last_variant[0] == 'march' and k.last_variant[1].ZSUM, k.last_variant
    assert o.stride()[-1] == int(np.prod(shape))
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=bh)
    refb = OE.evaluate(op.backward_assignments, {'diffout': d}, boundary_handling=bh)
    assert_close_rel(o.detach().cpu().numpy(), ref['out'], 1e-6, 'fzyx forward')
    assert_close_rel(xs.grad.cpu().numpy(), refb['diffu'], 1e-6, 'fzyx adjoint')
    assert torch.equal(o, oa) and torch.equal(xs.grad, xa.grad)


@pytest.mark.gpu
def test_fzyx_strided_inputs_and_2d_vector_gpu():
    """A C-order tensor handed to an fzyx op is reordered once; a 2-D fzyx vector stencil with mixed
    component offsets (curl-like, ``test_tfmad.py:355-376``) matches the oracle."""
    u, out = ps.fields("u(2), out(2): float32[2d]", layout='fzyx')
    ac = ps.AssignmentCollection([ps.Assignment(out.center(0), u[1, 0](1) - u[-1, 0](1) + 0.5 * u[0, 1](0)),
                                  ps.Assignment(out.center(1), u[0, 1](0) - u[0, -1](0) - 0.25 * u[0, 0](1))])
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(2)
    a = rng.uniform(-1, 1, (33, 70, 2)).astype(np.float32)
    (o,) = fn.apply(torch.from_numpy(a).cuda())          # C-order input
    torch.cuda.synchronize()
    ref = OE.evaluate(op.forward_assignments, {'u': a}, boundary_handling='zeros')
    assert_close_rel(o.cpu().numpy(), ref['out'], 1e-6, '2-D fzyx')
