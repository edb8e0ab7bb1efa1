"""The op's native autograd node (``csrc/psad_torch.cpp``, ``_torch_native._NativePath``).

``Op.apply`` runs the forward and adjoint launches as a C++ ``torch::autograd::Function`` whenever the call
fits a plan; otherwise the Python Function (``_torch_native.py:10-142`` restated) runs. Both launch the same
kernels, so results must be bit-identical between them (and the oracle parity of ``test_gpu_parity.py``,
which now runs through the native node, carries over). GPU tests compare the two paths on: the BASELINE
stencils in both boundary modes, fp16/fp32/fp64, multiple inputs and outputs, a missing output gradient,
non-contiguous and misaligned gradients/inputs (the latter fall back), scalar ``class_kwargs`` changes (one
plan per value), ``retain_graph`` double backward and ``no_grad``. CPU tests: the extension loads and
rejects inconsistent plans without touching a GPU."""
import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W

torch = pytest.importorskip('torch')


def _make(ac, bh, native, **kw):
    from pystencils_autodiff_amd.backends import _torch_native as TN
    saved = TN._native
    if not native:
        TN._native = False
    try:
        op = pa.AutoDiffOp(ac, boundary_handling=bh, **kw)
        return op, op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    finally:
        TN._native = saved


def _is_native(t):
    return 'StencilFunction' in t.grad_fn.name()


def _two_outputs():
    u, v, a, b = ps.fields("u, v, a, b: float64[2d]")
    return ps.AssignmentCollection({a.center: u[1, 0] * v.center + sp.sin(u[0, -1]),
                                    b.center: u.center * v[0, 1] - 2 * v[-1, 0]})


CASES = [
    ('diffusion7_zeros', W.diffusion_7pt, 'zeros', (20, 24, 136), torch.float32, 1),
    ('diffusion7_none', W.diffusion_7pt, None, (20, 24, 136), torch.float32, 1),
    ('laplace5_zeros', W.laplace_5pt, 'zeros', (40, 72), torch.float32, 1),
    ('laplace5_none', W.laplace_5pt, None, (40, 72), torch.float32, 1),
    ('stencil27_f16', W.stencil_27pt, 'zeros', (18, 20, 140), torch.float16, 1),
    ('readme_none', W.readme_op, None, (20, 30), torch.float32, 2),
    ('asym7_f64', lambda: W.asym_7pt(dtype='float64'), 'zeros', (11, 13, 17), torch.float64, 1),
    ('two_outputs_f64', _two_outputs, 'zeros', (21, 13), torch.float64, 2),
]


def _inputs(shape, dtype, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(shape, generator=g, dtype=torch.float64) + 0.5).to(dtype).cuda().requires_grad_(True)
            for _ in range(n)]


def _run(fn, ins, grads, retain=False):
    outs = fn.apply(*ins)
    torch.autograd.backward([o for o, g in zip(outs, grads) if g is not None],
                            [g for g in grads if g is not None], retain_graph=retain)
    res = [o.detach().clone() for o in outs] + [t.grad.clone() if t.grad is not None else None for t in ins]
    for t in ins:
        t.grad = None
    return outs, res


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert (x is None) == (y is None)
        if x is not None:
            assert torch.equal(x, y), float((x.double() - y.double()).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize('case,builder,bh,shape,dtype,nin', CASES, ids=[c[0] for c in CASES])
def test_native_node_matches_python_function(case, builder, bh, shape, dtype, nin):
    _, fn_n = _make(builder(), bh, True)
    _, fn_p = _make(builder(), bh, False)
    ins = _inputs(shape, dtype, nin)
    probe = fn_n.apply(*ins)
    g = torch.Generator().manual_seed(1)
    grads = [(torch.rand(o.shape, generator=g, dtype=torch.float64) * 2 - 1).to(dtype).cuda() for o in probe]
    from pystencils_autodiff_amd.backends._torch_native import native_module
    native_module().set_debug_poison(True)          # cells a kernel leaves unwritten would read NaN
    try:
        outs_n, res_n = _run(fn_n, ins, grads)
    finally:
        native_module().set_debug_poison(False)
    outs_p, res_p = _run(fn_p, ins, grads)
    assert all(_is_native(o) for o in outs_n), outs_n[0].grad_fn.name()
    assert not any(_is_native(o) for o in outs_p)
    _same(res_n, res_p)


@pytest.mark.gpu
def test_native_missing_output_gradient_and_noncontiguous_grad():
    _, fn_n = _make(_two_outputs(), 'zeros', True)
    _, fn_p = _make(_two_outputs(), 'zeros', False)
    ins = _inputs((21, 13), torch.float64, 2)
    big = torch.rand(13, 21, dtype=torch.float64).cuda()
    grads = [None, big.t()]                       # first output unused, second gradient transposed
    assert not grads[1].is_contiguous()
    _, res_n = _run(fn_n, ins, grads)
    _, res_p = _run(fn_p, ins, [None, grads[1].contiguous()])
    _same(res_n, res_p)


@pytest.mark.gpu
def test_native_misaligned_input_falls_back():
    _, fn = _make(W.laplace_5pt(), 'zeros', True)
    _, fn_p = _make(W.laplace_5pt(), 'zeros', False)
    base = torch.rand(40 * 72 + 1, device='cuda')
    u = base[1:].view(40, 72).detach().requires_grad_(True)      # 4-byte offset: not 32-byte aligned
    assert u.data_ptr() % 32
    d = torch.rand(40, 72, device='cuda')
    outs, res = _run(fn, [u], [d])
    assert not _is_native(outs[0])
    _, ref = _run(fn_p, [u], [d])
    _same(res, ref)
    ua = u.detach().clone().requires_grad_(True)                  # the same values, aligned: native
    outs_a, res_a = _run(fn, [ua], [d])
    assert _is_native(outs_a[0])
    _same(res_a, res)


@pytest.mark.gpu
def test_native_scalar_class_kwargs_patched_per_call():
    """Scalars are patched into the plan's argument buffers per call: changing ``class_kwargs`` reuses the plan
    (no plan per value), and the backward uses the forward's values even if they change in between."""
    from pystencils_autodiff_amd.backends._torch_native import native_module
    z, y, x = ps.fields("z, y, x: float32[20,40]")
    a = sp.Symbol('a')
    _, fn = _make(ps.AssignmentCollection({z[0, 0]: x[0, 0] * sp.log(a * x[0, 0] * y[0, 0])}), None, True)
    ins = _inputs((20, 40), torch.float32, 2)
    with pytest.raises(TypeError, match='class_kwargs'):
        fn.apply(*ins)
    g = torch.ones(20, 40, device='cuda')
    n0 = None
    for av in (5.0, 2.0, 5.0, 0.75):
        fn.class_kwargs['a'] = av
        outs, res = _run(fn, ins, [g])
        assert _is_native(outs[0])
        n0 = native_module().num_plans() if n0 is None else n0
        assert native_module().num_plans() == n0
        xn, yn = (t.detach().double() for t in ins)
        torch.testing.assert_close(res[0].double(), xn * torch.log(av * xn * yn), rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(res[1].double(), torch.log(av * xn * yn) + 1, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(res[2].double(), xn / yn, rtol=1e-6, atol=1e-6)
    # a value changed between forward and backward: the adjoint still uses the forward's value
    fn.class_kwargs['a'] = 3.0
    (o,) = fn.apply(*ins)
    fn.class_kwargs['a'] = 7.0
    o.backward(g)
    xn, yn = (t.detach().double() for t in ins)
    torch.testing.assert_close(ins[0].grad.double(), torch.log(3.0 * xn * yn) + 1, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_native_retain_graph_and_no_grad():
    _, fn = _make(W.asym_7pt(), 'zeros', True)
    (u,) = _inputs((11, 13, 17), torch.float32, 1)
    d = torch.rand(11, 13, 17, device='cuda')
    (o,) = fn.apply(u)
    o.backward(d, retain_graph=True)
    g1 = u.grad.clone()
    o.backward(d)
    torch.testing.assert_close(u.grad, 2 * g1)
    with torch.no_grad():
        (o2,) = fn.apply(u)
    assert o2.grad_fn is None and torch.equal(o2, o.detach())


@pytest.mark.gpu
def test_native_constant_input_has_no_gradient():
    _, fn = _make(W.readme_op(), None, True)
    ins = _inputs((20, 30), torch.float32, 2)
    ins[0].requires_grad_(False)
    (z,) = fn.apply(*ins)
    z.backward(torch.ones_like(z))
    assert ins[0].grad is None and ins[1].grad is not None


def _random_case(nd, tname, seed):
    import itertools
    rng = np.random.default_rng(seed)
    a, b, out = ps.fields(f"a, b, out: {tname}[{nd}d]")
    offs = list(itertools.product((-1, 0, 1), repeat=nd))
    rhs = 0
    for f in (a, b):
        for k in rng.choice(len(offs), 3, replace=False):
            rhs += sp.Float(round(float(rng.uniform(-1, 1)), 3)) * f[offs[k]]
    rhs += sp.Float(0.25) * sp.sin(a.center) * b[offs[rng.integers(len(offs))]]
    return ps.AssignmentCollection({out.center: rhs})


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(13, 17, 70), (6, 5, 3), (1, 9, 256), (40, 37), (2, 300), (1, 1)])
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_native_random_stencils_vs_oracle(shape, bh, dtype):
    """Random nonlinear two-input stencils through ``Op.apply`` + ``backward`` on the native node (uninitialised
    outputs poisoned) against the float64 oracle: forward and both TF-MAD gradients."""
    from oracle import evaluate as OE
    from pystencils_autodiff_amd.backends._torch_native import native_module
    from tests.conftest import assert_close_rel
    tname = 'float32' if dtype == np.float32 else 'float64'
    _, fn = _make(_random_case(len(shape), tname, sum(shape) + len(shape)), bh, True)
    op = fn.autodiff_op
    rng = np.random.default_rng(3)
    a, b, d = (rng.uniform(-1, 1, shape).astype(dtype) for _ in range(3))
    ta, tb = (torch.from_numpy(x).cuda().requires_grad_(True) for x in (a, b))
    native_module().set_debug_poison(True)
    try:
        (out,) = fn.apply(ta, tb)
        out.backward(torch.from_numpy(d).cuda())
        torch.cuda.synchronize()
    finally:
        native_module().set_debug_poison(False)
    # an interior-only launch over an empty interior (an extent below 3) has no plan: the Python Function
    assert _is_native(out) == (bh == 'zeros' or min(shape) >= 3)
    tol = 1e-6 if dtype == np.float32 else 1e-12
    ref = OE.evaluate(op.forward_assignments, {'a': a, 'b': b}, boundary_handling=bh)['out']
    refb = OE.evaluate(op.backward_assignments, {'a': a, 'b': b, 'diffout': d}, boundary_handling=bh)
    assert_close_rel(out.detach().cpu().numpy(), ref, tol, 'out')
    assert_close_rel(ta.grad.cpu().numpy(), refb['diffa'], tol, 'diffa')
    assert_close_rel(tb.grad.cpu().numpy(), refb['diffb'], tol, 'diffb')


# --- CPU: the extension itself ---------------------------------------------------------------------------

def test_native_extension_loads_and_validates_plans():
    from pystencils_autodiff_amd.backends._torch_native import native_module
    m = native_module()
    assert m is not None and all(hasattr(m, f) for f in ('register_plan', 'apply', 'num_plans', 'set_debug_poison'))
    n0 = m.num_plans()
    args = b'\0' * 32
    ok = dict(name='t', device=0, in_shape=[[4, 4]], in_dtype=[6], fwd_shape=[[4, 4]], fwd_dtype=[6],
              fwd_zero=[False], fwd_fn=1, fwd_grid=1, fwd_block=256, fwd_args=args, fwd_slot=[0, 1],
              fwd_scal=[[16, 0, 0]], saved=[], bwd_shape=[[4, 4]], bwd_dtype=[6], bwd_zero=[False], bwd_fn=1,
              bwd_grid=1, bwd_block=256, bwd_args=args, bwd_slot=[0, 1], bwd_scal=[[24, 1, 0]], grad_of_input=[1],
              n_scalars=1)
    pid = m.register_plan(*ok.values())
    assert pid == n0 and m.num_plans() == n0 + 1
    for key, bad in (('fwd_slot', [0, 2]), ('saved', [5]), ('bwd_slot', [0, 3]), ('grad_of_input', [7]),
                     ('fwd_args', b'\0' * 8), ('fwd_scal', [[8, 0, 0]]), ('bwd_scal', [[28, 1, 0]]),
                     ('bwd_scal', [[24, 1, 1]]), ('fwd_scal', [[16, 0]])):
        kw = dict(ok, **{key: bad})
        with pytest.raises(RuntimeError):
            m.register_plan(*kw.values())
    assert m.num_plans() == n0 + 1
    x = torch.zeros(4, 4)                         # a CPU tensor never matches a plan: None, no launch
    assert m.apply(pid, [x], [1.0]) is None
    assert m.apply(pid, [], [1.0]) is None
    assert m.apply(pid, [torch.zeros(4, 4)], []) is None      # scalar count differs from the plan


@pytest.mark.gpu
def test_native_node_on_non_default_device():
    """Inputs on cuda:1 while cuda:0 is current: the plan's function handles belong to cuda:1's modules and the
    launches (native node and Python Function) run under a device guard — results equal the same op on cuda:0."""
    if torch.cuda.device_count() < 2:
        pytest.skip('one GPU visible')
    _, fn = _make(W.asym_7pt(), 'zeros', True)
    (u0,) = _inputs((11, 13, 70), torch.float32, 1)
    d0 = torch.rand(11, 13, 70, device='cuda:0')
    outs0, res0 = _run(fn, [u0], [d0])
    u1 = u0.detach().to('cuda:1').requires_grad_(True)
    d1 = d0.to('cuda:1')
    with torch.cuda.device(0):
        outs1, res1 = _run(fn, [u1], [d1])
    assert outs1[0].device == torch.device('cuda', 1)
    _same([r.to('cuda:0') if r is not None else None for r in res1], res0)
