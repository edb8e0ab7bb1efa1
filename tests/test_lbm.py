"""Lattice Boltzmann time-step op (§8 f3; reference ``lbm/_autodiff_lbstep.py``): forward steps against an
independent array-roll restatement (``oracle/lbm.py``), the adjoint steps against torch's reverse mode
through that restatement, conservation at full sizes. Parity with lbmpy itself is unpinned (lbmpy absent):
the oracle restates lbmpy's published SRT equations."""
import numpy as np
import pytest
import sympy as sp

from oracle import lbm as OL
from pystencils_autodiff_amd import lbm, ps


def _init(stencil, shape, compressible, seed=0):
    rng = np.random.default_rng(seed)
    D = len(shape)
    Q = {'D2Q9': 9, 'D3Q19': 19, 'D3Q27': 27}[stencil]
    rho = 1 + 0.05 * rng.standard_normal(shape)
    u = 0.04 * rng.standard_normal(shape + (D,))
    return OL.equilibrium(rho, u, stencil, compressible) + 0.01 * rng.standard_normal(shape + (Q,))


def _oracle_grad(f0, omega, T, stencil, compressible, g, device='cpu'):
    import torch
    ft = torch.tensor(f0, requires_grad=True, device=device)
    out = OL.run(ft, omega, T, stencil, compressible, xp=torch)
    (gref,) = torch.autograd.grad(out, ft, torch.as_tensor(g, device=device))
    return out.detach().cpu().numpy(), gref.cpu().numpy()


CPU_CASES = [('D2Q9', (10, 7), False, 'fzyx'), ('D2Q9', (9, 12), True, 'numpy'), ('D3Q19', (6, 5, 4), False, 'fzyx'),
             ('D3Q27', (5, 4, 6), True, 'fzyx')]


@pytest.mark.parametrize('stencil,shape,compressible,layout', CPU_CASES)
def test_lbm_steps_cpu_vs_oracle(stencil, shape, compressible, layout):
    """T forward steps (periodic sync, pull-stream-collide, swap) and T adjoint steps on the C kernels."""
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, layout=layout)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.4, target='cpu')
    f0 = _init(stencil, shape, compressible)
    T = 4
    step.set_pdfs(f0)
    step.run(T, record=True)
    g = np.random.default_rng(1).standard_normal(f0.shape)
    ref, gref = _oracle_grad(f0, 1.4, T, stencil, compressible, g)
    assert np.abs(step.pdf_array - ref).max() <= 1e-13 * np.abs(ref).max()
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref).max() <= 1e-12 * np.abs(gref).max()


def test_lbm_timestep_op_cpu_autograd():
    import torch
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(8, 6), relaxation_rate=1.1, target='cpu')
    Op = step.create_timestep_op(3)
    f0 = _init('D2Q9', (8, 6), True, seed=3)
    x = torch.tensor(f0, requires_grad=True)
    out = Op.apply(x)
    g = torch.tensor(np.random.default_rng(4).standard_normal(f0.shape))
    out.backward(g)
    ref, gref = _oracle_grad(f0, 1.1, 3, 'D2Q9', True, g.numpy())
    assert np.abs(out.detach().numpy() - ref).max() <= 1e-13
    assert np.abs(x.grad.numpy() - gref).max() <= 1e-12 * np.abs(gref).max()
    assert Op.num_time_steps == 3 and Op.lb_step is step


def test_lbm_field_guessing_and_names():
    rule = lbm.create_lb_update_rule('D2Q9')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(4, 4), relaxation_rate=1.0, target='cpu')
    assert step.pdf_field.name == 'src' and step.temporary_field.name == 'dst'
    assert step.backward_pdf_array_name == 'diffdst' and step._backward_tmp_array_name == 'diffsrc'
    a, b, c = ps.fields("a(9), b(9), c(9): float64[2D]")
    two_src = ps.AssignmentCollection([ps.Assignment(c.center(i), a.center(i) + b.center(i)) for i in range(9)])
    with pytest.raises(lbm.PdfFieldNotDetectedException):
        lbm.AutoDiffLatticeBoltzmannStep(two_src, domain_size=(4, 4), target='cpu')
    step2 = lbm.AutoDiffLatticeBoltzmannStep(two_src, a, c, domain_size=(4, 4), target='cpu', constant_fields=[b])
    assert step2.pdf_field == a
    with pytest.raises(ValueError):
        lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(4, 4), target='cpu')     # omega needs a value


def test_lbm_update_rule_lattice():
    for name, q in (('D2Q9', 9), ('D3Q19', 19), ('D3Q27', 27)):
        st = lbm.LBStencil(name)
        assert st.Q == q and sum(st.weights) == 1
        for i in range(q):
            assert st.directions[st.inverse_direction_index(i)] == tuple(-c for c in st.directions[i])


def test_lbm_macroscopic_ops_cpu():
    import torch
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(6, 5), relaxation_rate=1.0, target='cpu')
    setter = step.create_macroscopic_setter_op()
    getter = step.create_macroscopic_getter_op()
    rng = np.random.default_rng(2)
    rho = torch.tensor(1 + 0.1 * rng.standard_normal((6, 5)))
    vel = torch.tensor(0.05 * rng.standard_normal((6, 5, 2)))
    (pdfs,) = setter.apply(rho, vel)
    assert np.abs(pdfs.numpy() - OL.equilibrium(rho.numpy(), vel.numpy(), 'D2Q9', True)).max() < 1e-14
    r2, v2 = getter.apply(pdfs)
    assert np.abs(r2.numpy() - rho.numpy()).max() < 1e-13 and np.abs(v2.numpy() - vel.numpy()).max() < 1e-13


# --------------------------------------------------------------------------------------------------------
# GPU (HIP kernels)
# --------------------------------------------------------------------------------------------------------
GPU_CASES = [('D2Q9', (40, 33), False, 'fzyx', 'float64'), ('D2Q9', (37, 64), True, 'numpy', 'float64'),
             ('D2Q9', (64, 48), True, 'fzyx', 'float32'), ('D3Q19', (20, 17, 12), False, 'fzyx', 'float64'),
             ('D3Q19', (16, 12, 24), True, 'fzyx', 'float32')]


@pytest.mark.gpu
@pytest.mark.parametrize('schedule', ['lattice', 'autodiffop'])
@pytest.mark.parametrize('stencil,shape,compressible,layout,dtype', GPU_CASES)
def test_lbm_steps_gpu_vs_oracle(stencil, shape, compressible, layout, dtype, schedule, monkeypatch):
    """T steps and T adjoint steps on the owned arrays, through the lattice schedule and through the rule's
    AutoDiffOp kernels (PSAD_LBM_LATTICE=0), against the oracle and torch's reverse mode through it."""
    import torch
    monkeypatch.setenv('PSAD_LBM_LATTICE', '1' if schedule == 'lattice' else '0')
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, layout=layout, data_type=dtype)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target='gpu')
    f0 = _init(stencil, shape, compressible)
    T = 5
    tdt = getattr(torch, dtype)
    step.set_pdfs(torch.tensor(f0, dtype=tdt, device='cuda'))
    step.run(T, record=True)
    g = np.random.default_rng(1).standard_normal(f0.shape)
    ref, gref = _oracle_grad(f0, 1.3, T, stencil, compressible, g)
    tol = 1e-12 if dtype == 'float64' else 1e-5
    got = step.pdf_array.double().cpu().numpy()
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max()
    step.set_adjoint_pdfs(torch.tensor(g, dtype=tdt, device='cuda'))
    step.run_backward(T)
    gg = step.adjoint_pdf_array.double().cpu().numpy()
    assert np.abs(gg - gref).max() <= tol * 10 * np.abs(gref).max()
    assert (step._lattice is not None) == (schedule == 'lattice')
    kf = step.autodiff_op.forward_ast_gpu.compile()
    if layout == 'fzyx' and schedule == 'autodiffop':
        assert kf.last_variant[0] == 'generic'       # SoA components: one-thread-per-cell streaming schedule


@pytest.mark.gpu
@pytest.mark.parametrize('native_layout', [False, True])
def test_lbm_timestep_op_gpu_autograd(native_layout):
    """The T-step op: inputs and gradients in numpy layout (copied into fzyx) or already in the step's
    layout (``empty_pdfs``: used in place, never written)."""
    import torch
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True, data_type='float64')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(48, 40), relaxation_rate=1.7, target='gpu')
    Op = step.create_timestep_op(6)
    f0 = _init('D2Q9', (48, 40), True, seed=5)
    g = torch.tensor(np.random.default_rng(6).standard_normal(f0.shape), device='cuda')
    if native_layout:
        x = step.empty_pdfs()
        x.copy_(torch.tensor(f0, device='cuda'))
        x.requires_grad_(True)
        g2 = step.empty_pdfs()
        g2.copy_(g)
        g = g2
    else:
        x = torch.tensor(f0, requires_grad=True, device='cuda')
    g_before = g.clone()
    out = Op.apply(x)
    out.backward(g)
    assert torch.equal(g, g_before)
    ref, gref = _oracle_grad(f0, 1.7, 6, 'D2Q9', True, g.cpu().numpy(), device='cuda')
    assert np.abs(out.detach().cpu().numpy() - ref).max() <= 1e-12
    assert np.abs(x.grad.cpu().numpy() - gref).max() <= 1e-11 * np.abs(gref).max()


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape', [('D2Q9', (2048, 1024)), ('D3Q19', (128, 96, 160))])
def test_lbm_full_size_properties(stencil, shape):
    """Full sizes: mass is conserved by the periodic steps (fp64 sum), and the adjoint of T steps equals
    torch's reverse mode through the oracle run on the GPU (fp32 kernels vs fp64 oracle)."""
    import torch
    rule = lbm.create_lb_update_rule(stencil, compressible=False, data_type='float32')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.5, target='gpu')
    f0 = _init(stencil, shape, False, seed=9)
    step.set_pdfs(torch.tensor(f0, dtype=torch.float32, device='cuda'))
    m0 = step.pdf_array.double().sum().item()
    T = 3
    step.run(T, record=True)
    m1 = step.pdf_array.double().sum().item()
    assert abs(m1 - m0) <= 1e-6 * abs(m0)
    g = np.random.default_rng(10).standard_normal(f0.shape)
    _, gref = _oracle_grad(f0, 1.5, T, stencil, False, g, device='cuda')
    step.set_adjoint_pdfs(torch.tensor(g, dtype=torch.float32, device='cuda'))
    step.run_backward(T)
    gg = step.adjoint_pdf_array.double().cpu().numpy()
    assert np.abs(gg - gref).max() <= 1e-5 * np.abs(gref).max()


def _periodic_case():
    import sympy as sp
    u, v = ps.fields("u, v: float64[2D]")
    ac = ps.AssignmentCollection([ps.Assignment(v.center, 0.3 * u[1, 0] - 0.7 * u[0, -1] + 0.25 * u[-1, 1]
                                                + sp.Rational(1, 5) * u.center)])
    return ac


def _periodic_ref(x):
    return 0.3 * np.roll(x, -1, 0) - 0.7 * np.roll(x, 1, 1) + 0.25 * np.roll(np.roll(x, 1, 0), -1, 1) + 0.2 * x


def test_periodic_boundary_cpu():
    """``boundary_handling='periodic'`` (extension used by the LBM step): wrapped reads, forward and the
    TF-MAD adjoint (exact for this linear stencil) against array rolls."""
    import pystencils_autodiff_amd as pa
    op = pa.AutoDiffOp(_periodic_case(), boundary_handling='periodic')
    x = np.random.default_rng(0).standard_normal((9, 7))
    out = np.empty_like(x)
    op.forward_ast_cpu.compile()(u=x, v=out)
    assert np.abs(out - _periodic_ref(x)).max() < 1e-14
    g = np.random.default_rng(1).standard_normal((9, 7))
    gu = np.empty_like(x)
    op.backward_ast_cpu.compile()(diffv=g, diffu=gu)
    assert abs(np.vdot(_periodic_ref(x), g) - np.vdot(x, gu)) < 1e-12 * np.abs(g).sum()


@pytest.mark.gpu
def test_periodic_boundary_gpu():
    import torch
    import pystencils_autodiff_amd as pa
    op = pa.AutoDiffOp(_periodic_case(), boundary_handling='periodic')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    x = torch.tensor(np.random.default_rng(0).standard_normal((67, 129)), device='cuda', requires_grad=True)
    (out,) = fn.apply(x)
    assert np.abs(out.detach().cpu().numpy() - _periodic_ref(x.detach().cpu().numpy())).max() < 1e-13
    g = torch.tensor(np.random.default_rng(1).standard_normal((67, 129)), device='cuda')
    out.backward(g)
    lhs = float((out.detach() * g).sum())
    rhs = float((x.detach() * x.grad).sum())
    assert abs(lhs - rhs) < 1e-11 * float(g.abs().sum())
    assert op.forward_ast_gpu.compile().last_variant[0] == 'generic'


# --------------------------------------------------------------------------------------------------------
# walls (NoSlip, set_boundary_including_adjoint) and the end-to-end op (_autodiff_lbstep.py:162-187, 310-334)
# --------------------------------------------------------------------------------------------------------
def _channel(shape, obstacle=True):
    """A channel: walls on the first and last rows of axis 1, plus a small obstacle (bool mask)."""
    wall = np.zeros(shape, bool)
    wall[:, 0] = True
    wall[:, -1] = True
    if obstacle:
        c = tuple(n // 3 for n in shape)
        wall[tuple(slice(k, k + 2) for k in c)] = True
    return wall


def _set_channel(step, shape, obstacle=True):
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 0])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, -1])
    if obstacle:
        c = [n // 3 for n in shape]
        # the obstacle through a mask callback over cell midpoints (axis 0 first), lbmpy's convention
        step.set_boundary_including_adjoint(
            lbm.NoSlip('obstacle'), mask_callback=lambda *m: np.logical_and.reduce(
                [(mi > ci) & (mi < ci + 2) for mi, ci in zip(m, c)]))


@pytest.mark.parametrize('stencil,shape,compressible,layout', [('D2Q9', (12, 9), True, 'fzyx'),
                                                              ('D2Q9', (10, 8), False, 'numpy'),
                                                              ('D3Q19', (7, 8, 6), False, 'fzyx')])
def test_lbm_walls_cpu_vs_oracle(stencil, shape, compressible, layout):
    """No-slip channel with an obstacle: T forward steps vs the array-roll + bounce-back restatement, the
    adjoint of T steps vs torch's reverse mode through it, the flags equal the mask the API was given."""
    import torch
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, layout=layout)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.2, target='cpu')
    _set_channel(step, shape)
    wall = _channel(shape)
    assert np.array_equal(step.boundary_handling.flags.astype(bool), wall)
    f0 = _init(stencil, shape, compressible, seed=7)
    T = 4
    step.set_pdfs(f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_walls(ft, 1.2, torch.tensor(wall), T, stencil, compressible, xp=torch)
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    g = np.random.default_rng(8).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


def test_lbm_walls_api():
    rule = lbm.create_lb_update_rule('D2Q9')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(6, 5), relaxation_rate=1.0, target='cpu')
    assert step.backward_boundary_handling is step.boundary_handling
    step.set_boundary_including_adjoint(lbm.NoSlip(), mask_array=np.eye(6, 5, dtype=bool))
    assert np.array_equal(step.boundary_handling.flags, np.eye(6, 5, dtype=np.uint8))
    step.boundary_handling.set_boundary('domain', lbm.make_slice[2:, :])
    assert step.boundary_handling.flags.sum() == 2
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[4, 1:3],
                                        adjoint_boundary_condition=lbm.AdjointNoSlip())
    assert step.boundary_handling.flags[4, 1:3].all() and step.boundary_handling.flags.sum() == 4
    with pytest.raises(NotImplementedError):
        step.set_boundary_including_adjoint('UBB')
    with pytest.raises(NotImplementedError):
        lbm.AdjointBoundaryCondition(object())
    assert lbm.AdjointBoundaryCondition(lbm.NoSlip()) == lbm.AdjointBoundaryCondition(lbm.NoSlip())


def test_lbm_end_to_end_op_cpu():
    """rho, u → equilibrium → T steps (channel walls) → rho, u: values vs the oracle chain, gradients of a
    scalar loss w.r.t. rho and u vs torch's reverse mode through the oracle chain."""
    import torch
    shape, T = (10, 8), 4
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.4, target='cpu')
    _set_channel(step, shape, obstacle=False)
    rng = np.random.default_rng(12)
    rho0 = 1 + 0.05 * rng.standard_normal(shape)
    u0 = 0.03 * rng.standard_normal(shape + (2,))
    rho = torch.tensor(rho0, requires_grad=True)
    vel = torch.tensor(u0, requires_grad=True)
    res = step.create_end_to_end_op(T, vel, rho, num_times_steps_without_save=1)
    w = torch.tensor(rng.standard_normal(shape + (2,)))
    loss = (res.output_velocity_tensor * w).sum() + (res.output_density_tensor ** 2).sum()
    loss.backward()
    rt, vt = torch.tensor(rho0, requires_grad=True), torch.tensor(u0, requires_grad=True)
    f = OL.equilibrium(rt, vt, 'D2Q9', True, xp=torch)
    f = OL.run_walls(f, 1.4, torch.tensor(_channel(shape, False)), T, 'D2Q9', True, xp=torch)
    r_ref = f.sum(-1)
    dirs = OL.D2Q9[0]
    v_ref = torch.stack([sum(c[a] * f[..., i] for i, c in enumerate(dirs)) / r_ref for a in range(2)], -1)
    l_ref = (v_ref * w).sum() + (r_ref ** 2).sum()
    l_ref.backward()
    assert abs(float(loss) - float(l_ref)) <= 1e-12 * abs(float(l_ref))
    assert torch.allclose(rho.grad, rt.grad, rtol=0, atol=1e-11 * float(rt.grad.abs().max()))
    assert torch.allclose(vel.grad, vt.grad, rtol=0, atol=1e-11 * float(vt.grad.abs().max()))
    assert res.input_pdf_tensor.shape == shape + (9,)


# --- GPU: the lattice schedule ---------------------------------------------------------------------------
LATTICE_GPU_CASES = [('D2Q9', (64, 48), True, 'fzyx', 'float32', True), ('D2Q9', (37, 70), False, 'numpy', 'float64', True),
                     ('D3Q19', (20, 17, 70), False, 'fzyx', 'float32', True),
                     ('D3Q19', (16, 12, 24), True, 'fzyx', 'float64', False),
                     ('D3Q27', (10, 9, 66), True, 'fzyx', 'float64', True)]


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape,compressible,layout,dtype,walls', LATTICE_GPU_CASES)
def test_lbm_lattice_schedule_gpu_vs_oracle(stencil, shape, compressible, layout, dtype, walls):
    """The timestep op on the lattice schedule (walls or periodic, fzyx / AoS pdfs, fp32 / fp64): forward vs the
    oracle, the adjoint vs torch's reverse mode through it; the op's internal states are row-interleaved
    (their layout never reaches the caller: the output comes back in the field's layout, the gradient in the one
    torch's gradient accumulation gives the input)."""
    import torch
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, layout=layout, data_type=dtype)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target='gpu')
    wall = _channel(shape) if walls else np.zeros(shape, bool)
    if walls:
        _set_channel(step, shape)
    Op = step.create_timestep_op(5)
    f0 = _init(stencil, shape, compressible, seed=4)
    tdt = getattr(torch, dtype)
    x = torch.tensor(f0, dtype=tdt, device='cuda', requires_grad=True)
    out = Op.apply(x)
    assert out.stride() == step.empty_pdfs().stride()
    ft = torch.tensor(f0, requires_grad=True, device='cuda')
    ref = OL.run_walls(ft, 1.3, torch.tensor(wall, device='cuda'), 5, stencil, compressible, xp=torch)
    tol = 1e-12 if dtype == 'float64' else 1e-5
    assert float((out.double() - ref).abs().max()) <= tol * float(ref.abs().max())
    g = torch.tensor(np.random.default_rng(5).standard_normal(f0.shape), device='cuda')
    out.backward(g.to(tdt))
    (gref,) = torch.autograd.grad(ref, ft, g)
    assert float((x.grad.double() - gref).abs().max()) <= 10 * tol * float(gref.abs().max())


@pytest.mark.gpu
def test_lbm_end_to_end_op_gpu():
    import torch
    shape, T = (96, 64), 6
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True, data_type='float64')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.6, target='gpu')
    _set_channel(step, shape)
    rng = np.random.default_rng(13)
    rho0, u0 = 1 + 0.05 * rng.standard_normal(shape), 0.03 * rng.standard_normal(shape + (2,))
    rho = torch.tensor(rho0, requires_grad=True, device='cuda')
    vel = torch.tensor(u0, requires_grad=True, device='cuda')
    res = step.create_end_to_end_op(T, vel, rho, num_times_steps_without_save=2)
    loss = (res.output_velocity_tensor[..., 0] ** 2).sum() + res.output_density_tensor.sum()
    loss.backward()
    rt, vt = torch.tensor(rho0, requires_grad=True, device='cuda'), torch.tensor(u0, requires_grad=True, device='cuda')
    f = OL.equilibrium(rt, vt, 'D2Q9', True, xp=torch)
    f = OL.run_walls(f, 1.6, torch.tensor(_channel(shape), device='cuda'), T, 'D2Q9', True, xp=torch)
    r_ref = f.sum(-1)
    ux = sum(c[0] * f[..., i] for i, c in enumerate(OL.D2Q9[0])) / r_ref
    (ux ** 2).sum().add(r_ref.sum()).backward()
    assert torch.allclose(rho.grad, rt.grad, rtol=0, atol=1e-10 * float(rt.grad.abs().max()))
    assert torch.allclose(vel.grad, vt.grad, rtol=0, atol=1e-10 * float(vt.grad.abs().max()))


# --- moving walls (UBB) and the generic adjoint boundary (adjoint_boundaryconditions.py:7-46) -------------
LID_U = 0.05


def _cavity(shape):
    """Lid-driven cavity: no-slip walls on both ends of axis 0 and the low end of axis 1, the lid (UBB moving along
    axis 0) on the high end of axis 1. Returns (wall mask, wall velocity [*shape, 2])."""
    wall = np.zeros(shape, bool)
    wall[0, :] = wall[-1, :] = wall[:, 0] = wall[:, -1] = True
    vel = np.zeros(shape + (2,))
    vel[1:-1, -1, 0] = LID_U
    return wall, vel


def _set_cavity(step, shape, adjoint=None):
    lid = lbm.UBB((LID_U, 0.0), name='lid')
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[0, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[-1, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 0])
    step.set_boundary_including_adjoint(lid, lbm.make_slice[1:-1, -1], adjoint_boundary_condition=adjoint)
    return lid


def test_boundary_links_and_generic_adjoint():
    """The link assignments of NoSlip / UBB (lbmpy's form), the adjoint derived from them, and the (α, β, γ, βρ, γρ)
    the lattice kernels fuse (density-weighted links too); a link of another form is refused."""
    import sympy as sp
    from pystencils_autodiff_amd import AdjointField, ps
    st = lbm.LBStencil('D2Q9')
    f = ps.fields('f(9): [2D]')
    ubb = lbm.UBB((0.1, -0.2))
    (a,) = ubb(f, 6, st)                       # direction 6 = (1, 1): link into the wall at x + (1, 1), comes back as 7
    assert a.lhs == f[1, 1](7)
    assert sp.simplify(a.rhs - (f(6) - 6 * sp.Rational(1, 36) * (sp.Float(0.1) - sp.Float(0.2)))) == 0
    adj = lbm.AdjointBoundaryCondition(ubb)(AdjointField(f), 6, st)
    (b,) = adj.main_assignments
    g = AdjointField(f)
    assert b.lhs == g(6) and sp.simplify(b.rhs - g[1, 1](7)) == 0     # the transpose: diff f(6) <- diff f[1,1](7)
    # the reference's heuristic: a field named diff<name> is the adjoint of <name>
    assert lbm.AdjointBoundaryCondition(ubb)(ps.fields('difff(9): [2D]'), 6, st).main_assignments[0].lhs.field.name == \
        'difff'
    co = lbm.link_coefficients(ubb, lbm.AdjointBoundaryCondition(ubb), st)
    for d, (al, be, ga, br, gr) in enumerate(co):
        c = st.directions[d]
        assert al == 1.0 and ga == 1.0 and br == 0.0 and gr == 0.0
        assert be == pytest.approx(-6 * float(st.weights[d]) * (0.1 * c[0] - 0.2 * c[1]))
    assert lbm.link_coefficients(lbm.NoSlip(), lbm.AdjointNoSlip(), st) == \
        tuple((1.0, 0.0, 1.0, 0.0, 0.0) for _ in range(9))

    class DensityUBB(lbm.Boundary):
        """A link weighted by the cell's density, inline (no subexpression): fused as βρ = -0.1."""
        def __call__(self, pdf_field, direction, lb_method, **kw):
            c = st.directions[direction]
            rho = sum(pdf_field(i) for i in range(9))
            return [ps.Assignment(pdf_field[c](st.inverse_direction_index(direction)), pdf_field(direction) - 0.1 * rho)]
    co = lbm.link_coefficients(DensityUBB(), lbm.AdjointBoundaryCondition(DensityUBB()), st)
    assert all(tuple(t) == pytest.approx((1.0, 0.0, 1.0, -0.1, -0.1)) for t in co[1:])
    # lbmpy's compressible UBB (density subexpression): βρ = −6 w_d (c_d·u)
    dub = lbm.UBB((0.1, -0.2), density_weighted=True)
    for d, (al, be, ga, br, gr) in enumerate(lbm.link_coefficients(dub, lbm.AdjointBoundaryCondition(dub), st)):
        c = st.directions[d]
        assert al == pytest.approx(1.0) and be == 0.0 and ga == pytest.approx(1.0)
        assert br == pytest.approx(-6 * float(st.weights[d]) * (0.1 * c[0] - 0.2 * c[1])) and gr == pytest.approx(br)

    class Skewed(lbm.Boundary):
        """Not of the fused form (another pdf weighted on its own)."""
        def __call__(self, pdf_field, direction, lb_method, **kw):
            c = st.directions[direction]
            return [ps.Assignment(pdf_field[c](st.inverse_direction_index(direction)),
                                  pdf_field(direction) - 0.1 * pdf_field(0))]
    with pytest.raises(NotImplementedError):
        lbm.link_coefficients(Skewed(), lbm.AdjointBoundaryCondition(Skewed()), st)
    # ... it is a link program instead: the forward value and the Jacobian row of the cell's own pdfs
    kind, prog = lbm.link_form(Skewed(), lbm.AdjointBoundaryCondition(Skewed()), st)
    assert kind == 'program' and prog[0] is None
    lines, val, jac = prog[6]
    assert sorted(k for k, _, _ in jac) == [0, 6] and dict((k, e) for k, _, e in jac)[6] in ('(T)1', '(T)1.0')

    class Remote(lbm.Boundary):
        """Reads a population of another cell: neither form."""
        def __call__(self, pdf_field, direction, lb_method, **kw):
            c = st.directions[direction]
            return [ps.Assignment(pdf_field[c](st.inverse_direction_index(direction)), pdf_field[-c[0], -c[1]](direction))]
    step = lbm.AutoDiffLatticeBoltzmannStep(lbm.create_lb_update_rule('D2Q9', compressible=True),
                                            domain_size=(6, 5), relaxation_rate=1.0, target='cpu')
    with pytest.raises(NotImplementedError):
        step.set_boundary_including_adjoint(Remote())
    step.set_boundary_including_adjoint(Skewed(), lbm.make_slice[0, :])


@pytest.mark.parametrize('adjoint', ['derived', 'noslip'])
@pytest.mark.parametrize('compressible', [True, False])
def test_lbm_lid_driven_cavity_cpu(adjoint, compressible):
    """D2Q9 lid-driven cavity (NoSlip walls + a UBB lid) on the C lattice kernels: T forward steps vs the array-roll
    + moving-wall restatement (oracle/lbm.py), the adjoint of T steps vs torch's reverse mode through it — with the
    default adjoint (AdjointBoundaryCondition(UBB), derived by AD) and an explicit AdjointNoSlip (the same
    transposed link)."""
    import torch
    shape, T = (14, 11), 6
    rule = lbm.create_lb_update_rule('D2Q9', compressible=compressible)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target='cpu')
    _set_cavity(step, shape, None if adjoint == 'derived' else lbm.AdjointNoSlip())
    wall, vel = _cavity(shape)
    assert np.array_equal(step.boundary_handling.flags != 0, wall)
    assert step._links() is not None
    f0 = _init('D2Q9', shape, compressible, seed=21)
    step.set_pdfs(f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_moving_walls(ft, 1.3, torch.tensor(wall), torch.tensor(vel), T, 'D2Q9', compressible, xp=torch)
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    # the lid drives the flow: the moving-wall terms are in (the no-slip-only run differs)
    still = OL.run_walls(torch.tensor(f0), 1.3, torch.tensor(wall), T, 'D2Q9', compressible, xp=torch)
    assert float((ref - still).abs().max()) > 1e-3
    g = np.random.default_rng(22).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


def test_lbm_link_tables_derived_once_per_boundary_change(monkeypatch):
    """The wall kernels' link tables (sympy AD of each boundary's link, ~20 ms) are derived once per boundary change,
    not per time step (a per-step derivation made the walled LBM configs 19x slower)."""
    calls = []
    from pystencils_autodiff_amd.lbm.boundaries import BoundaryHandling
    orig = BoundaryHandling.link_tables

    def counted(self, method):
        calls.append(1)
        return orig(self, method)
    monkeypatch.setattr(BoundaryHandling, "link_tables", counted)
    shape = (14, 11)
    step = lbm.AutoDiffLatticeBoltzmannStep(lbm.create_lb_update_rule('D2Q9'), domain_size=shape,
                                            relaxation_rate=1.3, target='cpu')
    _set_cavity(step, shape, None)
    step.set_pdfs(_init('D2Q9', shape, False, seed=3))
    step.run(4, record=True)
    step.set_adjoint_pdfs(np.ones_like(step.pdf_array))
    step.run_backward(4)
    assert len(calls) == 1
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 1])    # a boundary change: derived again
    step.run(1)
    assert len(calls) == 2


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', ['float64', 'float32'])
def test_lbm_lid_driven_cavity_gpu(dtype):
    """The lid-driven cavity through the timestep op on the HIP lattice kernels: forward vs the moving-wall
    restatement, the adjoint vs torch's reverse mode through it."""
    import torch
    shape, T = (70, 64), 8
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True, data_type=dtype)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.5, target='gpu')
    _set_cavity(step, shape)
    wall, vel = _cavity(shape)
    Op = step.create_timestep_op(T)
    f0 = _init('D2Q9', shape, True, seed=23)
    tdt = getattr(torch, dtype)
    x = torch.tensor(f0, dtype=tdt, device='cuda', requires_grad=True)
    out = Op.apply(x)
    ft = torch.tensor(f0, requires_grad=True, device='cuda')
    ref = OL.run_moving_walls(ft, 1.5, torch.tensor(wall, device='cuda'), torch.tensor(vel, device='cuda'), T, 'D2Q9',
                              True, xp=torch)
    tol = 1e-12 if dtype == 'float64' else 1e-5
    assert float((out.double() - ref).abs().max()) <= tol * float(ref.abs().max())
    g = torch.tensor(np.random.default_rng(24).standard_normal(f0.shape), device='cuda')
    out.backward(g.to(tdt))
    (gref,) = torch.autograd.grad(ref, ft, g)
    assert float((x.grad.double() - gref).abs().max()) <= 10 * tol * float(gref.abs().max())


FORCE_CASES = [('D2Q9', (10, 7), False, 'guo'), ('D2Q9', (9, 12), True, 'guo'), ('D2Q9', (8, 6), True, 'simple'),
               ('D3Q19', (6, 5, 4), False, 'guo')]


def _forced(stencil, shape, compressible, model, target, dtype='float64', schedule='lattice'):
    """A constant body force: the lattice kernels (force terms compiled in) or, with PSAD_LBM_LATTICE=0, the rule's
    own AutoDiffOp kernels (Guo: the transposed derivation)."""
    import os
    force = (1e-3, -2e-3, 5e-4)[:len(shape)]
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, force_model=model, force=force,
                                     data_type=dtype)
    old = os.environ.get('PSAD_LBM_LATTICE')
    os.environ['PSAD_LBM_LATTICE'] = '1' if schedule == 'lattice' else '0'
    try:
        step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.4, target=target)
    finally:
        if old is None:
            os.environ.pop('PSAD_LBM_LATTICE')
        else:
            os.environ['PSAD_LBM_LATTICE'] = old
    assert (step._lattice is not None) == (schedule == 'lattice')
    return step, force


@pytest.mark.parametrize('schedule', ['lattice', 'autodiffop'])
@pytest.mark.parametrize('stencil,shape,compressible,model', FORCE_CASES)
def test_lbm_force_models_cpu_vs_oracle(stencil, shape, compressible, model, schedule):
    """A constant body force (lbmpy's 'simple' / 'guo' force models restated; parity unpinned vs lbmpy): T steps
    and the adjoint of T steps on the C kernels vs the oracle's forced collision and torch's reverse mode."""
    import torch
    step, force = _forced(stencil, shape, compressible, model, 'cpu', schedule=schedule)
    f0 = _init(stencil, shape, compressible, seed=5)
    T = 3
    step.set_pdfs(f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run(ft, 1.4, T, stencil, compressible, xp=torch, force_model=model, force=force)
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    unforced = OL.run(torch.tensor(f0), 1.4, T, stencil, compressible, xp=torch)
    assert float((ref - unforced).abs().max()) > 1e-5          # the force is in
    g = np.random.default_rng(6).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


def test_lbm_force_model_getter_shift():
    """Guo forcing: the macroscopic getter reports the velocity shifted by F/2 (/ρ)."""
    import torch
    step, force = _forced('D2Q9', (6, 5), True, 'guo', 'cpu')
    f0 = _init('D2Q9', (6, 5), True, seed=8)
    rho, vel = step.create_macroscopic_getter_op().apply(torch.tensor(f0))
    dirs, _ = OL.SETS['D2Q9']
    r = f0.sum(-1)
    for a in range(2):
        m = sum(c[a] * f0[..., i] for i, c in enumerate(dirs))
        assert np.abs(vel.numpy()[..., a] - (m + force[a] / 2) / r).max() < 1e-13
    with pytest.raises(NotImplementedError):
        lbm.create_lb_update_rule('D2Q9', force_model='luo', force=(0, 0))


@pytest.mark.gpu
@pytest.mark.parametrize('schedule', ['lattice', 'autodiffop'])
@pytest.mark.parametrize('stencil,shape,compressible,model', FORCE_CASES)
def test_lbm_force_models_gpu_vs_oracle(stencil, shape, compressible, model, schedule):
    """The forced rules on the HIP kernels: the lattice kernels with the force terms compiled in, and the rule's
    AutoDiffOp kernels (transposed-mode adjoint)."""
    import torch
    step, force = _forced(stencil, shape, compressible, model, 'gpu', schedule=schedule)
    f0 = _init(stencil, shape, compressible, seed=5)
    T = 3
    step.set_pdfs(torch.tensor(f0, device='cuda'))
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run(ft, 1.4, T, stencil, compressible, xp=torch, force_model=model, force=force)
    got = step.pdf_array.double().cpu().numpy()
    assert np.abs(got - ref.detach().numpy()).max() <= 1e-12 * np.abs(f0).max()
    g = np.random.default_rng(6).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(torch.tensor(g, device='cuda'))
    step.run_backward(T)
    gg = step.adjoint_pdf_array.double().cpu().numpy()
    assert np.abs(gg - gref.numpy()).max() <= 1e-11 * np.abs(gref.numpy()).max()


# a per-cell body force: a force FIELD (D components) in the update rule — an additional input of the step, its adjoint
# summed over the steps (the reference's additional / time-constant fields, _autodiff_lbstep.py:113-128, :284-306)
FIELD_FORCE_CASES = [('D2Q9', (9, 7), True, 'guo', 'numpy'), ('D2Q9', (8, 6), False, 'simple', 'fzyx'),
                     ('D2Q9', (7, 9), False, 'guo', 'fzyx'), ('D3Q19', (5, 4, 6), True, 'guo', 'numpy')]
# the remaining (model, compressible, layout) combinations, lattice kernels only (the AutoDiffOp derivation of a D3Q19
# rule takes ~1 min of sympy on the CPU)
FIELD_FORCE_CASES_LATTICE = [('D3Q19', (4, 6, 5), False, 'simple', 'numpy'), ('D3Q19', (4, 5, 4), True, 'simple', 'fzyx'),
                             ('D2Q9', (6, 8), True, 'simple', 'numpy'), ('D3Q19', (5, 5, 4), False, 'guo', 'fzyx')]
FIELD_FORCE_ALL = [c + ('lattice',) for c in FIELD_FORCE_CASES + FIELD_FORCE_CASES_LATTICE] + \
    [c + ('autodiffop',) for c in FIELD_FORCE_CASES]


def _force_field_case(stencil, shape, compressible, model, layout, target, T=3, schedule='lattice'):
    import os
    import torch
    D = len(shape)
    F = ps.fields(f"F({D}): float64[{D}D]", layout=layout)
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, force_model=model, force=F)
    old = os.environ.get('PSAD_LBM_LATTICE')
    os.environ['PSAD_LBM_LATTICE'] = '1' if schedule == 'lattice' else '0'
    try:
        step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.4, target=target)
    finally:
        if old is None:
            os.environ.pop('PSAD_LBM_LATTICE')
        else:
            os.environ['PSAD_LBM_LATTICE'] = old
    assert [f.name for f in step._additional_fields] == ['F']
    assert (step._lattice is not None) == (schedule == 'lattice')
    op = step.create_timestep_op(T)
    rng = np.random.default_rng(sum(shape))
    f0 = _init(stencil, shape, compressible, seed=9)
    Fv = 1e-3 * rng.standard_normal(shape + (D,))
    dev = 'cuda' if target == 'gpu' else 'cpu'
    x = torch.tensor(f0, device=dev, requires_grad=True)
    Ft = torch.tensor(Fv, device=dev, requires_grad=True)
    out = op.apply(x, Ft)
    ft, Fr = torch.tensor(f0, requires_grad=True), torch.tensor(Fv, requires_grad=True)
    ref = OL.run(ft, 1.4, T, stencil, compressible, xp=torch, force_model=model,
                 force=tuple(Fr[..., a] for a in range(D)))
    g = torch.tensor(rng.standard_normal(f0.shape))
    out.backward(g.to(dev))
    gx, gF = torch.autograd.grad(ref, (ft, Fr), g)
    return out.detach().cpu(), ref.detach(), x.grad.cpu(), gx, Ft.grad.cpu(), gF


@pytest.mark.parametrize('stencil,shape,compressible,model,layout,schedule', FIELD_FORCE_ALL)
def test_lbm_force_field_cpu_vs_oracle(stencil, shape, compressible, model, layout, schedule):
    """A per-cell force field through the timestep op on the C kernels — the lattice kernels (the force read per
    cell, its adjoint accumulated over the steps in the adjoint kernel) and the rule's AutoDiffOp kernels: pdfs after
    T steps, the pdf adjoint and the force adjoint (summed over the steps) vs the oracle's forced collision with
    per-cell forces and torch's reverse mode (parity unpinned vs lbmpy, which is absent)."""
    out, ref, gx, gxr, gF, gFr = _force_field_case(stencil, shape, compressible, model, layout, 'cpu',
                                                   schedule=schedule)
    assert float((out - ref).abs().max()) <= 1e-13 * float(ref.abs().max())
    assert float((gx - gxr).abs().max()) <= 1e-12 * float(gxr.abs().max())
    assert float((gF - gFr).abs().max()) <= 1e-12 * float(gFr.abs().max())


def test_lbm_force_field_end_to_end_and_errors():
    """create_end_to_end_op(force_input_tensor=…): setter → steps (force bound to every step) → getter (Guo's shifted
    velocity reads the force too); dloss/dF against central finite differences; a rule with a force field needs
    its tensor, a rule without one refuses it."""
    import torch
    F = ps.fields("F(2): float64[2D]")
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True, force_model='guo', force=F)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=(9, 7), relaxation_rate=1.4, target='cpu')
    rng = np.random.default_rng(1)
    rho = torch.tensor(1 + 0.01 * rng.standard_normal((9, 7)))
    vel = torch.tensor(0.01 * rng.standard_normal((9, 7, 2)))
    Ft = torch.tensor(1e-3 * rng.standard_normal((9, 7, 2)), requires_grad=True)

    def loss(Fv):
        r = step.create_end_to_end_op(4, vel, rho, force_input_tensor=Fv, num_times_steps_without_save=1)
        return (r.output_velocity_tensor ** 2).sum() + r.output_density_tensor.sum()
    loss(Ft).backward()
    e = 1e-6
    for idx in ((3, 2, 1), (0, 6, 0), (8, 0, 1)):
        Fp, Fm = Ft.detach().clone(), Ft.detach().clone()
        Fp[idx] += e
        Fm[idx] -= e
        fd = (float(loss(Fp)) - float(loss(Fm))) / (2 * e)
        assert abs(fd - float(Ft.grad[idx])) <= 1e-6 * abs(fd) + 1e-9, (idx, fd, float(Ft.grad[idx]))
    with pytest.raises(ValueError):
        step.create_end_to_end_op(4, vel, rho)
    plain = lbm.AutoDiffLatticeBoltzmannStep(lbm.create_lb_update_rule('D2Q9'), domain_size=(9, 7),
                                             relaxation_rate=1.4, target='cpu')
    with pytest.raises(ValueError):
        plain.create_end_to_end_op(4, vel, rho, force_input_tensor=Ft)
    with pytest.raises(ValueError):
        lbm.create_lb_update_rule('D2Q9', force_model='guo', force=ps.fields("G(3): float64[2D]"))


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape,compressible,model,layout,schedule', FIELD_FORCE_ALL)
def test_lbm_force_field_gpu_vs_oracle(stencil, shape, compressible, model, layout, schedule):
    """The per-cell force field on the HIP kernels: the lattice kernels (force array read per cell, force adjoint
    accumulated by the adjoint launches) and the rule's AutoDiffOp kernels (transposed-mode adjoint)."""
    out, ref, gx, gxr, gF, gFr = _force_field_case(stencil, shape, compressible, model, layout, 'gpu',
                                                   schedule=schedule)
    assert float((out.double() - ref).abs().max()) <= 1e-12 * float(ref.abs().max())
    assert float((gx.double() - gxr).abs().max()) <= 1e-11 * float(gxr.abs().max())
    assert float((gF.double() - gFr).abs().max()) <= 1e-11 * float(gFr.abs().max())


@pytest.mark.parametrize('target', ['cpu', pytest.param('gpu', marks=pytest.mark.gpu)])
@pytest.mark.parametrize('model,compressible', [('guo', True), ('simple', False)])
def test_lbm_force_driven_channel(target, model, compressible):
    """A body force along a no-slip channel on the lattice kernels (walls and force terms in one kernel): T steps and
    the adjoint vs the oracle's wall step with the forced collision; after many steps the profile across the channel
    is Poiseuille's parabola (Guo: the velocity with the F/2 shift against F (y − y0)(y1 − y) / (2ν) within a few %).
    """
    import torch
    shape, T = (12, 9), 4
    F = (0.0, 1e-5)                                   # along axis 1 (the channel's walls are the first / last axis-0 rows)
    rule = lbm.create_lb_update_rule('D2Q9', compressible=compressible, force_model=model, force=F)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.2, target=target)
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[0, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[-1, :])
    assert step._lattice is not None
    wall = np.zeros(shape, bool)
    wall[0, :] = wall[-1, :] = True
    f0 = _init('D2Q9', shape, compressible, seed=13)
    dev = 'cuda' if target == 'gpu' else 'cpu'
    step.set_pdfs(torch.tensor(f0, device=dev) if target == 'gpu' else f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_walls(ft, 1.2, torch.tensor(wall), T, 'D2Q9', compressible, xp=torch, force_model=model, force=F)
    got = step.pdf_array.double().cpu().numpy() if target == 'gpu' else step.pdf_array
    assert np.abs(got - ref.detach().numpy()).max() <= 1e-12 * np.abs(f0).max()
    g = np.random.default_rng(14).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(torch.tensor(g, device=dev) if target == 'gpu' else g)
    step.run_backward(T)
    ga = step.adjoint_pdf_array.double().cpu().numpy() if target == 'gpu' else step.adjoint_pdf_array
    assert np.abs(ga - gref.numpy()).max() <= 1e-11 * np.abs(gref.numpy()).max()
    if model == 'guo':
        # steady state from rest: Poiseuille across axis 0 (walls half-way between rows 0/1 and 10/11)
        rest = np.broadcast_to(np.asarray([float(w) for w in OL.SETS['D2Q9'][1]]), shape + (9,)).copy()
        step.set_pdfs(torch.tensor(rest, device=dev) if target == 'gpu' else rest)
        step.run(4000)
        f = step.pdf_array.double().cpu().numpy() if target == 'gpu' else step.pdf_array
        dirs = OL.SETS['D2Q9'][0]
        rho = f.sum(-1)
        u1 = (sum(c[1] * f[..., i] for i, c in enumerate(dirs)) + F[1] / 2) / rho
        nu = (1 / 1.2 - 0.5) / 3
        y = np.arange(shape[0]) - 0.5                 # distance from the lower wall (half-way bounce-back)
        H = shape[0] - 2
        prof = F[1] * y * (H - y) / (2 * nu)
        inner = slice(1, shape[0] - 1)
        assert np.abs(u1[inner].mean(1) - prof[inner]).max() <= 0.03 * prof[inner].max()


# ------------------------------------------------------------------------------------------------------ TRT method
# create_lb_update_rule(method='trt'): lbmpy's two-relaxation-time method restated (parity unpinned vs lbmpy, absent);
# checked against the oracle's TRT collision (oracle/lbm.py collide(omega_odd=…)) and torch's reverse mode through it
TRT_CASES = [('D2Q9', (9, 7), True, 'magic', 'fzyx', False), ('D2Q9', (8, 6), False, 'rate', 'numpy', True),
             ('D3Q19', (5, 4, 6), True, 'rate', 'fzyx', True), ('D3Q19', (4, 5, 4), False, 'magic', 'numpy', False)]


def _trt_case(stencil, shape, compressible, odd, layout, walls, target, schedule, force=None):
    import os
    rr = 1.4
    kw = dict(relaxation_rates=[rr, 1.1]) if odd == 'rate' else {}
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, layout=layout, method='trt',
                                     force_model='simple' if force else None, force=force, **kw)
    old = os.environ.get('PSAD_LBM_LATTICE')
    os.environ['PSAD_LBM_LATTICE'] = '1' if schedule == 'lattice' else '0'
    try:
        step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=rr, target=target)
    finally:
        if old is None:
            os.environ.pop('PSAD_LBM_LATTICE')
        else:
            os.environ['PSAD_LBM_LATTICE'] = old
    assert (step._lattice is not None) == (schedule == 'lattice')
    w_odd = 1.1 if odd == 'rate' else OL.trt_odd_rate(rr)
    wall = None
    if walls:
        _set_channel(step, shape)
        wall = _channel(shape)
    return step, rr, w_odd, wall


@pytest.mark.parametrize('schedule', ['lattice', 'autodiffop'])
@pytest.mark.parametrize('stencil,shape,compressible,odd,layout,walls', TRT_CASES)
def test_lbm_trt_cpu_vs_oracle(stencil, shape, compressible, odd, layout, walls, schedule):
    """TRT (ω₋ from lbmpy's magic number 3/16, or given): T steps and the adjoint of T steps on the C kernels (the
    lattice kernels, or the rule's AutoDiffOp kernels with the structured TRT adjoint) vs the oracle and torch's
    reverse mode, periodic and with no-slip walls."""
    import torch
    if schedule == 'autodiffop' and walls:
        pytest.skip('walls need the lattice schedule')
    step, rr, w_odd, wall = _trt_case(stencil, shape, compressible, odd, layout, walls, 'cpu', schedule)
    f0 = _init(stencil, shape, compressible, seed=4)
    T = 3
    step.set_pdfs(f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = (OL.run_walls(ft, rr, torch.tensor(wall), T, stencil, compressible, xp=torch, omega_odd=w_odd) if walls else
           OL.run(ft, rr, T, stencil, compressible, xp=torch, omega_odd=w_odd))
    srt = OL.run(torch.tensor(f0), rr, T, stencil, compressible, xp=torch)
    assert float((ref.detach() - srt).abs().max()) > 1e-6            # TRT is not SRT here
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    g = np.random.default_rng(5).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


@pytest.mark.parametrize('stencil,equal', [('D2Q9', True), ('D3Q19', True), ('D3Q27', False)])
def test_lbm_mrt_trt_equivalence_per_stencil(stencil, equal):
    """MRT with rates [ω, ω, ω₋, ω] relaxes the non-equilibrium part like TRT — ω on the even part (f + f_ī)/2, ω₋ on
    the odd part (f − f_ī)/2 — on D2Q9 and D3Q19, whose odd non-conserved moments are the third-order ones. Not on
    D3Q27: its odd fifth-order moments x²y²z, x²yz², xy²z² sit in the fourth-order group (rate ω)."""
    from pystencils_autodiff_amd.lbm._method import MRT_GROUPS, mrt_moments, mrt_relaxation_matrices
    st = lbm.LBStencil(stencil)
    Q = st.Q
    P = {g: np.array(m, dtype=np.float64) for g, m in mrt_relaxation_matrices(st).items()}
    cons = [np.array(r, dtype=np.float64) for g, r in mrt_moments(st) if g == 'conserved']
    w_even, w_odd = 1.3, 0.7
    R = sum({'third': w_odd}.get(g, w_even) * P[g] for g in MRT_GROUPS)
    inv = [st.inverse_direction_index(i) for i in range(Q)]
    Pi = np.zeros((Q, Q))
    Pi[np.arange(Q), inv] = 1.0
    T = w_even * (np.eye(Q) + Pi) / 2 + w_odd * (np.eye(Q) - Pi) / 2
    rng = np.random.default_rng(7)
    A = np.stack(cons)                                     # non-equilibrium parts carry no conserved moments
    for _ in range(4):
        v = rng.normal(size=Q)
        v -= A.T @ np.linalg.lstsq(A @ A.T, A @ v, rcond=None)[0]
        assert np.allclose(A @ v, 0, atol=1e-12)
        assert np.allclose(R @ v, T @ v, atol=1e-12) == equal


def test_lbm_trt_rule_api():
    """The TRT rule: ω₊ = ω₋ is SRT; lbmpy's magic-number relation; the odd rate as a kernel symbol runs on the
    AutoDiffOp kernels; unsupported combinations raise."""
    import sympy as sp
    w = sp.Symbol('omega')
    wo = lbm.relaxation_rate_from_magic_number(w)
    lam = sp.simplify((1 / w - sp.Rational(1, 2)) * (1 / wo - sp.Rational(1, 2)))
    assert lam == sp.Rational(3, 16)
    assert abs(float(wo.subs(w, 1.4)) - OL.trt_odd_rate(1.4)) < 1e-14
    rule = lbm.create_lb_update_rule('D2Q9', method='trt', relaxation_rates=[1.3, 1.3])
    srt = lbm.create_lb_update_rule('D2Q9', relaxation_rate=1.3)
    for a, b in zip(rule.main_assignments, srt.main_assignments):
        assert sp.simplify(a.rhs - b.rhs) == 0
    sym = lbm.create_lb_update_rule('D2Q9', method='trt', relaxation_rates=[w, sp.Symbol('omega_odd')])
    step = lbm.AutoDiffLatticeBoltzmannStep(sym, domain_size=(6, 5), kernel_params={'omega': 1.2, 'omega_odd': 1.0},
                                            target='cpu')
    assert step._lattice is None
    with pytest.raises(NotImplementedError):
        lbm.create_lb_update_rule('D2Q9', method='cumulant')
    for m in ('trt', 'mrt'):                      # Guo with TRT / MRT: lbmpy's shear-rate prefactor (tested below)
        assert lbm.create_lb_update_rule('D2Q9', method=m, force_model='guo', force=(1e-3, 0)).force_model == 'guo'
    with pytest.raises(ValueError):
        lbm.create_lb_update_rule('D2Q9', relaxation_rates=[1.2, 1.1])


def test_lbm_trt_force_field_cpu():
    """TRT with a per-cell 'simple' force field on the lattice kernels: pdfs, pdf adjoint and force adjoint vs the
    oracle and torch's reverse mode."""
    import torch
    shape, D, T = (7, 8), 2, 3
    F = ps.fields(f"F({D}): float64[{D}D]")
    step, rr, w_odd, _ = _trt_case('D2Q9', shape, True, 'magic', 'fzyx', False, 'cpu', 'lattice', force=F)
    op = step.create_timestep_op(T)
    rng = np.random.default_rng(2)
    f0 = _init('D2Q9', shape, True, seed=3)
    Fv = 1e-3 * rng.standard_normal(shape + (D,))
    x, Ft = torch.tensor(f0, requires_grad=True), torch.tensor(Fv, requires_grad=True)
    out = op.apply(x, Ft)
    ft, Fr = torch.tensor(f0, requires_grad=True), torch.tensor(Fv, requires_grad=True)
    ref = OL.run(ft, rr, T, 'D2Q9', True, xp=torch, force_model='simple', force=tuple(Fr[..., a] for a in range(D)),
                 omega_odd=w_odd)
    assert float((out - ref).detach().abs().max()) <= 1e-13 * float(ref.detach().abs().max())
    g = torch.tensor(rng.standard_normal(f0.shape))
    out.backward(g)
    gx, gF = torch.autograd.grad(ref, (ft, Fr), g)
    assert float((x.grad - gx).abs().max()) <= 1e-12 * float(gx.abs().max())
    assert float((Ft.grad - gF).abs().max()) <= 1e-12 * float(gF.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize('schedule', ['lattice', 'autodiffop'])
@pytest.mark.parametrize('stencil,shape,compressible,odd,layout,walls', TRT_CASES)
def test_lbm_trt_gpu_vs_oracle(stencil, shape, compressible, odd, layout, walls, schedule):
    """TRT on the HIP kernels (lattice kernels and the rule's AutoDiffOp kernels) vs the oracle and torch's reverse
    mode."""
    import torch
    if schedule == 'autodiffop' and walls:
        pytest.skip('walls need the lattice schedule')
    step, rr, w_odd, wall = _trt_case(stencil, shape, compressible, odd, layout, walls, 'gpu', schedule)
    f0 = _init(stencil, shape, compressible, seed=4)
    T = 3
    step.set_pdfs(torch.tensor(f0, device='cuda'))
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = (OL.run_walls(ft, rr, torch.tensor(wall), T, stencil, compressible, xp=torch, omega_odd=w_odd) if walls else
           OL.run(ft, rr, T, stencil, compressible, xp=torch, omega_odd=w_odd))
    got = step.pdf_array.double().cpu().numpy()
    assert np.abs(got - ref.detach().numpy()).max() <= 1e-12 * np.abs(f0).max()
    g = np.random.default_rng(5).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(torch.tensor(g, device='cuda'))
    step.run_backward(T)
    gg = step.adjoint_pdf_array.double().cpu().numpy()
    assert np.abs(gg - gref.numpy()).max() <= 1e-11 * np.abs(gref.numpy()).max()


def _density_cavity(target, compressible, trt=False):
    shape, T = (14, 11), 5
    kw = dict(method='trt') if trt else {}
    rule = lbm.create_lb_update_rule('D2Q9', compressible=compressible, **kw)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target=target)
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[0, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[-1, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 0])
    step.set_boundary_including_adjoint(lbm.UBB((LID_U, 0.0), density_weighted=True), lbm.make_slice[1:-1, -1])
    wall, vel = _cavity(shape)
    assert step._lattice_kernels().rho_links
    return step, shape, T, wall, vel, (OL.trt_odd_rate(1.3) if trt else None)


@pytest.mark.parametrize('compressible,trt', [(True, False), (False, False), (True, True)])
def test_lbm_density_weighted_ubb_cpu(compressible, trt):
    """Lid-driven cavity with lbmpy's compressible UBB (the wall term times the fluid cell's density): the link is
    affine in all the cell's pdfs, fused into the C lattice kernels (ρ(x) from the cell's own pdfs in the forward, a
    second adjoint pass for the density term); T steps vs the oracle, the adjoint vs torch's reverse mode."""
    import torch
    step, shape, T, wall, vel, w_odd = _density_cavity('cpu', compressible, trt)
    f0 = _init('D2Q9', shape, compressible, seed=23)
    step.set_pdfs(f0)
    step.run(T, record=True)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_moving_walls(ft, 1.3, torch.tensor(wall), torch.tensor(vel), T, 'D2Q9', compressible, xp=torch,
                              density_weighted=True, omega_odd=w_odd)
    plain = OL.run_moving_walls(torch.tensor(f0), 1.3, torch.tensor(wall), torch.tensor(vel), T, 'D2Q9', compressible,
                                xp=torch, omega_odd=w_odd)
    assert float((ref.detach() - plain).abs().max()) > 1e-4        # the density weighting is in
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    g = np.random.default_rng(24).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


@pytest.mark.gpu
@pytest.mark.parametrize('compressible,trt', [(True, False), (False, False), (True, True)])
def test_lbm_density_weighted_ubb_gpu(compressible, trt):
    """The density-weighted UBB cavity on the HIP lattice kernels (two adjoint passes), through ``run`` and the
    timestep op, vs the oracle and torch's reverse mode."""
    import torch
    step, shape, T, wall, vel, w_odd = _density_cavity('gpu', compressible, trt)
    f0 = _init('D2Q9', shape, compressible, seed=23)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_moving_walls(ft, 1.3, torch.tensor(wall), torch.tensor(vel), T, 'D2Q9', compressible, xp=torch,
                              density_weighted=True, omega_odd=w_odd)
    g = np.random.default_rng(24).standard_normal(f0.shape)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    step.set_pdfs(torch.tensor(f0, device='cuda'))
    step.run(T, record=True)
    assert np.abs(step.pdf_array.cpu().numpy() - ref.detach().numpy()).max() <= 1e-12 * np.abs(f0).max()
    step.set_adjoint_pdfs(torch.tensor(g, device='cuda'))
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array.cpu().numpy() - gref.numpy()).max() <= 1e-11 * np.abs(gref.numpy()).max()
    op = step.create_timestep_op(T)
    x = torch.tensor(f0, device='cuda', requires_grad=True)
    out = op.apply(x)
    out.backward(torch.tensor(g, device='cuda'))
    assert float((out.detach().cpu() - ref.detach()).abs().max()) <= 1e-12 * np.abs(f0).max()
    assert float((x.grad.cpu() - gref).abs().max()) <= 1e-11 * float(gref.abs().max())


# --- pressure boundaries (lbmpy FixedDensity) and other link programs ----------------------------------------
RHO_IN, RHO_OUT = 1.02, 0.98


def _pressure_channel(stencil, shape, compressible, target, trt=False, dtype='float64'):
    """A channel along axis 0: no-slip walls on both ends of axis 1 (and axis 2), FixedDensity inlet / outlet
    planes at the ends of axis 0 (lbmpy's pressure boundary, a link program of the lattice kernels)."""
    kw = dict(method='trt') if trt else {}
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, data_type=dtype, **kw)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target=target)
    D = len(shape)
    wall = np.zeros(shape, bool)
    for ax in range(1, D):
        for end in (0, -1):
            sl = [slice(None)] * D
            sl[ax] = end
            step.set_boundary_including_adjoint(lbm.NoSlip(), tuple(sl))
            wall[tuple(sl)] = True
    inner = tuple(slice(1, -1) for _ in range(1, D))
    step.set_boundary_including_adjoint(lbm.FixedDensity(RHO_IN, name='inlet'), (0,) + inner)
    step.set_boundary_including_adjoint(lbm.FixedDensity(RHO_OUT, name='outlet'), (-1,) + inner)
    pressure = np.zeros(shape, bool)
    pressure[(0,) + inner] = pressure[(-1,) + inner] = True
    wall |= pressure
    rho_w = np.ones(shape)
    rho_w[(0,) + inner], rho_w[(-1,) + inner] = RHO_IN, RHO_OUT
    assert np.array_equal(step.boundary_handling.flags != 0, wall)
    K = step._lattice_kernels()
    assert K.programs is not None and (K.link_pass or target == "gpu")
    return step, wall, pressure, rho_w, (OL.trt_odd_rate(1.3) if trt else None)


def _pressure_ref(f0, step_args, stencil, compressible, T, g, device='cpu'):
    import torch
    _, wall, pressure, rho_w, w_odd = step_args
    ft = torch.tensor(f0, requires_grad=True, device=device)
    tw = [torch.tensor(a, device=device) for a in (wall, pressure, rho_w)]
    ref = OL.run_pressure_walls(ft, 1.3, *tw, T, stencil, compressible, xp=torch, omega_odd=w_odd)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g, device=device))
    return ref.detach().cpu().numpy(), gref.cpu().numpy()


PRESSURE_CASES = [('D2Q9', (16, 9), True, False), ('D2Q9', (15, 10), False, False), ('D2Q9', (12, 9), True, True),
                  ('D3Q19', (9, 6, 5), True, False)]


@pytest.mark.parametrize('stencil,shape,compressible,trt', PRESSURE_CASES)
def test_lbm_pressure_channel_cpu(stencil, shape, compressible, trt):
    """A pressure-driven channel (FixedDensity inlet / outlet, no-slip walls) on the C lattice kernels: T steps vs
    the anti-bounce-back restatement (oracle/lbm.py ``run_pressure_walls``), the adjoint (link-program Jacobians
    through the second pass) vs torch's reverse mode through it."""
    T = 5
    args = _pressure_channel(stencil, shape, compressible, 'cpu', trt)
    step = args[0]
    f0 = _init(stencil, shape, compressible, seed=31)
    g = np.random.default_rng(32).standard_normal(f0.shape)
    ref, gref = _pressure_ref(f0, args, stencil, compressible, T, g)
    step.set_pdfs(f0)
    step.run(T, record=True)
    assert np.abs(step.pdf_array - ref).max() <= 1e-13 * np.abs(f0).max()
    # the pressure links are in: the same walls bouncing back everywhere give another flow
    import torch
    still = OL.run_walls(torch.tensor(f0), 1.3, torch.tensor(args[1]), T, stencil, compressible, xp=torch,
                         omega_odd=args[4]).numpy()
    assert np.abs(ref - still).max() > 1e-4
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref).max() <= 1e-12 * np.abs(gref).max()


def test_lbm_pressure_drives_flow():
    """Physics check of the pressure boundary: from rest, a density difference between inlet and outlet drives a
    flow from high to low density along the channel (positive mean axis-0 velocity in the interior)."""
    shape = (24, 11)
    step, wall, *_ = _pressure_channel('D2Q9', shape, True, 'cpu')
    f0 = OL.equilibrium(np.ones(shape), np.zeros(shape + (2,)), 'D2Q9', True)
    step.set_pdfs(f0)
    step.run(150)
    f = step.pdf_array
    dirs = OL.D2Q9[0]
    rho = f.sum(-1)
    ux = sum(c[0] * f[..., i] for i, c in enumerate(dirs)) / rho
    interior = ux[2:-2, 2:-2]
    assert interior.mean() > 1e-4
    assert rho[1, 5] > rho[-2, 5]


def test_lbm_fixed_density_symbolic_raises_clearly():
    """A FixedDensity with a symbolic density: a clear NotImplementedError from the link program (the lattice
    kernels compile the wall density in), not a bare TypeError from float(); the forward link itself stays symbolic."""
    st = lbm.LBStencil('D2Q9')
    view = lbm.boundaries.LBMethodView(st, True)
    rho = sp.Symbol('rho_w')
    fd = lbm.FixedDensity(rho)
    with pytest.raises(NotImplementedError, match='numeric wall density'):
        fd.program(view)
    with pytest.raises(NotImplementedError):
        lbm.link_program(fd, lbm.AdjointBoundaryCondition(fd), view)
    f = ps.fields('pdf(9): [2D]')
    assert any(rho in a.rhs.free_symbols for a in fd(f, 1, view))


def test_lbm_link_program_paths_agree():
    """The link program of FixedDensity three ways agree: written out by the boundary (``FixedDensity.program``,
    what the kernels use), differentiated by sympy from the printed link (any ``AdjointBoundaryCondition``), and read
    off the adjoint object's assignments (the transposed AD of the link, the general path)."""
    st = lbm.LBStencil('D2Q9')
    view = lbm.boundaries.LBMethodView(st, True)
    fd = lbm.FixedDensity(1.03)
    fast = lbm.link_program(fd, lbm.AdjointBoundaryCondition(fd), view)
    # a subclass of the adjoint object: not taken as the plain derived adjoint, so its assignments are parsed

    class Parsed(lbm.AdjointBoundaryCondition):
        pass
    slow = lbm.link_program(fd, Parsed(fd), view)

    class NoProgram(lbm.FixedDensity):
        program = None                                  # the derivative of the printed link by sympy
    mid = lbm.link_program(NoProgram(1.03), lbm.AdjointBoundaryCondition(NoProgram(1.03)), view)
    rng = np.random.default_rng(5)
    env = {f'c{q}': v for q, v in enumerate(rng.uniform(0.05, 0.3, 9))}

    def ev(lines, e):
        loc = dict(env)
        for ln in lines:
            name, rhs = ln[len('const T '):].rstrip(';').split(' = ', 1)
            loc[name] = eval(rhs.replace('(T)', ''), {}, loc)
        return eval(e.replace('(T)', ''), {}, loc)
    for a, b, m in zip(fast, slow, mid):
        assert (a is None) == (b is None) == (m is None)
        if a is not None:
            assert ev(a[0], a[1]) == pytest.approx(ev(m[0], m[1]), rel=1e-13)
            jm = {k: ev(l, e) for k, l, e in m[2]}
            assert all(jm[k] == pytest.approx(ev(l, e), rel=1e-12, abs=1e-15) for k, l, e in a[2])
        if a is None:
            continue
        assert ev(a[0], a[1]) == pytest.approx(ev(b[0], b[1]), rel=1e-13)
        ja, jb = {k: ev(l, e) for k, l, e in a[2]}, {k: ev(l, e) for k, l, e in b[2]}
        assert ja.keys() == jb.keys() and all(ja[k] == pytest.approx(jb[k], rel=1e-12, abs=1e-15) for k in ja)


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape,compressible,trt,dtype', [('D2Q9', (70, 33), True, False, 'float64'),
                                                                   ('D2Q9', (64, 40), False, True, 'float32'),
                                                                   ('D3Q19', (20, 12, 10), True, False, 'float64')])
def test_lbm_pressure_channel_gpu(stencil, shape, compressible, trt, dtype):
    """The pressure-driven channel on the HIP lattice kernels (link programs compiled in, two adjoint passes),
    through ``run`` / ``run_backward`` and the timestep op, vs the oracle and torch's reverse mode."""
    import torch
    T = 6
    args = _pressure_channel(stencil, shape, compressible, 'gpu', trt, dtype)
    step = args[0]
    f0 = _init(stencil, shape, compressible, seed=33)
    g = np.random.default_rng(34).standard_normal(f0.shape)
    ref, gref = _pressure_ref(f0, args, stencil, compressible, T, g)
    tdt = getattr(torch, dtype)
    tol = 1e-12 if dtype == 'float64' else 2e-5
    step.set_pdfs(torch.tensor(f0, dtype=tdt, device='cuda'))
    step.run(T, record=True)
    assert np.abs(step.pdf_array.double().cpu().numpy() - ref).max() <= tol * np.abs(f0).max()
    step.set_adjoint_pdfs(torch.tensor(g, dtype=tdt, device='cuda'))
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array.double().cpu().numpy() - gref).max() <= 10 * tol * np.abs(gref).max()
    op = step.create_timestep_op(T)
    x = torch.tensor(f0, dtype=tdt, device='cuda', requires_grad=True)
    out = op.apply(x)
    out.backward(torch.tensor(g, dtype=tdt, device='cuda'))
    assert float((out.detach().double().cpu() - torch.tensor(ref)).abs().max()) <= tol * np.abs(f0).max()
    assert float((x.grad.double().cpu() - torch.tensor(gref)).abs().max()) <= 10 * tol * np.abs(gref).max()


@pytest.mark.parametrize('target', ['cpu', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_lbm_pressure_with_density_weighted_lid(target):
    """Both second-pass terms in one lattice: a density-weighted moving lid (UBB, fused form with the density term)
    and a FixedDensity outlet (link program) with no-slip walls elsewhere — forward vs the oracle, the adjoint vs
    torch's reverse mode."""
    import torch
    shape, T = (14, 11), 5
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target=target)
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[0, :])
    step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 0])
    step.set_boundary_including_adjoint(lbm.UBB((LID_U, 0.0), density_weighted=True), lbm.make_slice[1:-1, -1])
    step.set_boundary_including_adjoint(lbm.FixedDensity(0.99), lbm.make_slice[-1, 1:-1])
    K = step._lattice_kernels()
    assert K.rho_links and K.programs is not None
    wall = step.boundary_handling.flags != 0
    pressure = np.zeros(shape, bool)
    pressure[-1, 1:-1] = True
    rho_w = np.where(pressure, 0.99, 1.0)
    vel = np.zeros(shape + (2,))
    vel[1:-1, -1, 0] = LID_U
    f0 = _init('D2Q9', shape, True, seed=41)
    g = np.random.default_rng(42).standard_normal(f0.shape)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_pressure_walls(ft, 1.3, torch.tensor(wall), torch.tensor(pressure), torch.tensor(rho_w), T, 'D2Q9',
                                True, xp=torch, wall_velocity=torch.tensor(vel), density_weighted=True)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    ref, gref = ref.detach().numpy(), gref.numpy()
    if target == 'gpu':
        step.set_pdfs(torch.tensor(f0, device='cuda'))
    else:
        step.set_pdfs(f0)
    step.run(T, record=True)
    pdf = step.pdf_array.cpu().numpy() if target == 'gpu' else step.pdf_array
    assert np.abs(pdf - ref).max() <= 1e-12 * np.abs(f0).max()
    step.set_adjoint_pdfs(torch.tensor(g, device='cuda') if target == 'gpu' else g)
    step.run_backward(T)
    adj = step.adjoint_pdf_array.cpu().numpy() if target == 'gpu' else step.adjoint_pdf_array
    assert np.abs(adj - gref).max() <= 1e-11 * np.abs(gref).max()


# --- MRT (lbmpy's weighted-orthogonal moment groups, restated) --------------------------------------------------
MRT_RATES = dict(shear=1.3, bulk=1.1, third=0.9, fourth=1.2)


def _mrt_case(stencil, shape, compressible, target, walls, dtype='float64', force=None):
    kw = dict(force_model='simple', force=force) if force is not None else {}
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, method='mrt', data_type=dtype,
                                     relaxation_rates=[sp_omega(), MRT_RATES['bulk'], MRT_RATES['third'],
                                                       MRT_RATES['fourth']], **kw)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=MRT_RATES['shear'], target=target)
    wall = np.zeros(shape, bool)
    if walls:
        for end in (0, -1):
            sl = [slice(None)] * len(shape)
            sl[1] = end
            step.set_boundary_including_adjoint(lbm.NoSlip(), tuple(sl))
            wall[tuple(sl)] = True
    assert step._lattice is not None and step._lattice_mrt is not None
    return step, wall, OL.mrt_matrix(stencil, MRT_RATES)


def sp_omega():
    import sympy as sp
    return sp.Symbol('omega')


MRT_CASES = [('D2Q9', (10, 7), True, False), ('D2Q9', (9, 12), False, True), ('D3Q19', (6, 5, 4), True, True),
             ('D3Q19', (5, 6, 4), False, False), ('D3Q27', (5, 6, 4), True, True)]


@pytest.mark.parametrize('stencil,shape,compressible,walls', MRT_CASES)
def test_lbm_mrt_cpu_vs_oracle(stencil, shape, compressible, walls):
    """MRT on the C lattice kernels (relaxation matrix ω P_ω + C compiled in): T steps vs the oracle's moment-space
    collision (its own Gram–Schmidt basis, ``M⁻¹ S M`` by numpy), the adjoint (h = Aᵀ g) vs torch's reverse mode."""
    import torch
    T = 4
    step, wall, A = _mrt_case(stencil, shape, compressible, 'cpu', walls)
    f0 = _init(stencil, shape, compressible, seed=51)
    g = np.random.default_rng(52).standard_normal(f0.shape)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_walls(ft, None, torch.tensor(wall), T, stencil, compressible, xp=torch, mrt=A)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    srt = OL.run_walls(torch.tensor(f0), MRT_RATES['shear'], torch.tensor(wall), T, stencil, compressible, xp=torch)
    assert float((ref.detach() - srt).abs().max()) > 1e-6          # the other rates are in
    step.set_pdfs(f0)
    step.run(T, record=True)
    assert np.abs(step.pdf_array - ref.detach().numpy()).max() <= 1e-13 * np.abs(f0).max()
    step.set_adjoint_pdfs(g)
    step.run_backward(T)
    assert np.abs(step.adjoint_pdf_array - gref.numpy()).max() <= 1e-12 * np.abs(gref.numpy()).max()


def test_lbm_mrt_special_cases_and_generic_schedule():
    """MRT with every rate ω is SRT and with [ω, ω, ω₋, ω] TRT (the only odd non-conserved moments are the third-order
    ones); a rate that is another symbol runs on the rule's AutoDiffOp kernels and matches the lattice kernels."""
    import sympy as sp
    shape = (9, 8)
    f0 = _init('D2Q9', shape, True, seed=53)
    res = {}
    for name, kw in (('srt', {}), ('mrt_all', dict(method='mrt')),
                     ('trt', dict(method='trt', relaxation_rates=[sp.Symbol('omega'), 0.8])),
                     ('mrt_trt', dict(method='mrt', relaxation_rates=[sp.Symbol('omega'), sp.Symbol('omega'), 0.8]))):
        step = lbm.AutoDiffLatticeBoltzmannStep(lbm.create_lb_update_rule('D2Q9', compressible=True, **kw),
                                                domain_size=shape, relaxation_rate=1.3, target='cpu')
        step.set_pdfs(f0)
        step.run(3)
        res[name] = step.pdf_array.copy()
    assert np.abs(res['srt'] - res['mrt_all']).max() <= 1e-14
    assert np.abs(res['trt'] - res['mrt_trt']).max() <= 1e-14
    sb = sp.Symbol('s_bulk')
    rule = lbm.create_lb_update_rule('D2Q9', compressible=True, method='mrt',
                                     relaxation_rates=[sp.Symbol('omega'), sb, 0.9, 1.2])
    generic = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.3, target='cpu',
                                               kernel_params={'s_bulk': 1.1})
    assert generic._lattice is None                   # a rate that is neither ω nor a number: the AutoDiffOp kernels
    lattice, _, _ = _mrt_case('D2Q9', shape, True, 'cpu', False)
    for st in (generic, lattice):
        st.set_pdfs(f0)
        st.run(3)
    assert np.abs(generic.pdf_array - lattice.pdf_array).max() <= 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape,compressible,walls,dtype', [('D2Q9', (66, 40), True, True, 'float64'),
                                                                     ('D3Q19', (20, 12, 10), False, False, 'float64'),
                                                                     ('D3Q19', (16, 12, 10), True, True, 'float32'),
                                                                     ('D3Q27', (12, 10, 8), True, True, 'float64')])
def test_lbm_mrt_gpu_vs_oracle(stencil, shape, compressible, walls, dtype):
    """MRT on the HIP lattice kernels through the timestep op vs the oracle and torch's reverse mode."""
    import torch
    T = 5
    step, wall, A = _mrt_case(stencil, shape, compressible, 'gpu', walls, dtype)
    f0 = _init(stencil, shape, compressible, seed=54)
    g = np.random.default_rng(55).standard_normal(f0.shape)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_walls(ft, None, torch.tensor(wall), T, stencil, compressible, xp=torch, mrt=A)
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    tdt = getattr(torch, dtype)
    tol = 1e-12 if dtype == 'float64' else 2e-5
    op = step.create_timestep_op(T)
    x = torch.tensor(f0, dtype=tdt, device='cuda', requires_grad=True)
    out = op.apply(x)
    out.backward(torch.tensor(g, dtype=tdt, device='cuda'))
    assert float((out.detach().double().cpu() - ref.detach()).abs().max()) <= tol * np.abs(f0).max()
    assert float((x.grad.double().cpu() - gref).abs().max()) <= 10 * tol * float(gref.abs().max())


@pytest.mark.parametrize('target', ['cpu', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_lbm_mrt_pressure_channel(target):
    """MRT with link-program walls: a D3Q19 pressure-driven channel (FixedDensity inlet / outlet, no-slip walls) on
    the MRT lattice kernels — on the GPU through the fix-up kernels — vs the oracle and torch's reverse mode."""
    import sympy as sp
    import torch
    stencil, shape, T = 'D3Q19', (10, 7, 6), 4
    rule = lbm.create_lb_update_rule(stencil, compressible=True, method='mrt',
                                     relaxation_rates=[sp.Symbol('omega'), MRT_RATES['bulk'], MRT_RATES['third'],
                                                       MRT_RATES['fourth']])
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=MRT_RATES['shear'], target=target)
    wall = np.zeros(shape, bool)
    for ax in (1, 2):
        for end in (0, -1):
            sl = [slice(None)] * 3
            sl[ax] = end
            step.set_boundary_including_adjoint(lbm.NoSlip(), tuple(sl))
            wall[tuple(sl)] = True
    step.set_boundary_including_adjoint(lbm.FixedDensity(RHO_IN), (0, slice(1, -1), slice(1, -1)))
    step.set_boundary_including_adjoint(lbm.FixedDensity(RHO_OUT), (-1, slice(1, -1), slice(1, -1)))
    pressure = np.zeros(shape, bool)
    pressure[0, 1:-1, 1:-1] = pressure[-1, 1:-1, 1:-1] = True
    wall |= pressure
    rho_w = np.where(pressure, np.where(np.arange(shape[0])[:, None, None] == 0, RHO_IN, RHO_OUT), 1.0)
    K = step._lattice_kernels()
    assert K.programs is not None and K.mrt is not None
    f0 = _init(stencil, shape, True, seed=61)
    g = np.random.default_rng(62).standard_normal(f0.shape)
    ft = torch.tensor(f0, requires_grad=True)
    ref = OL.run_pressure_walls(ft, None, torch.tensor(wall), torch.tensor(pressure), torch.tensor(rho_w), T, stencil,
                                True, xp=torch, mrt=OL.mrt_matrix(stencil, MRT_RATES))
    (gref,) = torch.autograd.grad(ref, ft, torch.tensor(g))
    ref, gref = ref.detach().numpy(), gref.numpy()
    dev = (lambda a: torch.tensor(a, device='cuda')) if target == 'gpu' else (lambda a: a)
    host = (lambda a: a.cpu().numpy()) if target == 'gpu' else (lambda a: a)
    step.set_pdfs(dev(f0))
    step.run(T, record=True)
    assert np.abs(host(step.pdf_array) - ref).max() <= 1e-12 * np.abs(f0).max()
    step.set_adjoint_pdfs(dev(g))
    step.run_backward(T)
    assert np.abs(host(step.adjoint_pdf_array) - gref).max() <= 1e-11 * np.abs(gref).max()


# --- Guo forcing with TRT / MRT (lbmpy's Guo model: prefactor 1 − ω/2 with the shear rate, velocity shift F/2) --------
GUO_METHOD_CASES = [('D2Q9', (9, 7), True, 'trt', 'const', 'lattice'), ('D2Q9', (8, 9), False, 'mrt', 'const', 'lattice'),
                    ('D2Q9', (7, 8), True, 'mrt', 'field', 'lattice'), ('D3Q19', (5, 4, 6), True, 'trt', 'field', 'lattice'),
                    ('D3Q19', (4, 5, 4), False, 'mrt', 'field', 'lattice'),
                    ('D2Q9', (6, 7), True, 'mrt', 'field', 'autodiffop'), ('D2Q9', (7, 6), False, 'trt', 'const', 'autodiffop')]


def _guo_method_case(stencil, shape, compressible, method, force_kind, schedule, target, T=3):
    import os
    import sympy as sp
    import torch
    D = len(shape)
    w = sp.Symbol('omega')
    if method == 'trt':
        kw = dict(method='trt', relaxation_rates=[w, 0.9])
        okw = dict(omega_odd=0.9)
    else:
        kw = dict(method='mrt', relaxation_rates=[w, MRT_RATES['bulk'], MRT_RATES['third'], MRT_RATES['fourth']])
        okw = dict(mrt=OL.mrt_matrix(stencil, dict(MRT_RATES, shear=1.4)))
    F = ps.fields(f"F({D}): float64[{D}D]", layout='fzyx') if force_kind == 'field' else (1e-3, -2e-3, 5e-4)[:D]
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, force_model='guo', force=F, **kw)
    old = os.environ.get('PSAD_LBM_LATTICE')
    os.environ['PSAD_LBM_LATTICE'] = '1' if schedule == 'lattice' else '0'
    try:
        step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.4, target=target)
    finally:
        if old is None:
            os.environ.pop('PSAD_LBM_LATTICE')
        else:
            os.environ['PSAD_LBM_LATTICE'] = old
    assert (step._lattice is not None) == (schedule == 'lattice')
    op = step.create_timestep_op(T)
    rng = np.random.default_rng(sum(shape) + 7)
    f0 = _init(stencil, shape, compressible, seed=71)
    dev = 'cuda' if target == 'gpu' else 'cpu'
    x = torch.tensor(f0, device=dev, requires_grad=True)
    ft = torch.tensor(f0, requires_grad=True)
    g = torch.tensor(rng.standard_normal(f0.shape))
    if force_kind == 'field':
        Fv = 1e-3 * rng.standard_normal(shape + (D,))
        Ft, Fr = torch.tensor(Fv, device=dev, requires_grad=True), torch.tensor(Fv, requires_grad=True)
        out = op.apply(x, Ft)
        ref = OL.run(ft, 1.4, T, stencil, compressible, xp=torch, force_model='guo',
                     force=tuple(Fr[..., a] for a in range(D)), **okw)
        out.backward(g.to(dev))
        gx, gF = torch.autograd.grad(ref, (ft, Fr), g)
        return out.detach().cpu(), ref.detach(), x.grad.cpu(), gx, Ft.grad.cpu(), gF
    out = op.apply(x)
    ref = OL.run(ft, 1.4, T, stencil, compressible, xp=torch, force_model='guo', force=F, **okw)
    out.backward(g.to(dev))
    (gx,) = torch.autograd.grad(ref, ft, g)
    return out.detach().cpu(), ref.detach(), x.grad.cpu(), gx, None, None


def _check_guo(res, tol):
    out, ref, gx, gxr, gF, gFr = res
    assert float((out - ref).abs().max()) <= tol * float(ref.abs().max())
    assert float((gx - gxr).abs().max()) <= 10 * tol * float(gxr.abs().max())
    if gF is not None:
        assert float((gF - gFr).abs().max()) <= 10 * tol * float(gFr.abs().max())


@pytest.mark.parametrize('stencil,shape,compressible,method,force_kind,schedule', GUO_METHOD_CASES)
def test_lbm_guo_trt_mrt_cpu(stencil, shape, compressible, method, force_kind, schedule):
    """Guo forcing with the TRT and MRT collisions (constant and per-cell forces) on the C kernels — the lattice kernels
    (the force term's adjoint sums over g beside the equilibrium's over h) and the rule's AutoDiffOp kernels — vs the
    oracle's collisions with Guo's term and torch's reverse mode (parity unpinned vs lbmpy)."""
    _check_guo(_guo_method_case(stencil, shape, compressible, method, force_kind, schedule, 'cpu'), 1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize('stencil,shape,compressible,method,force_kind,schedule',
                         [c for c in GUO_METHOD_CASES if c[-1] == 'lattice'])
def test_lbm_guo_trt_mrt_gpu(stencil, shape, compressible, method, force_kind, schedule):
    """The same on the HIP lattice kernels."""
    _check_guo(_guo_method_case(stencil, shape, compressible, method, force_kind, schedule, 'gpu'), 1e-12)
