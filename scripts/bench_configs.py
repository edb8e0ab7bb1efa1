"""Measure every BASELINE.json config on one GPU through the drop-in op (fwd + TF-MAD bwd per step).

Prints one JSON line per config: Mcells/s, fwd/bwd ms (HIP events), algorithmic GB/s of each sweep and
its fraction of the 8 TB/s HBM peak. Bytes per cell per sweep: (fields read + fields written) x size.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def graph_step(fn, ins, grads, steps):
    """Seconds per step of the same apply + backward captured once in a HIP graph (torch.cuda.graph on
    static inputs / gradients) and replayed: what a stepped solver with fixed shapes pays once the
    host-side autograd / launch overhead is gone."""
    import torch
    static = [t.detach().clone().requires_grad_(True) for t in ins]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.autograd.backward(list(fn.apply(*static)), grads)
            for t in static:
                t.grad = None
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        # torch.autograd.grad: the gradients come back as new tensors (backward() would accumulate into .grad, one
        # more elementwise pass per replay that the eager loop, which resets .grad, does not run)
        keep = torch.autograd.grad(list(fn.apply(*static)), static, grads)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps * 10):
        graph.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (steps * 10)


def graph_sweeps(fn, ins, grads, K=20, reps=30):
    """Per-sweep GPU time of a small op without the host in it: K forward applies captured in one HIP graph, K
    backward passes of ONE eager forward (``autograd.grad(..., retain_graph=True)``) in a second, each replayed
    ``reps`` times between two HIP events on the stream: forward = the first graph / K, adjoint = the second / K —
    each sweep timed on its own, both writing K fresh output blocks per replay. (Until round 6 the adjoint was
    (K apply + backward steps − K applies) / K: that charged the adjoint with what the forward loses when the
    adjoint's writes share the Infinity Cache with it — config 2's "adjoint 7–12 % slower than the forward".)
    For configs whose kernels take tens of µs, events around each eager apply / backward time the host's launch
    latency as much as the kernel (BASELINE config 2 measured 0.024–0.037 ms per sweep from run to run that way,
    VERDICT r04 item 5). Returns (fwd, adjoint, adjoint by the old subtraction)."""
    import torch
    static = [t.detach().clone().requires_grad_(True) for t in ins]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            torch.autograd.backward(list(fn.apply(*static)), grads)
            for t in static:
                t.grad = None
    torch.cuda.current_stream().wait_stream(s)
    gf, gs, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
        keep = [fn.apply(*static) for _ in range(K)]
    with torch.cuda.graph(gs):
        keep2 = [torch.autograd.grad(list(fn.apply(*static)), static, grads) for _ in range(K)]
    with torch.cuda.stream(s):
        outs0 = list(fn.apply(*static))             # one eager forward: its autograd graph is replayed K times below
        torch.autograd.grad(outs0, static, grads, retain_graph=True)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(gb):
        keep3 = [torch.autograd.grad(outs0, static, grads, retain_graph=True) for _ in range(K)]
    out = []
    for g in (gf, gs, gb):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / (reps * K))
    del keep, keep2, keep3, outs0
    return out[0], out[2], out[1] - out[0]


SETTLE_MS = 400.0


def settle(step, ms=SETTLE_MS):
    """Run ``step`` as a continuous load until ``ms`` have passed: a sustained HBM-bound load first drives
    the chip into a power-management transient (27-point 768³ dispatches rise from ~368 to ~510 us and settle
    at ~375 us; kernel trace in profiles/r02_power_transient_27pt.txt; 0.08 s of settling still left the
    27-point op at 0.409 ms, 0.5 s gave 0.377 ms = the kernel, profiles/r02_op_vs_kernel27_settled.log) — timed
    steps start after it."""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):          # a continuous load (no host sync between steps)
            step()
        torch.cuda.synchronize()


def run(name, builder, shape, dtype, bh, nin, steps=20, warmup=3, bytes_fwd=None, bytes_bwd=None):
    import torch

    import pystencils_autodiff_amd as pa
    op = pa.AutoDiffOp(builder(), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    g = torch.Generator(device='cuda').manual_seed(0)
    ins = [(torch.rand(shape, generator=g, device='cuda') + (0.5 if name.startswith('readme') else 0.0)).to(dtype)
           .requires_grad_(True) for _ in range(nin)]
    outs = fn.apply(*ins)
    grads = [(torch.rand(o.shape, generator=g, device='cuda') * 2 - 1).to(dtype) for o in outs]
    ev = []

    def one():
        o_ = fn.apply(*ins)
        torch.autograd.backward(list(o_), grads)
        for t in ins:
            t.grad = None
    settle(one)
    for i in range(warmup + steps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        outs = fn.apply(*ins)
        e1.record()
        torch.autograd.backward(list(outs), grads)
        e2.record()
        for t in ins:
            t.grad = None
        if i >= warmup:
            ev.append((e0, e1, e2))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        outs = fn.apply(*ins)
        torch.autograd.backward(list(outs), grads)
        for t in ins:
            t.grad = None
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # the same loop with torch's autograd device thread off (torch.autograd.set_multithreading_enabled):
    # the backward runs in the calling thread, which removes the engine's thread hand-off (~60-75 µs
    # per step measured, scripts/op_overhead_2d.py) from launch-bound configs
    torch.autograd.set_multithreading_enabled(False)
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            outs = fn.apply(*ins)
            torch.autograd.backward(list(outs), grads)
            for t in ins:
                t.grad = None
        torch.cuda.synchronize()
        el_st = time.perf_counter() - t0
    finally:
        torch.autograd.set_multithreading_enabled(True)
    cells = 1
    for s in shape[:3]:
        cells *= s
    el_graph = graph_step(fn, ins, grads, steps) if cells <= 1 << 26 else None
    f_ev = sorted(a.elapsed_time(b) for a, b, _ in ev)[len(ev) // 2]
    b_ev = sorted(b.elapsed_time(c) for _, b, c in ev)[len(ev) // 2]
    # small configs: the per-sweep GPU time from graph replays (events around eager calls time the host too)
    small = cells <= 1 << 26
    f_ms, b_ms, b_sub = graph_sweeps(fn, ins, grads) if small else (f_ev, b_ev, None)
    res = {'config': name, 'shape': list(shape), 'dtype': str(dtype).replace('torch.', ''),
           'mcells_per_s': round(cells * steps / el / 1e6, 1), 'ms_per_step': round(el / steps * 1e3, 4),
           'mcells_per_s_autograd_1thread': round(cells * steps / el_st / 1e6, 1),
           'ms_per_step_autograd_1thread': round(el_st / steps * 1e3, 4),
           **({'mcells_per_s_hip_graph': round(cells / el_graph / 1e6, 1),
               'ms_per_step_hip_graph': round(el_graph * 1e3, 4)} if el_graph else {}),
           'fwd_ms': round(f_ms, 4), 'bwd_ms': round(b_ms, 4),
           'sweep_timing': 'hip_graph_replay' if small else 'hip_events_per_call',
           **({'fwd_ms_events': round(f_ev, 4), 'bwd_ms_events': round(b_ev, 4),
               'bwd_ms_step_minus_fwd': round(b_sub, 4)} if small else {}),
           'fwd_schedule': op.forward_ast_gpu.compile().last_variant[0],
           'bwd_schedule': op.backward_ast_gpu.compile().last_variant[0]}
    if bytes_fwd:
        res['fwd_GBps'] = round(bytes_fwd * cells / (f_ms * 1e-3) / 1e9, 1)
        res['bwd_GBps'] = round(bytes_bwd * cells / (b_ms * 1e-3) / 1e9, 1)
        res['fwd_frac'] = round(res['fwd_GBps'] / PEAK, 4)
        res['bwd_frac'] = round(res['bwd_GBps'] / PEAK, 4)
    print(json.dumps(res))
    sys.stdout.flush()
    del ins, outs, grads
    torch.cuda.empty_cache()


def run_slab(name, builder, shape, dtype, full_cells, steps=20, warmup=3):
    """One rank's share of a z-slab decomposed step WITHOUT the exchange: interior planes, then both
    faces in one two-range launch reading halo planes, for the forward and the adjoint kernel — the
    per-rank compute time of the N-GPU run (zslab.py launch pattern)."""
    import torch

    import pystencils_autodiff_amd as pa
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    ks = [op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()]
    g = torch.Generator(device='cuda').manual_seed(0)
    args = []
    for k in ks:
        kw = {f.name: (torch.rand(shape, generator=g, device='cuda') * 2 - 1).to(dtype) for f in k.ir.fields}
        halos = {f.name: (kw[f.name][:1].clone(), kw[f.name][-1:].clone()) for f in k.ir.stencil_fields}
        args.append((k, kw, halos))
    Z = shape[0]

    def step():
        for k, kw, halos in args:
            k(z_range=(1, Z - 1), **kw)
            k(halos=halos, z_range=((0, 1), (Z - 1, Z)), **kw)
    for _ in range(warmup):
        step()
    settle(step)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    res = {'config': name, 'shape': list(shape), 'dtype': str(dtype).replace('torch.', ''),
           'ms_per_step_rank_compute': round(ms, 4),
           'implied_full_domain_mcells_per_s_no_exchange': round(full_cells / (ms * 1e-3) / 1e6, 1),
           'schedule': ks[0].last_variant[0] + ('/ws' if getattr(ks[0].last_variant[1], 'WS', False) else '')}
    print(json.dumps(res))
    sys.stdout.flush()


def run_lbm(name, stencil, shape, dtype, T=10, reps=5, compressible=False, walls=False, force_model=None,
            force_field=False, method='srt'):
    """Lattice Boltzmann time-step op (lbm.AutoDiffLatticeBoltzmannStep.create_timestep_op): T forward steps
    and the T adjoint steps, HIP events around Op.apply and backward (back-to-back applies). MLUPS = cells · T / time; algorithmic
    bytes per cell and step: forward 2q·s (read src, write dst), adjoint 3q·s (read diffdst and the recorded
    src, write diffsrc), s = element size; the ghost sync, state records and adjoint border fills are extra.
    ``force_field``: a per-cell force (a D-component fzyx field, an input of the op): + D·s per cell and step forward
    (the force read), + 3·D·s adjoint (the force read, its accumulated adjoint read and written)."""
    import sympy as sp
    import torch

    from pystencils_autodiff_amd import lbm
    from pystencils_autodiff_amd import ps
    D = len(shape)
    dts = str(dtype).replace('torch.', '')
    force = (1e-5, -2e-5, 5e-6)[:D] if force_model else None
    if force_model and force_field:
        force = ps.fields(f"F({D}): {dts}[{D}D]", layout='fzyx')
    mk = dict(method='mrt', relaxation_rates=[sp.Symbol('omega'), 1.1, 0.9, 1.2]) if method == 'mrt' else {}
    rule = lbm.create_lb_update_rule(stencil, compressible=compressible, data_type=dts, force_model=force_model,
                                     force=force, **mk)
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.5, target='gpu')
    if walls:
        # a channel: no-slip walls on the first and last rows of axis 1
        step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, 0])
        step.set_boundary_including_adjoint(lbm.NoSlip(), lbm.make_slice[:, -1])
    if walls == 'pressure':
        # ... driven by FixedDensity inlet / outlet planes at the ends of axis 0 (link programs)
        step.set_boundary_including_adjoint(lbm.FixedDensity(1.01, name='inlet'), lbm.make_slice[0, 1:-1])
        step.set_boundary_including_adjoint(lbm.FixedDensity(0.99, name='outlet'), lbm.make_slice[-1, 1:-1])
    Op = step.create_timestep_op(T)
    q = rule.stencil.Q
    g = torch.Generator(device='cuda').manual_seed(0)
    f0 = (torch.full(tuple(shape) + (q,), 1.0 / q, device='cuda', dtype=torch.float64) *
          (1 + 0.01 * torch.rand(tuple(shape) + (q,), generator=g, device='cuda', dtype=torch.float64))).to(dtype)
    # inputs in the step's fzyx layout (one plane per component): no layout copies inside the op
    x = step.empty_pdfs()
    x.copy_(f0)
    x.requires_grad_(True)
    gr = step.empty_pdfs()
    gr.copy_(torch.rand(tuple(shape) + (q,), generator=g, device='cuda', dtype=dtype))
    fw, bw = [], []
    extra = ()
    if force_field:
        Fv = torch.empty([D] + list(shape), device='cuda', dtype=dtype).permute(*range(1, D + 1), 0)
        Fv.copy_(1e-5 * (torch.rand(tuple(shape) + (D,), generator=g, device='cuda', dtype=dtype) - 0.5))
        extra = (Fv.requires_grad_(True),)

    def one():
        Op.apply(x, *extra).backward(gr)
        x.grad = None
    settle(one)
    # back-to-back applies as run() times the stencil configs (the queue stays ahead of the GPU: event times are
    # the op's GPU time, not the host latency to its first launch after an idle GPU)
    ev = []
    for i in range(reps + 2):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        out = Op.apply(x, *extra)
        e1.record()
        out.backward(gr)
        e2.record()
        x.grad = None
        if i >= 2:
            ev.append((e0, e1, e2))
    torch.cuda.synchronize()
    for e0, e1, e2 in ev:
        fw.append(e0.elapsed_time(e1))
        bw.append(e1.elapsed_time(e2))
    cells = 1
    for n in shape:
        cells *= n
    es = torch.tensor([], dtype=dtype).element_size()
    f_ms, b_ms = sorted(fw)[len(fw) // 2], sorted(bw)[len(bw) // 2]
    res = {'config': name, 'shape': list(shape), 'dtype': str(dtype).replace('torch.', ''), 'time_steps': T,
           'schedule': 'lattice' if step._lattice is not None else 'autodiffop',
           'walls': walls if isinstance(walls, str) else bool(walls),
           'fwd_mlups': round(cells * T / (f_ms * 1e-3) / 1e6, 1), 'bwd_mlups': round(cells * T / (b_ms * 1e-3) / 1e6, 1),
           'fwd_ms': round(f_ms, 4), 'bwd_ms': round(b_ms, 4),
           'fwd_GBps': round((2 * q + (D if force_field else 0)) * es * cells * T / (f_ms * 1e-3) / 1e9, 1),
           'bwd_GBps': round((3 * q + (3 * D if force_field else 0)) * es * cells * T / (b_ms * 1e-3) / 1e9, 1),
           'force': (f'{force_model}, per-cell field' if force_field else force_model) if force_model else None,
           'method': method}
    res['fwd_frac'] = round(res['fwd_GBps'] / PEAK, 4)
    res['bwd_frac'] = round(res['bwd_GBps'] / PEAK, 4)
    print(json.dumps(res))
    sys.stdout.flush()
    del x, out, gr, f0, Op
    torch.cuda.empty_cache()


def run_cpu(name, builder, shape, bh, nin, steps=2000):
    """BASELINE config 1 as stated: the op on the CPU backend (use_cuda=False, the C kernels), host
    wall time per forward + backward."""
    import torch

    import pystencils_autodiff_amd as pa
    op = pa.AutoDiffOp(builder(), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=False, backend='torch_native')
    g = torch.Generator().manual_seed(0)
    ins = [(torch.rand(shape, generator=g) + 0.5).requires_grad_(True) for _ in range(nin)]
    outs = fn.apply(*ins)
    grads = [torch.rand(o.shape, generator=g) * 2 - 1 for o in outs]
    for _ in range(50):
        torch.autograd.backward(list(fn.apply(*ins)), grads)
    t0 = time.perf_counter()
    for _ in range(steps):
        torch.autograd.backward(list(fn.apply(*ins)), grads)
    el = (time.perf_counter() - t0) / steps
    cells = 1
    for s in shape:
        cells *= s
    print(json.dumps({'config': name, 'shape': list(shape), 'backend': 'cpu (C kernels, use_cuda=False)',
                      'us_per_step': round(el * 1e6, 2), 'mcells_per_s': round(cells / el / 1e6, 2)}))
    sys.stdout.flush()


def main():
    import torch

    from pystencils_autodiff_amd import workloads as W
    only = [a for a in sys.argv[1:] if not a.startswith('--repeat=')]
    repeat = int(next((a.split('=')[1] for a in sys.argv[1:] if a.startswith('--repeat=')), 1))
    cfgs = [
        ('readme_op_f32_20x30', W.readme_op, (20, 30), torch.float32, None, 2, 12, 20),
        ('readme_op_f32_16384^2', lambda: W.readme_op(shape=None), (16384, 16384), torch.float32, None, 2, 12, 20),
        ('laplace5_f32_4096^2', lambda: W.laplace_5pt(), (4096, 4096), torch.float32, 'zeros', 1, 8, 8),
        ('diffusion7_f32_512^3', lambda: W.diffusion_7pt(), (512, 512, 512), torch.float32, 'zeros', 1, 8, 8),
        ('diffusion7_f32_1024^3', lambda: W.diffusion_7pt(), (1024, 1024, 1024), torch.float32, 'zeros', 1, 8, 8),
        ('stencil27_f16_768^3', lambda: W.stencil_27pt(), (768, 768, 768), torch.float16, 'zeros', 1, 4, 4),
        # not a BASELINE config: the non-power-of-two extent of config 5 on the config-4 sweep
        ('diffusion7_f32_768^3', lambda: W.diffusion_7pt(), (768, 768, 768), torch.float32, 'zeros', 1, 8, 8),
        ('diffusion7_f16_768^3', lambda: W.diffusion_7pt(dtype='float16'), (768, 768, 768), torch.float16, 'zeros', 1,
         4, 4),
        ('diffusion7_f64_512^3', lambda: W.diffusion_7pt(dtype='float64'), (512, 512, 512), torch.float64,
         'zeros', 1, 16, 16),
        # variable-coefficient diffusion (two inputs; the adjoint reads three fields and writes two)
        ('varcoef7_f32_768^3', lambda: W.varcoef_diffusion_7pt(), (768, 768, 768), torch.float32, 'zeros', 2, 12, 20),
        ('varcoef7_f32_512^3', lambda: W.varcoef_diffusion_7pt(), (512, 512, 512), torch.float32, 'zeros', 2, 12, 20),
        ('varcoef7_f16_768^3', lambda: W.varcoef_diffusion_7pt(dtype='float16'), (768, 768, 768), torch.float16, 'zeros',
         2, 6, 10),
        ('veclaplace7_f32_384^3x3', lambda: W.vector_laplace_7pt(), (384, 384, 384, 3), torch.float32, 'zeros', 1,
         24, 24),
    ]
    # row pitch: extents that are not a multiple of 16 bytes next to their power-of-two neighbours (VERDICT r03 item
    # 5: within 15 %)
    for n in (510, 512):
        cfgs.append((f'pitch_diffusion7_f16_{n}^3', lambda: W.diffusion_7pt(dtype='float16'), (n, n, n), torch.float16,
                     'zeros', 1, 4, 4))
    for n in (255, 256, 511, 512):
        cfgs.append((f'pitch_stencil27_f16_{n}^3', lambda: W.stencil_27pt(), (n, n, n), torch.float16, 'zeros', 1, 4, 4))
    if not only or 'readme_op_f32_20x30_cpu' in only:
        run_cpu('readme_op_f32_20x30_cpu', W.readme_op, (20, 30), None, 2)
    for name, b, shape, dt, bh, nin, bf, bb in cfgs:
        if only and name not in only:
            continue
        for _ in range(repeat):
            run(name, b, shape, dt, bh, nin, bytes_fwd=bf, bytes_bwd=bb)
    slabs = [('slab8_diffusion7_f32_128x1024^2', lambda: W.diffusion_7pt(), (128, 1024, 1024), torch.float32, 1024 ** 3),
             ('slab4_diffusion7_f32_256x1024^2', lambda: W.diffusion_7pt(), (256, 1024, 1024), torch.float32, 1024 ** 3),
             ('slab8_stencil27_f16_96x768^2', lambda: W.stencil_27pt(), (96, 768, 768), torch.float16, 768 ** 3)]
    for name, b, shape, dt, cells in slabs:
        if only and name not in only:
            continue
        run_slab(name, b, shape, dt, cells)
    lbms = [('lbm_d2q9_f32_2048^2', 'D2Q9', (2048, 2048), torch.float32, False),
            ('lbm_d3q19_f32_192^3', 'D3Q19', (192, 192, 192), torch.float32, False),
            ('lbm_d2q9_f32_2048^2_channel', 'D2Q9', (2048, 2048), torch.float32, True),
            ('lbm_d3q19_f32_192^3_channel', 'D3Q19', (192, 192, 192), torch.float32, True),
            ('lbm_d2q9_f32_2048^2_pressure', 'D2Q9', (2048, 2048), torch.float32, 'pressure'),
            ('lbm_d3q19_f32_192^3_pressure', 'D3Q19', (192, 192, 192), torch.float32, 'pressure'),
            ('lbm_d2q9_f32_2048^2_mrt', 'D2Q9', (2048, 2048), torch.float32, False, 'mrt'),
            ('lbm_d3q19_f32_192^3_mrt', 'D3Q19', (192, 192, 192), torch.float32, False, 'mrt')]
    for name, stencil, shape, dt, walls, *method in lbms:
        if only and name not in only:
            continue
        run_lbm(name, stencil, shape, dt, walls=walls, method=method[0] if method else 'srt')


if __name__ == '__main__':
    main()
