"""Why the per-sweep time measured around ``Op.apply`` (scripts/bench_configs.py) exceeded the kernel's own
time: the same 27-point fp16 768³ forward timed (a) with events around each apply inside the fwd+bwd
loop (bench_configs), (b) with events around 10 back-to-back applies (no backward), (c) with events
around 10 back-to-back direct kernel calls, (d) as (a) but with the outputs of the previous step kept
alive until the next apply.

Finding (profiles/r02_power_transient_27pt.txt): whichever loop runs FIRST after the fields are created
looks ~15 % slower — a sustained HBM-bound load drives the chip into a power-management transient
(dispatches rise from ~368 to ~510 us, then settle at ~385 us within ~40 dispatches). With ``SETTLE=1``
(default) every variant runs after 80 ms of warm-up load and (a)-(d) agree."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    wl = sys.argv[2] if len(sys.argv) > 2 else 'stencil27'
    builder, dt = {'stencil27': (W.stencil_27pt, torch.float16), 'diffusion7': (W.diffusion_7pt, torch.float32)}[wl]
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    k = op.forward_ast_gpu.compile()
    u = torch.rand((n, n, n), device='cuda').to(dt).requires_grad_(True)
    d = (torch.rand((n, n, n), device='cuda') * 2 - 1).to(dt)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    if os.environ.get('SETTLE', '1') == '1':
        import time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < float(os.environ.get('SETTLE_S', '0.08')):
            for _ in range(8):
                (o,) = fn.apply(u)
                o.backward(d)
                u.grad = None
            torch.cuda.synchronize()

    def loop_a(keep):
        held = None
        ts = []
        for i in range(23):
            e0, e1, e2 = ev(), ev(), ev()
            e0.record()
            (o,) = fn.apply(u)
            e1.record()
            o.backward(d)
            e2.record()
            u.grad = None
            if keep:
                held = o
            if i >= 3:
                ts.append((e0, e1, e2))
        torch.cuda.synchronize()
        del held
        f = sorted(a.elapsed_time(b) for a, b, _ in ts)
        b = sorted(b_.elapsed_time(c) for _, b_, c in ts)
        return f[len(f) // 2], b[len(b) // 2]

    fa = loop_a(False)
    print(f'(a) events around apply / backward in the fwd+bwd loop: fwd {fa[0]:.4f} ms  bwd {fa[1]:.4f} ms', flush=True)
    fd = loop_a(True)
    print(f'(d) same, previous output kept alive:                  fwd {fd[0]:.4f} ms  bwd {fd[1]:.4f} ms', flush=True)
    with torch.no_grad():
        for _ in range(3):
            fn.apply(u)
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(10):
            fn.apply(u)
        e1.record()
        torch.cuda.synchronize()
    print(f'(b) 10 back-to-back applies (no_grad):                  fwd {e0.elapsed_time(e1) / 10:.4f} ms', flush=True)
    out = torch.empty_like(u)
    uu = u.detach()
    for _ in range(3):
        k(u=uu, out=out)
    e0, e1 = ev(), ev()
    e0.record()
    for _ in range(10):
        k(u=uu, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(f'(c) 10 back-to-back kernel calls:                      fwd {e0.elapsed_time(e1) / 10:.4f} ms', flush=True)


if __name__ == '__main__' and (len(sys.argv) < 2 or sys.argv[1] not in ('patterns', 'alloc')):
    main()


def patterns():
    """Direct fwd / bwd kernel calls: each kernel writing the block the previous kernel wrote (ping-pong),
    a 3-block rotation, and fixed output blocks; per-kernel HIP-event times."""
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    tun = {}
    for kv in (sys.argv[3].split(',') if len(sys.argv) > 3 and sys.argv[3] else []):
        k_, v_ = kv.split('=')
        tun[k_] = int(v_)
    kf = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='pf', target='gpu',
                       gpu_indexing_params=tun).compile()
    kb = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='pb', target='gpu',
                       gpu_indexing_params=tun).compile()
    print('tuning', tun, flush=True)
    u = torch.rand((n, n, n), device='cuda').half()
    d = torch.rand((n, n, n), device='cuda').half()
    blocks = [torch.empty_like(u) for _ in range(3)]
    seqs = {'ping-pong (A,B,B,A,...)': lambda i: (blocks[i % 2], blocks[(i + 1) % 2]),
            'rotation of 3': lambda i: (blocks[(2 * i) % 3], blocks[(2 * i + 1) % 3]),
            'fixed (A,B)': lambda i: (blocks[0], blocks[1])}
    for name, pick in seqs.items():
        ts = []
        for i in range(24):
            o, g = pick(i)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            kf(u=u, out=o)
            e[1].record()
            kb(diffout=d, diffu=g)
            e[2].record()
            if i >= 4:
                ts.append(e)
        torch.cuda.synchronize()
        f = sorted(a.elapsed_time(b) for a, b, _ in ts)
        b = sorted(b_.elapsed_time(c) for _, b_, c in ts)
        print(f'{name:26s} fwd {f[len(f) // 2]:.4f} ms  bwd {b[len(b) // 2]:.4f} ms', flush=True)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'patterns':
    patterns()


def alloc_patterns():
    """The allocation pattern of the fwd+bwd loop reproduced with direct kernel calls and torch's caching
    allocator: outputs allocated per step, the adjoint freed right after its launch (as ``u.grad = None``),
    the previous forward output freed after the next one is allocated (as rebinding ``o``)."""
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    kf, kb = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    u = torch.rand((n, n, n), device='cuda').half()
    d = torch.rand((n, n, n), device='cuda').half()
    import contextlib
    pools = (torch.cuda.MemPool(), torch.cuda.MemPool())
    for name in ('loop-like (free adjoint at once)', 'adjoint freed one step later', 'fresh blocks each step',
                 'loop-like, fwd / bwd outputs from two MemPools'):
        ts = []
        o = None
        keep = []
        two = name.endswith('MemPools')
        for i in range(24):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            with (torch.cuda.use_mem_pool(pools[0]) if two else contextlib.nullcontext()):
                o_new = torch.empty_like(u)
            kf(u=u, out=o_new)
            o = o_new
            e[1].record()
            with (torch.cuda.use_mem_pool(pools[1]) if two else contextlib.nullcontext()):
                g = torch.empty_like(u)
            kb(diffout=d, diffu=g)
            e[2].record()
            if name.startswith('adjoint freed'):
                keep = [g]
            elif name.startswith('fresh'):
                keep.append(g)
                keep.append(o)
                if len(keep) > 8:
                    keep = keep[-8:]
            del g
            if i >= 4:
                ts.append(e)
        torch.cuda.synchronize()
        f = sorted(a.elapsed_time(b) for a, b, _ in ts)
        b = sorted(b_.elapsed_time(c) for _, b_, c in ts)
        print(f'{name:34s} fwd {f[len(f) // 2]:.4f} ms  bwd {b[len(b) // 2]:.4f} ms', flush=True)
        del keep, o


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'alloc':
    alloc_patterns()
