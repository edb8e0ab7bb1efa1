"""Per-rank step of the N=8 bench on one GPU: the 128x1024^2 slab through ZSlabOp.autograd_function()
apply+backward with a loopback RCCL communicator (both faces exchanged with itself), vs the plain
N=1 op on the same slab. Wall time per step and per-sweep event times."""
import sys
import time

import torch

sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp  # noqa: E402


def timed(fn, u, d, steps=50):
    uu = u.clone().requires_grad_(True)

    def step():
        (o,) = fn.apply(uu)
        o.backward(d)
        uu.grad = None
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    host = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, host


def main():
    zl = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    wl = sys.argv[2] if len(sys.argv) > 2 else 'diffusion7'
    n = 768 if wl == 'stencil27' else 1024
    op = pa.AutoDiffOp(W.stencil_27pt() if wl == 'stencil27' else W.diffusion_7pt(), boundary_handling='zeros')
    dt = torch.float16 if wl == 'stencil27' else torch.float32
    u = torch.rand((zl, n, n), device='cuda').to(dt)
    d = (torch.rand_like(u, dtype=torch.float32) * 2 - 1).to(dt)
    plain = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    zop = ZSlabOp(op, use_cuda=True)
    zop._halo = RcclHalo(loopback=True)
    zfn = zop.autograd_function()
    for name, fn in (('plain op', plain), ('zslab + RCCL loopback', zfn), ('plain op', plain),
                     ('zslab + RCCL loopback', zfn)):
        wall, host = timed(fn, u, d)
        print(f'{name:24s} {wl} {zl}x{n}^2: {wall:.4f} ms/step wall, {host:.4f} ms/step host enqueue, '
              f'implied N={n // zl} {n}^3 rate {n**3 / (wall * 1e-3) / 1e6:,.0f} Mcells/s')
    torch.autograd.set_multithreading_enabled(False)
    import os
    for native, faces in (('1', 'compute'), ('0', 'compute'), ('1', 'halo'), ('1', 'compute'), ('1', 'halo')):
        # the slab Function through the native node (csrc/psad_torch.cpp "z-slab sweeps") or the Python sweeps;
        # the native node's face launches on the compute stream after the interior, or on the halo stream
        os.environ['PSAD_NATIVE_SLAB'] = native
        os.environ['PSAD_SLAB_FACES'] = faces
        zop2 = ZSlabOp(op, use_cuda=True)          # a fresh plan per setting (the face placement is fixed at plan time)
        zop2._halo = zop._halo
        zfn = zop2.autograd_function()
        wall, host = timed(zfn, u, d)
        print(f'zslab {"native" if native == "1" else "python"} faces on {faces}, autograd 1 thread: {wall:.4f} ms/step wall, '
              f'{host:.4f} ms/step host enqueue, implied N={n // zl} {n}^3 rate '
              f'{n**3 / (wall * 1e-3) / 1e6:,.0f} Mcells/s', flush=True)
    zop.close()


def profile_host(zl=96, wl='stencil27', steps=300):
    """cProfile of the zslab step's host side (autograd in the calling thread so all of it is visible)."""
    import cProfile
    import pstats
    n = 768 if wl == 'stencil27' else 1024
    op = pa.AutoDiffOp(W.stencil_27pt() if wl == 'stencil27' else W.diffusion_7pt(), boundary_handling='zeros')
    dt = torch.float16 if wl == 'stencil27' else torch.float32
    u = torch.rand((zl, n, n), device='cuda').to(dt).requires_grad_(True)
    d = (torch.rand((zl, n, n), device='cuda') * 2 - 1).to(dt)
    zop = ZSlabOp(op, use_cuda=True)
    zop._halo = RcclHalo(loopback=True)
    fn = zop.autograd_function()
    torch.autograd.set_multithreading_enabled(False)
    for _ in range(10):
        (o,) = fn.apply(u)
        o.backward(d)
        u.grad = None
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        (o,) = fn.apply(u)
        o.backward(d)
        u.grad = None
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr, stream=sys.stdout).sort_stats('tottime').print_stats(22)
    zop.close()


def time_sweeps(zl=96, wl='stencil27', steps=300):
    """Host time inside ZSlabOp._sweep per forward / backward sweep, autograd multi- vs single-threaded."""
    import collections
    n = 768 if wl == 'stencil27' else 1024
    op = pa.AutoDiffOp(W.stencil_27pt() if wl == 'stencil27' else W.diffusion_7pt(), boundary_handling='zeros')
    dt = torch.float16 if wl == 'stencil27' else torch.float32
    u = torch.rand((zl, n, n), device='cuda').to(dt).requires_grad_(True)
    d = (torch.rand((zl, n, n), device='cuda') * 2 - 1).to(dt)
    zop = ZSlabOp(op, use_cuda=True)
    zop._halo = RcclHalo(loopback=True)
    fn = zop.autograd_function()
    acc = collections.defaultdict(float)
    orig = zop._sweep

    def timed(which, kwargs):
        t = time.perf_counter()
        orig(which, kwargs)
        acc[which] += time.perf_counter() - t
    zop._sweep = timed
    ex = zop._halo.exchange

    def timed_ex(*a):
        t = time.perf_counter()
        ex(*a)
        acc['exchange'] += time.perf_counter() - t
    zop._halo.exchange = timed_ex
    for mt in (True, False):
        torch.autograd.set_multithreading_enabled(mt)
        for _ in range(10):
            (o,) = fn.apply(u)
            o.backward(d)
            u.grad = None
        torch.cuda.synchronize()
        acc.clear()
        t0 = time.perf_counter()
        ta = tb = 0.0
        for _ in range(steps):
            t1 = time.perf_counter()
            (o,) = fn.apply(u)
            t2 = time.perf_counter()
            o.backward(d)
            t3 = time.perf_counter()
            ta += t2 - t1
            tb += t3 - t2
            u.grad = None
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e6
        print(f'multithreaded={mt}: wall {wall:.1f} us/step; apply {ta / steps * 1e6:.1f} us, backward() '
              f'{tb / steps * 1e6:.1f} us; inside _sweep: fwd {acc["forward"] / steps * 1e6:.1f} us, '
              f'bwd {acc["backward"] / steps * 1e6:.1f} us; exchange calls {acc["exchange"] / steps * 1e6:.1f} us')
    torch.autograd.set_multithreading_enabled(True)
    zop.close()


def trace(zl=128, wl='diffusion7', steps=20):
    """A short run for ``rocprofv3 --kernel-trace``: the plain op, then the native slab step (faces on the compute
    stream), ``steps`` fwd+bwd each after warm-up (``scripts/trace_timeline.py`` shows the last ones)."""
    n = 768 if wl == 'stencil27' else 1024
    op = pa.AutoDiffOp(W.stencil_27pt() if wl == 'stencil27' else W.diffusion_7pt(), boundary_handling='zeros')
    dt = torch.float16 if wl == 'stencil27' else torch.float32
    u = torch.rand((zl, n, n), device='cuda').to(dt)
    d = (torch.rand_like(u, dtype=torch.float32) * 2 - 1).to(dt)
    plain = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    zop = ZSlabOp(op, use_cuda=True)
    zop._halo = RcclHalo(loopback=True)
    zfn = zop.autograd_function()
    torch.autograd.set_multithreading_enabled(False)
    for name, fn in (('plain op', plain), ('zslab', zfn)):
        wall, host = timed(fn, u, d, steps)
        print(f'{name:10s} {wl} {zl}x{n}^2: {wall:.4f} ms/step wall, {host:.4f} ms/step host', flush=True)
        time.sleep(0.01)
    zop.close()


if __name__ == '__main__':
    if len(sys.argv) > 3 and sys.argv[3] == 'trace':
        trace(int(sys.argv[1]), sys.argv[2])
    elif len(sys.argv) > 3 and sys.argv[3] == 'profile':
        profile_host(int(sys.argv[1]), sys.argv[2])
    elif len(sys.argv) > 3 and sys.argv[3] == 'sweeps':
        time_sweeps(int(sys.argv[1]), sys.argv[2])
    else:
        main()
