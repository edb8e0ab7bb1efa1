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
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    u = torch.rand((zl, 1024, 1024), device='cuda')
    d = torch.rand_like(u) * 2 - 1
    plain = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    zop = ZSlabOp(op, use_cuda=True)
    zop._halo = RcclHalo(loopback=True)
    zfn = zop.autograd_function()
    for name, fn in (('plain op', plain), ('zslab + RCCL loopback', zfn), ('plain op', plain),
                     ('zslab + RCCL loopback', zfn)):
        wall, host = timed(fn, u, d)
        print(f'{name:24s} {zl}x1024^2: {wall:.4f} ms/step wall, {host:.4f} ms/step host enqueue, '
              f'implied N=8 1024^3 rate {1024**3 / (wall * 1e-3) / 1e6:,.0f} Mcells/s' if zl == 128 else
              f'{name:24s} {zl}x1024^2: {wall:.4f} ms/step wall, {host:.4f} ms/step host enqueue')
    torch.autograd.set_multithreading_enabled(False)
    wall, host = timed(zfn, u, d)
    print(f'zslab, autograd 1 thread  : {wall:.4f} ms/step wall, {host:.4f} ms/step host enqueue')
    zop.close()


if __name__ == '__main__':
    main()
