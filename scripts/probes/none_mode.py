"""boundary_handling=None (the reference default) through the op: fwd+bwd per step with outputs
allocated as torch.empty + one border-zeroing kernel vs one torch.zeros memset (BORDER_KERNEL)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends import _torch_native as TN  # noqa: E402


def step_ms(fn, u, d, steps=20):
    uu = u.clone().requires_grad_(True)
    for _ in range(3):
        (o,) = fn.apply(uu)
        o.backward(d)
        uu.grad = None
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        (o,) = fn.apply(uu)
        o.backward(d)
        uu.grad = None
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


for n in (512, 1024):
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling=None)
    u = torch.rand((n, n, n), device='cuda')
    d = torch.rand_like(u)
    res = {}
    for name, bk in (('border kernel', True), ('memset', False), ('border kernel', True), ('memset', False)):
        TN.BORDER_KERNEL = bk
        fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
        res.setdefault(name, []).append(step_ms(fn, u, d))
    zop = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros').create_tensorflow_op(use_cuda=True,
                                                                                          backend='torch_native')
    res['zeros mode (reference)'] = [step_ms(zop, u, d)]
    print(n, {k: [round(x, 4) for x in v] for k, v in res.items()}, 'ms per fwd+bwd step')

# kernel-level: the interior-only forward kernel vs the zeros-mode one, and the border fills alone
n = 1024
u = torch.rand((n, n, n), device='cuda')
out = torch.empty_like(u)
for bh in (None, 'zeros'):
    k = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling=bh).forward_ast_gpu.compile()
    k(u=u, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        k(u=u, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(f'forward kernel boundary={bh}: {e0.elapsed_time(e1) / 10:.4f} ms  variant={k.last_variant[0]} '
          f'WS={getattr(k.last_variant[1], "WS", None)}')
alloc = TN._allocator(pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling=None).forward_ast_gpu, 'out')
TN.BORDER_KERNEL = True
alloc((n, n, n), torch.float32, u.device)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    alloc((n, n, n), torch.float32, u.device)
e1.record()
torch.cuda.synchronize()
print(f'empty + border kernel: {e0.elapsed_time(e1) / 10:.4f} ms')
for d in range(3):
    e0.record()
    for _ in range(10):
        out.narrow(d, 0, 1).zero_()
        out.narrow(d, n - 1, 1).zero_()
    e1.record()
    torch.cuda.synchronize()
    print(f'  axis {d} faces: {e0.elapsed_time(e1) / 10:.4f} ms')
