"""The 1024^3 fp32 7-point op with bench.py's allocation sequence (variant 'bench': u from torch.rand, diffout from
rand * 2 - 1, two scratch blocks reserved) against diffout made in place (variant 'inplace': empty + uniform_(-1, 1),
no temporaries) and diffout allocated before u ('d_first'). One variant per process (the caching allocator's
history is the variable). Prints fwd / bwd ms (HIP events, median of 20 steps) and the block addresses.
python scripts/probes/bench_alloc.py bench|inplace|d_first"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else 'bench'
    n = 1024
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    g = torch.Generator(device='cuda').manual_seed(0)
    g1 = torch.Generator(device='cuda').manual_seed(1000)
    if variant == 'd_first':
        d = torch.rand((n, n, n), generator=g1, device='cuda') * 2 - 1
        u = torch.rand((n, n, n), generator=g, device='cuda')
    else:
        u = torch.rand((n, n, n), generator=g, device='cuda')
        if variant == 'inplace':
            d = torch.empty((n, n, n), device='cuda').uniform_(-1, 1, generator=g1)
        else:
            d = torch.rand((n, n, n), generator=g1, device='cuda') * 2 - 1
    scratch = [torch.empty_like(u), torch.empty_like(u)]
    del scratch
    torch.autograd.set_multithreading_enabled(False)
    uu = u.requires_grad_(True)
    fw, bw, addr = [], [], None
    for i in range(30):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        (o,) = fn.apply(uu)
        e1.record()
        o.backward(d)
        e2.record()
        addr = (u.data_ptr(), d.data_ptr(), o.data_ptr(), uu.grad.data_ptr())
        uu.grad = None
        if i >= 10:
            fw.append((e0, e1))
            bw.append((e1, e2))
    torch.cuda.synchronize()
    f = sorted(a.elapsed_time(b) for a, b in fw)
    b = sorted(a.elapsed_time(b) for a, b in bw)
    print(f'{variant:8s} fwd {f[len(f) // 2]:.4f} ms  bwd {b[len(b) // 2]:.4f} ms   u {addr[0]:#x} d {addr[1]:#x} '
          f'out {addr[2]:#x} grad {addr[3]:#x}', flush=True)


if __name__ == '__main__':
    main()
