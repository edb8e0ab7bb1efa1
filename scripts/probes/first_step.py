"""Where the first fwd+bwd step of bench.py spends its time after the bench's setup (kernel plans built,
caching-allocator blocks reserved, autograd engine started): host time per phase of steps 1-3 and a
cProfile of the first backward."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    fwd_k = op.forward_ast_gpu.compile()
    bwd_k = op.backward_ast_gpu.compile()
    u = torch.rand((n, n, n), device='cuda')
    d = torch.rand((n, n, n), device='cuda') * 2 - 1
    scratch = [torch.empty_like(u), torch.empty_like(u)]
    fwd_k.prepare(u=u, out=scratch[0])
    bwd_k.prepare(diffout=d, diffu=scratch[1])
    del scratch
    probe = torch.zeros(1, device='cuda', requires_grad=True)
    (probe * 2).backward(torch.ones_like(probe))
    torch.cuda.synchronize()
    uu = u.requires_grad_(True)
    for step in range(3):
        t0 = time.perf_counter()
        (o,) = fn.apply(uu)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if step == 0:
            pr = cProfile.Profile()
            pr.enable()
        o.backward(d)
        t3 = time.perf_counter()
        if step == 0:
            pr.disable()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        uu.grad = None
        print(f'step {step}: fwd host {1e3*(t1-t0):.2f} ms, fwd sync {1e3*(t2-t1):.2f}, bwd host {1e3*(t3-t2):.2f}, '
              f'bwd sync {1e3*(t4-t3):.2f}', flush=True)
        if step == 0:
            pstats.Stats(pr).sort_stats('cumulative').print_stats(18)


if __name__ == '__main__':
    main()
