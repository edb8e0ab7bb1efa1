"""HBM aliasing between a sweep's input and output: the 1024^3 fp32 7-point forward kernel (4 GiB in, 4 GiB out)
on views of one 18 GiB buffer, input at offset 0 and output at offset D, D = k * 4 GiB + delta. Prints the kernel
time per D (HIP events, median of 10 launches). python scripts/probes/alias_offsets.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

GiB, MiB = 1 << 30, 1 << 20


def main():
    n = 1024
    cells = n ** 3
    buf = torch.empty(18 * GiB // 4, dtype=torch.float32, device='cuda')
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    u = buf[:cells].view(n, n, n)
    u.uniform_(0, 1)
    for k4 in (1, 2, 3):
        for delta in (0, 1 * MiB, 2 * MiB, 8 * MiB, 24 * MiB, 64 * MiB, 256 * MiB, 1 * GiB, 2 * GiB):
            off = (k4 * 4 * GiB + delta) // 4
            if off + cells > buf.numel():
                continue
            out = buf[off:off + cells].view(n, n, n)
            for _ in range(3):
                k(u=u, out=out)
            ts = []
            for _ in range(10):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                k(u=u, out=out)
                b.record()
                ts.append((a, b))
            torch.cuda.synchronize()
            t = sorted(x.elapsed_time(y) for x, y in ts)[5]
            print(f'out - in = {k4} x 4 GiB + {delta / MiB:7.0f} MiB: {t:.4f} ms', flush=True)


if __name__ == '__main__':
    main()
