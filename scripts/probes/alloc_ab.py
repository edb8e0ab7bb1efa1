"""Forward / adjoint sweep times of the 1024³ 7-point op as a function of where the fields sit: the bench's
allocation order (u, then diffout), the swapped order, and both with a 1 GiB gap block in between — one process,
interleaved rounds, HIP events around Op.apply and backward (the driver's round-3 line had the adjoint 5 % slower than
the forward on one box; VERDICT r03 "what's weak" 3).
python scripts/probes/alloc_ab.py [edge]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    torch.autograd.set_multithreading_enabled(False)
    op = pa.AutoDiffOp(W.diffusion_7pt(), 'alloc_ab', boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    g = torch.Generator(device='cuda').manual_seed(0)
    layouts = {}
    for tag in ('u_then_d', 'd_then_u', 'u_gap_d'):
        keep = []
        if tag == 'd_then_u':
            d = torch.rand((n, n, n), generator=g, device='cuda') * 2 - 1
            u = torch.rand((n, n, n), generator=g, device='cuda')
        else:
            u = torch.rand((n, n, n), generator=g, device='cuda')
            if tag == 'u_gap_d':
                keep.append(torch.empty(1 << 28, device='cuda'))          # 1 GiB between the two fields
            d = torch.rand((n, n, n), generator=g, device='cuda') * 2 - 1
        layouts[tag] = (u.requires_grad_(True), d, keep)
    torch.cuda.synchronize()

    def rnd(u, d, steps=10):
        fw, bw = [], []
        for _ in range(steps):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            (o,) = fn.apply(u)
            e1.record()
            o.backward(d)
            e2.record()
            u.grad = None
            fw.append((e0, e1))
            bw.append((e1, e2))
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in fw], [a.elapsed_time(b) for a, b in bw]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        rnd(*layouts['u_then_d'][:2], steps=2)
    res = {k: ([], []) for k in layouts}
    for _ in range(5):
        for k, (u, d, _) in layouts.items():
            f, b = rnd(u, d)
            res[k][0].extend(f)
            res[k][1].extend(b)
    for k, (f, b) in res.items():
        f, b = sorted(f), sorted(b)
        u, d, _ = layouts[k]
        print(f'{k:10s} fwd {f[len(f) // 2]:.4f} ms  bwd {b[len(b) // 2]:.4f} ms   u @ {u.data_ptr():#x}  d @ '
              f'{d.data_ptr():#x}', flush=True)


if __name__ == '__main__':
    main()
