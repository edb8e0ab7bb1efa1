"""What the 'XM' rows cost (WS sweeps whose row pitch is not a multiple of 16 bytes): 7-point fp16 / fp32 through
the op on 512×512×X fields for X around 512 — pitch a multiple of 16 B (512, 504, 496) or not (510, 508, 506, 511),
same process, HIP events around Op.apply / backward.
python scripts/probes/xm_cost.py [dtype ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    dts = sys.argv[1:] or ['float16', 'float32']
    for dname in dts:
        dt = getattr(torch, dname)
        for X in (512, 510, 508, 506, 504, 511, 496):
            shape = (512, 512, X)
            op = pa.AutoDiffOp(W.diffusion_7pt(dtype=dname), boundary_handling='zeros')
            fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
            u = torch.rand(shape, device='cuda').to(dt).requires_grad_(True)
            d = (torch.rand(shape, device='cuda') * 2 - 1).to(dt)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                (o,) = fn.apply(u)
                o.backward(d)
                u.grad = None
            ev = []
            for _ in range(20):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                (o,) = fn.apply(u)
                e1.record()
                o.backward(d)
                e2.record()
                u.grad = None
                ev.append((e0, e1, e2))
            torch.cuda.synchronize()
            f = sorted(a.elapsed_time(b) for a, b, _ in ev)[10]
            b = sorted(b.elapsed_time(c) for _, b, c in ev)[10]
            cfg = op.forward_ast_gpu.compile().last_plan
            nb = 2 * u.element_size() * u.numel()
            print(f'7pt {dname} 512x512x{X} (pitch {X * u.element_size()} B): fwd {f:.4f} bwd {b:.4f} ms '
                  f'({nb / f / 1e9:.2f} / {nb / b / 1e9:.2f} TB/s)  {getattr(cfg, "variant", cfg)}', flush=True)
            del fn, op, u, d, o
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
