"""Rows whose byte pitch is not a multiple of 16 (X·esize % 16 != 0): the march schedule then drops to scalar
(VE=1) loads without the LDS-DMA loader. Time that default against the one-thread-per-cell generic schedule
(forward kernel, same process) on misaligned and aligned extents."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402


def bench(k, args, force, reps=30):
    for _ in range(3):
        k(force_schedule=force, **args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(reps):
            k(force_schedule=force, **args)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[2]


def main():
    cases = [('7pt f32', W.diffusion_7pt, torch.float32, (128, 300, 260)),
             ('7pt f32', W.diffusion_7pt, torch.float32, (128, 300, 261)),
             ('7pt f32', W.diffusion_7pt, torch.float32, (128, 300, 262)),
             ('7pt f32', W.diffusion_7pt, torch.float32, (255, 255, 255)),
             ('7pt f32', W.diffusion_7pt, torch.float32, (256, 256, 256)),
             ('7pt f16', lambda: W.diffusion_7pt(dtype='float16'), torch.float16, (128, 300, 264)),
             ('7pt f16', lambda: W.diffusion_7pt(dtype='float16'), torch.float16, (128, 300, 260)),
             ('27pt f16', W.stencil_27pt, torch.float16, (128, 300, 264)),
             ('27pt f16', W.stencil_27pt, torch.float16, (128, 300, 260)),
             ('27pt f16', W.stencil_27pt, torch.float16, (255, 255, 255)),
             ('27pt f16', W.stencil_27pt, torch.float16, (256, 256, 258)),
             ('27pt f16', W.stencil_27pt, torch.float16, (768, 768, 766)),
             ('7pt f16', lambda: W.diffusion_7pt(dtype='float16'), torch.float16, (256, 256, 258)),
             ('5pt f32', W.laplace_5pt, torch.float32, (4096, 4096)),
             ('5pt f32', W.laplace_5pt, torch.float32, (4097, 4097)),
             ('5pt f32', W.laplace_5pt, torch.float32, (4095, 4094))]
    for name, b, dt, shape in cases:
        op = pa.AutoDiffOp(b(), boundary_handling='zeros')
        k = op.forward_ast_gpu.compile()
        u = torch.rand(shape, device='cuda').to(dt)
        out = torch.empty_like(u)
        args = dict(u=u, out=out)
        t_def = bench(k, args, None)
        v = k.last_variant
        ref = out.clone()
        t_gen = bench(k, args, 'generic')
        same = torch.allclose(out.float(), ref.float(), rtol=0, atol=1e-3 if dt == torch.float16 else 1e-6)
        nbytes = 2 * u.numel() * u.element_size()
        vv = v[1] if len(v) > 1 else v
        desc = f'march VE={vv.VE} WS={vv.WS} CX={vv.CX} NR={vv.NR}' if v[0] == 'march' else str(v)
        print(f'{name:9s} {str(shape):18s} default {t_def * 1e3:8.1f} us ({nbytes / t_def / 1e6:6.0f} GB/s, {desc})  '
              f'generic {t_gen * 1e3:8.1f} us ({nbytes / t_gen / 1e6:6.0f} GB/s)  same={same}', flush=True)


if __name__ == '__main__':
    main()
