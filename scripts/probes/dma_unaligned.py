"""Probe: LDS-DMA 16-byte pieces from rows whose pitch is only 4-byte aligned (fp32, X % 4 != 0) — results vs
the generic schedule and timing vs the 8-byte register-prefetch default. """
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402


def t(k, args, force=None, reps=20):
    for _ in range(3):
        k(force_schedule=force, **args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        k(force_schedule=force, **args)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for shape in [(6, 9, 262), (16, 40, 261), (128, 300, 262), (128, 300, 261), (255, 255, 255)]:
    for b, name in ((W.diffusion_7pt, '7pt'), (lambda: W.stencil_27pt(dtype='float32'), '27pt_f32'),
                    (lambda: W.diffusion_7pt(dtype='float64'), '7pt_f64')):
        op = pa.AutoDiffOp(b(), boundary_handling='zeros')
        for k in (op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()):
            names = [f.name for f in k.ir.fields_read]
            dt = torch.float64 if name.endswith('f64') else torch.float32
            ins = {n: torch.rand(shape, device='cuda', dtype=dt) for n in names}
            out = {f.name: torch.full(shape, float('nan'), device='cuda', dtype=dt) for f in k.ir.fields_written}
            ref = {n: torch.empty_like(v) for n, v in out.items()}
            k(force_schedule='generic', **ins, **ref)
            us = t(k, {**ins, **out})
            v = k.last_variant
            ok = all(torch.allclose(out[n], ref[n], rtol=0, atol=1e-5) for n in out)
            print(f"{name:9s} {k.name[-20:]:20s} {str(shape):16s} {us:8.1f} us  VE={v[1].VE} WS={v[1].WS} XM={v[1].XM}  match_generic={ok}",
                  flush=True)
            assert ok
