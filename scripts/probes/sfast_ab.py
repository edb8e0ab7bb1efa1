"""A/B of the wave-uniform unguarded cells (MarchConfig.SFAST) against per-cell guarded ones, forward and adjoint
kernels alone, alternating in one process (HIP events, median of 20 after warm-up). Timing only. The zsum cases ran
with the same switch on the zsum store block (profiles/r05_sfast_ab.log: neutral, since reverted — SFAST now only
changes the march ring, and the zsum lines compare a kernel with itself).

python scripts/probes/sfast_ab.py [rounds=3]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

CASES = [('diffusion7_f32', W.diffusion_7pt, (1024, 1024, 1024), torch.float32),
         ('diffusion7_f32', W.diffusion_7pt, (768, 768, 768), torch.float32),
         ('diffusion7_f32', W.diffusion_7pt, (512, 512, 512), torch.float32),
         ('laplace5_f32', W.laplace_5pt, (4096, 4096), torch.float32),
         ('varcoef7_f32', W.varcoef_diffusion_7pt, (512, 512, 512), torch.float32)]


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for name, b, shape, dt in CASES:
        op = pa.AutoDiffOp(b(), boundary_handling='zeros')
        ins = {f.name: torch.rand(shape, device='cuda', dtype=dt) for f in op.forward_input_fields}
        outs = {f.name: torch.empty(shape, device='cuda', dtype=dt) for f in op.forward_output_fields}
        bins = {**ins, **{f'diff{n}': torch.rand(shape, device='cuda', dtype=dt) for n in outs}}
        bouts = {f.name: torch.empty(shape, device='cuda', dtype=dt) for f in op.backward_output_fields}
        ks = {}
        for tag, p in (('sfast', {}), ('guarded', {'SFAST': 0})):
            ks[tag] = (StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name=f'sf_{tag}_f',
                                     target='gpu', gpu_indexing_params=p or None).compile(),
                       StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name=f'sf_{tag}_b',
                                     target='gpu', gpu_indexing_params=p or None).compile())
        for r in range(rounds):
            line = []
            for tag, (fk, bk) in ks.items():
                tf = timed(lambda: fk(**ins, **outs))
                tb = timed(lambda: bk(**bins, **bouts))
                line.append(f'{tag} fwd {tf:.4f} bwd {tb:.4f} ms')
            print(f"{name} {'x'.join(map(str, shape))} round {r}: " + ' | '.join(line) +
                  f"  [{ks['sfast'][0].last_variant[0]}]", flush=True)
        del ins, outs, bins, bouts
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
