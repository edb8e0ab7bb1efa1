"""Run-to-run determinism of band variants on one input (27-point fp16 forward, (37, 48, 768)): each config runs
REPS times; prints, per config, how many cells differ between runs and from the BPAD=0 result, with the first
differing (z, y, x) cells. python scripts/probes/band_determinism.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

REPS = 6


def main():
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    g = torch.Generator().manual_seed(11)
    shape = tuple(int(v) for v in sys.argv[1].split(',')) if len(sys.argv) > 1 else (37, 48, 768)
    u = (torch.rand(shape, generator=g) * 2 - 1).half().cuda()
    base = None
    for tun in ({'BAND': 4, 'BPAD': 0}, {'BAND': 4, 'BPAD': 1}, {'BAND': 4, 'BPAD': 1, 'BTRIM': 1},
                {'BAND': 4, 'BPAD': 1, 'D': 1}, {'BAND': 4, 'BPAD': 0, 'BTRIM': 1}):
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='det', target='gpu',
                          gpu_indexing_params=tun).compile()
        outs = []
        for _ in range(REPS):
            o = torch.full_like(u, float('nan'))
            k(u=u, out=o)
            outs.append(o)
        torch.cuda.synchronize()
        if base is None:
            base = outs[0]
        cfg = k.last_variant[1]
        runs = [int((o != outs[0]).sum()) for o in outs[1:]]
        d = (outs[0].float() - base.float()).abs()
        where = torch.nonzero(d > 0)[:8].tolist()
        print(f'{str(tun):42s} BPAD={cfg.BPAD} BTRIM={cfg.BTRIM} ZMIN={cfg.ZMIN} D={cfg.D}: run-to-run differing cells '
              f'{runs}; vs first config {int((d > 0).sum())} cells (max {float(d.max()):.3g}) at {where}', flush=True)


if __name__ == '__main__':
    main()
