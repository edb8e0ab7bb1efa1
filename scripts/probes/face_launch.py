"""Cost of the two-face launch of a z-slab sweep (planes 0 and Zl-1 of a 128x1024^2 slab, halos read
in place) under different march configurations: event time per launch, back to back."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402


def main():
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    zl, n = 128, 1024
    u = torch.rand((zl, n, n), device='cuda')
    out = torch.empty_like(u)
    lo = torch.rand((1, n, n), device='cuda')
    hi = torch.rand((1, n, n), device='cuda')
    ref = None
    for spec in ['default', 'WS=0', 'WS=0,NR=2', 'WS=0,NR=1,CX=2', 'WS=0,NW=1,NR=2', 'WS=0,CX=1,NR=1', 'D=2',
                 'WS=0,NW=2,WX=1,NR=2']:
        tun = {} if spec == 'default' else {k: int(v) for k, v in (kv.split('=') for kv in spec.split(','))}
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='face', target='gpu',
                          gpu_indexing_params=tun).compile()
        args = dict(u=u, out=out, halos={'u': (lo, hi)}, z_range=((0, 1), (zl - 1, zl)))
        out.zero_()
        k(**args)
        torch.cuda.synchronize()
        faces = torch.stack([out[0], out[-1]]).clone()
        if ref is None:
            ref = faces
        ok = torch.allclose(faces, ref, rtol=0, atol=1e-6)
        for _ in range(20):
            k(**args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            k(**args)
        e1.record()
        torch.cuda.synchronize()
        print(f'{spec:24s} {e0.elapsed_time(e1) / 200 * 1e3:7.1f} us per two-face launch  variant={k.last_variant[1] if len(k.last_variant) > 1 else k.last_variant}'[:160] + f'  same={ok}')


if __name__ == '__main__':
    main()
