"""Where the half-ring 27-point kernel with DPP neighbour exchange differs from the oracle, per tuning."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from oracle import evaluate as OE
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    for shape in ((11, 21, 72), (9, 40, 300), (11, 21, 80), (11, 21, 256), (11, 21, 264), (11, 40, 72),
                  (30, 21, 72), (11, 8, 72), (1, 1, 72)):
        rng = np.random.default_rng(5)
        u = rng.uniform(0, 1, shape).astype(np.float16)
        ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling='zeros')['out']
        for params in (dict(CX=4, NR=2), dict(CX=4, NR=2, DPP=0)):
            k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='dbg', target='gpu',
                              gpu_indexing_params=params).compile()
            out = torch.zeros(shape, dtype=torch.float16, device='cuda')
            k(u=torch.from_numpy(u).cuda(), out=out)
            torch.cuda.synchronize()
            o = out.cpu().numpy().astype(np.float64)
            err = np.abs(o - ref)
            bad = np.argwhere(err > 1e-3 * np.abs(ref).max())
            info = ''
            if len(bad):
                zs, ys, xs = (sorted(set(bad[:, i].tolist())) for i in range(3))
                info = f' bad {len(bad)}: z {zs[:6]} y {ys[:12]} x {xs[:16]}'
            print(shape, params, k.last_variant[1].CX, k.last_variant[1].NR, f'max err {err.max():.3e}{info}', flush=True)


if __name__ == '__main__':
    main()
