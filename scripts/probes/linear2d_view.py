"""Config 2 (2-D 5-point Laplacian fp32 4096², forward and TF-MAD adjoint kernels) on the (1, Y, X) tiles of the zsum
schedule (default) against marching along axis 0 (VIEW2D='zy', rows as planes, LDS-DMA loader): 20 back-to-back launches
between two HIP events per variant (launch gaps amortised), fraction of 8 TB/s at 8 B/cell. Timing only.
python scripts/probes/linear2d_view.py [n=4096] [tiles=all]"""
import os
import sys

import sympy as sp
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import ps  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

TILES = {'default': {},
         'zy_cx2': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, ZSUM=1),
         'zy_cx4': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, ZSUM=1),
         'zy_cx4_z32': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, ZSUM=1, ZC=32),
         'zy_cx2_z64': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, ZSUM=1, ZC=64),
         'zy_cx2_z16': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, ZSUM=1, ZC=16)}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    names = sys.argv[2].split(',') if len(sys.argv) > 2 else list(TILES)
    u, out = ps.fields('u, out: float32[2d]')
    ac = ps.AssignmentCollection({out.center: u[1, 0] + u[-1, 0] + u[0, 1] + u[0, -1] - 4 * u.center})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    x = torch.rand((n, n), device='cuda')
    y = torch.empty_like(x)
    for name in names:
        p = TILES[name]
        res = []
        for asg, fn in ((op.forward_assignments, 'l2f'), (op.backward_assignments, 'l2b')):
            k = StencilKernel(asg, boundary_handling='zeros', function_name=fn, target='gpu',
                              gpu_indexing_params=p or None).compile()
            names_ = [f.name for f in k.ir.fields]
            kw = {names_[0]: x, names_[1]: y} if k.ir.fields_written[0].name == names_[1] else {names_[1]: x, names_[0]: y}
            for _ in range(10):
                k(**kw)
            ts = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    k(**kw)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) / 20)
            t = sorted(ts)[2]
            v = k.last_variant[1]
            res.append(f'{t * 1e3:.1f} us ({8 * n * n / t / 1e6 / 8000:.3f}) {v.VIEW2D} CX={v.CX} NR={v.NR} WS={v.WS}')
        print(f'lap2d {n}^2 {name:11s} fwd {res[0]}  bwd {res[1]}', flush=True)


if __name__ == '__main__':
    main()
