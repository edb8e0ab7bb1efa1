"""2-D variable-coefficient diffusion (5-point, nonlinear: ``u + α Σ₄ ½(k + k[nb])(u[nb] − u)``) through the op,
forward and TF-MAD adjoint kernels timed alone with HIP events (median of 20), fraction of 8 TB/s from the algorithmic
bytes (fwd 3, bwd 5 fields per cell). Timing only (parity: tests/test_varcoef.py::test_varcoef_2d_gpu_vs_oracle).
python scripts/probes/nonlinear2d.py [n=4096] [tiles=default,...] [f16|f32|f64]"""
import os
import sys

import sympy as sp
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import ps  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

TILES = {'default': {}, 'yx': dict(VIEW2D='yx'), 'old': dict(CX=4, NR=4), 'cx2nr2': dict(CX=2, NR=2), 'cx4nr2': dict(CX=4, NR=2), 'cx2nr4': dict(CX=2, NR=4),
         'cx4nr8': dict(CX=4, NR=8), 'cx8nr4': dict(CX=8, NR=4), 'cx4nr4_pr': dict(CX=4, NR=4, PR=1),
         'cx2nr2_pr': dict(CX=2, NR=2, PR=1), 'cx4nr1': dict(CX=4, NR=1), 'cx2nr8': dict(CX=2, NR=8),
         'nw1_cx4nr8': dict(NW=1, CX=4, NR=8), 'cx4wx2nr4': dict(CX=4, WX=2, NR=4),
         # march along axis 0 (VIEW2D='zy': rows are the ring's planes), waves side by side in x
         'zy_cx1': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=1), 'zy_cx2': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2),
         'zy_cx4': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4), 'zy_wx2': dict(VIEW2D='zy', NR=1, NW=2, WX=2, CX=2),
         'zy_cx2_pr': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, PR=1),
         # ... fed by the LDS-DMA loader wave (WS)
         'zyws_cx2': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2),
         'zyws_cx1': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=1, WS=1, D=2),
         'zyws_cx4': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2),
         'zyws_d4': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=4),
         'zyws_nw8': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=1, WS=1, D=2),
         'zyws_nw8c2': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=2, WS=1, D=2),
         'zyws_pr': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, PR=1),
         'zyws_pr4': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2, PR=1),
         'zyws_pr8': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=8, WS=1, D=2, PR=1),
         'zyws_pr4d3': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=3, PR=1),
         'zyws_pr4d1': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=1, PR=1),
         'zyws_pr_nw8': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=2, WS=1, D=2, PR=1),
         'zyws_pr4_nw8': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=4, WS=1, D=2, PR=1),
         'zyws_pr4_wx2': dict(VIEW2D='zy', NR=1, NW=2, WX=2, CX=4, WS=1, D=2, PR=1),
         'zyws_nw8c4': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=4, WS=1, D=2),
         'zyws_nw8d3': dict(VIEW2D='zy', NR=1, NW=8, WX=8, CX=2, WS=1, D=3),
         'zyws_cx8': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=8, WS=1, D=2),
         # chunking along axis 0 (rows per workgroup): ZMIN / ZMAX / BLK
         'zyws_c32': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, ZMIN=32, ZMAX=64, BLK=512),
         'zyws_c8': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, ZMIN=8, ZMAX=128, BLK=256),
         'zyws_c16': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, ZMIN=16, ZMAX=64, BLK=1024),
         'zyws_c64': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, ZMIN=64, ZMAX=128, BLK=256),
         'zyws_c128': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=2, WS=1, D=2, ZMIN=128, ZMAX=256, BLK=256),
         'zyws_pr4_c32': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2, PR=1, ZMIN=32, ZMAX=64, BLK=512),
         'zyws_pr4_c8': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2, PR=1, ZMIN=8, ZMAX=128, BLK=256),
         'zyws_pr4_c64': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2, PR=1, ZMIN=64, ZMAX=128, BLK=256),
         'zyws_pr4_c128': dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4, WS=1, D=2, PR=1, ZMIN=128, ZMAX=256, BLK=256)}


def varcoef2d(dts):
    u, k, out = ps.fields(f'u, k, out: {dts}[2d]')
    nb = [(1, 0), (-1, 0), (0, 1), (0, -1)]
    return ps.AssignmentCollection({out.center: u.center + 0.1 * sp.Add(
        *[sp.Rational(1, 2) * (k.center + k[o]) * (u[o] - u.center) for o in nb])})


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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    names = sys.argv[2].split(',') if len(sys.argv) > 2 else list(TILES)
    prec = sys.argv[3] if len(sys.argv) > 3 else 'f32'
    dts = {'f16': 'float16', 'f32': 'float32', 'f64': 'float64'}[prec]
    dt = getattr(torch, dts)
    es = dt.itemsize
    op = pa.AutoDiffOp(varcoef2d(dts), boundary_handling='zeros')
    shape = (n, n)
    u, k, d = (torch.rand(shape, device='cuda').to(dt) for _ in range(3))
    out, du, dk = (torch.empty(shape, device='cuda', dtype=dt) for _ in range(3))
    for name in names:
        p = dict(TILES[name])
        fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='v2f', target='gpu',
                           gpu_indexing_params=p or None).compile()
        bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='v2b', target='gpu',
                           gpu_indexing_params=p or None).compile()
        tf = timed(lambda: fk(u=u, k=k, out=out))
        tb = timed(lambda: bk(u=u, k=k, diffout=d, diffu=du, diffk=dk))
        v = fk.last_variant
        got = [t.float().clone() for t in (out, du, dk)]
        if name == names[0]:
            first = got            # (the first tiling's results: the others are compared with them)
        dev = max(float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, first))
        print(f'varcoef2d {n}^2 {prec} {name:12s} fwd {tf * 1e3:.1f} us ({3 * es * n * n / tf / 1e6 / 8000:.3f})  '
              f'bwd {tb * 1e3:.1f} us ({5 * es * n * n / tb / 1e6 / 8000:.3f})  {v[0]} '
              f'{dict(CX=v[1].CX, NR=v[1].NR, WS=v[1].WS, PR=v[1].PR, V=v[1].VIEW2D) if len(v) > 1 and hasattr(v[1], "CX") else ""}'
              f'  rel.dev {dev:.1e}',
              flush=True)


if __name__ == '__main__':
    main()
