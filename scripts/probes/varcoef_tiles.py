"""Tile sweep of the variable-coefficient diffusion (workloads.varcoef_diffusion_7pt) on the schedules a nonlinear
multi-field stencil can take, forward and TF-MAD adjoint kernels timed alone with HIP events (median of 20 after
warm-up), fraction of 8 TB/s from the algorithmic bytes (fwd 12, bwd 20 B/cell fp32). Timing only (parity:
tests/test_varcoef.py).  python scripts/probes/varcoef_tiles.py [n=512] [tiles=all] [f16]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends import hip_kernel as HK  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

TILES = {
    'default': {}, 'ws0': dict(WS=0), 'nt0': dict(NT_STORE=0), 'slp1': dict(SLP=1), 'ws0_slp1': dict(WS=0, SLP=1),
    'pr0': dict(PR=0), 'pr': dict(PR=1), 'ws0_pr': dict(WS=0, PR=1), 'ws0_pr0': dict(WS=0, PR=0),
    'pr_cx2nr4': dict(PR=1, WS=0, CX=2, NR=4), 'pr_cx4nr4': dict(PR=1, WS=0, CX=4, NR=4),
    'pr_ws_cx4nr2': dict(PR=1, WS=1, CX=4, NR=2, D=2), 'pr_ws8_cx4nr1': dict(PR=1, WS=1, NW=8, CX=4, NR=1, D=2),
    'pr_ws8_cx2nr2': dict(PR=1, WS=1, NW=8, CX=2, NR=2, D=2), 'pr_sf0': dict(PR=1, SFAST=0),
    'pd2': dict(PD=2, WS=0), 'pd2_pr': dict(PD=2, WS=0, PR=1), 'pd2_cx2nr4': dict(PD=2, WS=0, CX=2, NR=4),
    'pd2_cx2nr2': dict(PD=2, WS=0, CX=2, NR=2), 'pd2_cx4nr1': dict(PD=2, WS=0, CX=4, NR=1),
    'pd2_pr_cx2nr4': dict(PD=2, WS=0, PR=1, CX=2, NR=4), 'cx2nr2': dict(WS=0, CX=2, NR=2),
    'cx2nr2_pr': dict(WS=0, CX=2, NR=2, PR=1), 'cx2nr1': dict(WS=0, CX=2, NR=1), 'cx1nr2': dict(WS=0, CX=1, NR=2),
    'cx1nr4': dict(WS=0, CX=1, NR=4), 'cx2wx2nr2': dict(WS=0, CX=2, WX=2, NR=2), 'cx2wx2nr1': dict(WS=0, CX=2, WX=2, NR=1),
    'cx2nr2_nw2': dict(WS=0, CX=2, NR=2, NW=2), 'cx4nr1': dict(WS=0, CX=4, NR=1), 'cx2nr1_pr': dict(WS=0, CX=2, NR=1, PR=1),
    'cx2nr4': dict(WS=0, CX=2, NR=4), 'cx2nr2_nt0': dict(WS=0, CX=2, NR=2, NT_STORE=0),
    'cx4nr2_pr': dict(WS=0, CX=4, NR=2, PR=1), 'cx4nr1_pr': dict(WS=0, CX=4, NR=1, PR=1),
    'h_ws_cx4nr2': dict(PR=1, WS=1, CX=4, NR=2, D=2), 'h_ws_cx4nr4': dict(PR=1, WS=1, CX=4, NR=4, D=2),
    'h_ws_cx2nr2': dict(PR=1, WS=1, CX=2, NR=2, D=2), 'h_ws_cx2nr4': dict(PR=1, WS=1, CX=2, NR=4, D=2),
    'h_ws_cx4nr2_d3': dict(PR=1, WS=1, CX=4, NR=2, D=3), 'h_ws_cx2nr2_d3': dict(PR=1, WS=1, CX=2, NR=2, D=3),
    'h_ws8_cx4nr1': dict(PR=1, WS=1, NW=8, CX=4, NR=1, D=2), 'h_ws8_cx2nr2': dict(PR=1, WS=1, NW=8, CX=2, NR=2, D=2),
    'h_ws_cx4nr1': dict(PR=1, WS=1, CX=4, NR=1, D=2), 'h_ws_cx2nr1_d3': dict(PR=1, WS=1, CX=2, NR=1, D=3),
    'h_ws_cx2nr1': dict(PR=1, WS=1, CX=2, NR=1, D=2), 'h_ws8_cx2nr1': dict(PR=1, WS=1, NW=8, CX=2, NR=1, D=2),
    'h_ws8_cx2nr1_d3': dict(PR=1, WS=1, NW=8, CX=2, NR=1, D=3), 'h_ws8_cx2nr2_d3': dict(PR=1, WS=1, NW=8, CX=2, NR=2, D=3),
    'h_ws_cx2nr1_d4': dict(PR=1, WS=1, CX=2, NR=1, D=4), 'h_ws_cx2nr2_d4': dict(PR=1, WS=1, CX=2, NR=2, D=4),
    'h_ws_cx2wx2nr1_d3': dict(PR=1, WS=1, CX=2, WX=2, NR=1, D=3), 'h_ws_cx2wx2nr2': dict(PR=1, WS=1, CX=2, WX=2, NR=2, D=2),
    'reg': dict(CX=4, NR=4), 'reg_cx2nr2': dict(CX=2, NR=2), 'reg_cx1wx4nr4': dict(CX=1, WX=4, NR=4),
    'ws_cx4nr4': dict(WS=1, CX=4, NR=4, D=2), 'ws_cx4nr2': dict(WS=1, CX=4, NR=2, D=2),
    'ws_cx4nr2d3': dict(WS=1, CX=4, NR=2, D=3), 'ws_cx2nr4': dict(WS=1, CX=2, NR=4, D=2),
    'ws_cx2nr4d3': dict(WS=1, CX=2, NR=4, D=3), 'ws_cx2nr2d3': dict(WS=1, CX=2, NR=2, D=3),
    'ws_cx2nr2d4': dict(WS=1, CX=2, NR=2, D=4), 'ws_cx1nr4d3': dict(WS=1, CX=1, NR=4, D=3),
    'ws_cx2wx2nr2': dict(WS=1, CX=2, WX=2, NR=2, D=3), 'ws_cx4nr1d3': dict(WS=1, CX=4, NR=1, D=3),
    'ws_cx2nr2': dict(WS=1, CX=2, NR=2, D=2), 'ws_cx1nr4': dict(WS=1, CX=1, NR=4, D=2),
    'ws_cx1nr2': dict(WS=1, CX=1, NR=2, D=2), 'ws_cx2nr1': dict(WS=1, CX=2, NR=1, D=2),
    'ws_cx4nr1': dict(WS=1, CX=4, NR=1, D=2), 'ws_cx2nr2d1': dict(WS=1, CX=2, NR=2, D=1),
    'ws8_cx4nr1': dict(WS=1, NW=8, CX=4, NR=1, D=2), 'ws8_cx4nr2': dict(WS=1, NW=8, CX=4, NR=2, D=2),
    'ws8_cx2nr2': dict(WS=1, NW=8, CX=2, NR=2, D=2), 'ws8_cx2nr1': dict(WS=1, NW=8, CX=2, NR=1, D=2),
    'ws8_cx2wx2nr1': dict(WS=1, NW=8, WX=2, CX=2, NR=1, D=2), 'ws8_cx2nr4': dict(WS=1, NW=8, CX=2, NR=4, D=2),
    'ws_cx4nr1d4': dict(WS=1, CX=4, NR=1, D=4), 'ws8_cx4nr1d3': dict(WS=1, NW=8, CX=4, NR=1, D=3),
    'ws8_cx4nr1d4': dict(WS=1, NW=8, CX=4, NR=1, D=4), 'ws_cx2nr2d4': dict(WS=1, CX=2, NR=2, D=4),
    'ws8_cx2nr2d3': dict(WS=1, NW=8, CX=2, NR=2, D=3),
    # timing only (wrong results): the default ring with no plane loads — the compute waves' time alone
    'abl_noload': dict(BABL=3), 'abl_noload_ws8': dict(WS=1, NW=8, CX=4, NR=1, D=2, BABL=3),
    # chunk length along z (explicit ZC: the block-count path instead of the quantised chunk model)
    'zc24': dict(ZC=24), 'zc32': dict(ZC=32), 'zc48': dict(ZC=48), 'zc64': dict(ZC=64), 'zc96': dict(ZC=96),
    'zc128': dict(ZC=128), 'blk512': dict(BLOCKS=512), 'blk1024': dict(BLOCKS=1024),
}


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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    names = sys.argv[2].split(',') if len(sys.argv) > 2 else list(TILES)
    f16 = len(sys.argv) > 3 and sys.argv[3] == 'f16'
    dt, es = (torch.float16, 2) if f16 else (torch.float32, 4)
    op = pa.AutoDiffOp(W.varcoef_diffusion_7pt(dtype='float16' if f16 else 'float32'), boundary_handling='zeros')
    shape = (n, n, n)
    u, k, d = (torch.rand(shape, device='cuda').to(dt) for _ in range(3))
    out, du, dk = (torch.empty(shape, device='cuda', dtype=dt) for _ in range(3))
    cells = n ** 3
    for name in names:
        p = dict(TILES[name])
        HK.PROBE_KNOBS.clear()          # ablation knobs are not tile keys: the probe-only entry
        HK.PROBE_KNOBS.update({key: p.pop(key) for key in HK.PROBE_KEYS if key in p})
        fk = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='vcf', target='gpu',
                           gpu_indexing_params=p or None).compile()
        bk = StencilKernel(op.backward_assignments, boundary_handling='zeros', function_name='vcb', target='gpu',
                           gpu_indexing_params=p or None).compile()
        tf = timed(lambda: fk(u=u, k=k, out=out))
        tb = timed(lambda: bk(u=u, k=k, diffout=d, diffu=du, diffk=dk))
        HK.PROBE_KNOBS.clear()
        v = fk.last_variant[1] if len(fk.last_variant) > 1 else None
        bv = bk.last_variant[1] if len(bk.last_variant) > 1 else None
        print(f'varcoef {n}^3 {name:10s} fwd {tf:.4f} ms ({3 * es * cells / tf / 1e6 / 8000:.3f})  bwd {tb:.4f} ms '
              f'({5 * es * cells / tb / 1e6 / 8000:.3f})  fwd CX={getattr(v, "CX", "-")} NR={getattr(v, "NR", "-")} '
              f'WS={getattr(v, "WS", "-")} D={getattr(v, "D", "-")} | bwd CX={getattr(bv, "CX", "-")} NR={getattr(bv, "NR", "-")} '
              f'WS={getattr(bv, "WS", "-")} D={getattr(bv, "D", "-")}', flush=True)


if __name__ == '__main__':
    main()
