"""A nonlinear stencil on a vector field (index dimension, components fastest): first-order upwind-free advection
``out(c) = u(c) − α Σ_d u(d)·(u[+e_d](c) − u[−e_d](c))/2`` on u(3) fp32 — which schedule it takes and its forward /
adjoint rate through the op (HIP events, median of 20). Timing only.
python scripts/probes/vector_nonlinear.py [n=256] [dtype=float32] [2d: u(2) on n x n]"""
import os
import sys

import sympy as sp
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import ps  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dts = sys.argv[2] if len(sys.argv) > 2 else 'float32'
    D = 2 if len(sys.argv) > 3 and sys.argv[3] == '2d' else 3     # '2d': u(2) on n x n
    tdt = getattr(torch, dts)
    u, out = ps.fields(f'u({D}), out({D}): {dts}[{D}d]')
    e = [tuple(int(i == a) for i in range(D)) for a in range(D)]
    m = [tuple(-v for v in o) for o in e]
    ac = ps.AssignmentCollection({out.center(c): u.center(c) - 0.05 * sp.Add(
        *[u.center(d) * (u[e[d]](c) - u[m[d]](c)) / 2 for d in range(D)]) for c in range(D)})
    op = pa.AutoDiffOp(ac, boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    x = torch.rand((n,) * D + (D,), device='cuda').to(tdt).requires_grad_(True)
    g = torch.rand((n,) * D + (D,), device='cuda').to(tdt)
    for _ in range(5):
        (o,) = fn.apply(x)
        o.backward(g)
        x.grad = None
    fw, bw = [], []
    for _ in range(20):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        (o,) = fn.apply(x)
        ev[1].record()
        o.backward(g)
        ev[2].record()
        torch.cuda.synchronize()
        x.grad = None
        fw.append(ev[0].elapsed_time(ev[1]))
        bw.append(ev[1].elapsed_time(ev[2]))
    fw.sort()
    bw.sort()
    b = n ** D * D * tdt.itemsize
    print(f'vector advection {n}^{D}x{D} {dts}: fwd {fw[10]:.4f} ms ({2 * b / fw[10] / 1e6 / 8000:.3f} of 8 TB/s), '
          f'bwd {bw[10]:.4f} ms ({3 * b / bw[10] / 1e6 / 8000:.3f}); schedules '
          f'{op.forward_ast_gpu.compile().last_variant[0]} / {op.backward_ast_gpu.compile().last_variant[0]}', flush=True)


if __name__ == '__main__':
    main()
