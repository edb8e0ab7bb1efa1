"""fwd + bwd through the drop-in op for one workload / shape (HIP events, settled load): an op-level A/B of a
default against a PSAD_MARCH override run in another process.  python scripts/probes/op_ab.py diffusion7_f16 1024"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

B = {'diffusion7_f16': (lambda: W.diffusion_7pt(dtype='float16'), torch.float16),
     'diffusion7': (W.diffusion_7pt, torch.float32)}


def main():
    name, n = sys.argv[1], int(sys.argv[2])
    b, dt = B[name]
    op = pa.AutoDiffOp(b(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    u = torch.rand((n, n, n), device='cuda').to(dt).requires_grad_(True)
    d = (torch.rand((n, n, n), device='cuda') * 2 - 1).to(dt)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        (o,) = fn.apply(u)
        o.backward(d)
        u.grad = None
    torch.cuda.synchronize()
    fw, bw = [], []
    for _ in range(20):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        (o,) = fn.apply(u)
        e[1].record()
        o.backward(d)
        e[2].record()
        torch.cuda.synchronize()
        u.grad = None
        fw.append(e[0].elapsed_time(e[1]))
        bw.append(e[1].elapsed_time(e[2]))
    fw.sort()
    bw.sort()
    print(f"{name} {n}^3 PSAD_MARCH={os.environ.get('PSAD_MARCH', '')!r}: fwd {fw[10]:.4f} ms  bwd {bw[10]:.4f} ms  "
          f"variant {op.forward_ast_gpu.compile().last_variant[1].NR if op.forward_ast_gpu.compile().last_variant else None}",
          flush=True)


if __name__ == '__main__':
    main()
