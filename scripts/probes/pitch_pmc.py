"""A few band-schedule fwd+bwd steps per size, for rocprofv3 --pmc passes over rows of different pitch (the row-pitch
cliff: 27-point 510³ / 511³ against 512³).

rocprofv3 --pmc FETCH_SIZE -- python scripts/probes/pitch_pmc.py s27:510 s27:512"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

WL = {'h7': (lambda: W.diffusion_7pt(dtype='float16'), torch.float16), 's27': (W.stencil_27pt, torch.float16),
      'f7': (W.diffusion_7pt, torch.float32)}


def main():
    for spec in sys.argv[1:]:
        name, n = spec.split(':')
        b, dt = WL[name]
        fn = pa.AutoDiffOp(b(), boundary_handling='zeros').create_tensorflow_op(use_cuda=True, backend='torch_native')
        g = torch.Generator(device='cuda').manual_seed(0)
        n = int(n)
        u = torch.rand((n, n, n), device='cuda', generator=g).to(dt).requires_grad_(True)
        d = (torch.rand((n, n, n), device='cuda', generator=g) * 2 - 1).to(dt)
        for _ in range(4):
            (o,) = fn.apply(u)
            o.backward(d)
            u.grad = None
        torch.cuda.synchronize()
        print(spec, 'done', flush=True)


if __name__ == '__main__':
    main()
