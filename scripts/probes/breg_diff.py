"""Where BREG=2 (staged loader) differs from BREG=0 on a ragged-band shape: the first differing (z, y, x) cells.
python scripts/probes/breg_diff.py [Z,Y,X]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402


def main():
    shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '6,13,510').split(','))
    op = pa.AutoDiffOp(W.diffusion_7pt(dtype='float16'), boundary_handling='zeros')
    g = torch.Generator().manual_seed(5)
    u = (torch.rand(shape, generator=g) * 2 - 1).half().cuda()
    res = {}
    for breg in (0, 2):
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='bd', target='gpu',
                          gpu_indexing_params={'BAND': 4, 'BREG': breg}).compile()
        o = torch.full_like(u, float('nan'))
        k(u=u, out=o)
        torch.cuda.synchronize()
        res[breg] = o
        print(breg, k.last_variant[1])
    d = (res[0].float() - res[2].float()).abs()
    bad = torch.nonzero(~(d == 0))
    print('differing cells', bad.shape[0], 'rows', sorted(set(bad[:, 1].tolist()))[:20], 'x', sorted(set(bad[:, 2].tolist()))[:20],
          'planes', sorted(set(bad[:, 0].tolist())))


if __name__ == '__main__':
    main()
