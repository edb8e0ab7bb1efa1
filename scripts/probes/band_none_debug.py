"""Band schedule, boundary_handling=None: where does it differ from the zsum ring? (debug)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

shape = (11, 24, 256)
op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling=None)
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, shape).astype(np.float16)).cuda()
res = {}
for tag, tun in (('band', {'BAND': 4}), ('zsum', {'BAND': 0}), ('bandnt', {'BAND': 4, 'BTRIM': 0})):
    k = StencilKernel(op.forward_assignments, boundary_handling=None, function_name='dbg_' + tag, target='gpu',
                      gpu_indexing_params=tun).compile()
    out = torch.zeros(shape, dtype=torch.float16, device='cuda')
    k(u=x, out=out)
    torch.cuda.synchronize()
    res[tag] = out.float().cpu().numpy()
    print(tag, k.last_variant[1].BAND, k.last_variant[1].BMASK, k.last_plan.statics, flush=True)
for tag in ('band', 'bandnt'):
    d = np.abs(res[tag] - res['zsum'])
    bad = np.argwhere(d > 1e-2)
    print(tag, 'bad cells', len(bad), 'of', d.size)
    if len(bad):
        zs, ys, xs = bad[:, 0], bad[:, 1], bad[:, 2]
        print(' z', sorted(set(zs.tolist())), '\n y', sorted(set(ys.tolist())), '\n x', sorted(set(xs.tolist()))[:40])
        z, y, xx = bad[0]
        print(' first', bad[0], res[tag][z, y, xx], res['zsum'][z, y, xx])
