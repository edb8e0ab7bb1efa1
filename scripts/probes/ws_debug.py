"""Debug helper: a shifted-copy stencil through the WS zsum schedule, reports where it differs."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pystencils_autodiff_amd import ps  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else 'float16'
params = dict(kv.split('=') for kv in sys.argv[2].split(',')) if len(sys.argv) > 2 else {}
params = {k: int(v) for k, v in params.items()}
shape = (6, 9, 72)
for off in ((1, 0, 0), (0, 1, 0), (0, 0, 1), (0, 0, 0)):
    u, out = ps.fields(f"u, out: {dt}[3d]")
    ac = ps.AssignmentCollection({out.center: 1.0 * u[off] + (0.5 * u[-1, 0, 0] if off == (0, 0, 0) else 0)})
    k = StencilKernel(ac, boundary_handling='zeros', function_name='dbg', target='gpu',
                      gpu_indexing_params=dict(ZSUM=1, WS=1, **params)).compile()
    a = (np.arange(np.prod(shape)) % 1000).reshape(shape).astype(dt)
    ta = torch.from_numpy(a).cuda()
    o = torch.full(shape, -1.0, dtype=ta.dtype, device='cuda')
    k(u=ta, out=o)
    torch.cuda.synchronize()
    got = o.float().cpu().numpy()
    pad = np.zeros(tuple(s + 2 for s in shape), dtype=np.float64)
    pad[1:-1, 1:-1, 1:-1] = a
    ref = pad[1 + off[0]:1 + off[0] + shape[0], 1 + off[1]:1 + off[1] + shape[1], 1 + off[2]:1 + off[2] + shape[2]]
    if off == (0, 0, 0):
        ref = ref + 0.5 * pad[0:shape[0], 1:-1, 1:-1]
    bad = np.argwhere(np.abs(got - ref) > 1e-3 * np.abs(ref).max())
    print(off, k.last_variant[1], 'bad', len(bad), bad[:6].tolist(), [(got[tuple(b)], ref[tuple(b)]) for b in bad[:6]])
