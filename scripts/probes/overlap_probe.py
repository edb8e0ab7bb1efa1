"""Does a small kernel on a second stream (stand-in for RCCL's halo send/recv kernels) run while the
z-slab interior launch occupies every CU? Times the side kernel's completion relative to the start
of the interior launch (one rank of the 8-GPU 1024^3 run: 128x1024^2 fp32, planes 1..126)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
k = op.forward_ast_gpu.compile()
u = torch.rand((128, 1024, 1024), device='cuda')
out = torch.empty_like(u)
a = torch.rand((1, 1024, 1024), device='cuda')     # 4 MiB face
b = torch.empty_like(a)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for _ in range(3):
    with torch.cuda.stream(s1):
        k(u=u, out=out, z_range=(1, 127))
    with torch.cuda.stream(s2):
        b.copy_(a)
torch.cuda.synchronize()
res = []
for _ in range(10):
    e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    with torch.cuda.stream(s1):
        e0.record(s1)
        k(u=u, out=out, z_range=(1, 127))
        e1.record(s1)
    with torch.cuda.stream(s2):
        s2.wait_event(e0)
        b.copy_(a)
        e2.record(s2)
    torch.cuda.synchronize()
    res.append((e0.elapsed_time(e1), e0.elapsed_time(e2)))
torch.cuda.synchronize()
alone = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s2)
    b.copy_(a)
    e1.record(s2)
    torch.cuda.synchronize()
    alone.append(e0.elapsed_time(e1))
res.sort()
print('interior ms / side-copy done at ms (10 runs):', [(round(x, 4), round(y, 4)) for x, y in res])
print('side copy alone ms:', [round(x, 4) for x in alone])
print('variant:', k.last_variant[1])
