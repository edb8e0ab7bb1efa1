"""Print the emitted HIP source of a workload's forward kernel for a shape (no GPU needed).

python scripts/probes/dump_kernel.py stencil27 768,768,768 [KEY=VAL,...] > k.hip
"""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pystencils_autodiff_amd import AutoDiffOp, workloads as W
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel, default_march_config

wl = {'stencil27': W.stencil_27pt, 'diffusion7': W.diffusion_7pt}[sys.argv[1]]
shape = tuple(int(v) for v in sys.argv[2].split(','))
tun = {}
if len(sys.argv) > 3 and sys.argv[3]:
    for kv in sys.argv[3].split(','):
        k, v = kv.split('=')
        tun[k] = int(v)
which = sys.argv[4] if len(sys.argv) > 4 else 'forward'
op = AutoDiffOp(wl(), boundary_handling='zeros')
asg = op.forward_assignments if which == 'forward' else op.backward_assignments
k = StencilKernel(asg, boundary_handling='zeros', function_name='probe', target='gpu', gpu_indexing_params=tun)
hk = HipStencilKernel(k)
cfg = default_march_config(hk.ir, hk._vec_elems(), shape, tun)
print(hk.source(('march', cfg))[0])
print('//', cfg, file=sys.stderr)
