"""Sweep march-schedule tile shapes on the 1024³ 7-point forward sweep (interleaved rounds, one process).

python scripts/tune_march.py [--n 1024] [--rounds 5] [--configs "CX=2,WX=1,NR=2,ZC=512;..."]
Prints one line per config: median / min forward time and algorithmic GB/s. Kernel names carry the
config index (tune<i>_...) so a `rocprofv3 --pmc` run of this script attributes counters per config.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ';'.join([
    'CX=2,WX=1,NR=2,ZC=512', 'CX=2,WX=1,NR=2,ZC=64', 'CX=2,WX=1,NR=2,ZC=32', 'CX=2,WX=1,NR=2,ZC=16',
    'CX=2,WX=1,NR=4,ZC=512', 'CX=2,WX=1,NR=4,ZC=64', 'CX=2,WX=1,NR=4,ZC=32',
    'CX=4,WX=1,NR=2,ZC=512', 'CX=4,WX=1,NR=2,ZC=64', 'CX=4,WX=1,NR=4,ZC=64',
    'CX=1,WX=1,NR=4,ZC=64', 'CX=1,WX=1,NR=8,ZC=64', 'CX=2,WX=2,NR=4,ZC=64', 'CX=4,WX=1,NR=4,ZC=32',
    'CX=2,WX=1,NR=2,ZC=512,NT_STORE=1', 'CX=2,WX=1,NR=4,ZC=64,NT_STORE=1', 'CX=4,WX=1,NR=4,ZC=64,NT_STORE=1',
    'CX=2,WX=1,NR=8,ZC=64', 'CX=4,WX=1,NR=8,ZC=64',
])


def parse_cfg(s):
    d = {}
    if s.strip() == 'default':
        return d
    for kv in s.split(','):
        k, v = kv.split('=')
        k = k.strip()
        d[k] = {'0': 'zy', '1': 'yx'}.get(v.strip(), v.strip()) if k == 'VIEW2D' else int(v)
    return d


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--n', type=int, default=1024)
    p.add_argument('--rounds', type=int, default=5)
    p.add_argument('--reps', type=int, default=4)
    p.add_argument('--configs', default=DEFAULT)
    p.add_argument('--workload', default='diffusion7')
    p.add_argument('--configs-file')
    p.add_argument('--shape', help='Z,Y,X (overrides --n), e.g. 128,1024,1024 = one rank of 1024³ on 8 GPUs')
    a = p.parse_args()
    import torch

    from pystencils_autodiff_amd import AutoDiffOp
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel

    n = a.n
    builder = {'diffusion7': (W.diffusion_7pt, torch.float32), 'stencil27': (W.stencil_27pt, torch.float16),
               'laplace5': (W.laplace_5pt, torch.float32),
               'diffusion7_f64': (lambda: W.diffusion_7pt(dtype='float64'), torch.float64),
               'diffusion7_f16': (lambda: W.diffusion_7pt(dtype='float16'), torch.float16),
               'laplace5_f64': (lambda: W.laplace_5pt(dtype='float64'), torch.float64),
               'stencil27_f32': (lambda: W.stencil_27pt(dtype='float32'), torch.float32),
               'veclap3': (W.vector_laplace_7pt, torch.float32)}[a.workload]
    op = AutoDiffOp(builder[0](), boundary_handling='zeros')
    shape = (n, n) if a.workload == 'laplace5' else (n, n, n)
    if a.shape:
        shape = tuple(int(v) for v in a.shape.split(','))
    if a.workload == 'veclap3':
        shape = shape + (3,)
    cells = 1
    for s in shape:
        cells *= s
    esize = {torch.float16: 2, torch.float32: 4, torch.float64: 8}[builder[1]]
    u = torch.rand(shape, device='cuda').to(builder[1])
    out = torch.empty_like(u)
    spec = open(a.configs_file).read().strip() if a.configs_file else a.configs
    cfgs = [parse_cfg(s) for s in spec.split(';') if s.strip()]
    kernels = []
    for i, c in enumerate(cfgs):
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name=f'tune{i}',
                          target='gpu', gpu_indexing_params=c)
        ck = k.compile()
        ck(u=u, out=out)
        kernels.append(ck)
    ref = torch.empty_like(out)
    op_ref = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='tuneref', target='gpu')
    op_ref.compile()(u=u, out=ref, force_schedule='generic')
    torch.cuda.synchronize()
    maxdiff = [0.0] * len(cfgs)
    times = [[] for _ in cfgs]
    for r in range(a.rounds):
        for i, ck in enumerate(kernels):
            out.zero_()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                ck(u=u, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / a.reps)
            if r == 0:
                maxdiff[i] = (out.float() - ref.float()).abs().max().item()
    # achievable copy bandwidth in the same process (read+write of the same bytes)
    ct = []
    for _ in range(a.rounds):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out.copy_(u)
        e1.record()
        torch.cuda.synchronize()
        ct.append(e0.elapsed_time(e1))
    # a 16-byte-per-lane streaming copy through the emitter's pointwise schedule (out = u): the
    # practical read+write ceiling on this device, measured in the same process
    from pystencils_autodiff_amd import ps as _ps
    from pystencils_autodiff_amd.backends import hip_emitter as _he
    cu, co = _ps.fields(f"cu, co: {str(u.dtype).replace('torch.', '')}[{len(shape) if a.workload != 'veclap3' else 3}d]")
    if a.workload == 'veclap3':
        u, out = u.reshape(shape[0], shape[1], -1), out.reshape(shape[0], shape[1], -1)
    alg = 2 * esize * cells
    for nt_load, maxb in ((False, 2048), (True, 2048), (False, 0), (True, 0)):
        _he.POINTWISE_NT_LOAD = nt_load
        _he.POINTWISE_MAX_BLOCKS = maxb
        ck = StencilKernel(_ps.AssignmentCollection({co.center: cu.center}),
                           function_name=f'tunecopy{int(nt_load)}{maxb}', target='gpu').compile()
        ck(cu=u, co=out)
        pt = []
        for _ in range(a.rounds):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                ck(cu=u, co=out)
            e1.record()
            torch.cuda.synchronize()
            pt.append(e0.elapsed_time(e1) / a.reps)
        pmed = sorted(pt)[len(pt) // 2]
        print(f"pointwise copy{' (nt loads)' if nt_load else ''}{' one pass' if not maxb else ''}: median {pmed:.4f} ms = "
              f"{alg / (pmed * 1e-3) / 1e9:.0f} GB/s")
    _he.POINTWISE_NT_LOAD = True
    _he.POINTWISE_MAX_BLOCKS = 0
    # torch's own vectorised elementwise kernel (read + write of the same bytes) for reference
    mt = []
    for _ in range(a.rounds):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            torch.mul(u, 1.5, out=out)
        e1.record()
        torch.cuda.synchronize()
        mt.append(e0.elapsed_time(e1) / a.reps)
    mmed = sorted(mt)[len(mt) // 2]
    print(f"torch.mul (elementwise): median {mmed:.4f} ms = {alg / (mmed * 1e-3) / 1e9:.0f} GB/s")
    print(f"copy_: median {sorted(ct)[len(ct) // 2]:.4f} ms = {alg / (sorted(ct)[len(ct) // 2] * 1e-3) / 1e9:.0f} GB/s")
    for i, c in enumerate(cfgs):
        ts = sorted(times[i])
        med = ts[len(ts) // 2]
        plan = list(kernels[i]._plans.values())[-1]          # the launch actually timed
        geo = {'grid': plan.grid, 'zc': plan.statics[9]}
        print(f"tune{i:<3d} {','.join(f'{k}={v}' for k, v in c.items()) or 'default':34s} median {med:.4f} ms  min {ts[0]:.4f} ms  "
              f"{alg / (med * 1e-3) / 1e9:7.0f} GB/s  grid {geo['grid']} zc {geo['zc']}  maxdiff_vs_generic {maxdiff[i]:.2e}")
    sys.stdout.flush()


if __name__ == '__main__':
    main()
