"""Band schedule on / off through the drop-in op (fn.apply + backward, the native autograd node), same process,
settled A/B rounds: op A plans its kernels with PSAD_BAND=0 (zsum ring), op B with the band default.

python scripts/probes/op_band_ab.py [workload:edge[:PSAD_MARCH variant ...] ...]
  e.g. f7:512 s27:768 s27:1024:BTRIM=0,ZMIN=48,ZMAX=48:ZMIN=48,ZMAX=48 s27:96x768 (a slab) s27:512x510x512 (Z x Y x X)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd.backends import hip_kernel as HK  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

WL = {'f7': (W.diffusion_7pt, torch.float32), 'h7': (lambda: W.diffusion_7pt(dtype='float16'), torch.float16),
      's27': (W.stencil_27pt, torch.float16), 'f27': (lambda: W.stencil_27pt(dtype='float32'), torch.float32)}


_INPUTS = {}


def inputs(name, n):
    """One (u, diffout) pair per workload and size, shared by every variant: the variants differ in the kernels
    only, not in where their inputs sit in HBM (at 512³ fp32 two equal configurations on separately allocated
    inputs measured 0.357 vs 0.378 ms, profiles/r04_op_f7_ab.log)."""
    key = (name, n)
    if key not in _INPUTS:
        _INPUTS.clear()
        dt = WL[name][1]
        g = torch.Generator(device='cuda').manual_seed(0)
        shape = (n if len(n) == 3 else (n[0], n[1], n[1])) if isinstance(n, tuple) else (n, n, n)
        u = torch.rand(shape, device='cuda', generator=g).to(dt).requires_grad_(True)
        d = (torch.rand(shape, device='cuda', generator=g) * 2 - 1).to(dt)
        _INPUTS[key] = (u, d)
    return _INPUTS[key]


def make(name, n, band, march=''):
    b, dt = WL[name]
    os.environ['PSAD_BAND'] = '1' if band else '0'
    # ablation knobs (wrong results, timing only) go through the probe-only entry, the rest through PSAD_MARCH
    kv = [t for t in march.split(',') if t]
    HK.PROBE_KNOBS.clear()
    HK.PROBE_KNOBS.update({t.split('=')[0]: int(t.split('=')[1]) for t in kv if t.split('=')[0] in HK.PROBE_KEYS})
    tile = ','.join(t for t in kv if t.split('=')[0] not in HK.PROBE_KEYS)
    if tile:
        os.environ['PSAD_MARCH'] = tile
    op = pa.AutoDiffOp(b(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    u, d = inputs(name, n)

    def step():
        (o,) = fn.apply(u)
        o.backward(d)
        u.grad = None
    step()
    torch.cuda.synchronize()
    cfg = op.forward_ast_gpu.compile().last_variant[1]
    os.environ.pop('PSAD_BAND', None)
    if cfg.BAND:
        march = f'{march} BMASK={int(cfg.BMASK)} BPAD={cfg.BPAD} ZC={cfg.ZMIN}'.strip()
    os.environ.pop('PSAD_MARCH', None)
    HK.PROBE_KNOBS.clear()
    return step, f'BAND={cfg.BAND} BTY={cfg.BTY} {march}'


def main():
    torch.autograd.set_multithreading_enabled(False)
    for spec in sys.argv[1:] or ['f7:512', 'f7:768', 's27:768', 'h7:768']:
        name, n, *extra = spec.split(':')
        n = tuple(int(v) for v in n.split('x')) if 'x' in n else int(n)      # 'ZxN' = a Z x N x N slab
        runs = [make(name, n, False), make(name, n, True)] + [make(name, n, True, m) for m in extra]
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.0:
            runs[0][0]()
        torch.cuda.synchronize()
        res = [[] for _ in runs]
        for _ in range(5):
            for i, (fn, _) in enumerate(runs):
                for _ in range(10):
                    fn()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    fn()
                b.record()
                torch.cuda.synchronize()
                res[i].append(a.elapsed_time(b) / 20)
        for (fn, tag), r in zip(runs, res):
            v = sorted(r)
            print(f'{spec.split(":")[0]}:{str(n):<9s} {tag:44s} fwd+bwd {v[2]:.4f} ms  [{" ".join(f"{x:.4f}" for x in r)}]', flush=True)


if __name__ == '__main__':
    main()
