"""Row-band schedule (hip_band) vs the zsum half ring through the kernels the op launches, same process, settled
A/B rounds (every variant timed once per round after a warm start). Checks each band variant against the zsum
result (|diff| <= 1e-3 max|ref|, the fp16 tolerance of the parity tests) before timing.

python scripts/probes/band_ab.py [case ...]   cases: s27_768 s27_1024 s7_768 s7_1024 slab27 slab7
(profiles/r03_band_ab*.log were taken while the emitter still had a trimmed-chunk-edge option, BTRIM, since removed:
its "notrim" rows are today's kernels.)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402

CASES = {
    's27_768': (W.stencil_27pt, (768, 768, 768)),
    's27_1024': (W.stencil_27pt, (1024, 1024, 1024)),
    's7_768': (lambda: W.diffusion_7pt(dtype='float16'), (768, 768, 768)),
    's7_1024': (lambda: W.diffusion_7pt(dtype='float16'), (1024, 1024, 1024)),
    'slab27': (W.stencil_27pt, (96, 768, 768)),
    'slab7': (lambda: W.diffusion_7pt(dtype='float16'), (128, 1024, 1024)),
    'f7_1024': (W.diffusion_7pt, (1024, 1024, 1024)),
    'f7_768': (W.diffusion_7pt, (768, 768, 768)),
    'f7_512': (W.diffusion_7pt, (512, 512, 512)),
}
VARIANTS_F32 = {
    'zsum (BAND=0)': {'BAND': 0},
    'band R4 TY4 D2 zc8': {'BAND': 4, 'BTY': 4, 'D': 2, 'ZMIN': 8, 'ZMAX': 8},
    'band R4 TY4 D2 zc24': {'BAND': 4, 'BTY': 4, 'D': 2, 'ZMIN': 24, 'ZMAX': 24},
    'band R4 TY4 D2 zc64': {'BAND': 4, 'BTY': 4, 'D': 2, 'ZMIN': 64, 'ZMAX': 64},
    'band R2 TY4 D2 zc16': {'BAND': 2, 'BTY': 4, 'D': 2, 'ZMIN': 16, 'ZMAX': 16},
    'band R4 TY4 D1 zc16': {'BAND': 4, 'BTY': 4, 'D': 1, 'ZMIN': 16, 'ZMAX': 16},
    'band R4 TY4 D2 nt16': {'BAND': 4, 'BTY': 4, 'D': 2, 'ZMIN': 16, 'ZMAX': 16},
}
VARIANTS = {
    'zsum (BAND=0)': {'BAND': 0},
    'band default': {},
    'band zc16': {'ZMIN': 16, 'ZMAX': 16},
    'band zc8': {'ZMIN': 8, 'ZMAX': 8},
    'band notrim zc48': {'ZMIN': 48, 'ZMAX': 48},
    'band zc24 (default)': {},
    'band notrim zc12': {'ZMIN': 12, 'ZMAX': 12},
    'band R4 TY8 D2 nt': {'BAND': 4, 'BTY': 8, 'D': 2, 'ZMIN': 48, 'ZMAX': 48},
    'band R2 TY4 D3 nt': {'BAND': 2, 'BTY': 4, 'D': 3, 'ZMIN': 48, 'ZMAX': 48},
}


def timed(fn, reps=20):
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    v = sorted(x.elapsed_time(y) for x, y in ev)
    return v[len(v) // 2]


def settle(fn, sec):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < sec:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()


def main():
    cases = sys.argv[1:] or ['s27_768', 'slab27', 's7_768', 's27_1024']
    for case in cases:
        builder, shape = CASES[case]
        op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
        g = torch.Generator(device='cuda').manual_seed(0)
        for which, ac in (('fwd', op.forward_assignments), ('bwd', op.backward_assignments)):
            runs = []
            ref = None
            for vname, tun in (VARIANTS_F32 if case.startswith('f7') else VARIANTS).items():
                try:
                    k = StencilKernel(ac, boundary_handling='zeros', function_name=f'ab_{which}',
                                      target='gpu', gpu_indexing_params=tun).compile()
                except ValueError as e:
                    print(f'{case} {which} {vname}: {e}', flush=True)
                    continue
                dt = torch.float32 if case.startswith('f7') else torch.float16
                ins = {f.name: (torch.rand(shape, device='cuda', generator=g) * 2 - 1).to(dt)
                       for f in k.ir.fields_read} if ref is None else ins
                outs = {f.name: torch.full(shape, float('nan'), dtype=dt, device='cuda')
                        for f in k.ir.fields_written}
                try:
                    k(**ins, **outs)
                except ValueError as e:
                    print(f'{case} {which} {vname}: {e}', flush=True)
                    continue
                torch.cuda.synchronize()
                (o,) = outs.values()
                cfg = k.last_variant[1]
                tag = f'BAND={cfg.BAND} BTY={cfg.BTY} D={cfg.D} zc={k.last_plan.statics[9] if k.last_plan else "?"}'
                if ref is None:
                    ref = o.float()
                    err = 0.0
                else:
                    err = float((o.float() - ref).abs().max()) / max(1e-30, float(ref.abs().max()))
                    if not err <= (1e-6 if dt == torch.float32 else 1e-3):
                        print(f'{case} {which} {vname}: MISMATCH rel err {err:.3e}', flush=True)
                        continue
                runs.append((f'{case} {which} {vname:16s} {tag:32s} err {err:.1e}', (lambda k=k, a={**ins, **outs}: k(**a))))
            settle(runs[0][1], 1.0)
            res = {lab: [] for lab, _ in runs}
            for _ in range(4):
                for lab, fn in runs:
                    settle(fn, 0.1)
                    res[lab].append(timed(fn))
            nbytes = 2 * (4 if case.startswith('f7') else 2) * shape[0] * shape[1] * shape[2]
            for lab, _ in runs:
                v = sorted(res[lab])
                med = (v[1] + v[2]) / 2
                print(f'{lab} {med:.4f} ms {nbytes / med / 1e6:6.0f} GB/s  [{" ".join(f"{x:.4f}" for x in res[lab])}]',
                      flush=True)


if __name__ == '__main__':
    main()
