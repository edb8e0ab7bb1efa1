"""fp16 sweeps at odd row lengths: 255³ / 257³ against 256³ (the half-precision LDS-DMA ring with rows on half dwords
shifted in LDS, XO) and the register-prefetch path they took before (PSAD_XO=0); HIP events, one process.
python scripts/probes/odd_rows.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel

    def timed(fn, reps=30):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        v = sorted(a.elapsed_time(b) for a, b in ev)
        return v[len(v) // 2]
    for name, builder in (('27pt_f16', W.stencil_27pt), ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16'))):
        for n in (256, 255, 257, 254, 258, 511, 512, 510):
            for xo in ('1', '0'):
                if n % 2 == 0 and xo == '0':
                    continue                      # (even rows: XM, dword-aligned, no realignment)
                os.environ['PSAD_XO'] = xo
                op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
                k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name=f'odd{xo}',
                                  target='gpu').compile()
                u = torch.rand((n, n, n), device='cuda').half()
                out = torch.empty_like(u)
                ms = timed(lambda: k(u=u, out=out))
                cfg = k.last_variant[1]
                print(f'{name} {n}^3 XO={xo}: {ms:.4f} ms  {4 * n ** 3 / ms / 1e6:6.0f} GB/s  '
                      f'(WS={cfg.WS} XM={cfg.XM} XO={cfg.XO} VE={cfg.VE} NR={cfg.NR} BAND={cfg.BAND})', flush=True)
                if cfg.BAND:
                    # the same size on the zsum ring (what the unaligned neighbours run on)
                    kz = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='oddz',
                                       target='gpu', gpu_indexing_params={'BAND': 0}).compile()
                    ms = timed(lambda: kz(u=u, out=out))
                    print(f'{name} {n}^3 zsum: {ms:.4f} ms  {4 * n ** 3 / ms / 1e6:6.0f} GB/s', flush=True)
                if os.environ.get('NR_SWEEP') and xo == '1':
                    for nr in (2, 4):
                        kt = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name=f'oddnr{nr}',
                                           target='gpu', gpu_indexing_params={'NR': nr}).compile()
                        ms = timed(lambda: kt(u=u, out=out))
                        c2 = kt.last_variant[1]
                        print(f'{name} {n}^3 NR={nr}: {ms:.4f} ms  {4 * n ** 3 / ms / 1e6:6.0f} GB/s  '
                              f'(WS={c2.WS} XM={c2.XM} XO={c2.XO} TX={c2.TX} TY={c2.TY})', flush=True)


if __name__ == '__main__':
    main()
