"""Adjoint of the variable-coefficient diffusion (three fields read, two written, 512³ fp32) as a function of where
its five arrays start relative to each other: one allocation each (the caching allocator's 2 MiB-aligned blocks,
equal strides apart), and views into padded blocks with array i shifted by i × a stagger. Interleaved rounds in one
process, HIP events, median of 20. Timing only (the default schedule's kernel, same code for every layout).

python scripts/probes/stagger_ab.py [n=512] [rounds=3]
python scripts/probes/stagger_ab.py 1024 3 diffusion7     (the headline's forward: u read, out written)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

STAGGERS = [0, 4096, 65536 + 256, 1 << 20, (1 << 20) + 4096 * 3, 256, 2048]


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


HEADLINE_STAGGERS = [0, 1024, 2048, 4096, 8192, 12288, 16384, 32768, 65536, 131072, 262144, 524288, 1 << 20,
                     (1 << 20) + 4096]


def headline(shape, rounds):
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    fk = op.forward_ast_gpu.compile()
    layouts = {}
    for s in HEADLINE_STAGGERS:
        keep = []
        layouts[s] = (arrays(shape, s, keep, 2), keep)
    for r in range(rounds):
        line = []
        for s, ((u, o), _) in layouts.items():
            line.append(f'{s:>8d}: {timed(lambda: fk(u=u, out=o)):.4f}')
        print(f'diffusion7 {shape[0]}^3 forward round {r} (stagger bytes: ms) ' + ' | '.join(line), flush=True)


def arrays(shape, stagger, keep, count=5):
    n = shape[0] * shape[1] * shape[2]
    out = []
    for i in range(count):
        pad = (i * stagger) // 4
        blk = torch.rand(n + pad + 64, device='cuda')
        keep.append(blk)
        out.append(blk[pad:pad + n].view(shape))
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    shape = (n, n, n)
    if len(sys.argv) > 3 and sys.argv[3] == 'diffusion7':
        return headline(shape, rounds)
    op = pa.AutoDiffOp(W.varcoef_diffusion_7pt(), boundary_handling='zeros')
    fk, bk = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
    layouts = {}
    for s in STAGGERS:
        keep = []
        layouts[s] = (arrays(shape, s, keep), keep)
    for r in range(rounds):
        line = []
        for s, ((u, k, d, a, b), _) in layouts.items():
            tb = timed(lambda: bk(u=u, k=k, diffout=d, diffu=a, diffk=b))
            tf = timed(lambda: fk(u=u, k=k, out=a))
            line.append(f'{s:>8d}: fwd {tf:.4f} bwd {tb:.4f}')
        print(f'varcoef {n}^3 round {r} (stagger bytes: ms) ' + ' | '.join(line), flush=True)
    ptrs = {s: [hex(t.data_ptr() % (1 << 24)) for t in arrs] for s, (arrs, _) in layouts.items()}
    print('array start mod 16 MiB:', ptrs)


if __name__ == '__main__':
    main()
