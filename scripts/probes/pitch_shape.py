"""Row pitch vs plane pitch: the 27-point fp16 sweep (forward + adjoint through the op, HIP events, median of 20,
interleaved rounds in one process) on 512³ and on shapes that change only the row length (X = 511 / 510: rows off
the 1-KiB period, planes too) or only the plane size (Y = 511 / 510 with 1024-byte rows: planes off the power of
two, rows aligned). Timing only.  python scripts/probes/pitch_shape.py [rounds=3]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402

SHAPES = [(512, 512, 512), (512, 512, 511), (512, 512, 510), (512, 511, 512), (512, 510, 512), (511, 512, 512)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.autograd.set_multithreading_enabled(False)
    cases = []
    for shape in SHAPES:
        op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
        fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
        u = torch.rand(shape, device='cuda').half().requires_grad_(True)
        d = (torch.rand(shape, device='cuda') * 2 - 1).half()
        cases.append((shape, op, fn, u, d))
    for r in range(rounds):
        line = []
        for shape, op, fn, u, d in cases:
            for _ in range(5):
                (o,) = fn.apply(u)
                o.backward(d)
                u.grad = None
            fw, bw = [], []
            for _ in range(20):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record()
                (o,) = fn.apply(u)
                e[1].record()
                o.backward(d)
                e[2].record()
                torch.cuda.synchronize()
                u.grad = None
                fw.append(e[0].elapsed_time(e[1]))
                bw.append(e[1].elapsed_time(e[2]))
            fw.sort()
            bw.sort()
            cells = shape[0] * shape[1] * shape[2]
            t = fw[10] + bw[10]
            line.append(f"{'x'.join(map(str, shape))}: {fw[10]:.4f}/{bw[10]:.4f} ms "
                        f"({cells / (512 ** 3) * 1e3 / t * (t and 1):.0f} norm)")
        print(f'round {r}: ' + ' | '.join(line), flush=True)
    print('schedules:', [(c[0], c[1].forward_ast_gpu.compile().last_variant[0],
                          getattr(c[1].forward_ast_gpu.compile().last_variant[1], 'BAND', None)) for c in cases])


if __name__ == '__main__':
    main()
