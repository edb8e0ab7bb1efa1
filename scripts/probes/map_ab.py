"""Workgroup → tile mapping of the march schedule through the op, forward and adjoint: the XCD-aware remap
(``MAP=0``) against dispatch order (``MAP=1``), two ops on the same fields in one process, interleaved rounds,
HIP events around ``Op.apply`` / ``backward`` as ``scripts/bench_configs.py`` times them.
python scripts/probes/map_ab.py [workload:Z,Y,X ...]   (workloads: diffusion7, diffusion7_f16, diffusion7_f64,
stencil27)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CASES = ['diffusion7:384,384,384', 'diffusion7:512,512,512', 'diffusion7:640,640,640', 'diffusion7:768,768,768',
         'diffusion7:896,896,896', 'diffusion7:1024,1024,1024', 'diffusion7:128,1024,1024',
         'diffusion7:256,1024,1024', 'diffusion7:96,768,768', 'diffusion7_f16:768,768,768',
         'diffusion7_f16:1024,1024,1024', 'diffusion7_f64:512,512,512', 'diffusion7_f64:640,640,640']


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    builders = {'diffusion7': (W.diffusion_7pt, torch.float32),
                'diffusion7_f16': (lambda: W.diffusion_7pt(dtype='float16'), torch.float16),
                'diffusion7_f64': (lambda: W.diffusion_7pt(dtype='float64'), torch.float64),
                'stencil27': (W.stencil_27pt, torch.float16)}
    for case in (sys.argv[1:] or CASES):
        wl, sh = case.split(':')
        shape = tuple(int(v) for v in sh.split(','))
        b, dt = builders[wl]
        fns = []
        for m in (0, 1):
            op = pa.AutoDiffOp(b(), boundary_handling='zeros')
            for k in (op.forward_ast_gpu, op.backward_ast_gpu):
                k.tuning['MAP'] = m
            fns.append(op.create_tensorflow_op(use_cuda=True, backend='torch_native'))
        u = torch.rand(shape, device='cuda').to(dt).requires_grad_(True)
        d = (torch.rand(shape, device='cuda') * 2 - 1).to(dt)
        es = u.element_size()
        cells = u.numel()
        res = [([], []) for _ in fns]

        def one(fn):
            (o,) = fn.apply(u)
            o.backward(d)
            u.grad = None
        for r in range(4):
            for i, fn in enumerate(fns):
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.15:
                    one(fn)
                ev = []
                for _ in range(10):
                    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    e0.record()
                    (o,) = fn.apply(u)
                    e1.record()
                    o.backward(d)
                    e2.record()
                    u.grad = None
                    ev.append((e0, e1, e2))
                torch.cuda.synchronize()
                res[i][0].extend(a.elapsed_time(b_) for a, b_, _ in ev)
                res[i][1].extend(b_.elapsed_time(c) for _, b_, c in ev)

        def med(v):
            return sorted(v)[len(v) // 2]
        line = []
        for m, (f, bw) in enumerate(res):
            line.append(f'MAP={m} fwd {med(f):.4f} bwd {med(bw):.4f} ms ({2 * es * cells / med(f) / 1e9:.2f} / '
                        f'{2 * es * cells / med(bw) / 1e9:.2f} TB/s)')
        ratio = (med(res[1][0]) + med(res[1][1])) / (med(res[0][0]) + med(res[0][1]))
        print(f'{case:32s} ' + ' | '.join(line) + f' | MAP1/MAP0 {ratio:.3f}', flush=True)
        del fns, u, d
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
