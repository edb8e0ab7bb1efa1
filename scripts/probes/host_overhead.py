"""Host-side cost per call of the drop-in op on tiny fields (GPU work is negligible there):
raw compiled-kernel call, Function.apply, apply+backward; plus a cProfile of apply+backward."""
import cProfile
import pstats
import sys
import time

import torch

import pystencils_autodiff_amd as pa
from pystencils_autodiff_amd import workloads as W
from pystencils_autodiff_amd.backends import hip_runtime as rt


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    k = op.forward_ast_gpu.compile()
    u = torch.rand((8, 8, 64), device='cuda')
    out = torch.empty_like(u)
    d = torch.rand_like(u)
    k(u=u, out=out)
    plan = next(iter(k._plans.values()))
    packed = plan.pack([u.data_ptr(), out.data_ptr()], [], [0.1] * len(k.ir.scalars))
    stream = torch._C._cuda_getCurrentRawStream(0)
    res = {}
    res['rt.launch'] = per_call(lambda: rt.launch(plan.fn, (plan.grid,), (plan.block,), packed, stream))
    res['compiled(...)'] = per_call(lambda: k(u=u, out=out))
    res['torch.empty_like'] = per_call(lambda: torch.empty_like(u))
    with torch.no_grad():
        res['apply (no_grad)'] = per_call(lambda: fn.apply(u))
    uu = u.clone().requires_grad_(True)
    res['apply'] = per_call(lambda: fn.apply(uu))

    def step():
        (o,) = fn.apply(uu)
        o.backward(d)
        uu.grad = None
    res['apply+backward'] = per_call(step)
    res['torch mul+backward'] = per_call(lambda: (uu * 2.0).backward(d))

    class Twice(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 2.0

        @staticmethod
        def backward(ctx, g):
            return g * 2.0
    res['py Function mul+backward'] = per_call(lambda: Twice.apply(uu).backward(d))
    lib = rt.lib()

    def mk(body):
        class F(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x):
                return x * 2.0

            @staticmethod
            def backward(ctx, g):
                return body(g)
        return F

    def b_kernel(g):
        o = torch.empty_like(g)
        k(u=g, out=o)
        return o

    def b_launch(g):
        o = torch.empty_like(g)
        rt.launch(plan.fn, (plan.grid,), (plan.block,), packed, stream)
        return o

    def b_ctypes(g):
        lib.psad_abi_version()
        return g * 2.0

    def b_stream(g):
        torch._C._cuda_getCurrentRawStream(0)
        return g * 2.0
    for nm, b in (('kernel', b_kernel), ('rt.launch', b_launch), ('ctypes noop', b_ctypes), ('raw stream', b_stream)):
        F = mk(b)
        res[f'Function bwd={nm}'] = per_call(lambda: F.apply(uu).backward(d))
    torch.autograd.set_multithreading_enabled(False)
    res['apply+backward (1 thread)'] = per_call(step)
    res['py Function (1 thread)'] = per_call(lambda: Twice.apply(uu).backward(d))
    torch.autograd.set_multithreading_enabled(True)
    for k_, v in res.items():
        print(f'{k_:24s} {v:8.1f} us')
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2000):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr, stream=sys.stdout).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
