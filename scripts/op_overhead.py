"""Python-side cost of one Op.apply + backward on a tiny field (launch-bound), with cProfile."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    op = pa.AutoDiffOp(W.readme_op(), boundary_handling=None)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    x = (torch.rand(20, 30, device='cuda') + 0.5).requires_grad_(True)
    y = (torch.rand(20, 30, device='cuda') + 0.5).requires_grad_(True)
    g = torch.rand(20, 30, device='cuda')

    def step():
        (z,) = fn.apply(x, y)
        z.backward(g)
        x.grad = None
        y.grad = None
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    print(f"apply+backward: {(time.perf_counter() - t0) / n * 1e6:.1f} us per step")
    t0 = time.perf_counter()
    for _ in range(n):
        (z,) = fn.apply(x.detach(), y.detach())
    torch.cuda.synchronize()
    print(f"apply (no grad): {(time.perf_counter() - t0) / n * 1e6:.1f} us per call")
    # floor: a torch autograd.Function of the same shape (one elementwise kernel each way)
    class TorchFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, a, b):
            ctx.save_for_backward(a, b)
            return a * b

        @staticmethod
        def backward(ctx, gz):
            a, b = ctx.saved_tensors
            return gz * b, gz * a
    for _ in range(50):
        (TorchFn.apply(x, y)).backward(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        TorchFn.apply(x, y).backward(g)
        x.grad = None
        y.grad = None
    torch.cuda.synchronize()
    print(f"torch Function (1 mul fwd, 2 mul bwd) apply+backward: {(time.perf_counter() - t0) / n * 1e6:.1f} us per step")
    # host time of the two halves separately (kernels are tiny and asynchronous)
    ta = tb = 0.0
    for _ in range(n):
        t0 = time.perf_counter()
        (z,) = fn.apply(x, y)
        t1 = time.perf_counter()
        z.backward(g)
        t2 = time.perf_counter()
        x.grad = None
        y.grad = None
        ta += t1 - t0
        tb += t2 - t1
    torch.cuda.synchronize()
    print(f"host time: apply {ta / n * 1e6:.1f} us, backward {tb / n * 1e6:.1f} us")
    ta = tb = 0.0
    for _ in range(n):
        t0 = time.perf_counter()
        zz = TorchFn.apply(x, y)
        t1 = time.perf_counter()
        zz.backward(g)
        t2 = time.perf_counter()
        x.grad = None
        y.grad = None
        ta += t1 - t0
        tb += t2 - t1
    torch.cuda.synchronize()
    print(f"host time torch Function: apply {ta / n * 1e6:.1f} us, backward {tb / n * 1e6:.1f} us")
    # our backward body alone, called directly (no engine)
    (z,) = fn.apply(x, y)
    node = z.grad_fn
    t0 = time.perf_counter()
    for _ in range(n):
        node.apply(g)
    torch.cuda.synchronize()
    print(f"backward node.apply (no engine): {(time.perf_counter() - t0) / n * 1e6:.1f} us per call")
    k = op.forward_ast_gpu.compile()
    z = torch.empty(20, 30, device='cuda')
    t0 = time.perf_counter()
    for _ in range(n):
        k(x=x.detach(), y=y.detach(), z=z)
    torch.cuda.synchronize()
    print(f"kernel call: {(time.perf_counter() - t0) / n * 1e6:.1f} us per call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(500):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(25)


if __name__ == '__main__':
    main()
