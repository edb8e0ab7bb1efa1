"""Where the time goes for the 2-D 5-point op at 4096² (kernel ≈ 0.022 ms per sweep): steady-state
wall time per apply+backward step vs host time of each half vs the raw kernels back to back, and the
same step with torch's autograd device thread off (backward in the calling thread).

Measured (profiles/r01_op_overhead_2d.log): 121.5 µs per step with the default multithreaded
engine (host: apply 44.5 µs, backward 71.4 µs — the engine's hand-off to its device thread), 44.6 µs
with multithreading off = the raw kernels back to back (44.5 µs): the op itself adds nothing the
GPU can see once the engine's thread hand-off is gone."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    op = pa.AutoDiffOp(W.laplace_5pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    u = torch.rand(n, n, device='cuda').requires_grad_(True)
    d = torch.rand(n, n, device='cuda')
    steps = 200

    def step():
        (o,) = fn.apply(u)
        o.backward(d)
        u.grad = None
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"op apply+backward: {(time.perf_counter() - t0) / steps * 1e6:.1f} us per step (wall, steady)")
    ta = tb = 0.0
    for _ in range(steps):
        t0 = time.perf_counter()
        (o,) = fn.apply(u)
        t1 = time.perf_counter()
        o.backward(d)
        t2 = time.perf_counter()
        u.grad = None
        ta += t1 - t0
        tb += t2 - t1
    torch.cuda.synchronize()
    print(f"host: apply {ta / steps * 1e6:.1f} us, backward {tb / steps * 1e6:.1f} us")
    fk = op.forward_ast_gpu.compile()
    bk = op.backward_ast_gpu.compile()
    out = torch.empty_like(d)
    du = torch.empty_like(d)
    uu = u.detach()
    for _ in range(5):
        fk(u=uu, out=out)
        bk(diffout=d, diffu=du)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fk(u=uu, out=out)
        bk(diffout=d, diffu=du)
    torch.cuda.synchronize()
    print(f"raw kernels fwd+bwd: {(time.perf_counter() - t0) / steps * 1e6:.1f} us per step")
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fk(u=uu, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(f"fwd kernel (events, back to back): {e0.elapsed_time(e1) / steps * 1e3:.1f} us")
    # backward in the calling thread (no engine device thread): wall time + a profile of both halves
    import cProfile
    import pstats
    torch.autograd.set_multithreading_enabled(False)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    print(f"op apply+backward, autograd multithreading off: {(time.perf_counter() - t0) / steps * 1e6:.1f} us per step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(22)


if __name__ == '__main__':
    main()
