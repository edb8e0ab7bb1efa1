"""Where the autograd engine's device-thread hand-off costs time for a small op (2-D 5-point, 4096²).

Steady-state wall time per apply+backward step, default (multithreaded) engine, for:
  op        the drop-in op (Op.apply + backward)
  rawfn     a minimal Python autograd.Function launching the same two compiled kernels
  torchfn   a Python autograd.Function with torch elementwise kernels (u*2 / g*2)
  native    torch's own C++ autograd node (o = u*2)
  noop      a Python Function whose backward launches nothing
plus, for rawfn, the latency from ``backward()`` entry to the Python backward body and from its return
to ``backward()`` returning (device-thread wake-up / completion hand-off)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = 300
    op = pa.AutoDiffOp(W.laplace_5pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    fk = op.forward_ast_gpu.compile()
    bk = op.backward_ast_gpu.compile()
    u = torch.rand(n, n, device='cuda').requires_grad_(True)
    d = torch.rand(n, n, device='cuda')
    marks = {}

    class RawFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            o = torch.empty_like(x)
            fk(u=x, out=o)
            return o

        @staticmethod
        def backward(ctx, g):
            marks['b0'] = time.perf_counter()
            du = torch.empty_like(g)
            bk(diffout=g, diffu=du)
            marks['b1'] = time.perf_counter()
            return du

    class TorchFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 2

        @staticmethod
        def backward(ctx, g):
            return g * 2

    class NoopFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.view_as(x)

        @staticmethod
        def backward(ctx, g):
            return g

    def run(name, apply, leaf_grad=True):
        x = u if leaf_grad else u.detach().requires_grad_(True)

        def step():
            o = apply(x)
            o.backward(d)
            x.grad = None
        for _ in range(30):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e6
        ta = tb = 0.0
        enter = leave = 0.0
        for _ in range(steps):
            t0 = time.perf_counter()
            o = apply(x)
            t1 = time.perf_counter()
            o.backward(d)
            t2 = time.perf_counter()
            x.grad = None
            ta += t1 - t0
            tb += t2 - t1
            if 'b0' in marks:
                enter += marks['b0'] - t1
                leave += t2 - marks['b1']
        torch.cuda.synchronize()
        extra = ''
        if 'b0' in marks:
            extra = f", backward entry latency {enter / steps * 1e6:.1f} us, return latency {leave / steps * 1e6:.1f} us"
        marks.clear()
        print(f"{name:8s} {wall:7.1f} us/step wall; host apply {ta / steps * 1e6:.1f} us, "
              f"backward {tb / steps * 1e6:.1f} us{extra}", flush=True)

    for mt in (True, False):
        torch.autograd.set_multithreading_enabled(mt)
        print(f"-- autograd multithreading {'on' if mt else 'off'}")
        run('op', lambda x: fn.apply(x)[0])
        run('rawfn', RawFn.apply)
        run('torchfn', TorchFn.apply)
        run('native', lambda x: x * 2)
        run('noop', NoopFn.apply)
    # the same launches through a PyDLL handle: the foreign call keeps the GIL (ctypes.CDLL drops and
    # re-takes it around every call)
    import ctypes
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    P = ctypes.PyDLL(rt.library_path)
    P.psad_launch.argtypes = rt.lib().psad_launch.argtypes
    P.psad_launch.restype = ctypes.c_int
    cdll_launch = rt.launch

    def launch(fn_, grid, block, args_packed, stream, shared_bytes=0):
        gx, gy, gz = (tuple(grid) + (1, 1))[:3]
        bx, by, bz = (tuple(block) + (1, 1))[:3]
        rc = P.psad_launch(fn_, gx, gy, gz, bx, by, bz, shared_bytes, stream, args_packed, len(args_packed))
        if rc:
            raise RuntimeError(rc)
    rt.launch = launch
    for mt in (True, False):
        torch.autograd.set_multithreading_enabled(mt)
        print(f"-- PyDLL launch, autograd multithreading {'on' if mt else 'off'}")
        run('op', lambda x: fn.apply(x)[0])
        run('rawfn', RawFn.apply)
    rt.launch = cdll_launch


if __name__ == '__main__':
    main()
