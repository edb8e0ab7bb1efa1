"""The native z-slab sweep when every HIP stream shares one hardware queue (run under GPU_MAX_HW_QUEUES=1): the
cross-stream orderings must be ENQUEUED in a satisfiable order (a wait packet ahead of the launch or write that
satisfies it in one queue never completes), for every sync mode. Runs a few fwd+bwd steps of a 27-point fp16 and a
7-point fp32 slab on a loopback communicator per mode and compares with the Python sweeps bitwise.

GPU_MAX_HW_QUEUES=1 timeout -k 10 120 python scripts/probes/slab_shared_queue.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
import pystencils_autodiff_amd as pa  # noqa: E402
from pystencils_autodiff_amd import workloads as W  # noqa: E402
from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp  # noqa: E402


def run(builder, shape, dt, env):
    for k, v in env.items():
        os.environ[k] = v
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    g = torch.Generator(device='cuda').manual_seed(3)
    u = torch.rand(shape, device='cuda', generator=g).to(dt)
    d = (torch.rand(shape, device='cuda', generator=g) * 2 - 1).to(dt)
    z = ZSlabOp(op, use_cuda=True)
    z._halo = RcclHalo(loopback=True)
    res = []
    try:
        z.warm_exchange(u=u, diffout=d)
        fn = z.autograd_function()
        for native in ('1', '1', '1', '0'):
            os.environ['PSAD_NATIVE_SLAB'] = native
            uu = u.clone().requires_grad_(True)
            (o,) = fn.apply(uu)
            o.backward(d)
            torch.cuda.synchronize()
            res.append((o.detach().clone(), uu.grad.clone()))
    finally:
        z.close()
        for k in env:
            os.environ.pop(k, None)
    ok = all(torch.equal(r[0], res[-1][0]) and torch.equal(r[1], res[-1][1]) for r in res[:-1])
    return ok


def main():
    print('GPU_MAX_HW_QUEUES', os.environ.get('GPU_MAX_HW_QUEUES'), flush=True)
    from pystencils_autodiff_amd import _psad_torch as P
    bad = 0
    for env in ({}, {'PSAD_SLAB_START_SIG': '0'}, {'PSAD_SLAB_FACE_WAIT': '1'}, {'PSAD_SLAB_SYNC': 'event'},
                {'PSAD_SLAB_SYNC': 'mixed'}):
        for name, builder, shape, dt in (('27pt f16', W.stencil_27pt, (24, 64, 256), torch.float16),
                                         ('7pt f32', W.diffusion_7pt, (20, 48, 128), torch.float32)):
            s0, w0 = P.num_start_signal_sweeps(), P.num_face_wait_sweeps()
            ok = run(builder, shape, dt, env)
            bad += not ok
            print(f'{name} {env}: {"bitwise equal to the Python sweeps" if ok else "MISMATCH"}; start-signal sweeps '
                  f'{P.num_start_signal_sweeps() - s0}, face-wait sweeps {P.num_face_wait_sweeps() - w0}', flush=True)
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
