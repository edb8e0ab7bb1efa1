"""Where an LBM time step's wall time goes: raw kernel launches vs the step's loop vs the timestep op,
with the host time of the Python calls (no sync) beside the synchronised wall time.

python scripts/probes/lbm_host.py [D2Q9|D3Q19] [edge]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from pystencils_autodiff_amd import lbm
    st = sys.argv[1] if len(sys.argv) > 1 else 'D3Q19'
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    shape = (n, n) if st == 'D2Q9' else (n, n, n)
    rule = lbm.create_lb_update_rule(st, data_type='float32')
    step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.5, target='gpu')
    q = rule.stencil.Q
    f0 = torch.full(shape + (q,), 1.0 / q, device='cuda')
    step.set_pdfs(f0)
    kf, kb = step._kernels()
    a, b = step._alloc(), step._alloc()
    T = 10

    def timed(label, fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f'{label:28s} host {1e3 * (t1 - t0) / T:8.4f} ms/step   wall {1e3 * (t2 - t0) / T:8.4f} ms/step')

    def raw():
        for _ in range(T):
            kf(src=a, dst=b, omega=1.5)
    timed('raw forward launches', raw)

    def raw_b():
        for _ in range(T):
            kb(src=a, diffdst=b, diffsrc=a, omega=1.5)
    timed('raw adjoint launches', raw_b)
    timed('step.run', lambda: step.run(T))
    timed('step.run(record)', lambda: step.run(T, record=True))
    Op = step.create_timestep_op(T)
    x = f0.clone().requires_grad_(True)
    g = torch.rand_like(f0)

    def op_fwd():
        Op.apply(x)
    timed('Op.apply', op_fwd)

    def op_both():
        out = Op.apply(x)
        out.backward(g)
        x.grad = None
    timed('Op.apply + backward', op_both)
    e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e[0].record()
    raw()
    e[1].record()
    torch.cuda.synchronize()
    print(f'forward kernels alone (events) {e[0].elapsed_time(e[1]) / T:.4f} ms/step')


if __name__ == '__main__':
    main()
