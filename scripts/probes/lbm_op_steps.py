"""The LBM time-step op's overhead over its kernels: HIP events around Op.apply / backward (as bench_configs),
host enqueue time of the same calls (no sync), and the bare lattice kernels in the op's layouts (fzyx input →
row-interleaved states → fzyx output). Run under ``rocprofv3 --kernel-trace`` for the per-launch timeline.
python scripts/probes/lbm_op_steps.py [D2Q9|D3Q19 ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from pystencils_autodiff_amd import lbm
    from pystencils_autodiff_amd.lbm._lattice_kernels import row_interleaved_empty
    cases = [('D2Q9', (2048, 2048)), ('D3Q19', (192, 192, 192))]
    if len(sys.argv) > 1:
        cases = [c for c in cases if c[0] in sys.argv[1:]]
    T = 10
    for name, shape in cases:
        rule = lbm.create_lb_update_rule(name, data_type='float32')
        step = lbm.AutoDiffLatticeBoltzmannStep(rule, domain_size=shape, relaxation_rate=1.5, target='gpu')
        Op = step.create_timestep_op(T)
        q = rule.stencil.Q
        cells = 1
        for n in shape:
            cells *= n
        x = step.empty_pdfs()
        x.copy_(torch.rand(tuple(shape) + (q,), device='cuda') * 0.01 + 1.0 / q)
        x.requires_grad_(True)
        gr = step.empty_pdfs()
        gr.copy_(torch.rand(tuple(shape) + (q,), device='cuda'))

        def one():
            Op.apply(x).backward(gr)
            x.grad = None
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.4:
            one()
        torch.cuda.synchronize()
        fw, bw, hf, hb = [], [], [], []
        for _ in range(9):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            h0 = time.perf_counter()
            out = Op.apply(x)
            h1 = time.perf_counter()
            e1.record()
            h2 = time.perf_counter()
            out.backward(gr)
            h3 = time.perf_counter()
            e2.record()
            torch.cuda.synchronize()
            x.grad = None
            fw.append(e0.elapsed_time(e1))
            bw.append(e1.elapsed_time(e2))
            hf.append((h1 - h0) * 1e3)
            hb.append((h3 - h2) * 1e3)

        def med(v):
            return sorted(v)[len(v) // 2]
        fb, ab = 2 * q * 4 * cells * T, 3 * q * 4 * cells * T
        print(f'{name} {shape} op T={T}: fwd {med(fw):.4f} ms ({fb / med(fw) / 1e6 / 8000:.3f} of 8 TB/s), host '
              f'{med(hf):.4f} ms; bwd {med(bw):.4f} ms ({ab / med(bw) / 1e6 / 8000:.3f}), host {med(hb):.4f} ms',
              flush=True)
        # bare kernels in the op's layouts
        K = step._lattice_kernels()
        a = step.empty_pdfs()
        a.copy_(x.detach())
        r1, r2, r3 = (row_interleaved_empty(shape, q, torch.float32, 'cuda') for _ in range(3))
        r1.copy_(a)
        o = step.empty_pdfs()
        g2 = step.empty_pdfs()
        g2.copy_(gr)

        def timed(fn, reps=20):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ev = []
            for _ in range(reps):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                ev.append((s, e))
            torch.cuda.synchronize()
            return med([s.elapsed_time(e) for s, e in ev])
        om = step._omega_of()
        kf = {'fzyx->rowi': timed(lambda: K.forward(a, r2, om)), 'rowi->rowi': timed(lambda: K.forward(r1, r2, om)),
              'rowi->fzyx': timed(lambda: K.forward(r1, o, om))}
        ka = {'g fzyx, out rowi, src rowi': timed(lambda: K.adjoint(r1, g2, r2, om)),
              'g rowi, out rowi, src rowi': timed(lambda: K.adjoint(r1, r2, r3, om)),
              'g rowi, out fzyx, src fzyx': timed(lambda: K.adjoint(a, r1, o, om))}
        kf_sum = kf['fzyx->rowi'] + (T - 2) * kf['rowi->rowi'] + kf['rowi->fzyx']
        ka_sum = ka['g fzyx, out rowi, src rowi'] + (T - 2) * ka['g rowi, out rowi, src rowi'] + \
            ka['g rowi, out fzyx, src fzyx']
        for k, v in list(kf.items()) + list(ka.items()):
            print(f'  kernel {k:28s} {v:.4f} ms', flush=True)
        print(f'  sum of the op\'s kernels: fwd {kf_sum:.4f} ms ({fb / kf_sum / 1e6 / 8000:.3f}), adjoint {ka_sum:.4f} '
              f'ms ({ab / ka_sum / 1e6 / 8000:.3f})', flush=True)


if __name__ == '__main__':
    main()
