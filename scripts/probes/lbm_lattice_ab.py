"""LBM schedules, same process, HIP events: the AutoDiffOp one-thread-per-cell kernels (fzyx planes) against the
lattice kernels (``lbm/_lattice_kernels.py``) on fzyx planes and on the row-interleaved ``[z][y][q][x]`` layout, with
and without walls; forward and adjoint; GB/s of algorithmic bytes (fwd 2·q, adjoint 3·q values per cell).
python scripts/probes/lbm_lattice_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, reps=20):
    import torch
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def main():
    import numpy as np
    import torch

    from pystencils_autodiff_amd import AutoDiffOp
    from pystencils_autodiff_amd.lbm import LBStencil, create_lb_update_rule
    from pystencils_autodiff_amd.lbm._lattice_kernels import LatticeKernels, neighbour_mask, row_interleaved_empty
    from pystencils_autodiff_amd.lbm._method import create_lb_adjoint_rule
    cases = [('D3Q19', (192, 192, 192)), ('D2Q9', (2048, 2048))]
    if len(sys.argv) > 1:
        cases = [c for c in cases if c[0] in sys.argv[1:]]
    for name, shape in cases:
        st = LBStencil(name)
        Q = st.Q
        cells = int(np.prod(shape))
        fb, ab = 2 * Q * 4 * cells, 3 * Q * 4 * cells

        def fzyx():
            return torch.rand([Q] + list(shape), device='cuda').permute(*range(1, len(shape) + 1), 0)

        def rowi():
            t = row_interleaved_empty(shape, Q, torch.float32, 'cuda')
            t.copy_(torch.rand(t.shape, device='cuda'))
            return t
        rule = create_lb_update_rule(name, data_type='float32')
        op = AutoDiffOp(rule, 'LBM', boundary_handling='periodic', diff_mode='transposed',
                        backward_assignments=create_lb_adjoint_rule(rule))
        kf, kb = op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
        s, d, g, o = fzyx(), fzyx(), fzyx(), fzyx()
        res = {}
        res['generic fwd'] = (timed(lambda: kf(src=s, dst=d, omega=1.6)), fb)
        res['generic adj'] = (timed(lambda: kb(src=s, diffdst=g, diffsrc=o, omega=1.6)), ab)
        wall = torch.zeros(shape, dtype=torch.uint8, device='cuda')
        wall[:, 0] = 1
        wall[:, -1] = 1
        mask = neighbour_mask(wall, st, torch)
        for walls in (False, True):
            K = LatticeKernels(st, False, np.float32, walls, 'gpu')
            fl = mask if walls else None
            tag = ' walls' if walls else ''
            res['lattice fzyx fwd' + tag] = (timed(lambda: K.forward(s, d, 1.6, fl)), fb)
            res['lattice fzyx adj' + tag] = (timed(lambda: K.adjoint(s, g, o, 1.6, fl)), ab)
            rs, rd, rg, ro = rowi(), rowi(), rowi(), rowi()
            res['lattice rowi fwd' + tag] = (timed(lambda: K.forward(rs, rd, 1.6, fl)), fb)
            res['lattice rowi adj' + tag] = (timed(lambda: K.adjoint(rs, rg, ro, 1.6, fl)), ab)
        x = torch.rand(cells * Q, device='cuda')
        y = torch.empty_like(x)
        res['torch mul (2q values/cell)'] = (timed(lambda: torch.mul(x, 2.0, out=y)), fb)
        for k, (ms, b) in res.items():
            print(f'{name} {shape}: {k:32s} {ms:.4f} ms  {b / ms / 1e6:7.0f} GB/s  {b / ms / 1e6 / 8000:.3f}',
                  flush=True)


if __name__ == '__main__':
    main()
