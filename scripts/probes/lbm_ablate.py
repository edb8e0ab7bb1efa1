"""What bounds the LBM D3Q19 forward kernel (generic schedule, periodic, fzyx planes): the full
stream-pull-collide launch vs a pure pull-streaming copy of the same planes (same shifted reads, no
collision) vs an unshifted plane copy, all through AutoDiffOp's periodic HIP kernels, HIP events, same
process. python scripts/probes/lbm_ablate.py [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import sympy as sp
    import torch

    from pystencils_autodiff_amd import AutoDiffOp, ps
    from pystencils_autodiff_amd.lbm import LBStencil, create_lb_update_rule
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    st = LBStencil('D3Q19')
    src, dst = ps.fields(f"src(19), dst(19): float32[3D]", layout='fzyx')
    rules = {
        'collide': create_lb_update_rule('D3Q19', relaxation_rate=sp.Symbol('omega'), data_type='float32',
                                         src_field=src, dst_field=dst),
        'pull_copy': ps.AssignmentCollection([ps.Assignment(dst.center(i), src[tuple(-c for c in st.directions[i])](i))
                                              for i in range(19)]),
        'plain_copy': ps.AssignmentCollection([ps.Assignment(dst.center(i), src.center(i)) for i in range(19)]),
        'pull_copy_x2': ps.AssignmentCollection([ps.Assignment(dst.center(i), 2 * src[tuple(-c for c in st.directions[i])](i))
                                                 for i in range(19)]),
    }
    cells = n ** 3

    def planes(pad):
        # the 19 component planes of an fzyx pdf array, plane stride n³ + pad elements
        buf = torch.rand(19 * (cells + pad), device='cuda')
        return buf.as_strided((n, n, n, 19), (n * n, n, 1, cells + pad))
    pads = [int(v) for v in os.environ.get('PADS', '0').split(',')]
    for pad in pads:
        s_t, d_t = planes(pad), planes(pad)
        run(rules, s_t, d_t, cells, f'pad {pad}')


def run(rules, s_t, d_t, cells, tag):
    import torch

    from pystencils_autodiff_amd import AutoDiffOp
    for name, ac in rules.items():
        op = AutoDiffOp(ac, 'abl', boundary_handling='periodic', diff_mode='transposed')
        k = op.forward_ast_gpu.compile()
        kw = {'src': s_t, 'dst': d_t}
        if any(s.name == 'omega' for s in k.ir.scalars):
            kw['omega'] = 1.6
        for _ in range(3):
            k(**kw)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            k(**kw)
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]
        gbs = cells * 19 * 4 * 2 / (ms * 1e-3) / 1e9
        print(f'{tag:10s} {name:14s} {ms:.4f} ms  {gbs:7.1f} GB/s  variant {k.last_variant}', flush=True)
    x = torch.rand(19 * cells, device='cuda')
    y = torch.empty_like(x)
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.mul(x, 2.0, out=y)
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]
    print(f'torch.mul      {ms:.4f} ms  {cells * 19 * 8 / (ms * 1e-3) / 1e9:7.1f} GB/s', flush=True)


if __name__ == '__main__':
    main()
