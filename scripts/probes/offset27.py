"""Does the relative placement of the 27-point sweep's input and output arrays matter (HBM channel
conflicts between the plane being read and the plane being written)? The 768³ fp16 forward kernel with
``out`` placed at byte offsets from a fresh allocation, HIP events, same process, interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from pystencils_autodiff_amd import AutoDiffOp
    from pystencils_autodiff_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    op = AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    cells = n ** 3
    u = torch.rand((n, n, n), device='cuda').half()
    offs = [0, 256, 4096, 65536, 1 << 20, 3 << 20]       # bytes
    bufs = {o: torch.empty(cells + o // 2 + 64, dtype=torch.float16, device='cuda') for o in offs}
    outs = {o: bufs[o][o // 2:o // 2 + cells].view(n, n, n) for o in offs}
    for o in offs:
        k(u=u, out=outs[o])
    torch.cuda.synchronize()
    res = {o: [] for o in offs}
    for _ in range(5):
        for o in offs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                k(u=u, out=outs[o])
            e1.record()
            torch.cuda.synchronize()
            res[o].append(e0.elapsed_time(e1) / 4)
    base = torch.equal(outs[0], outs[offs[1]])
    for o in offs:
        v = sorted(res[o])
        print(f'out offset {o:8d} B: median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f} ms', flush=True)
    print('outputs equal across offsets:', base)


if __name__ == '__main__':
    main()
