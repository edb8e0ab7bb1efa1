"""Ablation of the 27-point fp16 half-ring kernel (n³ forward; argv: n [KEY=VAL,... tile overrides]): the default source, and copies edited
to drop work, launched through the same plan (same grid, chunks, arguments):
  full      - the shipped kernel
  fewfma    - every multiply-add chain keeps only its first term (≈1/9 of the FMAs)
  nocvt     - taps not converted (the fp16 dwords reinterpreted), FMAs kept
  memonly   - taps replaced by constants (the compiler folds the arithmetic): loader ring + barriers +
              stores of constants — the kernel's memory traffic alone (mem_plain: without nt; mem_x4: 16-byte
              stores from every other lane)
  nostore   - no output stores (the compiler then drops the arithmetic): loader ring + barriers + LDS reads
Prints median ms per variant (interleaved rounds)."""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from pystencils_autodiff_amd import AutoDiffOp, workloads as W
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    tun = dict((kv.split('=')[0], int(kv.split('=')[1])) for kv in sys.argv[2].split(',')) if len(sys.argv) > 2 else {}
    shape = (n, n, n)
    op = AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    u = torch.rand(shape, device='cuda').half()
    out = torch.empty_like(u)

    def fewfma(src):
        return re.sub(r'(= a\d+_\d+_\d+_\d+_\d+ \+ \([^;]*?\))( \+ \([^;]*?\))+;', r'\1;', src)

    def nocvt(src):
        return re.sub(r'\{\(float\)(h\w+)\[(\d)\], \(float\)(h\w+)\[(\d)\]\}',
                      r'{__builtin_bit_cast(float, \1) , __builtin_bit_cast(float, \3)}', src)

    def memonly(src):
        return re.sub(r'= \{\(float\)(h\w+)\[(\d)\], \(float\)(h\w+)\[(\d)\]\}', '= {0.5f, 0.25f}', src)

    def memonly_plain(src):
        return memonly(src).replace(', 0, 2);', ', 0, 0);')

    def memonly_x4(src):
        # 16-byte stores from every other lane (each covers its own quad and the next lane's)
        src = memonly(src)
        src = re.sub(r'__builtin_amdgcn_raw_buffer_store_b64\(__builtin_bit_cast\(u32x2, ([^)]*\))\), (\w+), (\w+), 0, (\d)\);',
                     r'if (!(lane & 1)) __builtin_amdgcn_raw_buffer_store_b128((u32x4)(0x3c003c00u), \2, \3, 0, \4);', src)
        return src.replace('typedef unsigned u32x2', 'typedef unsigned u32x4 __attribute__((ext_vector_type(4)));\ntypedef unsigned u32x2')

    def nostore(src):
        return '\n'.join(l for l in src.splitlines() if 'raw_buffer_store' not in l)
    variants = [('full', None), ('memonly', memonly), ('nostore', nostore)]
    kernels = []
    for i, (name, hack) in enumerate(variants):
        k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name=f'abl{i}', target='gpu',
                          gpu_indexing_params=tun).compile()
        v = ('march', k._march_cfg(8, shape))
        src, kname = k.source(v)
        if hack:
            new = hack(src)
            assert new != src, name
            k._variants[v] = (new, kname)
        k(u=u, out=out)
        kernels.append((name, k))
    torch.cuda.synchronize()
    times = {name: [] for name, _ in kernels}
    for r in range(7):
        for name, k in kernels:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                k(u=u, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 4)
    for name, ts in times.items():
        ts = sorted(ts)
        print(f'{name:8s} median {ts[len(ts) // 2]:.4f} ms  min {ts[0]:.4f} ms')


if __name__ == '__main__':
    main()
