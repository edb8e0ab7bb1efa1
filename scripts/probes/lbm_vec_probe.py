"""Memory-pattern probe for the lattice kernels: the D3Q19 pull stream alone (dst_q(x) = src_q(x − c_q), periodic,
fzyx fp32, no collision) with one cell per thread and 4-byte accesses (the lattice kernels' form) against four
consecutive x cells per thread with 16-byte buffer loads / stores at dword-aligned offsets. Timing only.

python scripts/probes/lbm_vec_probe.py [edge=192]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from pystencils_autodiff_amd.backends import hip_runtime as rt  # noqa: E402

DIRS = [(0, 0, 0), (0, 1, 0), (0, -1, 0), (-1, 0, 0), (1, 0, 0), (0, 0, 1), (0, 0, -1), (-1, 1, 0), (1, 1, 0),
        (-1, -1, 0), (1, -1, 0), (0, 1, 1), (0, -1, 1), (-1, 0, 1), (1, 0, 1), (0, 1, -1), (0, -1, -1), (-1, 0, -1),
        (1, 0, -1)]


def source():
    L = ['typedef unsigned u32x4 __attribute__((ext_vector_type(4)));']
    # axis order (z, y, x); a direction is (c_z, c_y, c_x) here
    L.append('extern "C" __global__ void __launch_bounds__(256) pull1(const float* __restrict__ src, '
             'float* __restrict__ dst, const int X, const int Y, const int Z)\n{')
    L.append('  const unsigned cell = blockIdx.x * 256u + threadIdx.x;')
    L.append('  if (cell >= (unsigned)X * Y * Z) return;')
    L.append('  const int x = cell % X, r = cell / X, y = r % Y, z = r / Y;')
    L.append('  const long long N = (long long)X * Y * Z;')
    for q, (cz, cy, cx) in enumerate(DIRS):
        L.append(f'  {{ const int xs = (x - ({cx}) + X) % X, ys = (y - ({cy}) + Y) % Y, zs = (z - ({cz}) + Z) % Z;')
        L.append(f'    dst[{q} * N + cell] = src[{q} * N + ((long long)zs * Y + ys) * X + xs]; }}')
    L.append('}')
    L.append('extern "C" __global__ void __launch_bounds__(256) pull4(const float* __restrict__ src, '
             'float* __restrict__ dst, const int X, const int Y, const int Z, const int nbytes)\n{')
    L.append('  const unsigned t = blockIdx.x * 256u + threadIdx.x;')
    L.append('  const unsigned X4 = X / 4;')
    L.append('  if (t >= X4 * Y * Z) return;')
    L.append('  const int x = (t % X4) * 4, r = t / X4, y = r % Y, z = r / Y;')
    L.append('  const unsigned N = (unsigned)X * Y * Z;')
    L.append('  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, '
             '0x00020000);')
    L.append('  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, nbytes, '
             '0x00020000);')
    L.append('  const unsigned dcell = ((unsigned)z * Y + y) * X + x;')
    for q, (cz, cy, cx) in enumerate(DIRS):
        L.append(f'  {{ const int ys = (y - ({cy}) + Y) % Y, zs = (z - ({cz}) + Z) % Z, xs = x - ({cx});')
        L.append(f'    const unsigned row = {q}u * N + ((unsigned)zs * Y + ys) * X;')
        L.append('    u32x4 v;')
        L.append('    if (xs >= 0 && xs + 4 <= X) {')
        L.append('      v = __builtin_amdgcn_raw_buffer_load_b128(rs, (row + xs) * 4u, 0, 0);')
        L.append('    } else {')
        L.append('      for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (row + (unsigned)(('
                 'xs + k + X) % X)) * 4u, 0, 0);')
        L.append('    }')
        L.append(f'    __builtin_amdgcn_raw_buffer_store_b128(v, rd, ({q}u * N + dcell) * 4u, 0, 0); }}')
    L.append('}')
    return '\n'.join(L) + '\n'


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    X = Y = Z = n
    Q = len(DIRS)
    src = torch.rand((Q, Z, Y, X), device='cuda')
    dst = torch.empty_like(src)
    ref = torch.stack([torch.roll(src[q], shifts=DIRS[q], dims=(0, 1, 2)) for q in range(Q)])
    code = rt.compile_hip(source(), name='lbm_vec_probe.hip')
    dev = torch.cuda.current_device()
    f1, f4 = rt.load_function(code, 'pull1', dev), rt.load_function(code, 'pull4', dev)
    st = torch.cuda.current_stream().cuda_stream
    a1 = rt.pack_args([('ptr', src.data_ptr()), ('ptr', dst.data_ptr()), ('i32', X), ('i32', Y), ('i32', Z)])
    a4 = rt.pack_args([('ptr', src.data_ptr()), ('ptr', dst.data_ptr()), ('i32', X), ('i32', Y), ('i32', Z),
                       ('i32', src.numel() * 4)])
    runs = {'1 cell / thread, 4-B accesses': (f1, -(-X * Y * Z // 256), a1),
            '4 cells / thread, 16-B accesses': (f4, -(-(X // 4) * Y * Z // 256), a4)}
    for name, (fn, nb, args) in runs.items():
        dst.zero_()
        rt.launch(fn, (nb,), (256,), args, st)
        torch.cuda.synchronize()
        assert torch.equal(dst, ref), name
    nbytes = 2 * src.numel() * 4
    for _ in range(2):
        for name, (fn, nb, args) in runs.items():
            for _ in range(5):
                rt.launch(fn, (nb,), (256,), args, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                rt.launch(fn, (nb,), (256,), args, st)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f'D3Q19 pull {n}^3 {name:34s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:6.2f} TB/s', flush=True)
    t = torch.empty_like(src)
    for _ in range(3):
        t.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        t.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f'torch copy_ of the same bytes {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:6.2f} TB/s')


if __name__ == '__main__':
    main()
