"""Write / copy patterns of the 27-point fp16 sweep on a 768³ fp16 field, no arithmetic (HIP events, one process).

The full 27-point sweep is bound by its load/store pattern (profiles/r02_ablate27_*.log: memory-only 0.355 ms, no
stores 0.160 ms, torch's elementwise kernel over the same bytes 0.294 ms). This probe separates the pattern from
the schedule: plain kernels that only WRITE the field (or copy plane p+1 of one field into plane p of another)
tile by tile like the sweep — 256×8 tiles marching z-chunks, lanes owning 4 x-adjacent halves per row (8-byte
stores, the sweep's pattern) — against 16-byte stores (two rows' quads swapped between lane pairs), full-row tiles
(768×TY, one contiguous block per plane), and a linear streaming write of the same bytes.
python scripts/probes/store_patterns.py [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SRC = r'''
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// tile marching writer: TXH halves wide (lanes own 4 x-adjacent halves), TY rows (4 waves x NR rows), zc planes
template <int NR, int MODE>
__device__ void tile_body(const _Float16* __restrict__ src, _Float16* __restrict__ dst, int N, int zc, int TXH) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntx = N / TXH, nty = N / (4 * NR);
  const int nt = ntx * nty;
  const int b = blockIdx.x;
  const int tile = b % nt, chunk = b / nt;
  const int x0 = (tile % ntx) * TXH, y0 = (tile / ntx) * (4 * NR);
  const long long YX = (long long)N * N;
  const int zb = chunk * zc, ze = min(zb + zc, N);
  for (int z = zb; z < ze; ++z) {
  for (int xw = 0; xw < TXH; xw += 256) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + (long long)z * YX), (short)0,
                                                                        (int)(YX * 2), 0x00020000);
    f16x4 v[NR];
    for (int r = 0; r < NR; ++r) {
      const int y = y0 + wave * NR + r, x = x0 + xw + 4 * lane;
      if (MODE == 2 && z + 1 < N) {
        v[r] = *(const f16x4*)(src + (long long)(z + 1) * YX + (long long)y * N + x);
      } else {
        v[r] = (f16x4)(_Float16)(z + r);
      }
    }
    if (MODE == 1 && NR % 2 == 0) {
      // lane pairs swap one row's quad: even lanes store row r [own, partner], odd lanes row r+1 [partner, own]
      for (int r = 0; r < NR; r += 2) {
        const bool odd = lane & 1;
        const u32x2 send = __builtin_bit_cast(u32x2, odd ? v[r] : v[r + 1]);
        u32x2 got;
        got.x = __builtin_amdgcn_update_dpp(0u, send.x, 0xB1, 0xf, 0xf, false);
        got.y = __builtin_amdgcn_update_dpp(0u, send.y, 0xB1, 0xf, 0xf, false);
        const u32x2 mine = __builtin_bit_cast(u32x2, odd ? v[r + 1] : v[r]);
        const u32x4 out = odd ? (u32x4){got.x, got.y, mine.x, mine.y} : (u32x4){mine.x, mine.y, got.x, got.y};
        const int y = y0 + wave * NR + r + (odd ? 1 : 0), x = x0 + xw + 4 * (lane & ~1);
        __builtin_amdgcn_raw_buffer_store_b128(out, rs, (unsigned)(y * N + x) * 2u, 0, 2);
      }
    } else {
      for (int r = 0; r < NR; ++r) {
        const int y = y0 + wave * NR + r, x = x0 + xw + 4 * lane;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[r]), rs, (unsigned)(y * N + x) * 2u, 0, 2);
      }
    }
  }
  }
}

extern "C" __global__ void __launch_bounds__(256) tile_w8(const _Float16* s, _Float16* d, int N, int zc, int TXH) { tile_body<2, 0>(s, d, N, zc, TXH); }
extern "C" __global__ void __launch_bounds__(256) tile_w16(const _Float16* s, _Float16* d, int N, int zc, int TXH) { tile_body<2, 1>(s, d, N, zc, TXH); }
extern "C" __global__ void __launch_bounds__(256) tile_copy8(const _Float16* s, _Float16* d, int N, int zc, int TXH) { tile_body<2, 2>(s, d, N, zc, TXH); }
extern "C" __global__ void __launch_bounds__(256) tile_w8_nr4(const _Float16* s, _Float16* d, int N, int zc, int TXH) { tile_body<4, 0>(s, d, N, zc, TXH); }
extern "C" __global__ void __launch_bounds__(256) tile_w16_nr4(const _Float16* s, _Float16* d, int N, int zc, int TXH) { tile_body<4, 1>(s, d, N, zc, TXH); }

// 1-D strips marching z: block = (strip of 2048 consecutive halves of a plane, z chunk), 16 B per lane
extern "C" __global__ void __launch_bounds__(256) strip_w16(_Float16* __restrict__ d, int N, int zc) {
  const long long YX = (long long)N * N;
  const int nstrip = (int)(YX / 2048);
  const int s = blockIdx.x % nstrip, chunk = blockIdx.x / nstrip;
  const int zb = chunk * zc, ze = min(zb + zc, N);
  for (int z = zb; z < ze; ++z)
    __builtin_nontemporal_store((f16x8)(_Float16)z, (f16x8*)(d + (long long)z * YX + (long long)s * 2048) + threadIdx.x);
}

extern "C" __global__ void __launch_bounds__(256) linear_w16(_Float16* __restrict__ d, long long n8) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n8) __builtin_nontemporal_store((f16x8)(_Float16)1, (f16x8*)d + i);
}
'''


def main():
    import struct

    import torch

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    code = rt.compile_hip(SRC, name='store_patterns.hip')
    dev = torch.cuda.current_device()
    src = torch.rand(N, N, N, device='cuda').half()
    dst = torch.empty_like(src)
    nbytes = dst.numel() * 2
    stream = torch.cuda.current_stream().cuda_stream

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        v = sorted(x.elapsed_time(y) for x, y in ts)
        return v[len(v) // 2]

    def tile(kname, nr, zc, txh):
        fn = rt.load_function(code, kname, dev)
        grid = (N // txh) * (N // (4 * nr)) * (-(-N // zc))
        args = struct.pack('<QQiii', src.data_ptr(), dst.data_ptr(), N, zc, txh) + b'\0' * 4
        return lambda: rt.launch(fn, (grid,), (256,), args, stream)
    res = []
    for zc in (1, 24, 96):
        for kname, nr in (('tile_w8', 2), ('tile_w16', 2), ('tile_w8_nr4', 4), ('tile_w16_nr4', 4)):
            for txh in (256, N):
                if N % txh:
                    continue
                ms = timed(tile(kname, nr, zc, txh))
                res.append((f'{kname:14s} tile {txh}x{4 * nr} zc {zc}', ms, nbytes))
        for txh in (256, N):
            ms = timed(tile('tile_copy8', 2, zc, txh))
            res.append((f'tile_copy8     tile {txh}x8 zc {zc} (read p+1, write p)', ms, 2 * nbytes))
    fs = rt.load_function(code, 'strip_w16', dev)
    for zc in (1, 4, 24, 96):
        nstrip = N * N // 2048
        args = struct.pack('<Qii', dst.data_ptr(), N, zc)
        res.append((f'strip_w16 (4 KB 1-D strips marching z) zc {zc}',
                    timed(lambda: rt.launch(fs, (nstrip * -(-N // zc),), (256,), args, stream)), nbytes))
    fl = rt.load_function(code, 'linear_w16', dev)
    n8 = dst.numel() // 8
    args = struct.pack('<Qq', dst.data_ptr(), n8)
    res.append(('linear_w16 (streaming write)', timed(lambda: rt.launch(fl, (-(-n8 // 256),), (256,), args, stream)),
                nbytes))
    res.append(('torch fill_', timed(lambda: dst.fill_(1.0)), nbytes))
    res.append(('torch mul (read + write)', timed(lambda: torch.mul(src, 2.0, out=dst)), 2 * nbytes))
    for name, ms, b in res:
        print(f'{name:52s} {ms:.4f} ms {b / ms / 1e6:7.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
