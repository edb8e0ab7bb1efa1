"""Cost of 16-byte global loads that start 4-byte aligned (the XM loader's pieces on rows whose pitch is not a
multiple of 16 bytes) against 16-byte aligned ones: a streaming read of 256 MB by raw buffer loads (to registers)
and by LDS-DMA (buffer_load ... lds) at byte offsets 0 / 4 / 8 / 12, streaming 8- and 16-byte stores at the same
offsets, plus a torch copy for scale.
python scripts/probes/dma_align.py"""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SRC = r'''
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// every lane reads 16 B per iteration at byte offset `off` + 16*i of the buffer; a sum keeps the loads alive
extern "C" __global__ void __launch_bounds__(256) rd_reg(const unsigned* __restrict__ src, unsigned* __restrict__ out,
                                                        unsigned n16, int off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  unsigned acc = 0;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16u + (unsigned)off, 0, 0);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA: each wave streams 1 KB pieces into its own 4 KB LDS ring slot (no consumer; at most 8 pieces in flight)
extern "C" __global__ void __launch_bounds__(256) rd_dma(const unsigned* __restrict__ src, unsigned* __restrict__ out,
                                                        unsigned n16, int off) {
  __shared__ __attribute__((aligned(1024))) unsigned lds[4 * 4 * 256];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned nw = gridDim.x * 4u;
  unsigned k = 0;
  for (unsigned w = blockIdx.x * 4u + wave; w * 64u < n16; w += nw, ++k) {
    __attribute__((address_space(3))) void* dst =
        (__attribute__((address_space(3))) void*)(&lds[(wave * 4 + (k & 3)) * 256]);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, (w * 64u + lane) * 16u + (unsigned)off, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F78);          // vmcnt <= 8
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (lds[threadIdx.x] == 0x12345678u && n16 == 0) out[0] = 1;
}

// LDS-DMA from ONE wave per workgroup (the WS loader's situation: one wave per CU issues every piece), up to
// `depth` pieces in flight
extern "C" __global__ void __launch_bounds__(64) rd_dma1(const unsigned* __restrict__ src, unsigned* __restrict__ out,
                                                        unsigned n16, int off) {
  __shared__ __attribute__((aligned(1024))) unsigned lds[16 * 256];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63;
  unsigned k = 0;
  for (unsigned w = blockIdx.x; w * 64u < n16; w += gridDim.x, ++k) {
    __attribute__((address_space(3))) void* dst = (__attribute__((address_space(3))) void*)(&lds[(k & 15) * 256]);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, (w * 64u + lane) * 16u + (unsigned)off, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F7C);          // vmcnt <= 12
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (lds[threadIdx.x] == 0x12345678u && n16 == 0) out[0] = 1;
}

// streaming writes of 8 / 16 B per lane at byte offset `off` (the XM sweeps' output rows start 4-byte aligned)
extern "C" __global__ void __launch_bounds__(256) wr_b64(unsigned* __restrict__ dst, unsigned n8, int off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 0x7fffffff, 0x00020000);
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n8; i += gridDim.x * 256u)
    __builtin_amdgcn_raw_buffer_store_b64((u32x2){i, i}, rs, i * 8u + (unsigned)off, 0, 0);
}
extern "C" __global__ void __launch_bounds__(256) wr_b128(unsigned* __restrict__ dst, unsigned n16, int off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, 0x7fffffff, 0x00020000);
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n16; i += gridDim.x * 256u)
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){i, i, i, i}, rs, i * 16u + (unsigned)off, 0, 0);
}
'''


def main():
    import torch

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    code = rt.compile_hip(SRC, name='dma_align.hip')
    dev = torch.cuda.current_device()
    nbytes = 256 << 20
    src = torch.empty(nbytes // 4 + 64, dtype=torch.int32, device='cuda').random_()
    out = torch.zeros(16, dtype=torch.int32, device='cuda')
    n16 = nbytes // 16
    stream = torch.cuda.current_stream().cuda_stream

    def timed(fn, reps=30):
        for _ in range(5):
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
        v = sorted(a.elapsed_time(b) for a, b in ev)
        return v[len(v) // 2]
    for kname, grid, block in (('rd_reg', 4096, 256), ('rd_dma', 4096, 256), ('rd_dma1', 256, 64),
                               ('rd_dma1', 512, 64)):
        fn = rt.load_function(code, kname, dev)
        for off in (0, 4, 8, 12, 16):
            args = struct.pack('<QQIi', src.data_ptr(), out.data_ptr(), n16, off)
            ms = timed(lambda: rt.launch(fn, (grid,), (block,), args, stream))
            label = kname if kname != 'rd_dma1' else f'rd_dma1 x{grid}'
            print(f'{label} offset {off:2d} B: {ms:.4f} ms {nbytes / ms / 1e6:7.0f} GB/s', flush=True)
    dst = torch.empty(nbytes // 4 + 64, dtype=torch.int32, device='cuda')
    for kname, w in (('wr_b64', 8), ('wr_b128', 16)):
        fn = rt.load_function(code, kname, dev)
        for off in (0, 2, 4, 8, 12):
            if off % 4 and w == 16:
                continue
            args = struct.pack('<QIi', dst.data_ptr(), nbytes // w, off)
            ms = timed(lambda: rt.launch(fn, (4096,), (256,), args, stream))
            print(f'{kname} offset {off:2d} B: {ms:.4f} ms {nbytes / ms / 1e6:7.0f} GB/s', flush=True)
    dst = dst[:nbytes // 4]
    ms = timed(lambda: dst.copy_(src[:nbytes // 4]))
    print(f'torch copy (read + write): {ms:.4f} ms {2 * nbytes / ms / 1e6:7.0f} GB/s', flush=True)


if __name__ == '__main__':
    main()
