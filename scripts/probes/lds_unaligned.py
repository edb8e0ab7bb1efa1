"""Throughput and results of 16-byte LDS reads (ds_read_b128) at 16-, 8-, 4- and 2-byte aligned addresses on
gfx950 (the driver runs LDS in unaligned mode; the compiler emits ds_read_b128 for 2-byte aligned vectors). Each
lane reads 16 bytes at ``off + 16·lane + 1040·i`` (bytes) for i < NIT, 768 workgroups of 256 threads.
python scripts/probes/lds_unaligned.py"""
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SRC = r'''
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(2)));
extern "C" __global__ void __launch_bounds__(256) rd(unsigned* out, int off, int nit)
{
  __shared__ __attribute__((aligned(16))) unsigned short lds[24576];       // 48 KB
  for (int i = threadIdx.x; i < 24576; i += 256) lds[i] = (unsigned short)(i * 2654435761u >> 7);
  __syncthreads();
  u32x4 acc = {0u, 0u, 0u, 0u};
  const char* base = (const char*)lds + off + 16 * threadIdx.x;
  for (int i = 0; i < nit; ++i) {
    const int o = (i * 1040) & 16383;
    const u32x4 v = *(const u32x4_u*)(base + o);
    acc ^= v + (unsigned)i;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// LDS-DMA of 16-byte pieces against a buffer range that ends inside a piece: which dwords land (values) and which
// read as zeros
extern "C" __global__ void __launch_bounds__(64) oob(const unsigned* src, unsigned* out, int nrec)
{
  __shared__ __attribute__((aligned(16))) unsigned lds[256];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nrec, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, threadIdx.x * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
'''


def main():
    import numpy as np
    import torch

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    code = rt.compile_hip(SRC, name='lds_unaligned.hip')
    fn = rt.load_function(code, 'rd', torch.cuda.current_device())
    fo = rt.load_function(code, 'oob', torch.cuda.current_device())
    src = torch.arange(1, 257, dtype=torch.int32, device='cuda')
    dst = torch.zeros(256, dtype=torch.int32, device='cuda')
    for nrec in (40, 38, 36, 34, 44):
        rt.launch(fo, (1,), (64,), struct.pack('<QQi', src.data_ptr(), dst.data_ptr(), nrec) + b'\0' * 4,
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        d = dst.cpu().numpy().astype('uint32')
        print(f'DMA range {nrec} B: dwords 8..11 (bytes 32..47) = {[hex(v) for v in d[8:12]]}', flush=True)
    nwg, nit = 768, 4096
    out = torch.zeros(nwg * 256, dtype=torch.int32, device='cuda')
    stream = torch.cuda.current_stream().cuda_stream

    def run(off, n):
        rt.launch(fn, (nwg,), (256,), struct.pack('<Qii', out.data_ptr(), off, n), stream)

    # expected values for workgroup 0 (host model of the LDS contents and the loop)
    lds = (((np.arange(24576, dtype=np.uint64) * 2654435761) & 0xffffffff) >> 7 & 0xffff).astype(np.uint16).tobytes()
    for off in (0, 16, 8, 4, 2, 6):
        run(off, 64)
        torch.cuda.synchronize()
        got = out[:256].cpu().numpy().astype(np.uint32)
        exp = np.zeros(256, dtype=np.uint32)
        for t in range(256):
            acc = np.zeros(4, dtype=np.uint32)
            for i in range(64):
                o = (i * 1040) & 16383
                v = np.frombuffer(lds[off + 16 * t + o: off + 16 * t + o + 16], dtype=np.uint32)
                acc ^= (v + np.uint32(i)).astype(np.uint32)
            exp[t] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3]
        ok = bool((got == exp).all())
        for _ in range(3):
            run(off, nit)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            run(off, nit)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 10
        tb = nwg * 256 * 16 * nit / (ms * 1e-3) / 1e12
        print(f'ds_read_b128 at byte offset {off:2d}: {ms:.4f} ms  {tb:6.1f} TB/s chip-wide  results '
              f'{"ok" if ok else "WRONG"}', flush=True)


if __name__ == '__main__':
    main()
