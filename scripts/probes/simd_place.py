"""Which SIMD each wave of a 4-wave workgroup lands on (HW_REG_HW_ID.SIMD_ID), for workgroups shaped like the band
kernel's (256 threads, 46 KB of LDS: three per CU). If wave 3 (the band kernel's loader) always lands on one SIMD, the
CU's three loaders share it and the compute waves crowd the other three SIMDs.
python scripts/probes/simd_place.py"""
import collections
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SRC = r'''
extern "C" __global__ void __launch_bounds__(256) place(unsigned* out, int spin)
{
  __shared__ float lds[11776];                       // 46 KB: three workgroups per CU
  lds[threadIdx.x] = 0.f;
  __syncthreads();
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);   // keep the workgroups co-resident
  if ((threadIdx.x & 63) == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[blockIdx.x * 4 + (threadIdx.x >> 6)] = hw + (unsigned)lds[threadIdx.x];
  }
}
'''


def main():
    import torch

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    code = rt.compile_hip(SRC, name='simd_place.hip')
    fn = rt.load_function(code, 'place', torch.cuda.current_device())
    nwg = 768
    out = torch.zeros(nwg * 4, dtype=torch.int32, device='cuda')
    args = struct.pack('<Qi', out.data_ptr(), 20) + b'\0' * 4
    rt.launch(fn, (nwg,), (256,), args, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hw = out.cpu().numpy().astype('uint32')
    simd = (hw >> 4) & 3
    per_wave = [collections.Counter(simd[w::4].tolist()) for w in range(4)]
    for w in range(4):
        print(f'wave {w}: SIMD histogram {dict(sorted(per_wave[w].items()))}')
    starts = collections.Counter(simd[0::4].tolist())
    print('start SIMD (wave 0) histogram:', dict(sorted(starts.items())))
    order = collections.Counter(tuple(simd[4 * b:4 * b + 4].tolist()) for b in range(nwg))
    print('wave->SIMD orders:', dict(order.most_common(8)))


if __name__ == '__main__':
    main()
