#include <hip/hip_runtime.h>
#include <cstdio>
// probe: buffer_load ... lds (16 B) with out-of-range offsets; does LDS get zeros or is the write skipped?
extern "C" __global__ void __launch_bounds__(64) probe(const float* __restrict__ src, float* __restrict__ out, int nrec)
{
  __shared__ __attribute__((aligned(16))) float lds[64 * 4];
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = -7.0f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nrec, 0x00020000);
  const int lane = threadIdx.x;
  const int voff = (lane & 1) ? 0x40000000 : lane * 16;   // odd lanes out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
int main() {
  float h[1024]; for (int i = 0; i < 1024; ++i) h[i] = i + 1;
  float *src, *out; hipMalloc(&src, 4096); hipMalloc(&out, 1024);
  hipMemcpy(src, h, 4096, hipMemcpyHostToDevice);
  for (int nrec : {4096, 0}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, nrec);
    float o[256]; hipMemcpy(o, out, 1024, hipMemcpyDeviceToHost);
    printf("nrec=%d: lane0 %g %g %g %g | lane1 %g %g %g %g | lane2 %g\n", nrec, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]);
  }
  return 0;
}
