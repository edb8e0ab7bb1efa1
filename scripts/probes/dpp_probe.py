"""What __builtin_amdgcn_update_dpp(old, src, 0x138 / 0x130, 0xf, 0xf, false) (wave_shr:1 / wave_shl:1) gives
each lane of a wave64 on gfx950 (the half-ring x-neighbour exchange relies on it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SRC = r'''
extern "C" __global__ void __launch_bounds__(64) dpp_probe(int* out) {
  const int lane = threadIdx.x;
  const int src = lane;
  const int old = 1000 + lane;
  out[lane] = __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
  out[64 + lane] = __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false);
}
'''


def main():
    import torch

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    fn = rt.load_function(rt.compile_hip(SRC), 'dpp_probe', 0)
    out = torch.zeros(128, dtype=torch.int32, device='cuda')
    import struct
    rt.launch(fn, (1,), (64,), struct.pack('<Q', out.data_ptr()), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().tolist()
    print('wave_shr:1 (0x138):', o[:64])
    print('wave_shl:1 (0x130):', o[64:])


if __name__ == '__main__':
    main()
