"""Row-block schedule probe for the 27-point fp16 sweep (768³): full-width bands of TY rows instead of 256×8 tiles.

A band of one plane is one contiguous block of memory (TY·X halves), so every wave-wide access is 1 KB contiguous:
the loader wave's LDS-DMA pieces (rows y0-1 … y0+TY of the plane, one contiguous block, 16 B per lane) and the
compute waves' 16-byte stores (lane-linear over the band: chunk c = 8 halves of row c / (X/8)). A lane's x
neighbours come from the adjacent lanes (DPP wave_shr/shl:1), the wave's end lanes read one LDS dword; full-width
rows make the x boundary a mask (column 0 / last column). Arithmetic: the zsum schedule (each input plane adds its
taps to outputs q+1, q, q-1), fp32 packed FMA over cell pairs (x_i, x_{i+4}) so every tap operand is a register pair
as converted, no realignment moves.

python scripts/probes/rowblock27.py [N]   (checks against torch conv3d, then times variants vs the op)"""
import itertools
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WEIGHTS = [(i - 13.3) / 50.0 for i in range(27)]


def source(X, TY, D, MODE, MAP, WPE=None, NCH=1):
    CPR = X // 8
    NPIECE = (TY + 2) * CPR
    NI = -(-NPIECE // 64)
    SLOT = NI * 512
    NS = D + 1
    NCT = TY * CPR // NCH          # compute threads: one chunk of 8 halves per lane and pass
    assert NCT * NCH == TY * CPR and NCT % 64 == 0 and NCT <= 960
    NT = NCT + 64
    wpe = f'__attribute__((amdgpu_waves_per_eu({WPE})))' if WPE else ''
    assert D * NI <= 63
    waits = '\n'.join(f'        case {a}: asm volatile("s_waitcnt vmcnt({a * NI})" ::: "memory"); break;'
                      for a in range(D))
    w = {}
    for i, (dz, dy, dx) in enumerate(itertools.product((-1, 0, 1), repeat=3)):
        w[(dz, dy, dx)] = f'{WEIGHTS[i]!r}f'

    def taps(dz, ind):
        out = []
        for p in range(4):
            terms = ' + '.join(f'{w[(dz, dy, dx)]} * P{dy + 1}[{p + dx + 1}]' for dy in (-1, 0, 1) for dx in (-1, 0, 1))
            out.append(terms)
        return out
    tp, t0, tm = taps(1, ''), taps(0, ''), taps(-1, '')
    if MODE == 1:   # memory only: the centre row's pairs stand in for the sums
        tp = t0 = tm = [f'P1[{p + 1}]' for p in range(4)]
    body_prev = '\n'.join(f'        const f32x2 o{p} = A0[i][{p}] + {tp[p]};' for p in range(4))
    body_mid = '\n'.join(f'        A0[i][{p}] = A1[i][{p}] + {t0[p]};' for p in range(4))
    body_next = '\n'.join(f'        A1[i][{p}] = {tm[p]};' for p in range(4))
    remap = ('const int per = nb >> 3, rem = nb & 7, xcd = b & 7, bi = b >> 3;\n'
             '  const int lb = (xcd < rem) ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;'
             if MAP == 0 else 'const int lb = b;')
    return f'''
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef long long i64;

extern "C" __global__ void __launch_bounds__({NT}) {wpe} rb27(const _Float16* __restrict__ u, _Float16* __restrict__ out,
                                                      const int Y, const int Z, const int zc, const int nbands)
{{
  __shared__ __attribute__((aligned(16))) _Float16 lds[{NS * SLOT + 64}];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = gridDim.x, b = blockIdx.x;
  {remap}
  const int band = lb % nbands, chunk = lb / nbands;
  const int y0 = band * {TY};
  const int zb = chunk * zc, ze = min(zb + zc, Z);
  if (zb >= ze) return;
  const i64 YX = (i64)Y * {X};
  const int nplanes = ze - zb + 2;
  if (wave == {NCT // 64}) {{
    int vo[{NI}];
    #pragma unroll
    for (int i = 0; i < {NI}; ++i) {{
      const int k = i * 64 + lane;
      vo[i] = k < {NPIECE} ? ((y0 - 1) * {X} * 2 + 16 * k) : 0x7ffffff0;
    }}
    auto issue = [&](const int q, const int slot) {{
      const bool in = q >= 0 && q < Z;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(u + (in ? (i64)q * YX : 0)), (short)0,
                                                                          in ? (int)(YX * 2) : 0, 0x00020000);
      _Float16* dst = lds + slot * {SLOT};
      #pragma unroll
      for (int i = 0; i < {NI}; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + i * 512), 16, vo[i], 0, 0, 0);
    }};
    for (int i = 0; i < {D}; ++i)
      if (i < nplanes) issue(zb - 1 + i, i);
    for (int j = 0; j < nplanes; ++j) {{
      const int after = min({D - 1}, nplanes - 1 - j);
      switch (after) {{
{waits}
      }}
      __builtin_amdgcn_s_barrier();
      if (j + {D} < nplanes) issue(zb - 1 + j + {D}, (j + {D}) % {NS});
    }}
    return;
  }}
  f32x2 A0[{NCH}][4], A1[{NCH}][4];
  #pragma unroll
  for (int i = 0; i < {NCH}; ++i)
    #pragma unroll
    for (int p = 0; p < 4; ++p) {{ A0[i][p] = (f32x2)(0.f); A1[i][p] = (f32x2)(0.f); }}
  // edge dword (in halves, relative to the lane's own chunk): lane 0 the dword left of it, lane 63 the one right of
  // it, the other lanes consecutive dwords of the wave's block (conflict-free, unused)
  const int eoff = 2 * (lane == 0 ? -1 : (lane == 63 ? 256 : lane)) - 8 * lane;   // NOLINT
  #pragma unroll 1
  for (int j = 0; j < nplanes; ++j) {{
    const int q = zb - 1 + j;
    __syncthreads();
    const _Float16* sl = lds + (j % {NS}) * {SLOT};
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (i64)(q - 1) * YX), (short)0,
                                                                         (int)(YX * 2), 0x00020000);
    #pragma unroll
    for (int i = 0; i < {NCH}; ++i) {{
      const int c = i * {NCT} + tid;
      const int col = c % {CPR};
      f32x2 P0[6], P1[6], P2[6];
      auto row = [&](const int dy, f32x2 (&P)[6]) {{
        const _Float16* rp = sl + c * 8 + dy * {X};
        const f16x8 v = *(const f16x8*)rp;
        const u32x4 d = __builtin_bit_cast(u32x4, v);
        const unsigned e = *(const unsigned*)(rp + eoff);
        const unsigned lw = __builtin_amdgcn_update_dpp(e, d.w, 0x138, 0xf, 0xf, false);   // wave_shr:1
        const unsigned rw = __builtin_amdgcn_update_dpp(e, d.x, 0x130, 0xf, 0xf, false);   // wave_shl:1
        const _Float16 l = col == 0 ? (_Float16)0 : __builtin_bit_cast(f16x2, lw)[1];
        const _Float16 r = col == {CPR - 1} ? (_Float16)0 : __builtin_bit_cast(f16x2, rw)[0];
        P[0] = (f32x2){{(float)l, (float)v[3]}};
        P[1] = (f32x2){{(float)v[0], (float)v[4]}};
        P[2] = (f32x2){{(float)v[1], (float)v[5]}};
        P[3] = (f32x2){{(float)v[2], (float)v[6]}};
        P[4] = (f32x2){{(float)v[3], (float)v[7]}};
        P[5] = (f32x2){{(float)v[4], (float)r}};
      }};
      row(0, P0);
      row(1, P1);
      row(2, P2);
{body_prev}
{body_mid}
{body_next}
      if (j >= 2) {{
        const f16x8 o = {{(_Float16)o0.x, (_Float16)o1.x, (_Float16)o2.x, (_Float16)o3.x,
                          (_Float16)o0.y, (_Float16)o1.y, (_Float16)o2.y, (_Float16)o3.y}};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ors, (unsigned)(y0 * {X} + c * 8) * 2u, 0, 2);
      }}
    }}
  }}
}}
'''


def main():
    import torch
    import torch.nn.functional as F

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    dev = torch.cuda.current_device()
    stream = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    u = torch.rand(N, N, N, device='cuda').half()
    out = torch.empty_like(u)
    up = F.pad(u.float()[None], (1, 1, 1, 1, 1, 1))[0]      # zero halo, no MIOpen (conv3d at 1024^3 stalls)
    ref = torch.zeros(N, N, N, device='cuda')
    for i, (dz, dy, dx) in enumerate(itertools.product((-1, 0, 1), repeat=3)):
        ref += WEIGHTS[i] * up[1 + dz:1 + dz + N, 1 + dy:1 + dy + N, 1 + dx:1 + dx + N]
    del up
    nbytes = 2 * u.numel() * 2

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
        v = sorted(x.elapsed_time(y) for x, y in ev)
        return v[len(v) // 2]

    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:     # settle clocks / power before the first timing
        torch.mul(u, 2.0, out=out)
    torch.cuda.synchronize()
    # the drop-in op's current kernel on the same field
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    with torch.no_grad():
        ms_op = timed(lambda: fn.apply(u))
    print(f'op forward (current schedule)            {ms_op:.4f} ms {nbytes / ms_op / 1e6:6.0f} GB/s', flush=True)
    ms_mul = timed(lambda: torch.mul(u, 2.0, out=out))
    print(f'torch mul                                {ms_mul:.4f} ms {nbytes / ms_mul / 1e6:6.0f} GB/s', flush=True)
    # (TY, NCH, D, MODE, MAP, zc, WPE)
    if N == 768:
        cfgs = [(8, 1, 3, 0, 0, 24, None), (8, 1, 3, 0, 1, 24, None), (8, 1, 3, 0, 0, 12, None),
                (8, 1, 3, 0, 0, 48, None), (8, 1, 2, 0, 0, 24, None), (8, 1, 4, 0, 0, 24, None),
                (4, 1, 3, 0, 0, 24, None), (4, 1, 5, 0, 0, 24, None), (8, 2, 3, 0, 0, 24, None),
                (2, 1, 5, 0, 0, 24, None), (8, 3, 3, 0, 0, 24, 3),
                (8, 1, 3, 1, 0, 24, None), (4, 1, 3, 1, 0, 24, None)]
    else:
        cfgs = [(4, 1, 3, 0, 0, 24, None), (4, 1, 3, 0, 1, 24, None), (4, 1, 2, 0, 0, 24, None),
                (6, 1, 3, 0, 0, 24, None), (4, 2, 3, 0, 0, 24, None), (2, 1, 5, 0, 0, 24, None),
                (4, 1, 3, 1, 0, 24, None)]
    compiled = {}
    for TY, NCH, D, MODE, MAP, zc, WPE in cfgs:
        CPR = N // 8
        if N % TY or (TY * CPR) % (64 * NCH) or D * -(-((TY + 2) * CPR) // 64) > 63 or TY * CPR // NCH > 960:
            continue
        NT = TY * CPR // NCH + 64
        key = (TY, NCH, D, MODE, MAP, WPE)
        if key not in compiled:
            code = rt.compile_hip(source(N, TY, D, MODE, MAP, WPE, NCH), name=f'rb27_{N}_{"_".join(map(str, key))}.hip')
            compiled[key] = rt.load_function(code, 'rb27', dev)
        f = compiled[key]
        nbands = N // TY
        grid = nbands * (-(-N // zc))
        args = struct.pack('<QQiiii', u.data_ptr(), out.data_ptr(), N, N, zc, nbands)
        launch = (lambda f=f, grid=grid, args=args, NT=NT: rt.launch(f, (grid,), (NT,), args, stream))
        out.zero_()
        launch()
        torch.cuda.synchronize()
        err = float((out.float() - ref).abs().max()) if MODE == 0 else float('nan')
        ms = timed(launch)
        print(f'TY {TY:2d} NCH {NCH} NT {NT:4d} D {D} MODE {MODE} MAP {MAP} zc {zc:2d}  {ms:.4f} ms {nbytes / ms / 1e6:6.0f} GB/s '
              f'maxerr {err:.2e}', flush=True)


if __name__ == '__main__':
    main()
