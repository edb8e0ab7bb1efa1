"""Row-band 27-point fp16 sweep with R rows per lane (register blocking in y), the follow-up of rowblock27.py.

rowblock27.py showed the full-width band's memory pattern is faster than the op's 256×8 tiles (memory-only 0.320 vs
0.355 ms at 768³) but its arithmetic does not hide: with one row per lane every input row is converted (fp16→fp32),
shifted (DPP) and masked three times, once per output row it feeds — ~21 VALU instructions per cell against 13.5
packed FMAs. A lane that owns R rows × 8 x-cells converts its R+2 input rows once per plane: (R+2)·10 conversions per
8R cells. The three z-partial sums (outputs q-1, q, q+1 of input plane q) live in a ring of three register sets
indexed by plane mod 3, with the plane loop unrolled by 3, so no accumulator moves.

MODE 0 = full, 1 = memory only (centre values stored), 2 = arithmetic only (no loads issued, no stores), 3 = 2 without
the per-plane workgroup barriers, 4 = loads only (1 without its stores). Optional 8th config value: store aux bits
(2 = non-temporal, default).
python scripts/probes/rowblock27r.py [N]"""
import itertools
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WEIGHTS = [(i - 13.3) / 50.0 for i in range(27)]


def source(X, TY, R, D, MODE, MAP, WPE=None, NCH=1, AUX=2, MIX=0, TRIM=0):
    CPR = X // 8
    G = TY // R
    NCT = G * CPR // NCH
    assert G * R == TY and NCT * NCH == G * CPR and NCT % 64 == 0 and NCT <= 960
    NT = NCT + 64
    NPIECE = (TY + 2) * CPR
    NI = -(-NPIECE // 64)
    SLOT = NI * 512
    NS = D + 1
    assert D * NI <= 63
    w = {}
    for i, (dz, dy, dx) in enumerate(itertools.product((-1, 0, 1), repeat=3)):
        w[(dz, dy, dx)] = f'{WEIGHTS[i]!r}f'
    waits = '\n'.join(f'        case {a}: asm volatile("s_waitcnt vmcnt({a * NI})" ::: "memory"); break;'
                      for a in range(D))
    wpe = f'__attribute__((amdgpu_waves_per_eu({WPE})))' if WPE else ''
    remap = ('const int per = nb >> 3, rem = nb & 7, xcd = b & 7, bi = b >> 3;\n'
             '  const int lb = (xcd < rem) ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;'
             if MAP == 0 else 'const int lb = b;')

    def S(s, i, o, p):
        return f'S{s}_{i}_{o}_{p}'

    # one plane step with static set roles: k = plane index mod 3
    def step(k, ind):
        sp, s0, sn = (k + 2) % 3, k, (k + 1) % 3       # out q-1, out q, out q+1
        L = []
        a = L.append
        a(f'{ind}if (jj < nplanes) {{')
        if MODE != 3:
            a(f'{ind}  __syncthreads();')
        a(f'{ind}  const _Float16* sl = lds + (jj % {NS}) * {SLOT};')
        if TRIM:
            a(f'{ind}  const bool nd_p = jj >= 2, nd_0 = jj >= 1 && jj + 1 < nplanes, nd_n = jj + 2 < nplanes;')
        for i in range(NCH):
            for r in range(R + 2):
                a(f'{ind}  {{')
                a(f'{ind}    const _Float16* rp = sl + lofs{i} + {r * X};')
                if MODE == 2:
                    a(f'{ind}    const f16x8 v = *(const f16x8*)rp;')
                else:
                    a(f'{ind}    const f16x8 v = *(const f16x8*)rp;')
                a(f'{ind}    const u32x4 d = __builtin_bit_cast(u32x4, v);')
                a(f'{ind}    const unsigned e = *(const unsigned*)(rp + eoff);')
                a(f'{ind}    const unsigned lw = __builtin_amdgcn_update_dpp(e, d.w, 0x138, 0xf, 0xf, false);')
                a(f'{ind}    const unsigned rw = __builtin_amdgcn_update_dpp(e, d.x, 0x130, 0xf, 0xf, false);')
                a(f'{ind}    const _Float16 l = lmask{i} ? (_Float16)0 : __builtin_bit_cast(f16x2, lw)[1];')
                a(f'{ind}    const _Float16 rr = rmask{i} ? (_Float16)0 : __builtin_bit_cast(f16x2, rw)[0];')
                if MIX:
                    a(f'{ind}    const _Float16 H0 = l, H9 = rr, ' + ', '.join(f'H{e + 1} = v[{e}]' for e in range(8)) + ';')
                else:
                    a(f'{ind}    const f32x2 P0 = {{(float)l, (float)v[3]}}, P1 = {{(float)v[0], (float)v[4]}}, '
                      f'P2 = {{(float)v[1], (float)v[5]}};')
                    a(f'{ind}    const f32x2 P3 = {{(float)v[2], (float)v[6]}}, P4 = {{(float)v[3], (float)v[7]}}, '
                      f'P5 = {{(float)v[4], (float)rr}};')
                if TRIM and MODE in (0, 2, 3) and not MIX:
                    # taps grouped per output set, each group behind a uniform branch: the first two and last two
                    # planes of a chunk feed outputs outside it, their taps for those outputs are skipped
                    for st, dz, flag in ((sp, 1, 'nd_p'), (s0, 0, 'nd_0'), (sn, -1, 'nd_n')):
                        a(f'{ind}    if ({flag}) {{')
                        for o in range(R):
                            dy = r - o - 1
                            if dy < -1 or dy > 1:
                                continue
                            for dx in (-1, 0, 1):
                                for p in range(4):
                                    acc = S(st, i, o, p)
                                    term = f'{w[(dz, dy, dx)]} * P{p + dx + 1}'
                                    if dz == -1 and dy == -1 and dx == -1:
                                        a(f'{ind}      {acc} = {term};')
                                    else:
                                        a(f'{ind}      {acc} = {acc} + {term};')
                        a(f'{ind}    }}')
                for o in range(R if not (TRIM and MODE in (0, 2, 3) and not MIX) else 0):
                    dy = r - o - 1
                    if dy < -1 or dy > 1:
                        continue
                    if MODE in (1, 4):
                        if dy == 0:
                            for p in range(8 if MIX else 4):
                                a(f'{ind}    {S(sp, i, o, p)} = ' + (f'(float)H{p + 1};' if MIX else f'P{p + 1};'))
                        continue
                    if MIX:
                        for dx in (-1, 0, 1):
                            for st, dz in ((sp, 1), (s0, 0), (sn, -1)):
                                for e in range(8):
                                    acc = S(st, i, o, e)
                                    hv = f'(float)H{e + dx + 1}'
                                    if dz == -1 and dy == -1 and dx == -1:
                                        a(f'{ind}    {acc} = {hv} * {w[(dz, dy, dx)]};')
                                    else:
                                        a(f'{ind}    {acc} = __builtin_fmaf({hv}, {w[(dz, dy, dx)]}, {acc});')
                        continue
                    # tap by tap across the 12 accumulators (3 sets x 4 pairs): consecutive FMAs independent
                    for dx in (-1, 0, 1):
                        for st, dz in ((sp, 1), (s0, 0), (sn, -1)):
                            for p in range(4):
                                acc = S(st, i, o, p)
                                term = f'{w[(dz, dy, dx)]} * P{p + dx + 1}'
                                if dz == -1 and dy == -1 and dx == -1:
                                    a(f'{ind}    {acc} = {term};')
                                else:
                                    a(f'{ind}    {acc} = {acc} + {term};')
                a(f'{ind}  }}')
        cond = 'jj >= 2' if MODE < 2 else 'jj >= 2 && st'
        if MODE == 4:
            cond = 'jj >= 2 && st'
        a(f'{ind}  if ({cond}) {{')
        a(f'{ind}    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc('
          f'(void*)(out + (i64)(zb - 2 + jj) * YX), (short)0, (int)(YX * 2), 0x00020000);')
        for i in range(NCH):
            for o in range(R):
                vals = ', '.join(f'(_Float16){S(sp, i, o, e)}' for e in range(8)) if MIX else \
                    ', '.join(f'(_Float16){S(sp, i, o, p)}.{c}' for c in 'xy' for p in range(4))
                a(f'{ind}    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, (f16x8){{{vals}}}), ors, '
                  f'sofs{i} + {o * X * 2}u, 0, {AUX});')
        a(f'{ind}  }}')
        a(f'{ind}  ++jj;')
        a(f'{ind}}}')
        return '\n'.join(L)

    decl = []
    for s in range(3):
        for i in range(NCH):
            for o in range(R):
                if MIX:
                    decl.append('float ' + ', '.join(f'{S(s, i, o, e)} = 0.f' for e in range(8)) + ';')
                else:
                    decl.append('f32x2 ' + ', '.join(f'{S(s, i, o, p)} = (f32x2)(0.f)' for p in range(4)) + ';')
    per_chunk = []
    for i in range(NCH):
        per_chunk.append(f'  const int t{i} = {i * NCT} + tid, g{i} = t{i} / {CPR}, col{i} = t{i} % {CPR};')
        per_chunk.append(f'  const int lofs{i} = g{i} * {R * X} + col{i} * 8;   // slot row g*R (input row y0+g*R-1)')
        per_chunk.append(f'  const unsigned sofs{i} = (unsigned)((y0 + g{i} * {R}) * {X} + col{i} * 8) * 2u;')
        per_chunk.append(f'  const bool lmask{i} = col{i} == 0, rmask{i} = col{i} == {CPR - 1};')
    issue_body = ((f'      if (st == 7)\n' if MODE in (2, 3) else '') + f'''      #pragma unroll
      for (int i = 0; i < {NI}; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + i * 512), 16, vo[i], 0, 0, 0);''')
    return f'''
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef long long i64;

extern "C" __global__ void __launch_bounds__({NT}) {wpe} rb27r(const _Float16* __restrict__ u, _Float16* __restrict__ out,
    const int Y, const int Z, const int zc, const int nbands, const int st)
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
{issue_body}
    }};
    for (int i = 0; i < {D}; ++i)
      if (i < nplanes) issue(zb - 1 + i, i);
    for (int j = 0; j < nplanes; ++j) {{
      const int after = min({D - 1}, nplanes - 1 - j);
      switch (after) {{
{waits}
      }}
      {'' if MODE == 3 else '__builtin_amdgcn_s_barrier();'}
      if (j + {D} < nplanes) issue(zb - 1 + j + {D}, (j + {D}) % {NS});
    }}
    return;
  }}
{chr(10).join(per_chunk)}
  const int eoff = 2 * (lane == 0 ? -1 : (lane == 63 ? 256 : lane)) - 8 * lane;
  {chr(10).join('  ' + d for d in decl).strip()}
  int jj = 0;
  #pragma unroll 1
  while (jj < nplanes) {{
{step(0, '    ')}
{step(1, '    ')}
{step(2, '    ')}
  }}
}}
'''


def main():
    import time

    import torch
    import torch.nn.functional as F

    from pystencils_autodiff_amd.backends import hip_runtime as rt
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    only = [tuple(int(v) for v in a.split(',')) for a in sys.argv[2:]]   # TY,R,NCH,D,MODE,MAP,zc (PMC runs)
    dev = torch.cuda.current_device()
    stream = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    u = torch.rand(N, N, N, device='cuda').half()
    out = torch.empty_like(u)
    ref = None
    if not only:       # PMC runs (configs given) skip the reference and the settle loops: every dispatch is profiled
        up = F.pad(u.float()[None], (1, 1, 1, 1, 1, 1))[0]
        ref = torch.zeros(N, N, N, device='cuda')
        for i, (dz, dy, dx) in enumerate(itertools.product((-1, 0, 1), repeat=3)):
            ref += WEIGHTS[i] * up[1 + dz:1 + dz + N, 1 + dy:1 + dy + N, 1 + dx:1 + dx + N]
        del up
    nbytes = 2 * u.numel() * 2

    def timed(fn, reps=30):
        for _ in range(1 if only else 5):
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

    t0 = time.perf_counter()
    while not only and time.perf_counter() - t0 < 1.0:
        torch.mul(u, 2.0, out=out)
    torch.cuda.synchronize()

    def settle(fn, sec=0.3):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < sec:
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    if only:
        with torch.no_grad():
            print(f'op forward (current schedule) {timed(lambda: fn.apply(u), 2):.4f} ms', flush=True)
    # (TY, R, NCH, D, MODE, MAP, zc)
    if N == 768:
        cfgs = [(8, 4, 1, 2, 0, 0, 48)]
        for zc in (8, 12, 16, 24, 32, 48):
            cfgs += [(8, 4, 1, 2, 0, 0, zc, 2, 0, 1)]
        cfgs += [(8, 4, 1, 2, 2, 0, 16, 2, 0, 1), (8, 4, 1, 2, 2, 0, 16, 2, 0, 0), (8, 4, 1, 3, 0, 0, 16, 2, 0, 1),
                 (6, 3, 1, 3, 0, 0, 16, 2, 0, 1), (6, 3, 1, 3, 0, 0, 12, 2, 0, 1)]
    else:
        cfgs = [(4, 2, 1, 3, 0, 0, 48)]
        for zc in (8, 16, 32):
            cfgs += [(4, 2, 1, 3, 0, 0, zc, 2, 0, 1), (4, 4, 1, 2, 0, 0, zc, 2, 0, 1)]
    if only:
        cfgs = only
    compiled = {}
    runs = []       # (label, launch)
    for cfg in cfgs:
        TY, R, NCH, D, MODE, MAP, zc = cfg[:7]
        AUX = cfg[7] if len(cfg) > 7 else 2
        MIX = cfg[8] if len(cfg) > 8 else 0
        TRIM = cfg[9] if len(cfg) > 9 else 0
        CPR = N // 8
        G = TY // R
        if N % TY or (G * CPR) % (64 * NCH) or D * -(-((TY + 2) * CPR) // 64) > 63 or G * CPR // NCH > 960:
            print('skip', (TY, R, NCH, D, MODE, MAP, zc), flush=True)
            continue
        NT = G * CPR // NCH + 64
        key = (TY, R, NCH, D, MODE, MAP, AUX, MIX, TRIM)
        if key not in compiled:
            code = rt.compile_hip(source(N, TY, R, D, MODE, MAP, None, NCH, AUX, MIX, TRIM), name=f'rb27r_{N}_{"_".join(map(str, key))}.hip')
            fn_ = rt.load_function(code, 'rb27r', dev)
            compiled[key] = (fn_, rt.function_attributes(fn_))
        f, attrs = compiled[key]
        nbands = N // TY
        grid = nbands * (-(-N // zc))
        args = struct.pack('<QQiiiii', u.data_ptr(), out.data_ptr(), N, N, zc, nbands, 1 if MODE < 2 else 0) + b'\0' * 4
        launch = (lambda f=f, grid=grid, args=args, NT=NT: rt.launch(f, (grid,), (NT,), args, stream))
        out.zero_()
        launch()
        torch.cuda.synchronize()
        err = float((out.float() - ref).abs().max()) if MODE == 0 and ref is not None else float('nan')
        label = (f'TY {TY:2d} R {R} NCH {NCH} NT {NT:4d} D {D} MODE {MODE} MAP {MAP} zc {zc:2d} aux {AUX} mix {MIX} trim {TRIM} maxerr {err:.1e} '
                 f'regs {attrs["num_regs"]} lds {attrs["shared_bytes"]}')
        runs.append((label, launch))
        if only:
            print(label, f'{timed(launch, 2):.4f} ms', flush=True)
    if only:
        return
    # A/B rounds: every config and the op timed once per round after a 2 s warm state (power / clocks settle
    # within the first ~20 ms of sweeps; the op measured first in a cold process reads 15-20 % slow)
    with torch.no_grad():
        runs.insert(0, ('op forward (current schedule)', lambda: fn.apply(u)))
        settle(runs[0][1], 2.0)
        res = {lab: [] for lab, _ in runs}
        for rnd in range(4):
            for lab, fn_ in runs:
                settle(fn_, 0.1)
                res[lab].append(timed(fn_, 20))
    for lab, _ in runs:
        v = sorted(res[lab])
        med = (v[1] + v[2]) / 2
        print(f'{lab:90s} {med:.4f} ms {nbytes / med / 1e6:6.0f} GB/s  [{" ".join(f"{x:.4f}" for x in res[lab])}]',
              flush=True)


if __name__ == '__main__':
    main()
