"""Row-band schedule for half-precision 3-D stencils (fp16 storage, fp32 arithmetic) on gfx950.

The ``zsum`` schedule tiles a plane in 256×8 tiles: a workgroup's share of a plane is eight 512-byte row segments,
and the stores of a sweep reach ~5.4 TB/s (``scripts/probes/store_patterns.py``). Here a workgroup owns a BAND:
``TY`` full rows of a plane, which in a dense row-major field is ONE contiguous block of ``TY·X`` halves.

* loader wave: the band's rows ``y0-1 … y0+TY`` of plane ``q`` are one contiguous block as well, streamed into an
  LDS slot by LDS-DMA (``buffer_load_dwordx4 … lds``, 1 KiB per wave instruction, rows outside the plane read as
  zeros by the buffer range check, planes outside the domain from the z-slab halo buffers or zeros);
  ``D`` planes in flight in a ring of ``D + 1`` slots, published by one workgroup barrier per plane.
* compute lanes: lane ``t`` owns the 16-byte chunk ``col = t mod X/8`` (8 x-adjacent cells) of the ``R`` rows of
  row group ``t div X/8``. Per plane it reads its ``R + 2`` input rows once (``ds_read_b128``), takes the x
  neighbours from the adjacent lanes (DPP ``wave_shr/shl:1``; the wave's end lanes read one LDS dword; full rows
  make columns 0 and X/8-1 the domain's x boundary), converts each value once to fp32 and runs packed FMAs over
  the cell pairs ``(x+e, x+e+4)`` so every tap operand is a register pair as converted.
* z partial sums (as ``zsum``): input plane ``q`` adds its taps to outputs ``q+1``, ``q``, ``q-1``; the three
  accumulator sets rotate with the plane index (loop unrolled by 3, no moves). (Skipping the taps of outputs outside
  a chunk in its first / last two planes behind uniform branches measured slower: profiles/r03_op_band_ab2.log.)
* stores: output ``q-1`` row by row, 16 bytes per lane, 1 KiB contiguous per wave instruction, non-temporal.

Eligible: 3-D, every field fp16 (fp32 storage compiles too: opt-in), one stencil field (radius ≤ 1), every store a linear combination of its taps
(``zsum_plan`` with no centre-plane remainder), rows a multiple of 16 bytes. Measured against the ``zsum`` half ring
in ``scripts/probes/rowblock27r.py`` (``profiles/r03_band_*.log``).
"""
import numpy as np

from .hip_emitter import (PRELUDE, MarchConfig, _field_params, _scalar_params, _ws_plane_base, extra_params,
                          halo_wait_lines, start_signal_lines, zsum_plan)
from .printer import KernelExprPrinter

__all__ = ['band_plans', 'band_geometry', 'band_choice', 'band_esize', 'emit_band']


def band_plans(ir):
    """Per-store tap weights ``{(dz, dy, dx): coefficient}`` if the kernel fits the band schedule, else None."""
    if ir.ndim != 3 or ir.has_index_dims or ir.periodic:
        return None
    if len({np.dtype(f.dtype.numpy_dtype).itemsize for f in ir.fields}) != 1 or \
            np.dtype(ir.fields[0].dtype.numpy_dtype).itemsize not in (2, 4):
        return None                     # fp16 (fp32 arithmetic) or fp32 storage
    stencil = ir.stencil_fields
    if len(stencil) != 1 or any(r > 1 for r in ir.radius):
        return None
    if set(ir.fields) - set(ir.fields_written) - set(stencil):
        return None                     # other (point) fields read
    plans = zsum_plan(ir, MarchConfig(VE=8, ZSUM=True))
    if plans is None or not 1 <= len(plans) <= 2:
        return None
    out = []
    for pl in plans:
        if pl['rest'] != 0 or pl['k'] != 0:
            return None
        w = {}
        for dz, terms in pl['lin'].items():
            for coeff, f, dy, dx, k in terms:
                if (f is not stencil[0] and f.name != stencil[0].name) or k != 0:
                    return None
                w[(dz, dy, dx)] = w.get((dz, dy, dx), 0) + coeff
        out.append(dict(field=pl['field'], w=w))
    return out


def band_esize(ir):
    return np.dtype(ir.fields[0].dtype.numpy_dtype).itemsize


def band_padded(X, es, pad):
    """Padded image rows (``BPAD``): rows of a 16-byte multiple only."""
    return bool(pad) and (X * es) % 16 == 0


def band_geometry(X, TY, R, D, es=2, pad=0, reg=0, free=0):
    """Launch / LDS geometry of a band of ``TY`` rows (``R`` per lane) on rows of ``X`` elements of ``es`` bytes.
    Rows whose pitch is not a multiple of 16 bytes (``X % VE``) take ``ceil(X / VE)`` chunks, the last one partial.
    ``pad``: every image row is preceded by one zero 16-byte piece and the slot ends with one (x neighbours of a row's
    end chunks read as zeros straight from LDS). ``reg``: rows of a partial last chunk on a padded image filled through
    registers (``BREG``). ``free``: the LDS handshake instead of plane barriers (``BFREE``), ``free - 1`` slots beyond
    ``D + 1``."""
    VE = 16 // es
    CPR = -(-X // VE)
    reg = bool(reg) and X % VE != 0
    padded = reg or band_padded(X, es, pad)
    # LDS image row pitch (elements, 16-byte multiple). Rows starting on half dwords (fp16, X odd) are loaded from the
    # dword at or below their start, one element early every other row: the image row then needs room for X + 2
    if padded:
        XP = (CPR + 1) * VE
    else:
        XP = CPR * VE if (X * es) % 4 == 0 else VE * -(-(X + 2) // VE)
    G = TY // R
    ntask = G * CPR
    NCT = -(-ntask // 64) * 64
    NPIECE = (TY + 2) * (XP // VE) + (1 if padded else 0)
    NI = -(-NPIECE // 64)
    SLOT = NI * 64 * VE
    NS = 3 if reg else D + 1 + max(0, int(free) - 1)
    return dict(VE=VE, CPR=CPR, XP=XP, G=G, ntask=ntask, NCT=NCT, NT=NCT + 64, NPIECE=NPIECE, NI=NI, SLOT=SLOT,
                NS=NS, lds_bytes=(NS * SLOT + 64) * es + (64 if free else 0))


def _fits(X, TY, R, D, es=2, pad=0, reg=0, idle=False):
    """Whether the geometry fits (compute lanes, the loader's vmcnt budget, 80 KB of LDS). Without ``idle`` every
    compute lane owns a task (``ntask`` a multiple of 64); with it the last compute wave may hold idle lanes."""
    g = band_geometry(X, TY, R, D, es, pad, reg)
    return (idle or g['ntask'] % 64 == 0) and g['NCT'] <= 960 and D * g['NI'] <= 63 and g['lds_bytes'] <= 80 * 1024


def band_choice(X, nstore=1, es=2, pad=0, reg=0, idle=False, star=False, wide16=True):
    """(TY, R, D) for rows of X elements, or None. fp16, measured (scripts/probes/band_ab.py,
    profiles/r03_band_ab*.log): 8-row bands of 4 rows per lane with 2 planes in flight at X = 768 and 1024
    (27-point 1024³: 0.895 ms vs 0.921 for 4-row bands of 2 rows per lane, 3 planes in flight); three workgroups
    per CU. fp32 rows hold half the cells per 16-byte chunk: 4-row bands of 4 rows per lane first (the loader's
    vmcnt budget and 80 KB of LDS).

    Round 5 (profiles/r05_band_geo1.log, through the op, same process): fp16 rows of at least 96 chunks whose
    16-row band of 2 rows per lane fills whole compute waves (X = 768: 12 compute waves, one workgroup per CU)
    take that band first — 27-point 768³ fwd+bwd 0.675 vs 0.705-0.711 ms with 8-row bands of 4 rows (2 planes in
    flight; 18 rows read per 16 stored instead of 10 per 8: the memory pattern alone 0.640 vs 0.662 ms), fp16
    7-point 768³ 0.604 vs 0.630 (``star``: 1 plane in flight, 0.626 with 2). 512-wide rows (8 compute waves) keep the
    8-row bands (0.210 vs 0.198 ms); 1024-wide rows do not fit 16 row groups of 128 chunks."""
    VE = 16 // es
    if X < 16 * VE:
        return None
    rmax = 4 if nstore == 1 else 2
    CPR = -(-X // VE)
    if wide16 and es == 2 and CPR >= 96 and X % VE == 0:
        first = (16, 2, 1 if star else 2)
        g = band_geometry(X, *first, es, pad, reg)
        # one workgroup per CU (up to 160 KB of LDS; the padded image at X = 768 takes 84 KB)
        if first[1] <= rmax and g['ntask'] % 64 == 0 and g['NCT'] <= 960 and first[2] * g['NI'] <= 63 and \
                g['lds_bytes'] <= 160 * 1024:
            return first
    # fp16: 16-row bands of 2 rows per lane before 4- / 8-row bands with 3 planes in flight (27-point 512²×640 0.279 vs
    # 0.335 ms, ×384 0.166 vs 0.170; fp16 7-point ×640 0.248 vs 0.252, ×384 0.149 vs 0.153: profiles/r04_op_band_823.log)
    cands = [(8, 4, 2), (16, 2, 2), (4, 2, 3), (8, 2, 3)] if es == 2 else [(4, 4, 2), (8, 4, 2), (4, 2, 2), (8, 2, 2)]
    cands += [(12, 4, 2), (16, 4, 2), (16, 2, 2), (32, 4, 2), (32, 2, 2)]
    for TY, R, D in cands:
        if R <= rmax and _fits(X, TY, R, D, es, pad, reg):
            return TY, R, D
    if idle:
        # rows whose chunk count leaves no band height of whole compute waves (X = 504 / 520 / 760 / 1000 halves: 63 /
        # 65 / 95 / 125 chunks): the last compute wave holds idle lanes. Measured through the op against the zsum
        # schedule these rows took before (profiles/r04_op_band_idle.log, fwd+bwd): 16-row bands of 2 rows per lane
        # first — 27-point 512²×520 0.246 vs 0.320 ms, ×504 0.217 vs 0.272, ×760 0.313 vs 0.400; fp16 7-point ×520
        # 0.194 vs 0.290, ×504 0.195 vs 0.249 — then 16-row bands of 4 rows per lane, one plane in flight (27-point
        # ×1000 0.402 vs 0.538). fp32: 8-row bands of 2 rows per lane (7-point ×520 0.389 vs 0.632 ms)
        order = [(16, 2, 2), (16, 4, 1), (8, 4, 2), (8, 2, 3)] if es == 2 else [(8, 2, 2), (8, 4, 2), (4, 4, 2)]
        for TY, R, D in order:
            g = band_geometry(X, TY, R, D, es, pad, reg)
            if R <= rmax and g['NCT'] <= 960 and D * g['NI'] <= 63 and g['lds_bytes'] <= 160 * 1024:
                return TY, R, D
    return None


def emit_band(ir, name, cfg):
    """HIP source of the band kernel (signature identical to the march / zsum kernels: fields, 2 halo pointers
    per stencil field, Z Y X zlo zhi ylo yhi xlo xhi zc zstep ntx nty, scalars)."""
    plans = band_plans(ir)
    if plans is None:
        raise ValueError('kernel is not eligible for the band schedule')
    fixed = [f for f in ir.fields if f.has_fixed_shape]
    es = band_esize(ir)
    X = cfg.BX
    TY, R, D = cfg.BTY, cfg.BAND, cfg.D
    breg = bool(cfg.BREG) and X % (16 // es) != 0     # partial rows on a padded image filled through registers
    padded = breg or band_padded(X, es, cfg.BPAD)
    g = band_geometry(X, TY, R, D, es, padded, breg, cfg.BFREE)
    VE, CPR, G, NCT, NT, NPIECE, NI, SLOT, NS = (g[k] for k in ('VE', 'CPR', 'G', 'NCT', 'NT', 'NPIECE', 'NI', 'SLOT',
                                                                 'NS'))
    assert D * NI <= 63 and NT <= 1024, (X, TY, R, D)
    assert not fixed or int(fixed[0].spatial_shape[-1]) == X, 'band kernel compiled for another row length'
    S = ir.stencil_fields[0]
    half = es == 2
    et = '_Float16' if half else 'float'            # storage element type
    XP = g['XP']                                    # row pitch in the LDS image (elements)
    NPR = XP // VE                                  # pieces per image row
    partial = X % VE != 0                           # a row's last chunk is partial (stores: tail of X % VE cells)
    bu = not padded and XP != X                     # rows not a multiple of 16 bytes: row-wise pieces, zero fill
    c0 = VE if padded else 0                        # image column of a row's first element
    bo = not breg and (X * es) % 4 != 0             # rows on half dwords (fp16, X odd): realigned in registers
    assert not partial or cfg.BMASK, 'rows of a partial last chunk need the masked stores'
    czf = bu and not cfg.BZF                        # BZF=0: the first element past a row zeroed in registers
    free = bool(cfg.BFREE)                          # LDS handshake instead of the plane barriers
    assert not (free and breg), 'the LDS handshake takes the LDS-DMA loader'
    assert not (cfg.HWAIT and breg), 'the halo wait is the LDS-DMA loader\'s'
    NCW = NCT // 64                                 # compute waves
    pr = KernelExprPrinter('float', dict(ir.symbol_names))
    W = []
    for pl in plans:
        W.append({k: f'(float)({pr.doprint_expr(v)})' for k, v in pl['w'].items() if v != 0})
    NP = len(plans)
    # accumulator slots per (set, row): fp16 = 4 fp32 pairs over the cells (x+a, x+a+4), fp32 = 4 floats
    at, azero = ('f32x2', '(f32x2)(0.f)') if half else ('float', '0.f')

    def A(si, s, o, a):
        return f'S{si}_{s}_{o}_{a}'

    def operand(a, dx):
        return f'P{a + dx + 1}' if half else f'H{a + dx + 1}'

    def cell(si, s, o, q):
        """Cell q (0..VE-1) of a row's chunk as a storage-type value."""
        if half:
            return f'(_Float16){A(si, s, o, q % 4)}.{"x" if q < 4 else "y"}'
        return A(si, s, o, q)

    params = _field_params(ir)
    params += [f'const {et}* __restrict__ hlo_{S.name}', f'const {et}* __restrict__ hhi_{S.name}']
    params += ['const int Z', 'const int Y', 'const int X', 'const int zlo', 'const int zhi', 'const int ylo',
               'const int yhi', 'const int xlo', 'const int xhi', 'const int zc', 'const int zstep', 'const int ntx',
               'const int nty']
    params += extra_params(cfg)
    params += _scalar_params(ir)
    L = [PRELUDE, 'typedef unsigned u32x4 __attribute__((ext_vector_type(4)));',
         'typedef unsigned u32x3 __attribute__((ext_vector_type(3)));', 'typedef unsigned u32x2 __attribute__((ext_vector_type(2)));']
    L.append(f'// band schedule: {TY}-row bands of full {X}-element rows, {R} rows x {VE} cells per lane, {NCT // 64} '
             f'compute waves + LDS-DMA loader wave, {NS}-slot {et} plane ring ({D} planes in flight), z partial sums '
             f'in 3 rotating register sets, LDS {g["lds_bytes"]} B')
    L.append(f'extern "C" __global__ void __launch_bounds__({NT}) {name}({", ".join(params)})\n{{')
    if cfg.SIG:
        L += start_signal_lines()
    L.append(f'  __shared__ __attribute__((aligned(1024))) {et} lds[{NS * SLOT + 64}];')
    L.append('  const int tid = threadIdx.x, lane = tid & 63;')
    L.append('  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);')
    if free:
        # hs[0]: planes landed (the loader's), hs[1 + w]: planes compute wave w has finished reading (its own word).
        # Set before the one workgroup barrier of the kernel; the plane steps then never meet at a barrier
        L.append(f'  __shared__ unsigned hs[{NCW + 1}];          // (relaxed workgroup atomics: ds_read / ds_write, not flat)')
        L.append('  auto hs_ld = [&](const int i) { return __hip_atomic_load(&hs[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };')
        L.append('  auto hs_st = [&](const int i, const unsigned v) { __hip_atomic_store(&hs[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };')
        L.append(f'  if (tid <= {NCW}) hs[tid] = 0u;')
        L.append('  __syncthreads();')
    if cfg.MAP == 1:
        L.append('  const int lb = blockIdx.x;')
    else:
        L.append('  // XCD-aware, bijective block remap: consecutive bands share one XCD (and its L2)')
        L.append('  const int nb = gridDim.x, b = blockIdx.x;')
        L.append('  const int per = nb >> 3, rem = nb & 7, xcd = b & 7, bi = b >> 3;')
        L.append('  const int lb = (xcd < rem) ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;')
    L.append('  const int band = lb % nty, chunk = lb / nty;')
    L.append(f'  const int y0 = band * {TY};')
    L.append('  const int zb = zlo + chunk * zstep;       // zstep = zc, or the gap of a two-range launch')
    L.append('  const int ze = min(zb + zc, zhi);')
    L.append('  if (zb >= ze) return;')
    L.append(f'  const i64 YX = (i64)Y * {X};')
    L.append('  const int nplanes = ze - zb + 2;')
    # ---- loader wave
    L.append(f'  const int ldw = {NCT // 64};')
    L.append('  if (wave == ldw) {')
    if not breg:
        L.append(f'    int vo[{NI}];')
        if bo:
            L.append(f'    int vo1[{NI}];')
            L.append('    auto hpar = [&](const void* b) { return (int)(((unsigned long long)b >> 1) & 1); };   // 0 for nullptr')
        L.append('    #pragma unroll')
        L.append(f'    for (int i = 0; i < {NI}; ++i) {{')
        L.append('      const int k = i * 64 + lane;')
        if padded:
            # image row rr = one zero piece (out of range: the DMA writes zeros) + the row's pieces; one zero piece ends
            # the slot (the right neighbour of the last row's end)
            L.append(f'      const int rr = k / {NPR}, pc = k - rr * {NPR}, yy = y0 - 1 + rr;')
            L.append(f'      vo[i] = (pc > 0 && rr < {TY + 2} && yy >= 0 && yy < Y) ? (yy * {X * es} + 16 * (pc - 1)) : '
                     '0x7ffffff0;')
        elif not bu:
            L.append(f'      vo[i] = k < {NPIECE} ? ((y0 - 1) * {X * es} + 16 * k) : 0x7ffffff0;   // row -1 / past Y: range '
                     'check')
        elif not bo:
            # rows of a pitch that is not a multiple of 16 bytes: each row's pieces start at the row (dword-aligned, the
            # LDS image keeps a 16-byte row pitch XP); the last piece runs past the row end (zero-filled below)
            L.append(f'      const int rr = k / {NPR}, pc = k - rr * {NPR}, yy = y0 - 1 + rr;')
            L.append(f'      vo[i] = (k < {NPIECE} && yy >= 0 && yy < Y) ? (yy * {X * es} + 16 * pc) : 0x7ffffff0;')
        else:
            # rows on half dwords: a row starting on an odd element (plane parity pp of the plane's first element, the
            # row's own parity) is loaded from one element early; offsets from the plane's dword-aligned base, one set
            # per plane parity
            L.append(f'      const int rr = k / {NPR}, pc = k - rr * {NPR}, yy = y0 - 1 + rr;')
            L.append(f'      const bool ok = k < {NPIECE} && yy >= 0 && yy < Y;')
            L.append(f'      const int s0 = yy * {X} - (yy & 1), s1 = 1 + yy * {X} - ((yy & 1) ^ 1);   // even elements')
            L.append(f'      vo[i] = ok ? 2 * s0 + 16 * pc : 0x7ffffff0;')
            L.append(f'      vo1[i] = ok ? 2 * s1 + 16 * pc : 0x7ffffff0;')
        L.append('    }')
        L.append('    auto issue = [&](const int q, const int slot) {')
        L.append(f'      const {et}* pb = {_ws_plane_base(S, 1, "q")};')
        if bo:
            L.append('      const int pp = hpar(pb);')
            L.append(f'      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(pb ? pb - pp : '
                     f'f_{S.name}), (short)0, pb ? (int)((YX * 2 + 2 * pp + 3) & ~3ll) : 0, 0x00020000);')
        else:
            L.append(f'      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(pb ? pb : '
                     f'f_{S.name}), (short)0, pb ? (int)(YX * {es}) : 0, 0x00020000);')
        L.append(f'      {et}* dst = lds + slot * {SLOT};')
        if cfg.BABL == 3:
            L.append('      if (Z < 0)   // ablation probe: no plane loads')
        L.append('      #pragma unroll')
        L.append(f'      for (int i = 0; i < {NI}; ++i)')
        L.append(f'        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + i * '
                 f'{64 * VE}), 16, {"pp ? vo1[i] : vo[i]" if bo else "vo[i]"}, 0, 0, 0);')
        L.append('    };')
        if free:
            # slot reuse: plane p goes into the slot of plane p - NS, which every compute wave must have released
            # (hs[1 + w] >= p - NS + 1); one LDS dword per lane, a wave-wide vote, s_sleep between polls
            L.append('    auto wait_free = [&](const int need) {')
            L.append('      if (need <= 0) return;')
            L.append('      while (true) {')
            L.append(f'        const unsigned v = lane < {NCW} ? hs_ld(1 + lane) : 0xffffffffu;')
            L.append('        if (__builtin_amdgcn_ballot_w64(v < (unsigned)need) == 0ull) break;')
            L.append('        __builtin_amdgcn_s_sleep(1);')
            L.append('      }')
            L.append('      asm volatile("" ::: "memory");')
            L.append('    };')
        if cfg.HWAIT:
            L += halo_wait_lines()
        L.append(f'    for (int i = 0; i < {D}; ++i)')
        L.append('      if (i < nplanes) issue(zb - 1 + i, i);')
        L.append('    for (int j = 0; j < nplanes; ++j) {')
        L.append('      // barrier j publishes plane j: the planes issued after it stay in flight')
        L.append(f'      const int after = min({D - 1}, nplanes - 1 - j);')
        L.append('      switch (after) {')
        for a in range(D):
            L.append(f'        case {a}: asm volatile("s_waitcnt vmcnt({a * NI})" ::: "memory"); break;')
        L.append('      }')
        if bo and not czf:
            # plane j has landed: zeros over the image columns past each row's last element (X + the row's parity .. XP)
            nz = XP - X
            L.append('      {')
            L.append(f'        const int ppj = hpar({_ws_plane_base(S, 1, "(zb - 1 + j)")});')
            L.append(f'        {et}* img = lds + (j % {NS}) * {SLOT};')
            L.append(f'        for (int i = lane; i < {(TY + 2) * nz}; i += 64) {{')
            L.append(f'          const int rr = i / {nz}, c = i - rr * {nz}, pos = {X} + (ppj ^ ((y0 - 1 + rr) & 1)) + c;')
            L.append(f'          if (pos < {XP}) img[rr * {XP} + pos] = ({et})0;')
            L.append('        }')
            L.append('        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");')
            L.append('      }')
        elif bu and not czf:
            # plane j has landed: zeros over the image columns X .. XP of every row (the straddling last piece brought
            # the next row's first elements), which the row's last cells read as their right neighbours
            ndw = (XP - X) * es // 4
            L.append('      {')
            L.append(f'        unsigned* img = (unsigned*)(lds + (j % {NS}) * {SLOT});')
            L.append(f'        for (int i = lane; i < {(TY + 2) * ndw}; i += 64) '
                     f'img[(i / {ndw}) * {XP * es // 4} + {X * es // 4} + i % {ndw}] = 0u;')
            L.append('        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");')
            L.append('      }')
        if free:
            # publish plane j (its DMA landed: the vmcnt wait above; the zero fill: its lgkmcnt wait), then refill
            L.append('      if (lane == 0) hs_st(0, (unsigned)(j + 1));')
            L.append(f'      if (j + {D} < nplanes) {{ wait_free(j + {D} - {NS} + 1); issue(zb - 1 + j + {D}, (j + {D}) % {NS}); }}')
        else:
            L.append('      __builtin_amdgcn_s_barrier();')
            L.append(f'      if (j + {D} < nplanes) issue(zb - 1 + j + {D}, (j + {D}) % {NS});')
        L.append('    }')
        L.append('    return;')
        L.append('  }')
    if breg:
        # register-staged loader for rows whose pitch is not a multiple of 16 bytes: each lane owns 16-byte image
        # pieces (pads, rows outside the plane: zeros); a row piece is read with 16-byte (and, on half-dword rows,
        # one more 4-byte) buffer loads at the dword at or below it, realigned by v_alignbyte, its cells past X
        # zeroed, and written to the padded image with ds_write_b128 -- aligned image, no zero fill, no DMA at a
        # row's misaligned start.
        nrs = 1
        L.append(f'    int go[{NI}];                        // byte offset of the piece in its plane (row piece)')
        L.append('    unsigned okm = 0u, lastm = 0u;       // pieces that are row data / a row\'s partial last piece')
        L.append('    #pragma unroll')
        L.append(f'    for (int i = 0; i < {NI}; ++i) {{')
        L.append('      const int k = i * 64 + lane;')
        L.append(f'      const int rr = k / {NPR}, pc = k - rr * {NPR}, yy = y0 - 1 + rr;')
        L.append(f'      const bool ok = pc > 0 && rr < {TY + 2} && yy >= 0 && yy < Y;')
        L.append(f'      go[i] = ok ? (yy * {X} + (pc - 1) * {VE}) * {es} : 0;')
        L.append('      okm |= ok ? (1u << i) : 0u;')
        L.append(f'      lastm |= (ok && pc == {CPR}) ? (1u << i) : 0u;')
        L.append('    }')
        for sname in ('a', 'b')[:nrs]:
            L.append(f'    u32x4 r{sname}[{NI}];')
            if half:
                L.append(f'    unsigned e{sname}[{NI}];')
            L.append(f'    int a{sname} = 0;')

        def load(sname, q):
            B = ['    {',
                 f'      const {et}* pb = {_ws_plane_base(S, 1, "(" + q + ")")};',
                 f'      a{sname} = pb ? (int)((unsigned long long)pb & 3ull) : 0;',
                 f'      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(pb ? '
                 f'(const char*)pb - a{sname} : (const char*)f_{S.name}), (short)0, pb ? (int)((a{sname} + YX * {es} + 3) '
                 f'& ~3ll) : 0, 0x00020000);',
                 '      #pragma unroll',
                 f'      for (int i = 0; i < {NI}; ++i) {{',
                 f'        const int o = ((okm >> i) & 1u) ? ((a{sname} + go[i]) & ~3) : 0x7ffffff0;',
                 f'        r{sname}[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);']
            if half:
                B.append(f'        e{sname}[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 16, 0, 0);')
            B += ['      }', '    }']
            return B

        kx = X % VE                                      # valid cells of a row's last piece
        keep = []                                        # per dword of the last piece: mask of the bits kept
        for dwi in range(4):
            lo_el, hi_el = dwi * (4 // es), dwi * (4 // es) + (4 // es) - 1
            if hi_el < kx:
                keep.append(0xffffffff)
            elif lo_el < kx:
                keep.append(0x0000ffff)
            else:
                keep.append(0)

        def store(sname, slot):
            B = ['    {',
                 f'      {et}* img = lds + {slot} * {SLOT};',
                 '      #pragma unroll',
                 f'      for (int i = 0; i < {NI}; ++i) {{',
                 f'        u32x4 v = r{sname}[i];']
            if half:
                B += [f'        if ((a{sname} + go[i]) & 2) {{            // the piece starts on a half dword',
                      f'          v = (u32x4){{__builtin_amdgcn_alignbyte(v.y, v.x, 2u), __builtin_amdgcn_alignbyte(v.z, v.y, 2u), '
                      f'__builtin_amdgcn_alignbyte(v.w, v.z, 2u), __builtin_amdgcn_alignbyte(e{sname}[i], v.w, 2u)}};',
                      '        }']
            B += ['        if ((lastm >> i) & 1u) {                // cells past X: zeros (right neighbour of cell X-1)',
                  '          ' + ' '.join(f'v.{"xyzw"[d]} &= {keep[d]:#x}u;' for d in range(4) if keep[d] != 0xffffffff),
                  '        }',
                  f'        *(u32x4*)(img + (i * 64 + lane) * {VE}) = v;',
                  '      }',
                  '    }']
            return B
        # planes 0 and 1 before the first barrier, then plane j+2 between barriers j and j+1 (loads, wait, writes:
        # the load latency is the loader's alone, hidden behind the compute of plane j; three slots: slot (j+2) % 3
        # held plane j-1, which every compute wave finished before barrier j). No registers live across a barrier
        # or the loop's back edge, so the compiler's own vmcnt waits are exact.
        L += load('a', 'zb - 1')
        L += store('a', '0')
        L.append('    if (nplanes > 1) {')
        L += load('a', 'zb')
        L += store('a', '1')
        L.append('    }')
        L.append('    for (int j = 0; j < nplanes; ++j) {')
        L.append('      asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");')
        L.append('      if (j + 2 < nplanes) {')
        L += load('a', '(zb + 1 + j)')
        L += store('a', f'((j + 2) % {NS})')
        L.append('      }')
        L.append('    }')
        L.append('    return;')
        L.append('  }')
    # ---- compute lanes
    if bo:
        L.append('  auto hpar = [&](const void* b) { return (int)(((unsigned long long)b >> 1) & 1); };   // 0 for nullptr')
    L.append('  const int ctid = (wave - (wave > ldw ? 1 : 0)) * 64 + lane;   // compute task')
    L.append(f'  const bool active = ctid < {g["ntask"]};')
    L.append(f'  const int t = active ? ctid : {g["ntask"] - 1};')
    L.append(f'  const int grp = t / {CPR}, col = t - grp * {CPR};')
    L.append(f'  const int lofs = grp * {R * XP} + {c0} + col * {VE};   // slot row grp*R = input row y0 + grp*R - 1')
    L.append(f'  const int x = col * {VE};')
    L.append(f'  const bool lmask = col == 0, rmask = col == {CPR - 1};')
    if bo:
        # the x-boundary zeros of half-dword rows as per-lane AND masks held in VGPRs (opaque to the compiler, so they
        # are not folded back into selects on 64-bit lane masks: those, with the per-plane v_perm selectors, ran the
        # kernel out of SGPRs — v_writelane / v_readlane spills in the plane loop)
        L.append('  unsigned lk0 = lmask ? 0xffff0000u : 0xffffffffu, rk = rmask ? 0u : 0xffffffffu, '
                 'rk0 = rmask ? 0xffff0000u : 0xffffffffu;')
        L.append('  asm volatile("" : "+v"(lk0), "+v"(rk), "+v"(rk0));')
    if cfg.BMASK:
        L.append(f'  const bool xfull = x >= xlo && x + {VE} <= xhi;')
        L.append(f'  const bool xtail = x + {VE} > {X};                 // the row\'s partial last chunk (unaligned rows)')
    L.append(f'  const int yrow0 = y0 + grp * {R};')
    L.append(f'  const unsigned sofs = (unsigned)(yrow0 * {X} + x) * {es}u;')
    if cfg.BMASK:
        L.append('  unsigned rowok = 0u;                           // rows of the lane inside [ylo, yhi), one bit each')
        L.append(f'  for (int o = 0; o < {R}; ++o) rowok |= (active && yrow0 + o >= ylo && yrow0 + o < yhi) ? (1u << o) : 0u;')
    L.append("  // edge dword (elements, from the lane's chunk): lane 0 the dword left of it, lane 63 the one right of it,")
    L.append("  // the other lanes dwords of the wave's block no other lane of their 32-lane half reads (unused): banks")
    L.append("  // (a/4) mod 32 all distinct per half (the compiler pairs these reads into ds_read2st64_b32). Lane 0 of")
    L.append("  // column 0 (x boundary, masked) reads its own first dword instead of the one before the slot.")
    dw = 4 // es                                          # elements per dword
    # dword targets relative to the wave's block (64 chunks of 4 dwords): -1, 0 .. 30 | 33 .. 63, 256
    if padded:
        pass                                              # x neighbours read from the image (zero pads at row ends)
    elif cfg.BEDGE:
        L.append(f'  const int eoff = {dw} * (lane == 0 ? (col == 0 ? 0 : -1) : (lane == 63 ? 256 : (lane < 32 ? lane - 1 '
                 f': lane + 1))) - {VE} * lane;')
    else:
        L.append(f'  const int eoff = {dw} * (lane == 0 ? -1 : (lane == 63 ? 256 : lane)) - {VE} * lane;')
    for si in range(NP):
        for s_ in range(3):
            for o in range(R):
                L.append(f'  {at} ' + ', '.join(f'{A(si, s_, o, a)} = {azero}' for a in range(4)) + ';')
    store_field = [pl['field'] for pl in plans]

    def row_prologue(ind, r):
        B = [f'{ind}    const {et}* rp = sl + {r * XP};']
        if bo:
            # image row r starts one element early when the input row starts on an odd element: realign the lane's
            # 10 elements x-1 .. x+8 as five dwords (v_perm over adjacent dwords; selector per row and plane parity)
            sel = 'selA' if r % 2 else 'selB'
            cq = '' if czf else 'const '
            B += [f'{ind}    const u32x4 d = *(const u32x4*)rp;',
                  f'{ind}    const unsigned e = *(const unsigned*)(rp + eoff);',
                  f'{ind}    const unsigned lw = __builtin_amdgcn_update_dpp(e, d.w, 0x138, 0xf, 0xf, false);   // wave_shr:1',
                  f'{ind}    const unsigned rw = __builtin_amdgcn_update_dpp(e, d.x, 0x130, 0xf, 0xf, false);   // wave_shl:1',
                  f'{ind}    {cq}f16x2 w0 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(d.x, lw, {sel}) & lk0), '
                  f'w1 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(d.y, d.x, {sel}));',
                  f'{ind}    {cq}f16x2 w2 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(d.z, d.y, {sel})), '
                  f'w3 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(d.w, d.z, {sel}));',
                  # the row's last chunk: x+7 and x+8 both lie at or past X (8·CPR - 1 >= X for odd X) and on a row
                  # loaded one element early both come from the next lane, which may hold another row: zeros
                  f'{ind}    const f16x2 w4 = __builtin_bit_cast(f16x2, __builtin_amdgcn_perm(rw, d.w, {sel}) & rk);',
                  f'{ind}    const _Float16 l = w0[0], rr = w4[1];',
                  *([f'{ind}    w{(X % VE + 1) // 2} = __builtin_bit_cast(f16x2, __builtin_bit_cast(unsigned, '
                     f'w{(X % VE + 1) // 2}) & rk0);   // the first element past the row end (no loader zero fill)']
                    if czf and (X % VE + 1) // 2 < 4 else []),
                  f'{ind}    const f32x2 P0 = {{(float)l, (float)w2[0]}}, P1 = {{(float)w0[1], (float)w2[1]}}, '
                  'P2 = {(float)w1[0], (float)w3[0]};',
                  f'{ind}    const f32x2 P3 = {{(float)w1[1], (float)w3[1]}}, P4 = {{(float)w2[0], (float)w4[0]}}, '
                  'P5 = {(float)w2[1], (float)rr};']
            return B
        if padded:
            # the dwords left and right of the lane's chunk straight from the image (a row's end chunks meet the zero
            # pads): no DPP, no boundary selects (one ds_read2_b32 per row)
            B += [f'{ind}    const unsigned el = *(const unsigned*)(rp - {dw}), er = *(const unsigned*)(rp + {VE});']
        if padded:
            if half:
                B += [f'{ind}    const f16x8 v = *(const f16x8*)rp;',
                      f'{ind}    const _Float16 l = __builtin_bit_cast(f16x2, el)[1], rr = __builtin_bit_cast(f16x2, er)[0];',
                      f'{ind}    const f32x2 P0 = {{(float)l, (float)v[3]}}, P1 = {{(float)v[0], (float)v[4]}}, '
                      'P2 = {(float)v[1], (float)v[5]};',
                      f'{ind}    const f32x2 P3 = {{(float)v[2], (float)v[6]}}, P4 = {{(float)v[3], (float)v[7]}}, '
                      'P5 = {(float)v[4], (float)rr};']
            else:
                B += [f'{ind}    const f32x4 v = *(const f32x4*)rp;',
                      f'{ind}    const float H0 = __builtin_bit_cast(float, el), H5 = __builtin_bit_cast(float, er);',
                      f'{ind}    const float H1 = v.x, H2 = v.y, H3 = v.z, H4 = v.w;']
            return B
        vt = 'f16x8' if half else 'f32x4'
        if czf:
            # the last chunk's element X % VE is the next row's first (no loader zero fill): zero, as the right
            # neighbour of cell X-1
            B += [f'{ind}    {vt} v = *(const {vt}*)rp;',
                  f'{ind}    v[{X % VE}] = rmask ? ({et})0 : v[{X % VE}];',
                  f'{ind}    const u32x4 d = __builtin_bit_cast(u32x4, v);']
        else:
            B += [f'{ind}    const {vt} v = *(const {vt}*)rp;',
                  f'{ind}    const u32x4 d = __builtin_bit_cast(u32x4, v);']
        B += [f'{ind}    const unsigned e = *(const unsigned*)(rp + eoff);',
              f'{ind}    const unsigned lw = __builtin_amdgcn_update_dpp(e, d.w, 0x138, 0xf, 0xf, false);   // wave_shr:1',
              f'{ind}    const unsigned rw = __builtin_amdgcn_update_dpp(e, d.x, 0x130, 0xf, 0xf, false);   // wave_shl:1']
        if half:
            B += [f'{ind}    const _Float16 l = lmask ? (_Float16)0 : __builtin_bit_cast(f16x2, lw)[1];',
                  f'{ind}    const _Float16 rr = rmask ? (_Float16)0 : __builtin_bit_cast(f16x2, rw)[0];',
                  f'{ind}    const f32x2 P0 = {{(float)l, (float)v[3]}}, P1 = {{(float)v[0], (float)v[4]}}, '
                  'P2 = {(float)v[1], (float)v[5]};',
                  f'{ind}    const f32x2 P3 = {{(float)v[2], (float)v[6]}}, P4 = {{(float)v[3], (float)v[7]}}, '
                  'P5 = {(float)v[4], (float)rr};']
        else:
            B += [f'{ind}    const float H0 = lmask ? 0.f : __builtin_bit_cast(float, lw), '
                  'H5 = rmask ? 0.f : __builtin_bit_cast(float, rw);',
                  f'{ind}    const float H1 = v.x, H2 = v.y, H3 = v.z, H4 = v.w;']
        return B

    def taps(ind, r, sets, first):
        """FMA statements of input row r into the given (set, dz) accumulators, dx outer."""
        B = []
        if cfg.BABL == 1:
            # ablation probe: one add per row and set (the row's loads and one convert stay live)
            for st, dz in sets:
                for si in range(NP):
                    o = min(max(r - 1, 0), R - 1)
                    acc = A(si, st, o, 0)
                    if dz == -1 and (si, o, 0) not in first:
                        first.add((si, o, 0))
                        B.append(f'{ind}{acc} = {operand(0, 0)};')
                    else:
                        B.append(f'{ind}{acc} = {acc} + {operand(0, 0)};')
            return B
        for dx in (-1, 0, 1):
            for st, dz in sets:
                for si in range(NP):
                    for o in range(R):
                        dy = r - o - 1
                        wv = W[si].get((dz, dy, dx)) if -1 <= dy <= 1 else None
                        if wv is None:
                            continue
                        for a in range(4):
                            acc = A(si, st, o, a)
                            term = f'{wv} * {operand(a, dx)}'
                            if dz == -1 and (si, o, a) not in first:
                                first.add((si, o, a))
                                B.append(f'{ind}{acc} = {term};')
                            else:
                                B.append(f'{ind}{acc} = {acc} + {term};')
        return B

    # the partial last chunk stored as one shifted 16-byte chunk (BTAIL): needs a left neighbour chunk of the same row in
    # the same wave for every row group's tail lane (never lane 0 of a wave)
    tail_sb = ((VE - X % VE) % VE) * es                 # bytes the row's last chunk lacks
    tail_shift = bool(cfg.BTAIL) and partial and cfg.BXW and CPR >= 2 and \
        all((grp * CPR + CPR - 1) % 64 != 0 for grp in range(G))

    def tail_shift_lines(src, dst):
        """``dst`` = the 16 bytes ending at the row's end: the left lane's last ``tail_sb`` bytes, then ``src``'s
        first 16 - tail_sb bytes (dword selects, and v_alignbyte when the shift is not whole dwords)."""
        q, b = tail_sb // 4, tail_sb % 4
        k0 = 4 - q - (1 if b else 0)                      # first dword of the result in (left lane | own)
        need = sorted({k0 + i for i in range(4)} | ({k0 + i + 1 for i in range(4)} if b else set()))
        out = []
        seq = {}
        for k in need:
            if k < 4:                                     # the left lane's dword k (wave_shr:1)
                out.append(f'const unsigned nb{k} = __builtin_amdgcn_update_dpp(0u, {src}.{"xyzw"[k]}, 0x138, 0xf, 0xf, '
                           'false);')
                seq[k] = f'nb{k}'
            else:
                seq[k] = f'{src}.{"xyzw"[k - 4]}'
        if b:
            parts = [f'__builtin_amdgcn_alignbyte({seq[k0 + i + 1]}, {seq[k0 + i]}, {4 - b}u)' for i in range(4)]
        else:
            parts = [seq[k0 + i] for i in range(4)]
        out.append(f'const u32x4 {dst} = {{{", ".join(parts)}}};')
        return out

    def stores(ind, si, sp, fld, rows=None):
        B = [f'{ind}{{',
             f'{ind}  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc('
             f'(void*)(f_{fld.name} + (i64)(zb - 2 + jj) * YX), (short)0, (int)(YX * {es}), 0x00020000);']
        vt = 'f16x8' if half else 'f32x4'
        for o in (range(R) if rows is None else rows):
            vals = ', '.join(cell(si, sp, o, q) for q in range(VE))
            st = (f'__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ov), ors, sofs + '
                  f'{o * X * es}u, 0, 2);')
            if not cfg.BMASK:
                # every row of every band inside [ylo, yhi), x range = whole rows (checked at plan time)
                B.append(f'{ind}  {{ const {vt} ov = {{{vals}}}; {st} }}')
                continue
            nb_t = (X % VE) * es if partial else 0           # bytes of a row's partial last chunk
            ndw_t, nh_t = nb_t // 4, (nb_t % 4) // 2       # whole dwords, then one half (X odd)
            if cfg.BXW:
                # whole rows: no branches. A row outside [ylo, yhi) (or an idle lane's) stores at an offset past the
                # buffer's range, which the range check drops; a partial last chunk stores its whole dwords (and
                # half) at the row offset while its 16-byte store is dropped, every other lane the reverse
                ro = f'((rowok & {1 << o}u) ? sofs + {o * X * es}u : 0x7ffffff0u)'
                B.append(f'{ind}  {{ const {vt} ov = {{{vals}}}; const unsigned ro = {ro};')
                if partial and tail_shift:
                    # the row's partial last chunk as ONE 16-byte store of the row's last VE cells, shifted left by
                    # the sb bytes the chunk lacks: the first of them are the left lane's last cells (DPP wave_shr:1,
                    # the same row; that lane stores the same values there), so the row takes one store instruction
                    # instead of three (16-byte, then dword and half stores that drop 63 lanes each)
                    B.append(f'{ind}    const u32x4 ow = __builtin_bit_cast(u32x4, ov);')
                    B += [f'{ind}    {ln}' for ln in tail_shift_lines('ow', 'tw')]
                    B.append(f'{ind}    __builtin_amdgcn_raw_buffer_store_b128(xtail ? tw : ow, ors, xtail ? ro - {tail_sb}u : ro, '
                             f'0, 2);')
                elif partial:
                    c = 'xyzw'
                    B.append(f'{ind}    const u32x4 ow = __builtin_bit_cast(u32x4, ov);')
                    B.append(f'{ind}    __builtin_amdgcn_raw_buffer_store_b128(ow, ors, xtail ? 0x7ffffff0u : ro, 0, 2);')
                    # (the tail store under a branch on the tail lanes measured slower: profiles/r05_pitch_btb.log)
                    B.append(f'{ind}    const unsigned rt = xtail ? ro : 0x7ffffff0u;')
                    tb = []
                    if ndw_t:
                        ty = {1: 'unsigned', 2: 'u32x2', 3: 'u32x3'}[ndw_t]
                        tb.append(f'__builtin_amdgcn_raw_buffer_store_b{32 * ndw_t}(({ty})ow.{c[:ndw_t]}, ors, rt, 0, 2);')
                    if nh_t:
                        tb.append(f'__builtin_amdgcn_raw_buffer_store_b16((unsigned short)ow.{c[ndw_t]}, ors, '
                                  f'rt + {4 * ndw_t}u, 0, 2);')
                    B += [f'{ind}    {t}' for t in tb]
                else:
                    B.append(f'{ind}    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ov), ors, ro, 0, 2);')
                B.append(f'{ind}  }}')
                continue
            B.append(f'{ind}  if (rowok & {1 << o}u) {{')
            B.append(f'{ind}    const {vt} ov = {{{vals}}};')
            B.append(f'{ind}    if (xfull) {{')
            B.append(f'{ind}      {st}')
            B.append(f'{ind}    }} else {{')
            # not a whole in-range chunk. 'bu' rows: the partial last chunk holds X % VE cells of the row (the rest is
            # the next row's), stored as whole dwords (X·es is a multiple of 4)

            def tail_store(vec):
                """The partial last chunk of vector ``vec``: whole dwords, then the odd element's half."""
                out, c = [], 'xyzw'
                if ndw_t:
                    ty = {1: 'unsigned', 2: 'u32x2', 3: 'u32x3'}[ndw_t]
                    out.append(f'__builtin_amdgcn_raw_buffer_store_b{32 * ndw_t}(({ty}){vec}.{c[:ndw_t]}, ors, '
                               f'sofs + {o * X * es}u, 0, 2);')
                if nh_t:
                    out.append(f'__builtin_amdgcn_raw_buffer_store_b16((unsigned short){vec}.{c[ndw_t]}, ors, '
                               f'sofs + {o * X * es + 4 * ndw_t}u, 0, 2);')
                return ' '.join(out)

            def tail_load(dst):
                """Read the current contents of the partial last chunk into ``dst`` (read-modify-write)."""
                out, c = [], 'xyzw'
                if ndw_t == 1:
                    out.append(f'{dst}.x = __builtin_amdgcn_raw_buffer_load_b32(ors, sofs + {o * X * es}u, 0, 0);')
                elif ndw_t:
                    ty = {2: 'u32x2', 3: 'u32x3'}[ndw_t]
                    out.append(f'{{ const {ty} t = __builtin_amdgcn_raw_buffer_load_b{32 * ndw_t}(ors, '
                               f'sofs + {o * X * es}u, 0, 0); ' + ' '.join(f'{dst}.{c[i]} = t.{c[i]};'
                                                                        for i in range(ndw_t)) + ' }')
                if nh_t:
                    out.append(f'{dst}.{c[ndw_t]} = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(ors, '
                               f'sofs + {o * X * es + 4 * ndw_t}u, 0, 0);')
                return ' '.join(out)
            if cfg.XB:
                # x border cells: zeros (the row is stored whole); each cell selected on its own
                sel = ', '.join(f'(x + {q} >= xlo && x + {q} < xhi) ? {cell(si, sp, o, q)} : ({et})0' for q in range(VE))
                B.append(f'{ind}      const {vt} zv = {{{sel}}};')
                full = (f'__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, zv), ors, '
                        f'sofs + {o * X * es}u, 0, 2);')
                if partial:
                    B.append(f'{ind}      const u32x4 zw = __builtin_bit_cast(u32x4, zv);')
                    B.append(f'{ind}      if (xtail) {{ {tail_store("zw")} }} else {{ {full} }}')
                else:
                    B.append(f'{ind}      {full}')
            else:
                # cells outside [xlo, xhi) keep their contents: read-modify-write of the lane's chunk (the whole chunk,
                # or the partial last one), cells selected one by one (per-cell stores cost ~30 VGPRs in the loop)
                B.append(f'{ind}      const u32x4 ow = __builtin_bit_cast(u32x4, ov);')
                B.append(f'{ind}      u32x4 old;')
                if partial:
                    B.append(f'{ind}      if (xtail) {{ old = (u32x4)(0u); {tail_load("old")} }}')
                    B.append(f'{ind}      else old = __builtin_amdgcn_raw_buffer_load_b128(ors, sofs + {o * X * es}u, 0, 0);')
                else:
                    B.append(f'{ind}      old = __builtin_amdgcn_raw_buffer_load_b128(ors, sofs + {o * X * es}u, 0, 0);')
                nw = []
                for d in range(4):
                    if half:
                        lo = f'(x + {2 * d} >= xlo && x + {2 * d} < xhi)'
                        hi = f'(x + {2 * d + 1} >= xlo && x + {2 * d + 1} < xhi)'
                        nw.append(f'(({lo} ? ow.{"xyzw"[d]} : old.{"xyzw"[d]}) & 0xffffu) | '
                                  f'(({hi} ? ow.{"xyzw"[d]} : old.{"xyzw"[d]}) & 0xffff0000u)')
                    else:
                        nw.append(f'(x + {d} >= xlo && x + {d} < xhi) ? ow.{"xyzw"[d]} : old.{"xyzw"[d]}')
                B.append(f'{ind}      const u32x4 nw = {{{", ".join(nw)}}};')
                full = f'__builtin_amdgcn_raw_buffer_store_b128(nw, ors, sofs + {o * X * es}u, 0, 2);'
                if partial:
                    B.append(f'{ind}      if (xtail) {{ {tail_store("nw")} }} else {{ {full} }}')
                else:
                    B.append(f'{ind}      {full}')
            B.append(f'{ind}    }}')
            B.append(f'{ind}  }}')
        B.append(f'{ind}}}')
        if cfg.BNT != 2:
            # store cache policy probe (2 = non-temporal, the default)
            B = [ln.replace(', 0, 2);', f', 0, {cfg.BNT});') if 'raw_buffer_store' in ln else ln for ln in B]
        return B

    def step(k, ind, part='full', guard='jj < nplanes', store='jj >= 2'):
        """One plane with static set roles (k = plane index mod 3). ``part`` drops the taps of outputs outside the
        chunk: 'p0' = the chunk's first input plane (feeds output zb only), 'p1' = its second (not output zb-1),
        'e0' = the second to last (not output ze), 'e1' = the last (feeds output ze-1 only)."""
        sp, s0, sn = (k + 2) % 3, k, (k + 1) % 3
        sets = {'full': ((sp, 1), (s0, 0), (sn, -1)), 'p0': ((sn, -1),), 'p1': ((s0, 0), (sn, -1)),
                'e0': ((sp, 1), (s0, 0)), 'e1': ((sp, 1),)}[part]
        # the plane barrier as one asm statement with a memory clobber: the previous plane's LDS reads complete
        # (lgkmcnt) before it and none of them moves past it, none of this plane's moves above it (with
        # __syncthreads() hipcc 7.2 sank a peeled step's reads below the next step's barrier on the padded-row
        # image: the loader had already refilled that slot; scripts/probes/band_determinism.py)
        B = [f'{ind}if ({guard}) {{' if guard else f'{ind}{{']
        if free:
            # acquire: plane jj has landed once the loader's word exceeds jj (the last value seen is kept, so a wave
            # behind the loader polls no more); the memory clobbers keep this plane's LDS reads below the poll
            B += [f'{ind}  while ((int)seen <= jj) {{',
                  f'{ind}    seen = __builtin_amdgcn_readfirstlane(hs_ld(0));',
                  f'{ind}    if ((int)seen <= jj) __builtin_amdgcn_s_sleep(1);',
                  f'{ind}  }}',
                  f'{ind}  asm volatile("" ::: "memory");']
        else:
            B.append(f'{ind}  asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");')
        B.append(f'{ind}  const {et}* sl = lds + (jj % {NS}) * {SLOT} + lofs;')
        if bo:
            # v_perm selectors: input row parity = plane parity ^ (y0 - 1 + row) & 1, y0 and R even -> odd rows r of
            # the lane take the plane's parity (selA), even rows the other one (selB); 0x05040302 = elements shifted
            # by one (the row was loaded one element early), 0x07060504 = the dword as it is
            B += [f'{ind}  const int ppq = hpar({_ws_plane_base(S, 1, "(zb - 1 + jj)")});',
                  # (scalar arithmetic, not selects: a select becomes a 64-bit lane mask per unrolled step)
                  f'{ind}  const unsigned selA = 0x05040302u + (unsigned)ppq * 0x02020202u, '
                  'selB = 0x07060504u - (unsigned)ppq * 0x02020202u;']
        # sets a trimmed step leaves alone are dead (outputs already stored or outside the chunk): overwrite them first
        # so their old values are not live through the step (a full step overwrites its q+1 set; +16-45 VGPRs else)
        for s_ in sorted({sp, s0, sn} - {st for st, _ in sets}):
            for si in range(NP):
                for o in range(R):
                    B.append(f'{ind}  ' + ' '.join(f'{A(si, s_, o, a)} = {azero};' for a in range(4)))
        first = set()
        # idle lanes (band tasks not a multiple of 64) compute on a clamped task with wrong x neighbours: no stores
        act = 'active' if g['ntask'] != NCT else ''
        cond = ' && '.join(c for c in (store, act) if c) if store is not None else None

        for r in range(R + 2):
            B.append(f'{ind}  {{')
            B += row_prologue(ind, r)
            # every set every plane, one block: dx outer, then the three sets, rows and slots (12-36 independent
            # FMAs between two dependent ones)
            B += taps(f'{ind}    ', r, sets, first)
            B.append(f'{ind}  }}')
        if free:
            # release: this plane's LDS reads are complete; the loader may refill its slot
            B += [f'{ind}  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");',
                  f'{ind}  if (lane == 0) hs_st(1 + wave, (unsigned)(jj + 1));',
                  f'{ind}  asm volatile("" ::: "memory");']
        # outputs of q+1 that received no tap this plane (no dz = -1 taps) start from zero
        if any(dz == -1 for _, dz in sets):
            for si in range(NP):
                for o in range(R):
                    for a in range(4):
                        if (si, o, a) not in first:
                            B.append(f'{ind}  {A(si, sn, o, a)} = {azero};')
        if cfg.BABL == 2 and cond is not None:
            cond = f'({cond}) && Z < 0' if cond else 'Z < 0'          # ablation probe: no output stores
        if store is not None:
            B.append(f'{ind}  if ({cond}) {{' if cond else f'{ind}  {{')
            for si, fld in enumerate(store_field):
                B += stores(f'{ind}    ', si, sp, fld)
            B.append(f'{ind}  }}')
        B.append(f'{ind}  ++jj;')
        B.append(f'{ind}}}')
        return B

    if free:
        L.append('  unsigned seen = 0u;                               // planes known landed (hs[0])')
    L.append('  int jj = 0;')
    if cfg.BTRIM == 1:
        # the chunk's first two input planes run peeled steps without the taps of outputs before it (27 of 27·(zc+2)
        # FMAs per cell column); every chunk has >= 3 planes, so no fallback loop
        L += step(0, '  ', 'p0', None, None)
        L += step(1, '  ', 'p1', None, None)
        L.append('  #pragma unroll 1')
        L.append('  while (jj < nplanes) {')
        for k in (2, 0, 1):
            L += step(k, '    ', 'full', 'jj < nplanes', '')
        L.append('  }')
    elif cfg.BTRIM == 3:
        # chunks of exactly ZMIN planes (every chunk but a ragged last one): peeled first two planes, the main loop
        # over planes 2 .. ZMIN-1, the last two planes peeled after it at their static set roles (ZMIN is a compile-time
        # constant here); other chunks run the full loop
        zc = int(cfg.ZMIN)
        assert cfg.ZMIN == cfg.ZMAX and zc >= 3, 'BTRIM=3 needs a fixed chunk length of >= 3 planes'
        L.append(f'  if (nplanes == {zc + 2}) {{')
        L += step(0, '    ', 'p0', None, None)
        L += step(1, '    ', 'p1', None, None)
        L.append('    #pragma unroll 1')
        L.append(f'    while (jj < {zc}) {{')
        for k in (2, 0, 1):
            L += step(k, '      ', 'full', f'jj < {zc}', '')
        L.append('    }')
        k_end = zc % 3                     # set role of plane jj = zc (= nplanes - 2)
        L += step(k_end, '    ', 'e0', None, '')
        L += step((k_end + 1) % 3, '    ', 'e1', None, '')
        L.append('  } else {                         // a ragged chunk: peeled first two planes only (BTRIM=1)')
        L += step(0, '    ', 'p0', None, None)
        L += step(1, '    ', 'p1', None, None)
        L.append('    #pragma unroll 1')
        L.append('    while (jj < nplanes) {')
        for k in (2, 0, 1):
            L += step(k, '      ', 'full', 'jj < nplanes', '')
        L.append('    }')
        L.append('  }')
    else:
        if cfg.BTRIM == 2:
            # also the last two input planes (the taps of outputs after the chunk; 54 of 27·(zc+2) FMAs per cell
            # column), inside the unrolled loop at each static set role (a switch on jj % 3 after the loop made the
            # compiler select between the register sets: 192 VGPRs instead of 156); chunks of >= 3 planes
            L.append('  if (nplanes >= 5) {')
            L += step(0, '    ', 'p0', None, None)
            L += step(1, '    ', 'p1', None, None)
            L.append('    const int nend = nplanes - 2;')
            L.append('    #pragma unroll 1')
            L.append('    while (jj < nplanes) {')
            for k in (2, 0, 1):
                full = step(k, '      ', 'full', 'jj < nend', '')
                e0 = step(k, '      ', 'e0', 'jj == nend', '')
                e1 = step(k, '      ', 'e1', 'jj < nplanes', '')
                e0[0] = e0[0].replace('if', 'else if', 1)
                e1[0] = e1[0].replace('if', 'else if', 1)
                L += full + e0 + e1
            L.append('    }')
            L.append('  } else {')
        L.append('  #pragma unroll 1')
        L.append('  while (jj < nplanes) {')
        for k in range(3):
            L += step(k, '    ')
        L.append('  }')
        if cfg.BTRIM == 2:
            L.append('  }')
    L.append('}')
    return '\n'.join(L) + '\n'
