"""The lattice Boltzmann schedule: stream-pull-collide SRT forward and adjoint kernels, written for the lattice.

``AutoDiffLatticeBoltzmannStep`` drives rules made by ``create_lb_update_rule`` (lbmpy's SRT
``stream_pull_collide`` kernel [ext], ``/root/reference/src/pystencils_autodiff/lbm/_autodiff_lbstep.py:189-247,
372-398``) through these kernels instead of the general one-thread-per-cell lowering of the rule's
``AssignmentCollection``: the general lowering reads and writes each pdf component as its own field, in the
layout of the caller's tensors, with every cell's 2·Q streams in Q separate component planes.

What this schedule does differently:

* **Layouts by strides.** A pdf array is addressed as ``q·s_q + z·s_z + y·s_y + x·s_x``: the caller's fzyx
  (lbmpy's default, one plane per component) or AoS arrays are read and written in place. The time-step op's
  intermediate states, which only the op sees, use the row-interleaved layout ``[z][y][q][x]``: the Q
  components of a lattice row are one contiguous block (Q·X elements), so a wave's 2·Q accesses per row land
  in ~10 neighbouring row blocks instead of 2·Q planes a whole field apart.
* **Walls.** An optional flag array (``uint8``, one per cell, C order, 1 = no-slip obstacle) turns on lbmpy's
  half-way bounce-back fused into the pull: ``f_i(x) = src_ī(x)`` where ``x − c_i`` is an obstacle
  (``lbmpy.boundaries.NoSlip`` [ext] writes ``src_ī(x + c_i) := src_i(x)`` into the obstacle cell before the
  pull, ``adjoint_boundaryconditions.py:49-72`` moves the adjoint back); obstacle cells keep their state
  (``dst = src`` there — lbmpy's values in obstacle cells are not part of the flow).
* **Adjoint in scatter form through the collision's structure** (``_method.create_lb_adjoint_rule``):
  ``v_j = (1 − ω) g_j + ω (A + Σ_a B_a ∂u_a/∂f_j)`` with two moment-like sums, stored to the cell the forward
  pulled ``f_j`` from — ``(x − c_j, j)``, or ``(x, ī)`` for a bounced ``f_j``. Every (component, cell) of
  the result is written exactly once (for fluid ``x``: by ``x + c_k`` if that cell is fluid, else by ``x``
  itself; obstacle cells by themselves), so the output needs no zero fill and no atomics.

One source is printed for both targets: a HIP kernel (one thread per cell, wave64 along x) compiled by hiprtc,
and a C loop nest (``use_cuda=False`` / ``target='cpu'``) compiled by gcc.
"""
import ctypes
import os
import re
import struct

import numpy as np

__all__ = ['LatticeKernels', 'LaunchPlan', 'lattice_strides', 'row_interleaved_empty', 'neighbour_mask']


def _c(v):
    """A rational / float constant as a C literal of the compute type."""
    return repr(float(v))


SELF_BIT = 30      # bit of a cell's neighbour mask: the cell itself is an obstacle (bits 0..Q-1: x − c_i is one)
FIX_BIT = 31       # ... the cell is a fluid cell next to a wall with a link program (the HIP fix-up kernels' cells)
FIX_BLOCK = 64     # threads per workgroup of the fix-up kernel


def _emit(stencil, compressible, ctype, walls, target, idx, addr='ptr', links=None, force_model=None, force=None,
          force_field=False, trt=None, programs=None, mode='inline', mrt=None):
    """Source of the forward (``lbm_fwd``) and adjoint (``lbm_adj``) kernels.

    ``addr='buf'`` (HIP): every pdf array is one buffer resource (its bytes below 2³²); a component's plane
    offset ``q·s_q`` rides in the instruction's scalar offset and each distinct neighbour cell's byte offset is
    ONE 32-bit VGPR shared by all components that pull from it — no 64-bit address arithmetic per access.
    ``'ptr'``: plain pointers (the C target, and arrays of 4 GiB and more). ``walls``: a ``uint32`` neighbour
    mask per cell (bit i: ``x − c_i`` is an obstacle; bit ``SELF_BIT``: ``x`` is one), one load per cell.
    ``links``: None (every wall a plain bounce-back), or per wall id (the flag array's values) the boundary's link
    coefficients per direction (``boundaries.link_coefficients``): a bounced component then becomes
    ``α·src_ī(x) + β`` (id of the wall cell ``x − c_i`` from the flag array) and its adjoint is scaled by γ.
    ``force_model`` 'simple' / 'guo' with a constant body force ``force`` (D numbers, ``_method._force``): 'simple'
    adds the constant 3 w_i (c_i·F) to every fluid cell's post-collision value (its adjoint is unchanged); 'guo'
    shifts the velocity by F/2 (/ρ) and adds w_i (1 − ω/2)(3 (c_i − u)·F + 9 (c_i·u)(c_i·F)), whose derivative through
    u joins the adjoint's velocity sensitivities: B_a += C_a / ω with
    C_a = (1 − ω/2) Σ_i g_i w_i (9 c_ia (c_i·F) − 3 F_a).
    ``force_field``: the force is a per-cell vector field instead (``force`` unused): the kernels read ``F(x)`` from a
    ``[*domain, D]`` array by strides (an additional input of the rule, ``_autodiff_lbstep.py:113-128``) and the
    adjoint ACCUMULATES the force adjoint into ``dforce`` (same strides; every cell by one thread, so the T steps of
    the time-step op sum into one zeroed array): 'simple' ``dF_a = 3 Σ_i g_i w_i c_ia``; 'guo' — through the explicit
    term and the velocity shift ``∂u_a/∂F_a = 1/2 (/ρ)`` — ``dF_a = (1 − ω/2) Bf_a + ω B_a / 2 (/ρ)`` with ``Bf_a`` the
    equilibrium part of the velocity sensitivity (before the ρ scaling) and ``B_a`` the full one.
    ``trt``: the TRT method (``_method.create_lb_update_rule(method='trt')``): ``('magic', Λ)`` (ω₋ from ω and the
    magic number, computed per launch from the ω argument) or ``('rate', ω₋)`` (a constant). With a = (ω₊ + ω₋)/2,
    b = (ω₊ − ω₋)/2 the collision is ``dst_i = (1 − a) f_i − b f_ī + a feq_i + b feq_ī`` and the adjoint takes the
    equilibrium sums over h_i = a g_i + b g_ī: ``v_j = (1 − a) g_j − b g_ĵ + A_h + Σ_a B_h,a ∂u_a/∂f_j``.
    ``mrt``: the MRT method's relaxation matrix ``A = ω P_ω + C`` (``(P_ω, C)``, Q×Q numbers, ``_method.
    mrt_relaxation_matrices`` summed over the groups relaxing with the ω argument / with constant rates):
    ``dst = f − A (f − feq)``; the adjoint takes the equilibrium sums over h = Aᵀ g: ``v_j = g_j − h_j + A_h + Σ_a B_h,a
    ∂u_a/∂f_j``.
    ``programs``: per wall id None or the boundary's ``link_program`` (links of the cell's own pdfs the fused form does
    not take, ``boundaries.link_program``; their table rows are zeros): the forward evaluates the link from the
    cell's own pdfs ``c0 … c{Q-1}`` (loaded inside the link's branch), the adjoint's first pass stores ``v_j`` of each
    program-linked component j to a per-cell scratch array and the second pass (``lbm_adj_rho``) adds
    ``Σ_j J_jk(c) v_j`` to component k of the cell — the Jacobians are evaluated there, on the cells next to a wall,
    not in the first pass, whose registers they would take on every cell (``mode='inline'``, the C target).
    HIP (``mode='main'`` / ``'fix'``): the forward evaluates the programs inline as above; the main adjoint carries
    no program code and leaves the cells marked ``FIX_BIT`` (fluid cells next to a program wall) to ONE list-driven
    fix-up kernel (``lbm_adj_fix``): the regular scatter plus ``out_k(x) += G_k``, ``G_k = Σ_j J_jk v_j``. An entry
    out_k(x) that receives G_k is written by the cell x + c_k (or x itself, bounced); when that writer is a listed
    cell too (so it runs in the same fix-up launch), the main kernel's thread x zeroes the entry and both the
    writer's value and G_k arrive by atomic adds — two addends onto zero, the same sum in either order, so the result
    is the one the former second fix-up launch (``out += G`` after every other store) gave. The lattice's bulk runs
    the plain adjoint (measured: profiles/r05_lbm_pressure.jsonl, r06_lbm_fix_merge.jsonl)."""
    D, Q = stencil.D, stencil.Q
    dirs = [tuple(d) for d in stencil.directions]
    w = [float(x) for x in stencil.weights]
    fm = None if force_model is None else str(force_model).lower()
    ff = bool(fm) and bool(force_field)
    F = [float(v) for v in force] if fm and not ff else None
    cF = [sum(c * f for c, f in zip(d, F)) for d in dirs] if fm and not ff else None
    inv = [stencil.inverse_direction_index(i) for i in range(Q)]
    if mrt is not None and trt is not None:
        raise NotImplementedError('MRT and TRT lattice kernels at once')
    # Guo with TRT / MRT: the force term (prefactor 1 − ω/2 with the shear rate ω, as lbmpy's Guo model) is not
    # relaxed by the collision matrix, so its adjoint sums run over g while the equilibrium's run over h
    gsplit = fm == 'guo' and (trt is not None or mrt is not None)
    axes = ['z', 'y', 'x'][3 - D:]          # spatial axes, axis 0 slowest; x fastest
    ct = ctype
    hip = target == 'hip'
    buf = hip and addr == 'buf'
    esize = 8 if ctype == 'double' else 4
    L = []
    fn = '__device__ static inline' if hip else 'static inline'
    if not hip:
        L.append('#include <stdint.h>\ntypedef long long i64;')
    L.append(f'typedef {ctype} T;\ntypedef {idx} IDX;')
    if hip:
        L.append('typedef unsigned u32x2 __attribute__((ext_vector_type(2)));')
    # links whose value also depends on the fluid cell's density ρ(x) = Σ_k src_k(x) (a density-weighted moving wall):
    # forward f_j += βρ·ρ(x); the adjoint adds Σ_j βρ_j v_j to every component of the cell in a second pass
    rho_links = links is not None and any(len(t) > 3 and t[3] != 0 for lk in links for t in lk)
    gen = links is not None and programs is not None and any(p is not None for p in programs)
    fix = mode == 'fix'
    if fix and not gen:
        raise ValueError('fix-up kernels need link programs')
    # the adjoint's second pass over a per-cell scratch array: density-weighted links (any mode), link programs inline
    two = rho_links or (gen and mode == 'inline')
    if links is not None:
        # per (wall id, pulled component j): the link of direction d = ī_j (the population that left x towards the
        # wall cell x + c_d = x − c_j comes back as j)
        inv0 = [stencil.inverse_direction_index(i) for i in range(Q)]
        qual = '__constant__ T' if hip else 'static const T'
        cols = (('lk_a', 0), ('lk_b', 1), ('lk_g', 2)) + ((('lk_r', 3), ('lk_gr', 4)) if rho_links else ())
        for nm, col in cols:
            vals = [repr(float(links[k][inv0[j]][col] if col < len(links[k][inv0[j]]) else 0.0))
                    for k in range(len(links)) for j in range(Q)]
            L.append(f'{qual} {nm}[{len(vals)}] = {{{", ".join(vals)}}};')
    low = f'{(1 << Q) - 1}u'                 # neighbour-mask bits of the Q directions
    # the components q of a listed cell x that receive G_q = Σ_j J_jq v_j (link programs' Jacobian columns)
    gq_all = sorted({q for pg in (programs or ()) if pg is not None for row in pg if row is not None
                     for q, _, _ in row[2]}) if gen else []

    def c_(v):
        return f'({ct}){_c(v)}'

    def mat_terms(M, vec, transpose=False):
        """Σ_k M[i][k] vec_k (or M[k][i]) as C, zero entries left out (None when the row is all zeros)."""
        def row(i):
            t = []
            for k in range(Q):
                v = float(M[k][i] if transpose else M[i][k])
                if v != 0.0:
                    t.append(f'{c_(v)} * {vec}{k}')
            return ' + '.join(t) if t else None
        return row

    def Fa(a):
        """Force component a: a constant, or the cell's value (``force_field``)."""
        return f'F{a}' if ff else c_(F[a])

    def cFi(i, scale=1):
        """scale · (c_i · F) (None where it is the constant 0)."""
        if ff:
            if not any(dirs[i]):
                return None
            return f'cF{i}' if scale == 1 else f'({c_(scale)} * cF{i})'
        return c_(scale * cF[i]) if cF[i] else None

    def force_loads(L):
        """The cell's force vector and its projections c_i · F (``force_field``)."""
        if not ff:
            return
        fcell = ' + '.join(f'(IDX){a} * f_{a}' for a in axes)
        L.append(f'  const IDX fc = {fcell};')
        for a in range(D):
            L.append(f'  const {ct} F{a} = ({ct})force[(IDX){a} * f_c + fc];')
        for i in range(Q):
            t = [('+ ' if dirs[i][a] > 0 else '- ') + f'F{a}' for a in range(D) if dirs[i][a]]
            if t:
                e = ' '.join(t)
                L.append(f'  const {ct} cF{i} = {e[2:] if e.startswith("+ ") else "(" + e + ")"};')

    def key(d):
        return '_'.join({0: '0', 1: 'm', -1: 'p'}[c] for c in d)      # pull: x − c → m(inus) / p(lus)

    keys = sorted({key(d) for d in dirs})

    def coord(k, a):
        c = k.split('_')[axes.index(a)]
        return a if c == '0' else f'{a}{c}'

    def neighbour_offsets(L, prefix):
        """One element (ptr) or byte (buf) offset per distinct neighbour cell of tensor ``prefix``."""
        for k in keys:
            e = ' + '.join(f'(IDX){coord(k, a)} * {prefix}_{a}' for a in axes)
            if buf:
                L.append(f'  const unsigned {prefix}o_{k} = (unsigned)({e}) * {esize}u;')
            else:
                L.append(f'  const IDX {prefix}o_{k} = {e};')

    def soff(prefix, comp):
        return f'{comp} * {prefix}_qb' if buf else None

    def load(prefix, arr, comp, off):
        if buf:
            bits = 'b64' if esize == 8 else 'b32'
            ty = 'u32x2' if esize == 8 else 'unsigned'
            return (f'({ct})__builtin_bit_cast(T, ({ty})__builtin_amdgcn_raw_buffer_load_{bits}('
                    f'rs_{prefix}, {off}, {soff(prefix, comp)}, 0))')
        return f'({ct}){arr}[(IDX){comp} * {prefix}_q + {off}]'

    def store(prefix, arr, comp, off, val):
        if buf:
            bits = 'b64' if esize == 8 else 'b32'
            ty = 'u32x2' if esize == 8 else 'unsigned'
            return (f'__builtin_amdgcn_raw_buffer_store_{bits}(__builtin_bit_cast({ty}, (T)({val})), rs_{prefix}, '
                    f'{off}, {soff(prefix, comp)}, 0);')
        return f'{arr}[(IDX){comp} * {prefix}_q + {off}] = (T)({val});'

    def wrap_lines(L):
        for a in axes:
            N = a.upper()
            L.append(f'  const int {a}m = {a} == 0 ? {N} - 1 : {a} - 1, {a}p = {a} == {N} - 1 ? 0 : {a} + 1;')

    def rsrc(L, prefix, arr):
        if buf:
            L.append(f'  const __amdgpu_buffer_rsrc_t rs_{prefix} = __builtin_amdgcn_make_buffer_rsrc((void*){arr}, '
                     f'(short)0, (int){prefix}_bytes, 0x00020000);')
            L.append(f'  const int {prefix}_qb = (int){prefix}_q * {esize};')

    centre = '_'.join('0' for _ in axes)

    def load_v(prefix, voff):
        """One buffer load at a per-lane byte offset (plane offset folded in, no scalar offset)."""
        bits = 'b64' if esize == 8 else 'b32'
        ty = 'u32x2' if esize == 8 else 'unsigned'
        return (f'({ct})__builtin_bit_cast(T, ({ty})__builtin_amdgcn_raw_buffer_load_{bits}('
                f'rs_{prefix}, {voff}, 0, 0))')

    def store_v(prefix, voff, val):
        bits = 'b64' if esize == 8 else 'b32'
        ty = 'u32x2' if esize == 8 else 'unsigned'
        return (f'__builtin_amdgcn_raw_buffer_store_{bits}(__builtin_bit_cast({ty}, (T)({val})), rs_{prefix}, '
                f'{voff}, 0, 0);')

    def ncell(k):
        """C-order cell index of the neighbour ``x − c`` of pull key ``k`` (wrapped coordinates)."""
        if D == 3:
            return f'((IDX){coord(k, "z")} * Y + {coord(k, "y")}) * X + {coord(k, "x")}'
        return f'(IDX){coord(k, "y")} * X + {coord(k, "x")}'

    def program_cases(i):
        """(wall id, program of the link pulled as component i: direction ī) for the ids with link programs."""
        if not gen or not any(dirs[i]):
            return []
        return [(wid, pg[inv[i]]) for wid, pg in enumerate(programs) if pg is not None and pg[inv[i]] is not None]

    def own_loads(code, rd):
        """Loads of the cell's own pdfs a program's code reads (``const T c<q> = …;``; ``rd(q)``: the load)."""
        used = sorted({int(m) for m in re.findall(r'\bc(\d+)\b', code)})
        return ' '.join(f'const {ct} c{q} = {rd(q)};' for q in used)

    def pull_loads(L, prefix, arr, progs=True, hoisted=False):
        """``hoisted`` (the fix-up kernel, whose every cell has program links): the wall ids are loaded for every
        direction up front and the cell's own pdfs ``c<q>`` are already loaded, so no load waits on the mask."""
        for i in range(Q):
            k = key(dirs[i])
            cq = '' if links is not None and walls and any(dirs[i]) else 'const '
            if walls and any(dirs[i]):
                if hoisted and buf:
                    # (fix-up kernel: both candidates loaded, then selected — no load waits on the mask)
                    L.append(f'  const {ct} fb{i} = '
                             f'{load_v(prefix, f"{prefix}o_{centre} + (unsigned)({inv[i]} * {prefix}_qb)")}, '
                             f'fs{i} = {load_v(prefix, f"{prefix}o_{k} + (unsigned)({i} * {prefix}_qb)")};')
                    L.append(f'  {cq}{ct} f{i} = ((msk >> {i}) & 1u) ? fb{i} : fs{i};')
                elif buf:
                    # a bounced component is read from the cell itself: ONE load whose per-lane offset selects
                    # (component, cell) — not both loads and a select
                    L.append(f'  const unsigned vo{i} = ((msk >> {i}) & 1u) ? {prefix}o_{centre} + '
                             f'(unsigned)({inv[i]} * {prefix}_qb) : {prefix}o_{k} + (unsigned)({i} * {prefix}_qb);')
                    L.append(f'  {cq}{ct} f{i} = {load_v(prefix, f"vo{i}")};')
                else:
                    L.append(f'  {cq}{ct} f{i} = {arr}[(msk >> {i}) & 1u ? (IDX){inv[i]} * {prefix}_q + '
                             f'{prefix}o_{centre} : (IDX){i} * {prefix}_q + {prefix}o_{k}];')
                if links is not None:
                    # the wall cell's link (moving wall: α = 1, β = 6 w (c·u)); its id is loaded on this path only
                    rterm = f' + lk_r[id{i} * {Q} + {i}] * rs' if rho_links else ''
                    if hoisted:
                        L.append(f'  const unsigned id{i} = ((msk >> {i}) & 1u) ? (unsigned)wid{i} : 0u;')
                        L.append(f'  if ((msk >> {i}) & 1u) f{i} = lk_a[id{i} * {Q} + {i}] * f{i} + lk_b[id{i} * {Q} + '
                                 f'{i}]{rterm};')
                    else:
                        L.append(f'  unsigned id{i} = 0;')
                        L.append(f'  if ((msk >> {i}) & 1u) {{ id{i} = wallid[{ncell(k)}]; '
                                 f'f{i} = lk_a[id{i} * {Q} + {i}] * f{i} + lk_b[id{i} * {Q} + {i}]{rterm}; }}')
                    cases = program_cases(i) if progs else []
                    if cases:
                        L.append(f'  if ((msk >> {i}) & 1u) switch (id{i}) {{')
                        for wid, pg in cases:
                            lines, val, _ = pg
                            body = ' '.join(lines) + f' f{i} = {val};'
                            ld = '' if hoisted else own_loads(body, lambda q: load(prefix, arr, q, f'{prefix}o_{centre}'))
                            L.append(f'    case {wid}: {{ {ld} {body} }} break;')
                        L.append('    default: break;\n  }')
            else:
                L.append(f'  const {ct} f{i} = {load(prefix, arr, i, f"{prefix}o_{k}")};')

    def cell_density(L, prefix, arr):
        """ρ(x) of the cell's own (pre-streaming) pdfs, for density-weighted links, on cells next to a wall."""
        if not rho_links:
            return
        L.append(f'  {ct} rs = 0;')
        L.append(f'  if (msk & {low}) rs = ' + ' + '.join(load(prefix, arr, q, f'{prefix}o_{centre}')
                                                      for q in range(Q)) + ';')

    def moments(L):
        L.append(f'  const {ct} rho = ' + ' + '.join(f'f{i}' for i in range(Q)) + ';')
        for a in range(D):
            pos = [f'f{i}' for i in range(Q) if dirs[i][a] == 1]
            neg = [f'f{i}' for i in range(Q) if dirs[i][a] == -1]
            L.append(f'  const {ct} m{a} = (' + ' + '.join(pos) + ') - (' + ' + '.join(neg) + ');')
        if compressible:
            L.append(f'  const {ct} irho = ({ct})1 / rho;')
        for a in range(D):
            half = f'({ct})0.5 * F{a}' if ff else c_(F[a] / 2) if fm == 'guo' else None
            m = f'(m{a} + {half})' if fm == 'guo' else f'm{a}'      # Guo: velocity shifted by F/2
            L.append(f'  const {ct} u{a} = {m}' + (' * irho;' if compressible else ';'))
        L.append(f'  const {ct} usq = ' + ' + '.join(f'u{a} * u{a}' for a in range(D)) + ';')
        if fm == 'guo':
            L.append(f'  const {ct} uF = ' + ' + '.join(f'u{a} * {Fa(a)}' for a in range(D)) + ';')
            L.append(f'  const {ct} kg = ({ct})1 - ({ct})0.5 * omega;')
        if trt is not None:
            if trt[0] == 'magic':
                lam = c_(trt[1])
                wo = f'(({ct})4 - ({ct})2 * omega) / (({ct})4 * {lam} * omega + ({ct})2 - omega)'
            else:
                wo = c_(trt[1])
            L.append(f'  const {ct} w_odd = {wo};')
            L.append(f'  const {ct} ta = ({ct})0.5 * (omega + w_odd), tb = ({ct})0.5 * (omega - w_odd);')

    def cu_expr(i):
        t = [('+ ' if dirs[i][a] > 0 else '- ') + f'u{a}' for a in range(D) if dirs[i][a]]
        if not t:
            return f'({ct})0'
        s_ = ' '.join(t)
        return s_[2:] if s_.startswith('+ ') else '(' + s_ + ')'

    mask_param = 'const unsigned* __restrict__ nbmask, const unsigned char* __restrict__ wallid'
    fptr_f = ', const T* __restrict__ force' if ff else ''
    fptr_a = (', const T* __restrict__ force, T* __restrict__ dforce' if ff else '') + \
        (', T* __restrict__ rho_adj' if two else '')
    fstr = 'const IDX f_c, const IDX f_z, const IDX f_y, const IDX f_x, ' if ff else ''
    sig_fwd = (f'const T* __restrict__ src, T* __restrict__ dst, {mask_param}{fptr_f}, const int Z, const int Y, '
               'const int X, const IDX s_q, const IDX s_z, const IDX s_y, const IDX s_x, '
               f'const IDX d_q, const IDX d_z, const IDX d_y, const IDX d_x, {fstr}'
               f'const long long s_bytes, const long long d_bytes, const {ct} omega')
    sig_adj = (f'const T* __restrict__ src, const T* __restrict__ g, T* __restrict__ out, {mask_param}{fptr_a}, '
               'const int Z, const int Y, const int X, '
               'const IDX s_q, const IDX s_z, const IDX s_y, const IDX s_x, '
               'const IDX g_q, const IDX g_z, const IDX g_y, const IDX g_x, '
               f'const IDX o_q, const IDX o_z, const IDX o_y, const IDX o_x, {fstr}'
               f'const long long s_bytes, const long long g_bytes, const long long o_bytes, const {ct} omega')
    if ff and D == 2:
        fstr_unused = '(void)f_z; '
    else:
        fstr_unused = ''
    cell = '((IDX)z * Y + y) * X + x' if D == 3 else '(IDX)y * X + x'
    ncells = '(IDX)Z * Y * X'
    sig_rho = ('T* __restrict__ out, const unsigned* __restrict__ nbmask, const T* __restrict__ rho_adj, const int Z, '
               'const int Y, const int X, const IDX o_q, const IDX o_z, const IDX o_y, const IDX o_x')
    if gen and mode == 'inline':
        # the programs' Jacobians read the cell's own pdfs and the neighbours' wall ids
        sig_rho += (', const T* __restrict__ src, const unsigned char* __restrict__ wallid, '
                    'const IDX s_q, const IDX s_z, const IDX s_y, const IDX s_x')

    # ---- forward
    L.append(f'{fn} void lbm_fwd_cell({sig_fwd}, const int z, const int y, const int x)\n{{')
    L.append(f'  (void)Z; (void)s_bytes; (void)d_bytes; (void)wallid; {fstr_unused}')
    rsrc(L, 's', 'src')
    rsrc(L, 'd', 'dst')
    wrap_lines(L)
    neighbour_offsets(L, 's')
    L.append(f'  const IDX dc = ' + ' + '.join(f'(IDX){a} * d_{a}' for a in axes) + ';')
    if buf:
        L.append(f'  const unsigned dcb = (unsigned)dc * {esize}u;')
    dcoff = 'dcb' if buf else 'dc'
    if walls:
        L.append(f'  const unsigned msk = nbmask[{cell}];')
        L.append(f'  if ((msk >> {SELF_BIT}) & 1u) {{')
        for i in range(Q):
            L.append('    ' + store('d', 'dst', i, dcoff, load('s', 'src', i, f'so_{centre}')))
        L.append('    return;\n  }')

    force_loads(L)
    cell_density(L, 's', 'src')
    pull_loads(L, 's', 'src')
    moments(L)
    if trt is not None or mrt is not None:
        # TRT / MRT: every population's equilibrium first (the collision of i reads feq of other populations too)
        for i in range(Q):
            L.append(f'  {ct} fe{i};')
            L.append(f'  {{ const {ct} cu = {cu_expr(i)};')
            L.append(f'    const {ct} poly = cu * (({ct})3 + ({ct})4.5 * cu) - ({ct})1.5 * usq;')
            L.append(f'    fe{i} = ' + (f'{c_(w[i])} * rho * (({ct})1 + poly);' if compressible
                                        else f'{c_(w[i])} * (rho + poly);') + ' }')
        if mrt is not None:
            L.append(f'  const {ct} ' + ', '.join(f'nq{k} = f{k} - fe{k}' for k in range(Q)) + ';')   # f − feq
    for i in range(Q):
        L.append(f'  {{ const {ct} cu = {cu_expr(i)};')
        L.append(f'    const {ct} poly = cu * (({ct})3 + ({ct})4.5 * cu) - ({ct})1.5 * usq;')
        feq = f'{c_(w[i])} * rho * (({ct})1 + poly)' if compressible else f'{c_(w[i])} * (rho + poly)'
        term = ''
        if fm == 'simple' and cFi(i):
            term = f' + {c_(3 * w[i])} * {cFi(i)}' if ff else f' + {c_(3 * w[i] * cF[i])}'
        elif fm == 'guo':
            term = (f' + {c_(w[i])} * kg * (({ct})3 * ({cFi(i) or c_(0)} - uF)'
                    + (f' + {cFi(i, 9)} * cu' if cFi(i) else '') + ')')
        if trt is not None:
            j = inv[i]
            val = (f'(({ct})1 - ta) * f{i} - tb * f{j} + ta * fe{i} + tb * fe{j}{term}' if j != i else
                   f'f{i} + omega * (fe{i} - f{i}){term}')
        elif mrt is not None:
            pw, cc = mat_terms(mrt[0], 'nq')(i), mat_terms(mrt[1], 'nq')(i)
            val = f'f{i}' + (f' - omega * ({pw})' if pw else '') + (f' - ({cc})' if cc else '') + term
        else:
            val = f'f{i} + omega * ({feq} - f{i}){term}'
        L.append('    ' + store('d', 'dst', i, dcoff, val) + ' }')
    L.append('}')

    # ---- adjoint (scatter to where the forward pulled from)
    L.append(f'{fn} void lbm_adj_cell({sig_adj}, const int z, const int y, const int x'
             + ')\n{')
    L.append(f'  (void)Z; (void)s_bytes; (void)g_bytes; (void)o_bytes; (void)wallid; {fstr_unused}')
    rsrc(L, 's', 'src')
    rsrc(L, 'g', 'g')
    rsrc(L, 'o', 'out')
    wrap_lines(L)
    neighbour_offsets(L, 's')
    neighbour_offsets(L, 'o')
    L.append(f'  const IDX gc = ' + ' + '.join(f'(IDX){a} * g_{a}' for a in axes) + ';')
    if buf:
        L.append(f'  const unsigned gcb = (unsigned)gc * {esize}u;')
    gcoff = 'gcb' if buf else 'gc'
    if walls:
        L.append(f'  const unsigned msk = nbmask[{cell}];')
        L.append(f'  if ((msk >> {SELF_BIT}) & 1u) {{')
        for i in range(Q):
            L.append('    ' + store('o', 'out', i, f'oo_{centre}', load('g', 'g', i, gcoff)))
        L.append('    return;\n  }')
        if mode == 'main':
            # a cell next to a program wall is the fix-up kernel's: it only zeroes the entries out_q(x), q in gq, that
            # the fix-up kernel adds its G_q into and whose writer also runs there (the cell itself when x + c_q is a
            # wall, or a listed neighbour x + c_q) — both contributions then arrive by atomic adds onto that zero
            zl = []
            for q in gq_all:
                zero = store('o', 'out', q, f'oo_{centre}', c_(0))
                if any(dirs[q]):
                    kn = key(dirs[inv[q]])               # the neighbour x + c_q = x - c_(inv q)
                    zl.append(f'    if (((msk >> {inv[q]}) & 1u) || ((nbmask[{ncell(kn)}] >> {FIX_BIT}) & 1u)) {zero}')
                else:
                    zl.append(f'    {zero}')
            L.append(f'  if ((msk >> {FIX_BIT}) & 1u) {{')
            L += zl
            L.append('    return;\n  }')
    for i in range(Q):
        L.append(f'  const {ct} g{i} = {load("g", "g", i, gcoff)};')
    force_loads(L)
    cell_density(L, 's', 'src')
    adj_progs = gen and mode != 'main'          # the main HIP adjoint leaves the program cells to the fix-up kernels
    gq = gq_all if fix else []
    if gq:
        # the fix-up kernel: every listed cell has a program link, so its own pdfs (read by the links' programs and
        # their Jacobians) and the wall ids of all its neighbours are loaded once, up front, beside the mask — no load
        # of the kernel's latency-bound chain waits on the mask or on an id
        used = sorted({int(m) for pg in programs if pg is not None for row in pg if row is not None
                       for m in re.findall(r'\bc(\d+)\b', ' '.join(row[0]) + ' ' + row[1] + ' ' +
                                           ' '.join(' '.join(jl) + ' ' + je for _, jl, je in row[2]))})
        if used:
            L.append('  ' + ' '.join(f'const {ct} c{q} = {load("s", "src", q, f"so_{centre}")};' for q in used))
        if links is not None and walls:
            L.append('  ' + ' '.join(f'const unsigned char wid{i} = wallid[{ncell(key(dirs[i]))}];'
                                     for i in range(Q) if any(dirs[i])))
    pull_loads(L, 's', 'src', adj_progs, hoisted=bool(gq) and links is not None and walls)
    moments(L)
    if rho_links:
        L.append(f'  {ct} Rr = 0;')             # Σ_j βρ_j v_j over the cell's density-weighted links
    if gq:
        L.append(f'  {ct} ' + ', '.join(f'G{q} = 0' for q in gq) + ';')      # Σ_j J_jq v_j (link programs)
    if mrt is not None:
        # h = Aᵀ g
        for i in range(Q):
            pw, cc = mat_terms(mrt[0], 'g', True)(i), mat_terms(mrt[1], 'g', True)(i)
            hv = ' + '.join(t for t in ((f'omega * ({pw})' if pw else None), (f'({cc})' if cc else None)) if t)
            L.append(f'  const {ct} h{i} = {hv or c_(0)};')
    L.append(f'  {ct} S = 0, A = 0;')
    if gsplit:
        L.append(f'  {ct} Sg = 0;')                   # Σ_i g_i w_i (the force term's sums run over g)
    for a in range(D):
        L.append(f'  {ct} B{a} = 0;')
        if gsplit:
            L.append(f'  {ct} Bg{a} = 0;')            # Σ_i g_i w_i (3 + 9 c_i·u) c_ia
        if fm == 'guo':
            L.append(f'  {ct} E{a} = 0;')           # Σ_i g_i w_i c_ia (c_i·F)
        if ff and fm == 'simple':
            L.append(f'  {ct} M{a} = 0;')           # Σ_i g_i w_i c_ia (the 'simple' force adjoint / 3)
    for i in range(Q):
        L.append(f'  {{ const {ct} cu = {cu_expr(i)};')
        if trt is not None:
            # the equilibrium sums over h_i = a g_i + b g_ī (rest population: ω g_0)
            hi = f'(ta * g{i} + tb * g{inv[i]})' if inv[i] != i else f'omega * g{i}'
            L.append(f'    const {ct} gw = {hi} * {c_(w[i])};')
        elif mrt is not None:
            L.append(f'    const {ct} gw = h{i} * {c_(w[i])};')
        else:
            L.append(f'    const {ct} gw = g{i} * {c_(w[i])};')
        L.append('    S += gw;')
        if gsplit:
            L.append(f'    const {ct} gwg = g{i} * {c_(w[i])};')
            L.append('    Sg += gwg;')
        if compressible:
            L.append(f'    A += gw * (({ct})1 + cu * (({ct})3 + ({ct})4.5 * cu) - ({ct})1.5 * usq);')
        if any(dirs[i]):
            L.append(f'    const {ct} t = gw * (({ct})3 + ({ct})9 * cu);')
            for a in range(D):
                if dirs[i][a]:
                    L.append(f'    B{a} {"+" if dirs[i][a] > 0 else "-"}= t;')
            if gsplit:
                L.append(f'    const {ct} tg = gwg * (({ct})3 + ({ct})9 * cu);')
                for a in range(D):
                    if dirs[i][a]:
                        L.append(f'    Bg{a} {"+" if dirs[i][a] > 0 else "-"}= tg;')
            if fm == 'guo' and cFi(i):
                L.append(f'    const {ct} tf = {"gwg" if gsplit else "gw"} * {cFi(i)};')
                for a in range(D):
                    if dirs[i][a]:
                        L.append(f'    E{a} {"+" if dirs[i][a] > 0 else "-"}= tf;')
            if ff and fm == 'simple':
                gwm = f'(g{i} * {c_(w[i])})' if trt is not None or mrt is not None else 'gw'
                for a in range(D):
                    if dirs[i][a]:
                        L.append(f'    M{a} {"+" if dirs[i][a] > 0 else "-"}= {gwm};')
        L.append('  }')
    if not compressible:
        L.append('  A = S;')
    for a in range(D):
        L.append(f'  B{a} -= ({ct})3 * u{a} * S;')
        if ff and fm == 'guo':
            # the explicit force term's F-derivative sums (over g: Bg for TRT / MRT, = B before the ρ scaling for SRT)
            L.append(f'  const {ct} Bf{a} = ' + (f'Bg{a} - ({ct})3 * u{a} * Sg;' if gsplit else f'B{a};'))
        if compressible:
            L.append(f'  B{a} *= rho;')
        if gsplit:
            # the force term's derivative through u (TRT / MRT: v = g − h + A_h + Σ B_a ∂u_a/∂f_j, no ω factor)
            L.append(f'  B{a} += kg * (({ct})9 * E{a} - ({ct})3 * {Fa(a)} * Sg);')
        elif fm == 'guo':
            # the force term's derivative through u, scaled into B (v = … + ω (A + Σ B_a ∂u_a/∂f_j))
            L.append(f'  B{a} += kg * (({ct})9 * E{a} - ({ct})3 * {Fa(a)} * S) / omega;')
    if ff:
        # the force adjoint of this cell, accumulated over the op's steps
        for a in range(D):
            if fm == 'simple':
                val = f'({ct})3 * M{a}'
            else:
                # through the explicit term, and through the velocity shift ∂u_a/∂F_a = 1/2 (/ρ): Σ_i g_i ∂dst_i/∂u_a,
                # which is ω B_a for SRT (B carries 1/ω) and B_a for TRT / MRT
                sc = '' if gsplit else 'omega * '
                val = f'kg * Bf{a} + ({ct})0.5 * {sc}B{a}' + (' * irho' if compressible else '')
            L.append(f'  dforce[(IDX){a} * f_c + fc] += {val};')
    if compressible:
        L.append(f'  const {ct} Bu = ' + ' + '.join(f'B{a} * u{a}' for a in range(D)) + ';')
    for j in range(Q):
        cb = [('+ ' if dirs[j][a] > 0 else '- ') + f'B{a}' for a in range(D) if dirs[j][a]]
        cbs = ' '.join(cb)
        cbs = (cbs[2:] if cbs.startswith('+ ') else cbs) if cb else f'({ct})0'
        du = f'(({cbs}) - Bu) * irho' if compressible else f'({cbs})'
        vq = "" if links is not None and walls and any(dirs[j]) else "const "
        if trt is not None and inv[j] != j:
            L.append(f'  {{ {vq}{ct} v = (({ct})1 - ta) * g{j} - tb * g{inv[j]} + (A + {du});')
        elif trt is not None:
            L.append(f'  {{ {vq}{ct} v = (({ct})1 - omega) * g{j} + (A + {du});')
        elif mrt is not None:
            L.append(f'  {{ {vq}{ct} v = g{j} - h{j} + (A + {du});')
        else:
            L.append(f'  {{ {vq}{ct} v = (({ct})1 - omega) * g{j} + omega * (A + {du});')
        k = key(dirs[j])
        if walls and any(dirs[j]) and links is not None:
            if rho_links:
                L.append(f'    if ((msk >> {j}) & 1u) Rr += lk_gr[id{j} * {Q} + {j}] * v;')
            cases = program_cases(j) if adj_progs else []
            if cases and fix:
                # a program-linked component: Σ_j J_jq(c) v_j (c: the cell's own pre-streaming pdfs)
                L.append(f'    if ((msk >> {j}) & 1u) switch (id{j}) {{')
                for wid, pg in cases:
                    if len({jl for _, jl, _ in pg[2]}) == 1:
                        # one set of temporaries for the whole row (FixedDensity.program): emitted once
                        rows = ' '.join(pg[2][0][1]) + ' ' + ' '.join(f'G{q} += ({je}) * v;' for q, _, je in pg[2])
                    else:
                        rows = ' '.join('{ ' + ' '.join(jl) + f' G{q} += ({je}) * v; }}' for q, jl, je in pg[2])
                    L.append(f'      case {wid}: {{ {rows} }} break;')
                L.append('      default: break;\n    }')
            elif cases:
                # a program-linked component: its v for the second pass (the Jacobian row is evaluated there)
                L.append(f'    if ((msk >> {j}) & 1u) switch (id{j}) {{')
                L.append('      ' + ' '.join(f'case {wid}:' for wid, _ in cases) +
                         f' rho_adj[(IDX){j} * {ncells} + {cell}] = v; break;')
                L.append('      default: break;\n    }')
            L.append(f'    if ((msk >> {j}) & 1u) v *= lk_g[id{j} * {Q} + {j}];')
        if walls and any(dirs[j]) and fix and (j in gq or inv[j] in gq):
            # a store into a G entry (component q in gq of a listed cell) is an atomic add onto the entry the main
            # kernel zeroed: the cell itself (bounced, component ī) or a listed neighbour x − c_j (component j)
            ab = 'true' if inv[j] in gq else 'false'
            an = f'((nbmask[{ncell(k)}] >> {FIX_BIT}) & 1u)' if j in gq else 'false'
            if buf:
                L.append(f'    const unsigned vs = ((msk >> {j}) & 1u) ? oo_{centre} + (unsigned)({inv[j]} * o_qb) : '
                         f'oo_{k} + (unsigned)({j} * o_qb);')
                L.append(f'    if (((msk >> {j}) & 1u) ? {ab} : {an}) atomicAdd((T*)((char*)out + vs), (T)v); '
                         f'else {store_v("o", "vs", "v")} }}')
            else:
                L.append(f'    const IDX vs = ((msk >> {j}) & 1u) ? (IDX){inv[j]} * o_q + oo_{centre} : (IDX){j} * o_q + '
                         f'oo_{k};')
                L.append(f'    if (((msk >> {j}) & 1u) ? {ab} : {an}) atomicAdd(out + vs, (T)v); else out[vs] = (T)v; }}')
        elif walls and any(dirs[j]):
            if buf:
                L.append(f'    const unsigned vs = ((msk >> {j}) & 1u) ? oo_{centre} + (unsigned)({inv[j]} * o_qb) : '
                         f'oo_{k} + (unsigned)({j} * o_qb);')
                L.append(f'    {store_v("o", "vs", "v")} }}')
            else:
                L.append(f'    out[(msk >> {j}) & 1u ? (IDX){inv[j]} * o_q + oo_{centre} : (IDX){j} * o_q + oo_{k}] '
                         f'= (T)v; }}')
        elif fix and j in gq:
            # the rest population of a listed cell: its own G entry
            L.append(f'    atomicAdd(' + (f'(T*)((char*)out + oo_{k} + (unsigned)({j} * o_qb))' if buf else
                                         f'out + (IDX){j} * o_q + oo_{k}') + ', (T)v); }')
        else:
            L.append('    ' + store('o', 'out', j, f'oo_{k}', 'v') + ' }')
    inl = gen and mode == 'inline'
    if rho_links:
        # the density term: slot Q of the scratch array with inline link programs, its only slot without
        L.append(f'  if (msk & {low}) rho_adj[' + (f'(IDX){Q} * {ncells} + ' if inl else '') + f'{cell}] = Rr;')
    if gq:
        # out_q(x) += G_q: after the main launch's store of that entry, or (zeroed entry) in either order with this
        # launch's own atomic store into it — two addends onto zero, so the sum is the same either way
        L.append('  ' + ' '.join(f'atomicAdd(' + (f'(T*)((char*)out + oo_{centre} + (unsigned)({q} * o_qb))' if buf else
                                                 f'out + (IDX){q} * o_q + oo_{centre}') + f', G{q});' for q in gq))
    L.append('}')
    if two:
        # second adjoint pass: the density term of the cell's links reaches every component of the cell, whose
        # adjoint entries the first pass wrote from other threads
        L.append(f'{fn} void lbm_adj_rho_cell({sig_rho}, const int z, const int y, const int x)\n{{')
        L.append('  (void)Z;')
        L.append(f'  const unsigned msk = nbmask[{cell}];')
        L.append(f'  if (((msk >> {SELF_BIT}) & 1u) || !(msk & {low})) return;')
        L.append('  const IDX oc = ' + ' + '.join(f'(IDX){a} * o_{a}' for a in axes) + ';')
        if rho_links:
            L.append(f'  const {ct} R = rho_adj[' + (f'(IDX){Q} * {ncells} + ' if inl else '') + f'{cell}];')
            for q in range(Q):
                L.append(f'  out[(IDX){q} * o_q + oc] += R;')
        if inl:
            # Σ_j J_jk(c) v_j over the cell's program-linked components (c: the cell's own pre-streaming pdfs)
            wrap_lines(L)
            L.append('  const IDX sc = ' + ' + '.join(f'(IDX){a} * s_{a}' for a in axes) + ';')
            for j in range(Q):
                cases = program_cases(j)
                if not cases:
                    continue
                L.append(f'  if ((msk >> {j}) & 1u) {{')
                L.append(f'    const {ct} v = rho_adj[(IDX){j} * {ncells} + {cell}];')
                L.append(f'    switch (wallid[{ncell(key(dirs[j]))}]) {{')
                for wid, pg in cases:
                    rows = ' '.join('{ ' + ' '.join(jl) + f' out[(IDX){q} * o_q + oc] += ({je}) * v; }}'
                                    for q, jl, je in pg[2])
                    ld = own_loads(rows, lambda q: f'({ct})src[(IDX){q} * s_q + sc]')
                    L.append(f'      case {wid}: {{ {ld} {rows} }} break;')
                L.append('      default: break;\n    }\n  }')
        L.append('}')

    # ---- entry points
    fa_f, fa_a, fs = (', force', ', force, dforce', 'f_c, f_z, f_y, f_x, ') if ff else ('', '', '')
    fa_a += ', rho_adj' if two else ''
    args_r = 'out, nbmask, rho_adj, Z, Y, X, o_q, o_z, o_y, o_x' + \
        (', src, wallid, s_q, s_z, s_y, s_x' if gen and mode == 'inline' else '')
    args_f = (f'src, dst, nbmask, wallid{fa_f}, Z, Y, X, s_q, s_z, s_y, s_x, d_q, d_z, d_y, d_x, {fs}s_bytes, d_bytes, '
              'omega')
    args_a = (f'src, g, out, nbmask, wallid{fa_a}, Z, Y, X, s_q, s_z, s_y, s_x, g_q, g_z, g_y, g_x, o_q, o_z, o_y, o_x, '
              f'{fs}s_bytes, g_bytes, o_bytes, omega')
    if hip and fix:
        # the fix-up kernel: one thread per listed cell (the fluid cells next to a link-program wall)
        # one wave per workgroup (FIX_BLOCK lanes): the few listed cells spread over as many CUs as possible — each wave
        # runs a long, branchy, latency-bound chain, and waves of one CU would share its scalar unit
        L.append(f'extern "C" __global__ void __launch_bounds__({FIX_BLOCK}) lbm_adj_fix({sig_adj}, const int* __restrict__ '
                 'cells, const int ncell)\n{')
        L.append(f'  const int t = (int)(blockIdx.x * {FIX_BLOCK}u + threadIdx.x);')
        L.append('  if (t >= ncell) return;')
        L.append('  const unsigned cell = (unsigned)cells[t];')
        L.append('  const unsigned r = cell / (unsigned)X;')
        L.append('  const int x = (int)(cell - r * (unsigned)X);')
        L.append('  const int z = (int)(r / (unsigned)Y), y = (int)(r - (unsigned)z * Y);')
        L.append(f'  lbm_adj_cell({args_a}, z, y, x);\n}}')
    elif hip:
        # a block = 256 consecutive cells of the lattice in C order (rows of x), and consecutive blocks on one XCD
        # (bijective remap of the round-robin dispatch): a lattice row's x-shifted loads and the adjoint's
        # x-shifted stores cover cache lines that the neighbouring wave also touches — in one block, or in a
        # block on the same XCD's L2, not split between two L2s (partial-line write-backs)
        for nm, sig, args in (('lbm_fwd', sig_fwd, args_f), ('lbm_adj', sig_adj, args_a)) + \
                ((('lbm_adj_rho', sig_rho, args_r),) if two else ()):
            L.append(f'extern "C" __global__ void __launch_bounds__(256) {nm}({sig})\n{{')
            L.append('  const unsigned nb = gridDim.x, b = blockIdx.x;')
            L.append('  const unsigned per = nb >> 3, rem = nb & 7, xcd = b & 7, bi = b >> 3;')
            L.append('  const unsigned lb = (xcd < rem) ? xcd * (per + 1) + bi : rem * (per + 1) + (xcd - rem) * per + bi;')
            L.append('  const unsigned cell = lb * 256u + threadIdx.x;     // cells < 2^32 (checked at launch)')
            L.append('  if (cell >= (unsigned)X * (unsigned)Y * (unsigned)Z) return;')
            L.append('  const unsigned r = cell / (unsigned)X;')
            L.append('  const int x = (int)(cell - r * (unsigned)X);')
            L.append('  const int z = (int)(r / (unsigned)Y), y = (int)(r - (unsigned)z * Y);')
            L.append(f'  {nm}_cell({args}, z, y, x);\n}}')
    else:
        for nm, kind in (('lbm_fwd', 'f'), ('lbm_adj', 'a')):
            # the CPU kernels' ctypes signature (backends.cpu_kernel.compile_c): pointers, extents, strides, -, scalars
            L.append(f'void {nm}(void** P, const i64* N, const i64* S, const i64* B_, const double* Dv)\n{{')
            L.append('  (void)B_; const int Z = (int)N[0], Y = (int)N[1], X = (int)N[2];')
            L.append(f'  const {ct} omega = ({ct})Dv[0];')
            if kind == 'f':
                L.append('  const T* src = (const T*)P[0]; T* dst = (T*)P[1]; const unsigned* nbmask = '
                         '(const unsigned*)P[2]; const unsigned char* wallid = (const unsigned char*)P[3];')
                L.append('  const IDX s_q = S[0], s_z = S[1], s_y = S[2], s_x = S[3], d_q = S[4], d_z = S[5], '
                         'd_y = S[6], d_x = S[7];')
                if ff:
                    L.append('  const T* force = (const T*)P[4];')
                    L.append('  const IDX f_c = S[8], f_z = S[9], f_y = S[10], f_x = S[11];')
                L.append('  const long long s_bytes = 0, d_bytes = 0;')
                call = f'lbm_fwd_cell({args_f}, z, y, x);'
            else:
                L.append('  const T* src = (const T*)P[0]; const T* g = (const T*)P[1]; T* out = (T*)P[2]; '
                         'const unsigned* nbmask = (const unsigned*)P[3]; '
                         'const unsigned char* wallid = (const unsigned char*)P[4];')
                L.append('  const IDX s_q = S[0], s_z = S[1], s_y = S[2], s_x = S[3], g_q = S[4], g_z = S[5], '
                         'g_y = S[6], g_x = S[7], o_q = S[8], o_z = S[9], o_y = S[10], o_x = S[11];')
                if ff:
                    L.append('  const T* force = (const T*)P[5]; T* dforce = (T*)P[6];')
                    L.append('  const IDX f_c = S[12], f_z = S[13], f_y = S[14], f_x = S[15];')
                if two:
                    L.append(f'  T* rho_adj = (T*)P[{7 if ff else 5}];')
                L.append('  const long long s_bytes = 0, g_bytes = 0, o_bytes = 0;')
                call = f'lbm_adj_cell({args_a}, z, y, x);'
            L.append('  #pragma omp parallel for collapse(2) schedule(static)')
            L.append('  for (int z = 0; z < Z; ++z)\n    for (int y = 0; y < Y; ++y)\n      for (int x = 0; x < X; ++x)')
            L.append(f'        {call}')
            if kind == 'a' and two:
                # the density pass after every cell's scatter (the C target runs both passes in one call)
                L.append('  #pragma omp parallel for collapse(2) schedule(static)')
                L.append('  for (int z = 0; z < Z; ++z)\n    for (int y = 0; y < Y; ++y)\n      for (int x = 0; x < X; ++x)')
                L.append(f'        lbm_adj_rho_cell({args_r}, z, y, x);')
            L.append('}')
    return '\n'.join(L) + '\n'


def fix_cells(flags, stencil, program_ids):
    """Bool over the domain: fluid cells with a neighbour ``x − c_i`` (periodic) among the walls of ``program_ids``
    (the flag ids whose boundary is a link program) — the cells the HIP fix-up kernels recompute."""
    f = np.asarray(flags)
    prog = np.isin(f, np.asarray(sorted(program_ids), dtype=f.dtype))
    near = np.zeros(f.shape, bool)
    for c in stencil.directions:
        if any(c):
            near |= np.roll(prog, tuple(int(v) for v in c), axis=tuple(range(len(c))))
    return near & (f == 0)


def neighbour_mask(flags, stencil, xp, fix=None):
    """``uint32`` per cell: bit i set where ``x − c_i`` is a wall cell (periodic), bit ``SELF_BIT`` where ``x`` is
    one (``flags``: wall ids over the domain, 0 = fluid, numpy or torch); bit ``FIX_BIT`` where ``fix`` (a numpy
    bool array, ``fix_cells``) is set — then computed on the host, and a torch result comes back as the uint32
    bits in an int32 tensor on ``flags``' device."""
    is_torch = xp.__name__ == 'torch'
    if fix is not None:
        m = neighbour_mask(flags.cpu().numpy() if is_torch else flags, stencil, np)
        m = m | (np.asarray(fix, bool).astype(np.uint32) << np.uint32(FIX_BIT))
        return xp.from_numpy(np.ascontiguousarray(m).view(np.int32)).to(flags.device) if is_torch else m
    f = (flags != 0).to(xp.int32) if is_torch else (np.asarray(flags) != 0).astype(np.int64)
    m = f * 0
    for i, c in enumerate(stencil.directions):
        if not any(c):
            continue
        r = f
        for ax, sh in enumerate(c):
            if sh:
                r = xp.roll(r, shifts=sh, dims=ax) if is_torch else np.roll(r, sh, axis=ax)
        m = m | (r << i)
    m = m | (f << SELF_BIT)
    return m.to(xp.int32).contiguous() if is_torch else np.ascontiguousarray(m.astype(np.uint32))


def lattice_strides(t, D):
    """``(s_q, s_z, s_y, s_x)`` in elements of a pdf tensor ``[*spatial, q]`` (2-D: ``s_z`` = 0)."""
    st = [int(s) for s in (t.stride() if hasattr(t, 'stride') and callable(t.stride) else
                           [s // t.itemsize for s in t.strides])]
    sp_ = st[:D]
    if D == 2:
        sp_ = [0] + sp_
    return (st[D],) + tuple(sp_)


def row_interleaved_empty(domain, Q, dtype, device):
    """An uninitialised pdf tensor ``[*domain, Q]`` in the row-interleaved layout ``[z][y][q][x]`` (each lattice
    row's Q components one contiguous block) — the time-step op's internal states."""
    import torch
    dims = list(domain)
    base = torch.empty(dims[:-1] + [Q, dims[-1]], dtype=dtype, device=device)
    return base.transpose(-1, -2)


class LatticeKernels:
    """Compiled forward / adjoint lattice kernels of one (stencil, compressible, dtype, walls, links, target).
    ``mask`` arguments are the cells' neighbour masks (``neighbour_mask``), ``None`` without walls; ``ids`` the
    cells' wall ids (the ``uint8`` flag array, C order) when ``links`` is given (walls other than plain
    bounce-back)."""

    def __init__(self, stencil, compressible, dtype, walls, target, links=None, force_model=None, force=None,
                 force_field=False, trt=None, programs=None, mrt=None):
        self.stencil = stencil
        # MRT: (P_ω, C) relaxation matrices as float tuples (``_method.mrt_relaxation_matrices``)
        self.mrt = None if mrt is None else tuple(tuple(tuple(float(v) for v in row) for row in M) for M in mrt)
        self.trt = None if trt is None else (str(trt[0]), float(trt[1]))
        self.force_model = force_model
        self.force_field = bool(force_model) and bool(force_field)
        self.force = None if force_model is None or self.force_field else tuple(float(v) for v in force)
        self.compressible = bool(compressible)
        self.dtype = np.dtype(dtype)
        if self.dtype not in (np.float32, np.float64):
            raise NotImplementedError(f'lattice kernels for {self.dtype} pdfs')
        self.ct = 'double' if self.dtype == np.float64 else 'float'
        self.walls = bool(walls)
        self.links = links if walls else None
        # density-weighted links: the adjoint takes a second pass (lbm_adj_rho) over a per-cell scratch array
        self.rho_links = self.links is not None and any(len(t) > 3 and t[3] != 0 for lk in self.links for t in lk)
        # link programs (boundaries.link_program). C: inline, a Q-component scratch array per cell and the second
        # pass; HIP: the main kernels skip the FIX_BIT cells, the fix-up kernels (a module of their own) redo them
        self.programs = programs if self.links is not None and programs is not None and \
            any(p is not None for p in programs) else None
        self.link_pass = self.rho_links or (self.programs is not None and target != 'gpu')
        self.program_ids = tuple(k for k, p in enumerate(self.programs or ()) if p is not None)
        self._rho_bufs = {}
        self.target = target
        self._fns = {}
        self._plans = {}

    def source(self, idx='int', addr='buf', fix=False):
        """The C source (inline link programs), or a HIP module: the main kernels, or (``fix``) the fix-up kernels
        of the cells next to link-program walls."""
        if self.target != 'gpu':
            return _emit(self.stencil, self.compressible, self.ct, self.walls, 'c', 'i64', 'ptr', self.links,
                         self.force_model, self.force, self.force_field, self.trt, self.programs, mrt=self.mrt)
        if fix:
            return _emit(self.stencil, self.compressible, self.ct, self.walls, 'hip', idx, addr, self.links,
                         self.force_model, self.force, self.force_field, self.trt, self.programs, mode='fix',
                         mrt=self.mrt)
        return _emit(self.stencil, self.compressible, self.ct, self.walls, 'hip', idx, addr, self.links,
                     self.force_model, self.force, self.force_field, self.trt, self.programs,
                     mode='main' if self.programs is not None else 'inline', mrt=self.mrt)

    # -- GPU ---------------------------------------------------------------------------------------
    def _gpu_fn(self, which, idx, addr, device):
        key = (which, idx, addr, device)
        fn = self._fns.get(key)
        if fn is None:
            from ..backends import hip_runtime as rt
            code = rt.compile_hip(self.source(idx, addr, fix=which.endswith('fix')), name='psad_lbm.hip')
            fn = self._fns[key] = rt.load_function(code, f'lbm_{which}', device)
        return fn

    def build(self):
        from ..backends import hip_runtime as rt
        if self.target == 'gpu':
            return [rt.compile_hip(self.source('int', a, f), name='psad_lbm.hip') for a in ('buf', 'ptr')
                    for f in ((False, True) if self.programs is not None else (False,))]
        return self._cpu_fn('fwd')

    def _check(self, tensors, mask, ids=None):
        D, Q = self.stencil.D, self.stencil.Q
        shape = tuple(tensors[0].shape)
        for t in tensors:
            if tuple(t.shape) != shape or len(shape) != D + 1 or int(shape[D]) != Q:
                raise ValueError(f'pdf tensors must be [*domain, {Q}] of one shape, got {tuple(t.shape)}')
            if t.dtype != tensors[0].dtype or not t.is_cuda or t.device != tensors[0].device:
                raise ValueError('pdf tensors must share dtype and device')
        if self.walls != (mask is not None):
            raise ValueError('the wall kernels need the neighbour mask (and the periodic ones none)')
        if mask is not None and (tuple(mask.shape) != shape[:D] or not mask.is_contiguous()
                                 or mask.dtype.itemsize != 4 or mask.device != tensors[0].device):
            raise ValueError(f'neighbour mask of shape {tuple(mask.shape)} does not match the domain {shape[:D]}')
        if min(shape[:D]) < 2:
            raise ValueError('the periodic lattice needs at least 2 cells per axis')
        if (self.links is not None) != (ids is not None):
            raise ValueError('kernels with boundary links need the wall ids (and the others none)')
        if ids is not None and (tuple(ids.shape) != shape[:D] or not ids.is_contiguous() or ids.dtype.itemsize != 1
                                or ids.device != tensors[0].device):
            raise ValueError(f'wall ids of shape {tuple(ids.shape)} do not match the domain {shape[:D]}')

    @staticmethod
    def _reach(t):
        """Elements from the tensor's base to its last element (+1)."""
        return sum(abs(int(s)) * (int(n) - 1) for s, n in zip(t.stride(), t.shape)) + 1

    def _mode(self, tensors):
        reach = max(self._reach(t) for t in tensors)
        idx = 'int' if reach < 2 ** 31 - 1 else 'long long'
        esz = tensors[0].element_size()
        addr = 'buf' if reach * esz < 2 ** 31 and all(min(t.stride()) >= 0 for t in tensors) else 'ptr'
        if os.environ.get('PSAD_LBM_ADDR') == 'ptr':       # A/B of the addressing modes (probes)
            addr = 'ptr'
        return idx, addr

    def _common(self, tensors, mask, ids=None):
        self._check(tensors, mask, ids)
        idx, addr = self._mode(tensors)
        fn_args = []
        for t in tensors:
            fn_args += list(lattice_strides(t, self.stencil.D))
        return idx, addr, fn_args

    def _force_check(self, shape, force, dforce, which, xp_tensor=True):
        """The per-cell force (and, for the adjoint, its accumulated adjoint): ``[*domain, D]`` of the pdf dtype,
        ``dforce`` with the strides of ``force``; none without a force field."""
        D = self.stencil.D
        need = [force] + ([dforce] if which == 'adj' else [])
        if not self.force_field:
            if force is not None or dforce is not None:
                raise ValueError('these lattice kernels take no force field')
            return
        if any(t is None for t in need):
            raise ValueError(f'the force-field lattice kernels need the force{" and its adjoint" if which == "adj" else ""}')
        for t in need:
            if tuple(t.shape) != tuple(shape[:D]) + (D,):
                raise ValueError(f'force field of shape {tuple(t.shape)}: expected {tuple(shape[:D]) + (D,)}')
            if (t.dtype != self.dtype) if not xp_tensor else (str(t.dtype).split('.')[-1] != self.dtype.name):
                raise ValueError(f'force field dtype {t.dtype}: expected {self.dtype}')
        if which == 'adj' and tuple(dforce.stride() if xp_tensor else dforce.strides) != \
                tuple(force.stride() if xp_tensor else force.strides):
            raise ValueError('the force adjoint must have the strides of the force')

    def plan(self, which, tensors, mask, omega, ids=None, force=None, dforce=None, fix=None):
        """The launch of ``which`` ('fwd' / 'adj') on tensors of these shapes, strides, dtype and device (with or
        without walls): a ``LaunchPlan`` whose pointer slots and relaxation rate are patched per launch — the
        time-step op launches T of them per apply. ω is not part of the key (a trained or scheduled rate reuses the
        plan); the plan is built with the first ω it sees. ``fix``: (cells,) — the fix-up kernel of ``which`` over
        the listed cells (int32 cell indices)."""
        key = (which, mask is not None) + tuple((tuple(t.shape), tuple(t.stride()), t.dtype, t.device)
                                                for t in tensors) + \
            ((tuple(force.shape), tuple(force.stride())) if force is not None else ()) + \
            ((fix[0].data_ptr(), int(fix[0].numel())) if fix is not None else ())
        plan = self._plans.get(key)
        if plan is not None:
            return plan
        self._force_check(tuple(tensors[0].shape), force, dforce, which)
        idx, addr, strides = self._common(tensors, mask, ids)
        if force is not None:
            # the force is read (and its adjoint accumulated) through plain pointers with IDX offsets
            if max(self._reach(force), self._reach(dforce) if dforce is not None else 0) >= 2 ** 31 - 1:
                idx = 'long long'
            strides += list(lattice_strides(force, self.stencil.D))
        dev = tensors[0].device.index
        fn = self._gpu_fn(which + ('_fix' if fix is not None else ''), idx, addr, dev)
        Z, Y, X = self._extent(tensors[0])
        code = 'i' if idx == 'int' else 'q'
        nblocks = self._blocks(X, Y, Z) if fix is None else -(-int(fix[0].numel()) // FIX_BLOCK)
        reach = [self._reach(t) * t.element_size() for t in tensors]
        ptrs = [t.data_ptr() for t in tensors] + [mask.data_ptr() if mask is not None else 0,
                                                  ids.data_ptr() if ids is not None else 0]
        if force is not None:
            ptrs += [force.data_ptr()] + ([dforce.data_ptr()] if which == 'adj' else [])
        if which == 'adj' and self.link_pass:
            ptrs += [0]                                  # the second pass's scratch array (patched per launch)
        fmt = 'Q' * len(ptrs) + 'iii' + code * len(strides) + 'q' * len(tensors) + \
            ('d' if self.ct == 'double' else 'f')
        vals = [*ptrs, Z, Y, X, *strides, *reach, float(omega)]
        om_i = len(fmt) - 1
        if fix is not None:
            # the fix-up kernel: the cell list and its length after the main kernel's arguments
            fmt += 'Qi'
            vals += [fix[0].data_ptr(), int(fix[0].numel())]
        args = _pack(fmt, *vals)
        plan = self._plans[key] = LaunchPlan(fn, nblocks, args, len(ptrs), dev, _offset(fmt, om_i), fmt[om_i])
        if fix is not None:
            plan.block = FIX_BLOCK
        return plan

    def fix_launch(self, which, tensors, mask, omega, ids, force, dforce, cells, stream):
        """The fix-up launch after a main adjoint launch on ``tensors`` (HIP with link programs; nothing for the
        forward, which runs them inline, or when no cell is listed): the listed cells' adjoint with their programs'
        Jacobian terms, added atomically into the entries the main launch left zeroed (no second fix-up launch)."""
        if which != 'adj' or self.programs is None or self.target != 'gpu' or cells is None or \
                int(cells.numel()) == 0:
            return
        plan = self.plan(which, tensors, mask, omega, ids, force, dforce, fix=(cells,))
        ptrs = tuple(t.data_ptr() for t in tensors) + (mask.data_ptr(), ids.data_ptr())
        if force is not None:
            ptrs += (force.data_ptr(),) + ((dforce.data_ptr(),) if which == 'adj' else ())
        if which == 'adj' and self.link_pass:
            ptrs += (self.rho_buffer(tensors[0]).data_ptr(),)
        plan(ptrs, stream, omega)

    def rho_buffer(self, t):
        """The per-cell scratch array of the second adjoint pass (one per domain and device, reused: stream-ordered):
        one value per cell (density-weighted links), Q per cell with link programs."""
        import torch
        key = (tuple(int(n) for n in t.shape[:self.stencil.D]), t.device, t.dtype)
        b = self._rho_bufs.get(key)
        if b is None:
            # (HIP: link programs run in the fix-up kernels, so the density pass alone uses it — one slot)
            shape = ((self.stencil.Q + int(self.rho_links),) if self.programs is not None and self.target != 'gpu'
                     else ()) + key[0]
            b = self._rho_bufs[key] = torch.empty(shape, dtype=t.dtype, device=t.device)
        return b

    def rho_plan(self, out, mask, rho, src=None, ids=None):
        """The second pass of the adjoint (``lbm_adj_rho``: every component of a cell next to a density-weighted
        wall gets the cell's Σ_j βρ_j v_j added; with link programs, component k of a cell next to a program wall
        gets Σ_j J_jk v_j, the Jacobians evaluated at the cell's own pdfs in ``src``) on ``out``'s shape and strides.
        The plan's pointer slots: out, mask, scratch (+ src, ids with link programs)."""
        key = ('rho', tuple(out.shape), tuple(out.stride()), out.dtype, out.device) + \
            ((tuple(src.stride()),) if self.programs is not None else ())
        plan = self._plans.get(key)
        if plan is not None:
            return plan
        tensors = [out] + ([src] if self.programs is not None else [])
        idx, addr = self._mode(tensors)
        dev = out.device.index
        fn = self._gpu_fn('adj_rho', idx, addr, dev)
        Z, Y, X = self._extent(out)
        code = 'i' if idx == 'int' else 'q'
        if self.programs is None:
            fmt = 'QQQ' + 'iii' + code * 4
            args = _pack(fmt, out.data_ptr(), mask.data_ptr(), rho.data_ptr(), Z, Y, X,
                         *lattice_strides(out, self.stencil.D))
            nptr = 3
        else:
            fmt = 'QQQ' + 'iii' + code * 4 + 'QQ' + code * 4
            args = _pack(fmt, out.data_ptr(), mask.data_ptr(), rho.data_ptr(), Z, Y, X,
                         *lattice_strides(out, self.stencil.D), src.data_ptr(), ids.data_ptr(),
                         *lattice_strides(src, self.stencil.D))
            nptr = 3
        plan = self._plans[key] = LaunchPlan(fn, self._blocks(X, Y, Z), args, nptr, dev, None, None)
        if self.programs is not None:
            plan.extra = _offset(fmt, 3 + 3 + 4)          # the src / ids slots, patched per launch
        return plan

    def forward(self, src, dst, omega, mask=None, stream=None, ids=None, force=None, cells=None):
        """``dst = stream-pull-collide(src)`` (torch tensors ``[*domain, q]``, any strides; ``force``: the per-cell
        force ``[*domain, D]`` of force-field kernels)."""
        if self.target != 'gpu':
            return self._cpu('fwd', [src, dst], omega, mask, ids, force)
        st = _stream(stream, src)
        self.plan('fwd', [src, dst], mask, omega, ids, force)(
            (src.data_ptr(), dst.data_ptr(), mask.data_ptr() if mask is not None else 0,
             ids.data_ptr() if ids is not None else 0) + ((force.data_ptr(),) if force is not None else ()),
            st, omega)

    def adjoint(self, src, g, out, omega, mask=None, stream=None, ids=None, force=None, dforce=None, cells=None):
        """``out = (∂ step / ∂ src)ᵀ g`` at the state ``src``; force-field kernels also ADD ``(∂ step / ∂ F)ᵀ g`` to
        ``dforce``."""
        if self.target != 'gpu':
            return self._cpu('adj', [src, g, out], omega, mask, ids, force, dforce)
        st = _stream(stream, src)
        rho = self.rho_buffer(src) if self.link_pass else None
        self.plan('adj', [src, g, out], mask, omega, ids, force, dforce)(
            (src.data_ptr(), g.data_ptr(), out.data_ptr(), mask.data_ptr() if mask is not None else 0,
             ids.data_ptr() if ids is not None else 0) +
            ((force.data_ptr(), dforce.data_ptr()) if force is not None else ()) +
            ((rho.data_ptr(),) if rho is not None else ()), st, omega)
        self.fix_launch('adj', [src, g, out], mask, omega, ids, force, dforce, cells, st)
        if rho is not None:
            self.rho_pass(out, mask, rho, src, ids, st)

    def rho_pass(self, out, mask, rho, src, ids, stream):
        """Launch the adjoint's second pass (``rho_plan``) for this launch's ``out`` / ``src``."""
        plan = self.rho_plan(out, mask, rho, src, ids)
        plan((out.data_ptr(), mask.data_ptr(), rho.data_ptr()), stream,
             extra=(src.data_ptr(), ids.data_ptr()) if self.programs is not None else None)

    def _extent(self, t):
        shape = [int(n) for n in t.shape[:self.stencil.D]]
        return [1] + shape if self.stencil.D == 2 else shape

    @staticmethod
    def _blocks(X, Y, Z):
        """One block per 256 consecutive cells (cell indices are 32-bit in the kernel)."""
        if X * Y * Z + 255 >= 2 ** 32:
            raise ValueError('lattice of 2^32 cells or more: too large for one launch')
        return -(-(X * Y * Z) // 256)

    # -- CPU ---------------------------------------------------------------------------------------
    def _cpu_fn(self, which):
        fn = self._fns.get(which)
        if fn is None:
            from ..backends.cpu_kernel import compile_c
            fn = self._fns[which] = compile_c(self.source(), f'lbm_{which}', openmp=True)
        return fn

    def _cpu(self, which, arrays, omega, mask, ids=None, force=None, dforce=None):
        arrays = [np.asarray(a) for a in arrays]
        for a in arrays:
            if a.dtype != self.dtype:
                raise TypeError(f'pdf arrays must be {self.dtype}, got {a.dtype}')
        D = self.stencil.D
        shape = tuple(arrays[0].shape)
        for a in arrays:
            if tuple(a.shape) != shape or int(shape[D]) != self.stencil.Q:
                raise ValueError('pdf arrays must be [*domain, q] of one shape')
        if self.walls != (mask is not None):
            raise ValueError('the wall kernels need the neighbour mask (and the periodic ones none)')
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint32)
            if m.shape != shape[:D]:
                raise ValueError('neighbour mask does not match the domain')
        if (self.links is not None) != (ids is not None):
            raise ValueError('kernels with boundary links need the wall ids (and the others none)')
        idv = None
        if ids is not None:
            idv = np.ascontiguousarray(ids, dtype=np.uint8)
            if idv.shape != shape[:D]:
                raise ValueError('wall ids do not match the domain')
        self._force_check(shape, force, dforce, which, xp_tensor=False)
        fn = self._cpu_fn(which)
        ptrs = [a.ctypes.data for a in arrays] + [m.ctypes.data if m is not None else 0,
                                                  idv.ctypes.data if idv is not None else 0]
        strides = []
        for a in arrays:
            strides += list(lattice_strides(a, D))
        if force is not None:
            ptrs += [force.ctypes.data] + ([dforce.ctypes.data] if which == 'adj' else [])
            strides += list(lattice_strides(force, D))
        rho = None
        if which == 'adj' and self.link_pass:
            # the second pass's scratch (both passes in one call)
            rho = np.empty(((self.stencil.Q + int(self.rho_links),) if self.programs is not None else ()) + shape[:D],
                           self.dtype)
            ptrs += [rho.ctypes.data]
        ext = list(shape[:D]) if D == 3 else [1] + list(shape[:D])
        P = (ctypes.c_void_p * len(ptrs))(*ptrs)
        N = (ctypes.c_longlong * 3)(*ext)
        S = (ctypes.c_longlong * len(strides))(*strides)
        B = (ctypes.c_longlong * 1)(0)
        Dv = (ctypes.c_double * 1)(float(omega))
        fn(P, N, S, B, Dv)


class LaunchPlan:
    """One lattice kernel launch with its argument buffer; ``plan(ptrs, stream, omega)`` patches the leading pointer
    slots (the pdf arrays, then the neighbour mask) and the relaxation rate, and launches on the plan's device
    (made current for the launch when it is not: the function handle belongs to that device's module)."""
    __slots__ = ('fn', 'nblocks', 'template', 'fmt', 'device', 'om_off', 'om_fmt', 'extra', 'block')

    def __init__(self, fn, nblocks, template, nptr, device, om_off, om_code):
        self.fn, self.nblocks, self.template, self.fmt = fn, nblocks, template, f'<{nptr}Q'
        self.device, self.om_off, self.om_fmt = device, om_off, None if om_code is None else '<' + om_code
        self.extra = None              # byte offset of two more pointer slots patched per launch (second pass)
        self.block = 256

    def __call__(self, ptrs, stream, omega=None, extra=None):
        from ..backends import hip_runtime as rt
        buf = bytearray(self.template)
        struct.pack_into(self.fmt, buf, 0, *ptrs)
        if extra is not None:
            struct.pack_into('<2Q', buf, self.extra, *extra)
        if omega is not None and self.om_off is not None:
            struct.pack_into(self.om_fmt, buf, self.om_off, float(omega))
        import torch
        if self.device is not None and self.device != torch.cuda.current_device():
            with torch.cuda.device(self.device):
                rt.launch(self.fn, (self.nblocks,), (self.block,), bytes(buf), stream)
        else:
            rt.launch(self.fn, (self.nblocks,), (self.block,), bytes(buf), stream)


def _stream(stream, t):
    if stream is not None:
        return stream
    import torch
    return torch._C._cuda_getCurrentRawStream(t.device.index)


def _offset(fmt, i):
    """Byte offset of argument ``i`` in ``_pack(fmt, ...)``."""
    off = 0
    for j, c in enumerate(fmt):
        size = struct.calcsize(c)
        off += (-off) % size
        if j == i:
            return off
        off += size
    raise IndexError(i)


def _pack(fmt, *vals):
    """Kernel arguments at natural alignment (``HIP_LAUNCH_PARAM_BUFFER``)."""
    out, off = b'', 0
    for c, v in zip(fmt, vals):
        size = struct.calcsize(c)
        pad = (-off) % size
        out += b'\0' * pad + struct.pack('<' + c, v)
        off += pad + size
    return out + b'\0' * ((-off) % 8)
