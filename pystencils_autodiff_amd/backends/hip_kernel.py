"""A compiled GPU stencil kernel: schedule choice, hiprtc build, launch.

Replaces the reference's generated ``call_<kernel>`` wrapper
(``backends/astnodes.py:56-65,143-146``: ``at::Tensor`` → ``data_ptr<T>()``,
then ``kernel<<<grid, block>>>`` from ``indexing.call_parameters``,
``printer.py:88-108``). Calling convention kept: ``kernel(x=..., y=..., z=..., a=5.)``
with every field tensor and scalar passed by name, outputs written in place.
Launches go to torch's current HIP stream (the reference used the legacy
default stream, ``printer.py:106``).
"""
import math
import os

import numpy as np

from . import hip_runtime as rt
from .hip_band import band_choice, band_esize, band_geometry, band_plans, emit_band
from .hip_emitter import (MarchConfig, emit_generic, emit_march, emit_pointwise, emit_zsum, march_geometry, pair_ok,
                          storage_ctype, ws_geometry, zsum_plan)

__all__ = ['HipStencilKernel', 'default_march_config']


# row-band defaults, settled A/B rounds through the op (fn.apply + backward, same process;
# scripts/probes/op_band_ab.py, profiles/r03_op_band_ab*.log): box stencils (27 taps) 48-plane chunks without the
# trimmed chunk-edge planes (fwd+bwd 1024³ 1.707 vs 1.809 ms zsum, trimmed 24-plane chunks 2.01; 768³ 0.731 vs
# 0.762), star stencils 8-plane chunks (fp16 7-point 1024³ 1.461 vs 1.538, 768³ 0.635 vs 0.682). Launches of fewer
# than BAND_MIN_WG workgroups (z-slabs of a few planes) keep the zsum ring.
BAND_ZC_BOX, BAND_ZC_STAR = 48, 8
# round 4 (profiles/r04_op_band_ab1.log, same process, fwd+bwd through the op): the chunk's first two planes peeled
# without the taps of outputs before it (BTRIM=1) — 27-point 768³ 0.744 vs 0.768 ms, 1024³ 16-row bands 1.718 vs 1.744
# (and 1.679 with 32-plane chunks), fp16 7-point 768³ 0.602 vs 0.626
BAND_ZC_BOX16 = 32
# round 4 (profiles/r04_op_band_ab3.log .. _ab5.log): both chunk ends peeled at a compile-time chunk length (BTRIM=3)
# — 27-point 768³ 0.715 vs 0.724 ms (BTRIM=1), 1024³ 1.617 vs 1.640, fp16 7-point 768³ 0.594 vs 0.595-0.633
BAND_TRIM_DEFAULT = 3
# box-stencil chunk length: the longest of BAND_ZC_BOX_LADDER that still gives BAND_ROUND_WG workgroups (one
# round of three per CU; profiles/r04_op_zc_sweep.log): 27-point 512³ 32 planes 0.209 ms vs 16 0.243, 8 0.235;
# 256³ 8 planes 0.028 vs 11 0.036, 16 0.045; a 96×768² slab 12 planes 0.091 vs 8 0.095, 24 0.109
BAND_ZC_BOX_LADDER = (48, 32, 24, 16, 12, 8)
BAND_ROUND_WG = 768
BAND_MIN_WG = 768
# star stencils: 8-plane chunks, but 64-plane chunks on rows of <= 512 elements when that still gives >= 512
# workgroups (profiles/r04_op_zc_sweep.log, _ab6.log): fp16 7-point 512³ 0.184 vs 0.197 ms, 510³ 0.204 vs 0.229;
# 768³ keeps 8 (0.629 vs 0.675 at 96 planes, 0.699 at 64), 256³ too (0.024 vs 0.038 at 32)
BAND_ZC_STAR_LONG, BAND_STAR_LONG_MAX_X, BAND_STAR_LONG_MIN_WG = 64, 512, 512
# fp32 storage (4 cells per 16-byte chunk): 4-row bands measured slower through the op (7-point 512³ 0.387 vs
# 0.373 ms, 768³ 1.325 vs 1.261); 8-row bands of 4 rows per lane (4 compute waves, 60 KB of LDS) faster for star
# stencils on rows of <= 512 on every box (profiles/r04_op_f7_ab2.log .. _ab4.log, shared inputs): 512³
# 0.365-0.368 vs 0.373-0.389 ms; at 768 (6 compute waves, one workgroup per CU) it won on one box (1.189 vs 1.219)
# and lost on another (1.283-1.318 vs 1.261): zsum there. Box stencils in fp32 stay on zsum unless BAND=R asks.
BAND_F32_STAR_MAX_X = 512
BAND_ZC_STAR_F32 = 16
BAND_TRIM = BAND_TRIM_DEFAULT
# zero-padded image rows (x neighbours read from LDS, no DPP / boundary selects) for box stencils
# (profiles/r04_op_band_ab6.log): 27-point 768³ 0.699 vs 0.715 ms, 1024³ 1.581 vs 1.603, 512³ 0.198 vs 0.201;
# fp16 7-point 768³ 0.631 vs 0.629, 1024³ 1.444 vs 1.438 (not for star stencils)
BAND_PAD_BOX = 1
# partial rows on a padded image filled through registers (BREG) for star stencils on fp16 rows of odd length
# (profiles/r04_op_band_ab9.log): 7-point 511³ 0.210 vs 0.217 ms (DMA row pieces + v_perm realignment); even rows
# (510³ 0.207 vs 0.201) and box stencils (27-point 510³ 0.259 vs 0.245, 511³ 0.259 vs 0.252) keep the DMA pieces
BAND_REG_STAR_ODD = 1
# fp32 star stencils on rows with no whole-wave band height (idle lanes, hip_band.band_choice): the band up to this
# row length (7-point 512²×520 0.389 vs 0.632 ms on zsum, profiles/r04_op_band_idle.log)
BAND_F32_IDLE_MAX_X = 1024

# (CX, NR) candidates of the LDS-DMA plane ring for stencils that are not linear off the centre plane
# (hip_emitter._ring_ws_geometry), widest first: the first whose ring fits the LDS
RING_WS_TILES = ((4, 4), (4, 2), (2, 4), (2, 2), (1, 4), (1, 2), (1, 1))

# gpu_indexing_params keys of pystencils' own GPU indexing (``block_size``, ``maximum_block_size``, …, e.g.
# ``gpu_indexing_params={'block_size': (8, 4, 2)}`` in the reference's tests/test_graph_datahandling.py:70): they
# describe a one-thread-per-cell launch these schedules do not have, so they are accepted and ignored. Upper-case
# keys are this layer's tile parameters; an unknown one is a typo and raises.
TILE_KEYS = ('CX', 'WX', 'NR', 'ZMIN', 'ZMAX', 'BLK', 'D', 'NW', 'NT_STORE', 'ZSUM', 'PK', 'WS', 'AR', 'VIEW2D', 'ZC',
             'BLOCKS', 'MAP', 'BAND', 'BTY', 'BTRIM', 'BEDGE', 'BPAD', 'BZF', 'BREG', 'BNT', 'BFREE', 'BTAIL',
             'SFAST', 'SLP', 'PR', 'PD')
# Ablation knobs that make results WRONG (timing probes: ``BABL``). They are not tile keys — ``gpu_indexing_params`` and
# ``PSAD_MARCH`` reject them — and reach the planner only through this dict, which nothing on the op's path writes:
# a probe script sets it explicitly (``scripts/probes/op_band_ab.py``) and clears it again.
PROBE_KEYS = ('BABL',)
PROBE_KNOBS = {}


def _band_config(ir, ve, shape, over):
    """The row-band schedule (``hip_band``) for the stencils it fits — fp16 storage, and fp32 star stencils on rows of
    up to ``BAND_F32_STAR_MAX_X`` / ``BAND_F32_IDLE_MAX_X`` elements — when the row length is known and no tile
    override asks for another schedule (``BAND=0`` or ``PSAD_BAND=0`` turn it off, ``BAND=R`` / ``BTY`` pick
    rows per lane / band height)."""
    if shape is None or ir.ndim != 3 or os.environ.get('PSAD_BAND', '1') == '0':
        return None
    if 'BAND' in over:
        if not int(over['BAND']):
            return None
    elif any(k in over for k in ('CX', 'WX', 'NR', 'NW', 'ZSUM', 'PK', 'WS', 'AR', 'VIEW2D')):
        return None
    plans = band_plans(ir)
    X = int(shape[-1])
    es = band_esize(ir) if plans else 0
    ntaps = max(len(pl['w']) for pl in plans) if plans else 0
    whole = band_choice(X, len(plans), es, star=ntaps <= 12) if plans else None
    if whole is not None and whole[:2] == (16, 2) and 'BAND' not in over:
        # the wide-row 16-row band (one workgroup per CU) only where its launch still fills three rounds of the
        # chip with the chunk length it would take (a 96×768² slab would get 576 workgroups: 8-row bands there)
        nty16, Z = -(-int(shape[-2]) // 16), int(shape[0])
        zc16 = BAND_ZC_STAR if ntaps <= 12 else next((c for c in BAND_ZC_BOX_LADDER if nty16 * -(-Z // c) >=
                                                      BAND_ROUND_WG), BAND_ZC_BOX_LADDER[-1])
        if nty16 * -(-Z // zc16) < BAND_ROUND_WG:
            whole = band_choice(X, len(plans), es, star=ntaps <= 12, wide16=False)
    if plans and es == 4 and 'BAND' not in over and \
            not (ntaps <= 12 and X <= (BAND_F32_STAR_MAX_X if whole else BAND_F32_IDLE_MAX_X)):
        return None
    # rows with no band height of whole compute waves: a band whose last compute wave holds idle lanes
    choice = whole or (band_choice(X, len(plans), es, idle=True) if plans else None)
    if choice is None:
        return None
    TY, R, D = choice
    pad = int(over.get('BPAD', BAND_PAD_BOX if ntaps > 12 else 0))
    reg = int(over.get('BREG', BAND_REG_STAR_ODD if ntaps <= 12 and es == 2 and X % 2 and not int(over.get('BFREE', 0))
                       else 0))                 # (the LDS handshake takes the LDS-DMA loader)
    # fp32 star stencils: 8-row bands of 4 rows per lane (see BAND_F32_STAR_MAX_X) — one output only (band_choice's
    # rule: at most 2 rows per lane when a kernel stores two fields)
    g8 = band_geometry(X, 8, 4, 2, 4, pad, reg) if es == 4 and len(plans) == 1 else None
    if g8 and ntaps <= 12 and 'BAND' not in over and g8['ntask'] % 64 == 0 and g8['NCT'] <= 960 and \
            2 * g8['NI'] <= 63 and g8['lds_bytes'] <= 160 * 1024:
        TY, R, D = 8, 4, 2
    zc0 = int(over.get('ZMIN', BAND_ZC_BOX if ntaps > 12 else BAND_ZC_STAR))
    if ntaps > 12 and es == 2 and (X // 8) % 128 == 0 and R == 4 and \
            -(-int(shape[-2]) // 16) * -(-int(shape[0]) // zc0) >= BAND_MIN_WG:
        # box stencils on rows of a multiple of 1024 halves: 16-row bands, one plane in flight (18/16 rows read per
        # band instead of 10/8; 72 KB LDS): 27-point 1024³ fwd+bwd 1.712-1.719 vs 1.764-1.766 ms with 8-row bands
        # (profiles/r03_op_band_ab5.log, _ab6.log); the 7-point star stencil loses (1.65 vs 1.42), 768-wide rows too
        TY, D = 16, 1
        rule16 = True
    else:
        rule16 = False
    if 'BAND' in over:
        R = int(over['BAND'])
    TY = int(over.get('BTY', TY if TY % R == 0 else R * max(1, TY // R)))
    D = int(over.get('D', D))
    g = band_geometry(X, TY, R, D, es, pad, reg, free=int(over.get('BFREE', 0)))
    if TY % R or g['NCT'] > 960 or D * g['NI'] > 63 or g['lds_bytes'] > 160 * 1024 or g['NT'] > 1024:
        raise ValueError(f'band schedule: BTY={TY} BAND={R} D={D} do not fit rows of {X} elements')
    nty, Z = -(-int(shape[-2]) // TY), int(shape[0])
    min_wg = BAND_MIN_WG
    if ntaps <= 12 and es == 4:
        zc = BAND_ZC_STAR_F32
    elif ntaps <= 12:
        long_ok = X <= BAND_STAR_LONG_MAX_X and nty * -(-Z // BAND_ZC_STAR_LONG) >= BAND_STAR_LONG_MIN_WG
        zc = BAND_ZC_STAR_LONG if long_ok else BAND_ZC_STAR
        min_wg = BAND_STAR_LONG_MIN_WG if long_ok else BAND_MIN_WG
    elif TY == 16 and rule16:
        zc = BAND_ZC_BOX16              # (16-row bands of other rows — 2 rows per lane, idle lanes — take the ladder)
    else:
        zc = next((c for c in BAND_ZC_BOX_LADDER if nty * -(-Z // c) >= BAND_ROUND_WG), BAND_ZC_BOX_LADDER[-1])
    zc = int(over.get('ZMIN', zc))
    if 'BAND' not in over and nty * -(-Z // zc) < min_wg:
        return None
    zmax = int(over.get('ZMAX', zc))
    btrim = int(over.get('BTRIM', BAND_TRIM))
    if btrim == 3 and (zmax != zc or zc < 3):
        if 'BTRIM' in over:
            raise ValueError('band schedule: BTRIM=3 needs ZMIN == ZMAX >= 3')
        btrim = 1                       # chunk length not fixed at compile time: peel the chunk's first planes only
    return MarchConfig(VE=ve, BAND=R, BTY=TY, BX=X, D=D, ZSUM=True, NT_STORE=True, ZMIN=zc,
                       ZMAX=zmax, BLK=int(over.get('BLK', 512)), MAP=int(over.get('MAP', 0)),
                       BTRIM=btrim, BEDGE=int(over.get('BEDGE', 1)), BPAD=pad, BZF=int(over.get('BZF', 1)), BREG=reg,
                       BNT=int(over.get('BNT', 2)), BFREE=int(over.get('BFREE', 0)), BTAIL=int(over.get('BTAIL', 1)),
                       BABL=int(PROBE_KNOBS.get('BABL', 0)))


def ws_fallback_config(cfg):
    """The register-prefetch form of a WS (LDS-DMA loader) config, for planes beyond the loader's 32-bit buffer
    offsets: eight compute waves exist only on the LDS-DMA ring, so NW drops to 4 (and WX to at most 4) as in
    ``default_march_config``'s own fallback."""
    c = {**cfg.__dict__, 'WS': False}
    if c['NW'] == 8:
        c['NW'], c['WX'] = 4, min(c['WX'], 4)
    return MarchConfig(**c)


def default_march_config(ir, ve, shape=None, tuning=None, band=True):
    """Tile shape for a kernel and field shape (measured on MI355X).

    3-D stencils linear in their off-centre planes use the z-partial-sum schedule (``emit_zsum``):
    star stencils (7-point) with a 256×32 tile (CX=4, NR=8), box stencils (27-point) with a
    128×16 tile and 32-plane chunks; fp64 halves the tile width (register pressure). Other 3-D
    stencils use the LDS ring ("lite" ring when planes behind the centre are read only at (0,0)).
    2-D fields run as (1, Y, X) tiles of 256×16. Non-temporal stores for 3-D outputs (written
    once, never re-read by the sweep). Overrides: ``gpu_indexing_params`` or
    ``PSAD_MARCH="CX=..,NR=.."``.
    """
    from .hip_emitter import lite_fields
    star_ws = False
    cfg = dict(CX=4, WX=1, NR=8, NT_STORE=True, VIEW2D='yx', ZSUM=False, PK=False,
               ZMIN=32, ZMAX=64, BLK=512)
    probe = MarchConfig(VE=ve, **cfg)
    zsum_ok = zsum_plan(ir, probe) is not None
    if ir.ndim == 3 and set(ir.stencil_fields) - lite_fields(ir, probe):
        if zsum_ok:      # box stencil linear off-centre (27-point): z partial sums, small tile, short chunks
            # 768³ fp16: 0.460 ms (packed fp32 FMAs over column pairs, 2 waves side by side in x)
            # vs 0.469 scalar WX=1 vs 0.70 ms LDS ring; unrolling the plane loop 3x is slower (0.53-0.56)
            # chunks of 16..32 planes, ~2048 workgroups: 768³ 32 planes; one 8-GPU slab (96×768²) 16
            # planes, 0.067 vs 0.073 ms at 32
            # tap pairs by inline-asm ds_read2_b32 (AR): 0.421 vs 0.459 ms at 768³, 0.062 vs 0.067 ms per
            # 8-GPU slab (profiles/r01_tune_27pt_ar.log) — the compiler's adjacent-x merges cost 26 v_mov
            cfg.update(CX=2, WX=2, NR=4, ZSUM=True, PK=True, AR=True, ZMIN=16, ZMAX=32, BLK=2048)
            half = dict(CX=4, WX=1, NR=2, WS=True, D=3, ZMIN=24, ZMAX=24)
            if ws_geometry(ir, MarchConfig(VE=ve, **{**cfg, **half})):
                # fp16 storage: LDS-DMA loader wave into a half-precision ring, lanes own x-adjacent quads,
                # taps converted in registers (emit_zsum -> _emit_zsum_half), 256×8 tiles, 24-plane chunks:
                # 768³ 0.370-0.392 ms vs 0.431-0.448 ms for the register-prefetch AR form in the same
                # process; 96×768² slab 0.048-0.055 vs 0.059-0.069 ms (profiles/r02_tune_27pt_half*.log)
                cfg.update(half)
        else:
            cfg.update(CX=2, NR=4)                             # box stencil: full ring, LDS/VALU bound
    elif ir.ndim == 3 and zsum_ok:
        cfg.update(ZSUM=True)                                  # 1024³ 7-point: 1.495 ms vs 1.629 ms lite ring
        ws0 = ws_geometry(ir, MarchConfig(VE=ve, **{**cfg, 'WS': True}))
        if ws0:
            # star stencils, storage = compute type: LDS-DMA loader wave, 4 planes in flight, 256×16 tiles,
            # 128-plane chunks (one 5-wave workgroup per CU). 1024³ 7-point 1.411 ms vs 1.506 ms register
            # prefetch (128×32 tiles); one 8-GPU slab 0.182 vs 0.187 ms (profiles/r01_tune_ws_*.log).
            # fp16 storage (half-precision ring): 256×32 tiles, the same 16 KB per plane and workgroup:
            # 7-point fp16 1024³ 0.786 vs 0.889 ms, 768³ 0.372 vs 0.405, 128×1024² slab 0.092 vs 0.098,
            # 512³ 0.086 vs 0.087 (profiles/r02_tune_f16s_*.log). Chunks down to 8 planes: small domains are
            # latency bound with few long chunks (128³ 0.0106 vs 0.0197-0.021 ms, 256³ 0.0244 vs 0.032-0.036;
            # the chunk model keeps 1024³ / 768³ / 512³ / the 8-GPU slabs where they were,
            # profiles/r02_tune_small_*.log)
            cfg.update(WS=True, CX=4, NR=8 if ws0['kind'] == 'h' else 4, D=4, ZMIN=8, ZMAX=128, BLK=256)
            star_ws = True
    ring_ws = False                       # (the LDS-DMA plane ring of nonlinear stencils, 3-D or 2-D along axis 0)
    if ir.ndim == 3 and not zsum_ok:
        # stencils not linear off the centre plane (products / functions of neighbour taps): the plane ring fed by
        # an LDS-DMA loader wave, 2 planes in flight, the widest tile whose ring fits the LDS
        tiles = RING_WS_TILES
        if pair_ok(ir) and any(storage_ctype(f) == '_Float16' for f in ir.stencil_fields):
            # fp16 planes in the ring, taps as whole dwords of cell pairs (PR): 128×8 tiles, two planes in flight, for
            # two ring fields (varcoef forward), 128×4 and three in flight for more (its adjoint: three fields). 768³
            # fwd / bwd 0.618–0.634 / 1.066–1.095 ms vs 0.67–0.69 / 1.16–1.17 on the register ring
            # (profiles/r06_hring_f16.log, r06_hring_f16b.log: 20 tilings, 8 compute waves and deeper rings slower)
            two = len(ir.stencil_fields) <= 2
            tiles = [(2, 2 if two else 1)]
            cfg['PR'] = 1
        half_vec = ir.has_index_dims and any(storage_ctype(f) == '_Float16' for f in ir.stencil_fields)
        if half_vec:
            # vector fields in fp16 (fp16 images, taps converted): 128×8 tiles. Lanes own x-adjacent cell pairs with
            # packed fp32 statements (PR) where the statements allow — a lane's elements are then contiguous from an
            # even offset and its reads merge; eight compute waves for the adjoint's two ring fields. Advection u(3)
            # 256³ fwd / bwd 0.052 / 0.054 ms vs 0.063 / 0.063 per cell, 0.139 / 0.069 on the widest fitting tile
            # (256×16), 0.131 / 0.153 one thread per cell (profiles/r06_vec16_tiles.log, r06_vec16_pairs.log; fp32
            # vector fields measured slower as pairs: 0.075 / 0.12 vs 0.071 / 0.095)
            tiles = [(2, 2)]
            if pair_ok(ir, vectors=True):
                cfg['PR'] = 1
        for cx, nr in tiles:
            c = {**cfg, 'CX': cx, 'NR': nr, 'WS': True, 'D': 2 if nr == 2 or not cfg.get('PR') else 3, 'ZMIN': 8,
                 'ZMAX': 128, 'BLK': 256}
            if half_vec and len(ir.stencil_fields) > 1:
                c['NW'] = 8
            w = ws_geometry(ir, MarchConfig(VE=ve, **c))
            if w is not None and w['lds_bytes'] <= 160 * 1024:
                cfg.update(c)
                ring_ws = True
                break
        if not ring_ws:
            cfg['PR'] = 0                 # (the register ring stores fp32 images: pairs measured neutral there)
    if ir.ndim == 3 and not zsum_ok and not ring_ws:
        # nonlinear stencils on the register-prefetch ring (fp16 storage: the LDS-DMA ring holds the compute type):
        # 128×8 tiles, four workgroups per CU — varcoef fp16 768³ fwd / bwd 0.69–0.71 / 1.16–1.18 ms vs 0.81 / 1.31–1.34
        # with the budget's 256×16 / 256×8 (profiles/r06_varcoef_f16_tiles.log: latency, not VALU — packed cell pairs
        # or two planes in flight on the wide tiles gave nothing, r06_varcoef_pairs_f16.log, r06_varcoef_pd2_f16.log)
        cfg.update(CX=2, NR=2)
    if ir.ndim == 2:
        cfg.update(CX=4, WX=1, NR=4, VIEW2D='yx', NT_STORE=False)   # 256×16 tiles (4096²: 0.024 ms, 5.6 TB/s)
        plans2 = zsum_plan(ir, probe)
        if plans2 is None or any(pl['rest'] != 0 for pl in plans2):
            # nonlinear 2-D stencils (one tile per workgroup, nothing to pipeline): 128×8 tiles, more workgroups in
            # flight — 2-D varcoef 4096² fp32 fwd / bwd 0.52 / 0.51 of 8 TB/s vs 0.49 / 0.38 on 256×16, fp16 0.30 /
            # 0.35 vs 0.28 / 0.21 (profiles/r06_nl2d.log)
            cfg.update(CX=2, NR=2)
            # ... and on long 16-byte-piece rows: march along axis 0 (VIEW2D='zy', rows as the planes of the LDS-DMA
            # ring, four waves side by side in x: 512-cell row strips; fp16 as x-adjacent cell pairs), 512 / 1024
            # workgroups of 64 / 32 rows at 4096²: 2-D varcoef 4096² fp32 fwd / bwd 0.61 / 0.57–0.58 of 8 TB/s,
            # fp16 0.40–0.42 / 0.49 (profiles/r06_nl2d_zy.log: 40 tilings and chunkings; the register ring along
            # axis 0 was slower, 0.41 / 0.41, and 128-row chunks 0.51 / 0.49)
            # (fp64: 1024-cell strips, not halved below — fwd / bwd 0.56–0.62 / 0.58–0.61 vs 0.55–0.56 / 0.53–0.56 on
            # the (1, Y, X) tiles; 256-cell strips lost the adjoint, 0.53, profiles/r06_nl2d_f64.log)
            half2 = any(storage_ctype(f) == '_Float16' for f in ir.stencil_fields)
            wide = np.dtype(ir.compute_dtype).itemsize == 8
            zy = dict(VIEW2D='zy', NR=1, NW=4, WX=4, CX=4 if wide else 2, WS=True, D=2, ZMIN=16 if half2 else 32,
                      ZMAX=64, BLK=1024 if half2 else 512, PR=1 if half2 and pair_ok(ir, vectors=True) else 0)
            if ir.stencil_fields and (shape is None or int(shape[-1]) >= 64 * zy['CX'] * zy['WX']):
                w = ws_geometry(ir, MarchConfig(VE=ve, **{**cfg, **zy}))
                if w is not None and w['lds_bytes'] <= 160 * 1024:
                    cfg.update(zy)
                    ring_ws = True
    if ir.has_index_dims and not ring_ws:
        # vector fields (components interleaved in the plane image) linear off the centre plane: the zsum schedule;
        # narrower tiles keep the image (TX + 2H)·C elements wide (the plane ring picked its tile above)
        from .hip_emitter import ncomp
        cmax = max([ncomp(f) for f in ir.stencil_fields] + [1])
        cfg.update(ZSUM=True, PK=False, AR=False)
        while cfg['CX'] > 1 and cfg['CX'] * cmax > 4:
            cfg['CX'] //= 2
    if np.dtype(ir.compute_dtype).itemsize == 8 and not (ir.ndim == 2 and ring_ws):
        cfg['CX'] = max(1, cfg['CX'] // 2)                     # fp64: half-width tiles (512³: 0.380 vs 0.536 ms)
    elif ir.ndim == 3 and cfg['ZSUM'] and not cfg['PK'] and not cfg.get('WS'):
        # star stencils: 128×32 tiles, two workgroups per CU. 512³ / one 8-GPU slab of 1024³
        # (128×1024²): 0.191 / 0.187 ms vs 0.214 / 0.208 ms with 256×32 tiles; 1024³ a tie
        cfg['CX'] = 2
    env = os.environ.get('PSAD_MARCH')
    over = {k: v for k, v in dict(tuning or {}).items() if not k.islower()}     # pystencils indexing keys: ignored
    if env:
        for kv in env.split(','):
            k, v = kv.split('=')
            over[k.strip()] = v.strip() if k.strip() == 'VIEW2D' else int(v)
    view_yx = ir.ndim == 2 and str(over.get('VIEW2D', cfg['VIEW2D'])) != cfg['VIEW2D']
    if ring_ws and (any(k in over for k in ('CX', 'WX', 'NR', 'NW')) or view_yx) and 'WS' not in over:
        cfg.update(WS=False, D=3)           # a tile override on the ring: the register-prefetch form it was sized for
        if ir.ndim == 2:
            cfg.update(VIEW2D='yx', NW=4, WX=1, NR=2, PR=0, ZMIN=32, ZMAX=64, BLK=512,   # (the 2-D one: (1, Y, X) tiles)
                       CX=1 if np.dtype(ir.compute_dtype).itemsize == 8 else 2)
            if ir.has_index_dims:
                cfg.update(ZSUM=True, PK=False, AR=False)     # (vector fields: the zsum plane, as without the ring)
            ring_ws = False
    for k, v in over.items():
        if k not in TILE_KEYS:
            raise ValueError(f"unknown tile parameter '{k}' (gpu_indexing_params / PSAD_MARCH)")
        if k in ('CX', 'WX', 'NR', 'ZMIN', 'ZMAX', 'BLK', 'D', 'NW', 'MAP'):
            cfg[k] = int(v)
        elif k in ('NT_STORE', 'ZSUM', 'PK', 'WS', 'AR'):
            cfg[k] = bool(int(v)) if not isinstance(v, bool) else v
        elif k == 'VIEW2D':
            cfg[k] = str(v)
        elif k in ('SFAST', 'SLP', 'PR', 'PD'):
            cfg[k] = int(v)
    if cfg.get('PR') and 'PR' not in over and (cfg['CX'] % 2 or not pair_ok(ir, vectors=bool(cfg.get('WS')))):
        cfg['PR'] = 0          # a tile override the default pair form cannot take (odd CX; vector fields off the ring)
    if ring_ws and PROBE_KNOBS.get('BABL'):
        cfg['BABL'] = int(PROBE_KNOBS['BABL'])   # (timing probe of the march ring, as on the band: 3 = no plane loads)
    bc = _band_config(ir, ve, shape, over) if band else None
    if bc is not None:
        return bc
    if 'NW' in over and 'WX' not in over:
        cfg['WX'] = min(cfg['WX'], cfg['NW'])
    if cfg['ZSUM'] and zsum_plan(ir, MarchConfig(VE=ve, **cfg)) is None:
        cfg['ZSUM'] = False                                    # not eligible: LDS ring instead
    cmin = 2 if cfg.get('PR') and not cfg['ZSUM'] else 1      # packed cell pairs: two cells per lane and column
    if shape is not None:
        X = int(shape[-1])
        if 'CX' not in over:
            while cfg['CX'] > cmin and 64 * cfg['CX'] * cfg['WX'] // 2 >= X:
                cfg['CX'] //= 2
            tx = 64 * cfg['CX'] * cfg['WX']
            ws0 = ws_geometry(ir, MarchConfig(VE=ve, **cfg)) if cfg.get('WS') else None
            quads = ws0 is not None and ws0['kind'] == 'h'       # the half ring needs lanes owning quads
            if cfg.get('WS') and cfg['CX'] > cmin and -(-X // (tx // 2)) * (tx // 2) < -(-X // tx) * tx and \
                    (not quads or (cfg['CX'] // 2) % 4 == 0):
                # WS tiles: half width when it pads x less (384³ 7-point: 0.116 → 0.081 ms with 48-plane
                # chunks, profiles/r01_tune_odd_sizes.log)
                cfg['CX'] //= 2
        if 'WX' not in over:
            while cfg['WX'] > 1 and 64 * cfg['CX'] * cfg['WX'] // 2 >= X:
                cfg['WX'] //= 2
        ny = int(shape[-2]) if ir.ndim == 3 or cfg['VIEW2D'] == 'yx' else 1
        if 'NR' not in over:
            while cfg['NR'] > 1 and (cfg.get('NW', 4) // cfg['WX']) * cfg['NR'] // 2 >= ny:
                cfg['NR'] //= 2
    # LDS budget: two workgroups per CU (≤ 80 KB) for the register-prefetch defaults, the 160 KB hardware
    # limit for the LDS-DMA ring and for explicit tile overrides
    budget = 80 * 1024 if not ('CX' in over or 'NR' in over or cfg.get('WS')) else 160 * 1024

    def lds(c):
        mc = MarchConfig(VE=ve, **c)
        ws = ws_geometry(ir, mc)
        return ws['lds_bytes'] if ws else march_geometry(ir, mc)['lds_bytes']
    while cfg.get('WS') and cfg.get('D', 3) > 1 and lds(cfg) > 160 * 1024:
        cfg['D'] = cfg.get('D', 3) - 1                          # fewer planes in flight before smaller tiles
    while lds(cfg) > budget and (cfg['NR'] > 1 or cfg['CX'] > cmin):
        if (cfg['NR'] >= cfg['CX'] or cfg['CX'] <= cmin) and cfg['NR'] > 1:
            cfg['NR'] //= 2
        else:
            cfg['CX'] //= 2
    if cfg.get('WS') and not cfg['ZSUM'] and lds(cfg) > 160 * 1024:
        # a plane ring that does not fit even at the smallest tile (many fields of wide radius): the register form
        cfg['WS'] = False
        if cfg.get('NW', 4) == 8:                             # (eight compute waves only on the LDS-DMA ring)
            cfg['NW'], cfg['WX'] = 4, min(cfg['WX'], 4)
        while lds(cfg) > budget and (cfg['NR'] > 1 or cfg['CX'] > cmin):
            if (cfg['NR'] >= cfg['CX'] or cfg['CX'] <= cmin) and cfg['NR'] > 1:
                cfg['NR'] //= 2
            else:
                cfg['CX'] //= 2
    if ir.ndim == 3 and lds(cfg) > 160 * 1024:
        raise ValueError(f'no tile of this kernel fits the 160 KB LDS ({lds(cfg)} B at {cfg})')
    if star_ws and cfg.get('WS') and shape is not None and 'MAP' not in over:
        ntx = -(-int(shape[-1]) // (64 * cfg['CX'] * cfg['WX']))
        if ntx & (ntx - 1):
            # tiles per row not a power of two: dispatch order instead of the XCD-aware remap. Through the op,
            # fwd + bwd, same process (scripts/probes/map_ab.py, profiles/r03_map_ab.log): 768³ fp32 -8.6 %
            # (5.91 / 5.78 TB/s), 640³ -4.4 %, 768³ fp16 -4.7 %, 640³ fp64 -2.5 %; with 2 or 4 tiles per row
            # the dispatch order pins each XCD to the same x columns of every plane: 1024³ +10 %, 128×1024²
            # +10 %, 512³ fp64 +6 % — those keep the remap
            cfg['MAP'] = 1
    return MarchConfig(VE=ve, **cfg)


def _torch():
    import torch
    return torch


class HipStencilKernel:
    def __init__(self, kernel):
        from .kernel_ir import split_soa
        self.kernel = kernel
        # fzyx vector fields run as one scalar field per component (kernel_ir.split_soa)
        self.ir, self._soa = split_soa(kernel.ir)
        self.name = kernel.function_name
        self._variants = {}            # variant key -> (source, kernel name)
        self._plans = {}               # launch key -> _Plan
        self._specs = None
        self._ref_index = [f.name for f in self.ir.fields].index(self.ir.fields_written[0].name)
        self.last_variant = None
        self.last_plan = None

    # -- sources --------------------------------------------------------------------------------
    def schedule(self):
        ir = self.ir
        if ir.ndim not in (1, 2, 3) or ir.islice is not None:
            return 'generic'               # an iteration_slice: any rectangular subset, bound-checked reads
        if ir.pointwise:
            return 'generic' if ir.has_index_dims else 'pointwise'
        if ir.periodic:
            return 'generic'                   # wrapped reads: one thread per cell
        taps = {}
        for r in ir.reads:
            taps.setdefault(r.field, set()).add(r.offsets)
        if ir.stencil_fields and not ir.has_index_dims and all(len(taps.get(f, ())) == 1 for f in ir.stencil_fields):
            # every stencil field read at ONE offset (pull-streaming lattice Boltzmann: component i at -c_i):
            # staging planes in LDS buys no reuse, the one-thread-per-cell schedule streams each component
            return 'generic'
        if ir.ndim in (2, 3) and all(all(o == 0 for o in s[1]) for s in ir.stores) and \
                len({f.dtype for f in ir.fields}) == 1:
            if ir.has_index_dims:
                # vector fields: the zsum schedule (components interleaved in the plane image) when the
                # stencil is linear off the centre plane, the LDS-DMA plane ring (components interleaved the same
                # way) for other 3-D stencils, else one thread per cell
                probe = MarchConfig(VE=self._vec_elems(), ZSUM=True)
                if ir.stencil_fields and zsum_plan(ir, probe) is not None:
                    return 'march'
                ring = self._march_cfg(self._vec_elems())
                return 'march' if ir.stencil_fields and ring.WS and not ring.ZSUM else 'generic'
            return 'march'
        return 'generic'

    def _vec_elems(self):
        return 16 // self.ir.fields[0].dtype.itemsize

    def _march_cfg(self, ve, shape=None, band=True):
        return default_march_config(self.ir, ve, shape, self.kernel.tuning, band=band)

    def source(self, variant):
        if variant not in self._variants:
            kind = variant[0]
            kname = f"{self.name}_{kind}"
            if kind == 'pointwise':
                src = emit_pointwise(self.ir, kname)
            elif kind == 'march' and variant[1].BAND:
                kname = f"{self.name}_band"
                src = emit_band(self.ir, kname, variant[1])
            elif kind == 'march' and variant[1].ZSUM:
                kname = f"{self.name}_zsum"
                src = emit_zsum(self.ir, kname, variant[1])
            elif kind == 'march':
                src = emit_march(self.ir, kname, variant[1])
            else:
                src = emit_generic(self.ir, kname, idx32='idx32' in variant[1:], contig='contig' in variant[1:],
                                   shared='shared' in variant[1:])
            self._variants[variant] = (src, kname)
        return self._variants[variant]

    def primary_variant(self):
        s = self.schedule()
        if s == 'march':
            shape = None
            fixed = [f for f in self.ir.fields if f.has_fixed_shape]
            if fixed:
                shape = tuple(int(x) for x in fixed[0].spatial_shape)
            return ('march', self._march_cfg(self._vec_elems(), shape))
        return (s,)

    @property
    def code(self):
        return self.source(self.primary_variant())[0]

    @staticmethod
    def options(variant):
        """hiprtc options of a variant: the plane ring of nonlinear stencils (``emit_march``) compiles without the SLP
        vectorizer unless ``SLP=1`` — it paired scalar fp32 ops into ``v_pk_*`` at the price of register moves (varcoef
        fp16 adjoint: 1030 → 871 VALU instructions, 246 → 200 VGPRs); the zsum / band kernels form their packed math
        from explicit vector types and keep the default."""
        if variant[0] == 'march' and not variant[1].ZSUM and not variant[1].BAND and not variant[1].SLP:
            return rt.DEFAULT_OPTIONS + ('-fno-slp-vectorize',)
        return rt.DEFAULT_OPTIONS

    def function(self, variant, device):
        src, kname = self.source(variant)
        code = rt.compile_hip(src, self.options(variant))
        if variant[0] == 'pointwise':
            return {k: rt.load_function(code, f"{kname}_{k}", device) for k in ('v4', 'v1')}
        return rt.load_function(code, kname, device)

    def build(self):
        """Compile the primary variant ahead of time (hiprtc works without a GPU)."""
        v = self.primary_variant()
        return rt.compile_hip(self.source(v)[0], self.options(v))

    # -- launch ---------------------------------------------------------------------------------
    def _field_specs(self):
        if self._specs is None:
            torch = _torch()
            self._specs = [(f.name, getattr(torch, f.dtype.numpy_dtype.name), f.spatial_dimensions + f.index_dimensions,
                            tuple(int(x) for x in f.shape) if f.has_fixed_shape else None) for f in self.ir.fields]
        return self._specs

    def __call__(self, halos=None, stream=None, force_schedule=None, z_range=None, x_border=False, z_limits=None,
                 **kwargs):
        """Launch on the field tensors / scalars given by name.

        ``x_border=True`` asks the zsum schedule to also store zeros at x outside the iteration bounds of
        the rows it writes (returns True if the launch did). ``halos`` = ``{field: (lo_planes, hi_planes)}``: tensors holding the RZ planes just
        below plane 0 / above plane Z-1 of a stencil field (``None`` = zeros); ``z_range``
        restricts the written planes of axis 0 — ``(lo, hi)``, or two disjoint ranges of equal
        length ``((lo0, hi0), (lo1, hi1))`` written by ONE launch (the two slab faces; both:
        z-slab decomposition, ``zslab.py``). ``z_limits=(lo, hi)`` replaces the kernel's own axis-0
        iteration bounds (an interior-only kernel on a z-slab: the GLOBAL domain's interior, in local
        plane numbers).
        The first call for a given (shape, alignment, halo layout, z range) builds a launch plan
        (variant, function handle, grid, argument layout); later calls only re-pack pointers.
        """
        prep = self.prepare(halos=halos, force_schedule=force_schedule, z_range=z_range, x_border=x_border,
                            z_limits=z_limits, **kwargs)
        if prep is None:
            return None
        fn, grid, block, packed, xb, device = prep
        if grid == 0:
            return xb
        torch = _torch()
        if stream is None:
            stream = torch._C._cuda_getCurrentRawStream(device)
        if device != torch.cuda.current_device():
            # the function handle belongs to the module loaded on the tensors' device: launch with it current
            with torch.cuda.device(device):
                rt.launch(fn, (grid,), (block,), packed, stream)
        else:
            rt.launch(fn, (grid,), (block,), packed, stream)
        return xb

    def prepare(self, halos=None, force_schedule=None, z_range=None, x_border=False, z_limits=None,
                start_signal=False, halo_wait=False, **kwargs):
        """Everything of a launch but the launch: ``(function, grid, block, packed args, x_border done,
        device)``, or None for an empty domain (arguments as for ``__call__``). ``start_signal=True`` (march
        schedules, the z-slab interior): the kernel takes a signal word and a value after its extents, both zero in
        the packed arguments (no store) — the caller patches them at ``last_plan.sig_offsets``. ``halo_wait=True``
        (LDS-DMA loader schedules, the z-slab faces on the compute stream): the loader waits for a word to reach a
        value before its first plane load; both zero (no wait) until patched at ``last_plan.hwait_offsets``; a plan
        without an LDS-DMA loader raises ``ValueError``."""
        torch = _torch()
        ir = self.ir
        if self._soa:
            kwargs = self._bind_components(kwargs)
        tensors = []
        for name, dtype, ndim, fixed in self._field_specs():
            t = kwargs.get(name)
            if t is None:
                raise TypeError(f"{self.name}: missing field argument '{name}'")
            if not isinstance(t, (torch.Tensor, _Plane)) or not t.is_cuda:
                raise TypeError(f"{self.name}: field '{name}' must be a torch tensor on the GPU")
            if t.dtype != dtype:
                raise TypeError(f"{self.name}: field '{name}' has dtype {t.dtype}, kernel expects {dtype}")
            if t.dim() != ndim:
                raise ValueError(f"{self.name}: field '{name}' expects {ndim} dims, got {t.dim()}")
            if fixed is not None and tuple(t.shape) != fixed:
                raise ValueError(f"{self.name}: field '{name}' was declared with shape {fixed}, got {tuple(t.shape)}")
            tensors.append(t)
        scalars = []
        for s_ in ir.scalars:
            if s_.name not in kwargs:
                raise TypeError(f"{self.name}: missing scalar argument '{s_.name}'")
            scalars.append(float(kwargs[s_.name]))
        ref = tensors[self._ref_index]
        shape = tuple(ref.shape[:ir.ndim])
        for t, (name, _, _, _) in zip(tensors, self._specs):
            if tuple(t.shape[:ir.ndim]) != shape:
                raise ValueError(f"{self.name}: field '{name}' has spatial shape {tuple(t.shape[:ir.ndim])}, "
                                 f"expected {shape}")
        if any(n == 0 for n in shape):
            return None
        device = ref.device.index
        halo_list = []
        if halos:
            for f in ir.stencil_fields:
                lo, hi = halos.get(f.name, (None, None))
                halo_list += [lo, hi]
        ptrs = [t.data_ptr() for t in tensors]
        hptrs = [h.data_ptr() if h is not None else 0 for h in halo_list]
        contiguous = all(t.is_contiguous() for t in tensors)
        strides = None if contiguous else tuple(tuple(t.stride()) for t in tensors)
        # the alignment CLASS of every pointer (trailing zero bits, capped at 32 bytes): the plan's load path
        # depends on 16-, 8-, 4- and 2-byte alignment (LDS-DMA ring, narrower vectors, XM rows), so a plan built
        # for one class must not serve a pointer of another
        align = tuple(_align_class(p) for p in ptrs + hptrs)
        key = (force_schedule, bool(x_border), shape, strides, align,
               tuple(h.numel() if h is not None else -1 for h in halo_list), _zkey(z_range),
               tuple(z_limits) if z_limits is not None else None, device) + (('sig',) if start_signal else ()) + \
            (('hwait',) if halo_wait else ())
        plan = self._plans.get(key)
        if plan is None:
            if z_limits is not None:
                if not ir.ndim == 3 or not 0 <= int(z_limits[0]) <= int(z_limits[1]) <= shape[0]:
                    raise ValueError(f'z_limits {z_limits} must lie in [0, {shape[0]}] of a 3-D kernel')
            plan = self._make_plan(tensors, halo_list, shape, device, contiguous, force_schedule, z_range, x_border,
                                   z_limits, start_signal, halo_wait)
            self._plans[key] = plan
        self.last_variant = plan.variant
        self.last_plan = plan
        if plan.grid == 0:
            return plan.fn, 0, plan.block, b'', plan.xb, device
        return plan.fn, plan.grid, plan.block, plan.pack(ptrs, hptrs, scalars), plan.xb, device

    def _bind_components(self, kwargs):
        """fzyx vector tensors → one plane per component (``split_soa``'s scalar fields); any strides are
        accepted (a component whose plane is not C-contiguous takes the generic schedule). The planes are
        ``_Plane`` records (pointer arithmetic on the parent), not torch views: a D3Q19 adjoint binds 57
        planes per launch, ~4 µs of host time each as views."""
        torch = _torch()
        kwargs = dict(kwargs)
        sdim = self.ir.ndim
        for name, comps in self._soa.items():
            t = kwargs.pop(name, None)
            if t is None:
                raise TypeError(f"{self.name}: missing field argument '{name}'")
            if not isinstance(t, torch.Tensor):
                raise TypeError(f"{self.name}: field '{name}' must be a torch tensor on the GPU")
            nidx = len(comps[0][1])
            if t.dim() != sdim + nidx:
                raise ValueError(f"{self.name}: field '{name}' expects {sdim + nidx} dims, got {t.dim()}")
            shape, strides = tuple(t.shape), tuple(t.stride())
            base, esize = t.data_ptr(), t.element_size()
            for cfield, idx in comps:
                if any(not 0 <= i < n for i, n in zip(idx, shape[sdim:])):
                    raise ValueError(f"{self.name}: field '{name}' has component shape {shape[sdim:]}")
                off = sum(i * st for i, st in zip(idx, strides[sdim:]))
                kwargs[cfield.name] = _Plane(t, base + off * esize, shape[:sdim], strides[:sdim])
        return kwargs

    def _make_plan(self, tensors, halo_list, shape, device, contiguous, force_schedule, z_range, x_border=False,
                   z_limits=None, start_signal=False, halo_wait=False):
        torch = _torch()
        ir = self.ir
        sched = force_schedule or self.schedule()
        if sched != 'generic' and not contiguous:
            sched = 'generic'
        if (halo_list or z_range is not None or z_limits is not None or start_signal or halo_wait) and \
                sched != 'march':
            raise ValueError('halo planes / z ranges / start signals are only supported by the march schedule')
        with torch.cuda.device(device):
            if sched == 'pointwise':
                return self._plan_pointwise(tensors, shape, device)
            if sched == 'march':
                return self._plan_march(tensors, halo_list, shape, device, z_range, x_border, z_limits, start_signal,
                                        halo_wait)
            return self._plan_generic(tensors, shape, device)

    def _scalar_kind(self):
        return 'f64' if self.ir.compute_dtype == np.float64 else 'f32'

    def _plan_pointwise(self, tensors, shape, device):
        fns = self.function(('pointwise',), device)
        n = int(np.prod(shape))
        aligned = all(t.data_ptr() % 32 == 0 for t in tensors)
        from . import hip_emitter as he
        per_block = 256 * (4 * he.POINTWISE_UNROLL if aligned else 1)
        cap = (he.POINTWISE_MAX_BLOCKS or 2 ** 31 - 1) if aligned else 256 * 16
        blocks = max(1, min(math.ceil(n / per_block), cap))
        kinds = ['ptr'] * len(tensors) + ['i64'] + [self._scalar_kind()] * len(self.ir.scalars)
        return _Plan(('pointwise', 'v4' if aligned else 'v1'), fns['v4' if aligned else 'v1'], blocks, kinds,
                     len(tensors), 0, [n])

    def _plan_generic(self, tensors, shape, device):
        from .hip_emitter import magic_u32
        ir = self.ir
        if ir.periodic and any(r >= int(n) for r, n in zip(ir.radius, shape)):
            raise ValueError(f'periodic kernel: stencil radius {ir.radius} must be below the extent {shape}')
        bounds = ir.iteration_bounds(shape)
        ncell = int(np.prod([hi - lo for lo, hi in bounds]))
        idx32 = 0 < ncell < 2 ** 31
        contig = all(t.is_contiguous() for t in tensors)
        # one shape and one set of strides for every tensor, offsets within 32 bits: shared 32-bit addressing
        reach = max(list(ir.radius) + [0]) + 1
        shared = len({(tuple(t.shape), tuple(t.stride())) for t in tensors}) == 1 and \
            sum(abs(int(st)) * (int(n) - 1 + reach) for st, n in zip(tensors[0].stride(), tensors[0].shape)) < 2 ** 31 - 1
        variant = ('generic',) + (('idx32',) if idx32 else ()) + (('contig',) if contig else ()) + \
            (('shared',) if shared else ())
        fn = self.function(variant, device)
        statics = [int(n) for n in shape]
        for t in (tensors[:1] if shared else tensors):
            statics += [int(s_) for s_ in t.stride()]
        kinds = ['ptr'] * len(tensors) + ['i64'] * len(shape) + ['i32' if shared else 'i64'] * (len(statics) - len(shape))
        for lo, hi in bounds:
            statics += [lo, hi]
            kinds += ['i64', 'i64']
        if idx32:
            extra = [ncell]
            kinds.append('u32')
            for lo, hi in bounds[1:]:
                m, sh = magic_u32(max(1, hi - lo))
                extra += [m, sh]
                kinds += ['u32', 'i32']
            statics += extra
        kinds += [self._scalar_kind()] * len(ir.scalars)
        blocks = max(1, min(math.ceil(ncell / 256), 256 * 64)) if ncell > 0 else 0
        return _Plan(variant, fn, blocks, kinds, len(tensors), 0, statics)

    def _resident_slots(self, fn, block, device):
        """Workgroups of this kernel resident on the whole GPU at once (LDS, VGPR and wave limits per CU
        × CU count), from the loaded code object's attributes."""
        torch = _torch()
        a = rt.function_attributes(fn)
        regs, lds = a['num_regs'], a['shared_bytes']
        waves = -(-block // 64)
        per_simd = max(1, min(8, 512 // max(8, -(-regs // 8) * 8)))
        per_cu = max(1, min(4 * per_simd // waves, 163840 // max(1, lds), 32 // waves))
        return per_cu * torch.cuda.get_device_properties(device).multi_processor_count

    @staticmethod
    def quantized_chunk(nz, nt, slots, zmin, zmax, rz, wsat):
        """Chunk length for the WS schedule (few resident workgroups, each with a fixed number of bytes
        in flight): the chunk count c minimising Σ_rounds (planes per chunk + halo + fill) ·
        max(1, active / wsat) — a round takes at least one workgroup's march (latency bound below
        ``wsat`` concurrent workgroups, bandwidth bound above). The short last round of 128-plane
        chunks is what makes 768³ slower per cell than 1024³ (profiles/r01_tune_odd_sizes.log)."""
        best = None
        c0 = max(1, -(-nz // zmax))
        for c in range(c0, max(c0, nz // max(1, zmin)) + 1):
            zc = -(-nz // c)
            n = nt * -(-nz // zc)
            full, rem = divmod(n, slots)
            t = (zc + 2 * rz + 2) * (full * max(1.0, slots / wsat) + (max(1.0, rem / wsat) if rem else 0.0))
            if best is None or t < best[0] - 1e-9:
                best = (t, zc)
        return best[1]

    def march_launch_geometry(self, shape, cfg, z_range=None, slots=None, z_limits=None):
        """(Z, Y, X), bounds and grid of the march schedule for a field shape; ``slots`` = resident
        workgroups (``_resident_slots``) switches the WS schedule to quantisation-aware chunks."""
        ir = self.ir
        bounds = ir.iteration_bounds(shape)
        if z_limits is not None:
            bounds[0] = (int(z_limits[0]), int(z_limits[1]))
        if z_range is not None and _is_pair(z_range):
            (a0, a1), (b0, b1) = [(int(a), int(b)) for a, b in z_range]
            lo, hi = bounds[0]
            if ir.ndim == 2 and cfg.VIEW2D == 'yx':
                raise ValueError("z ranges need the 'zy' view of 2-D fields")
            if not (lo <= a0 < a1 <= b0 < b1 <= hi) or a1 - a0 != b1 - b0:
                raise ValueError(f'z_range pair {z_range} must be disjoint, ordered, of equal length '
                                 f'and inside [{lo}, {hi})')
            geo = self.march_launch_geometry(shape, cfg, (a0, b1), z_limits=z_limits)
            zc = a1 - a0
            geo.update(zlo=a0, zhi=b1, zc=zc, zstep=b0 - a0, grid=geo['ntx'] * geo['nty'] * 2)
            return geo
        if z_range is not None:
            lo, hi = bounds[0]
            bounds = [(max(lo, int(z_range[0])), min(hi, int(z_range[1])))] + list(bounds[1:])
        if ir.ndim == 3:
            Z, Y, X = shape
            (zlo, zhi), (ylo, yhi), (xlo, xhi) = bounds
        elif cfg.VIEW2D == 'yx':
            Z, (Y, X) = 1, shape
            (zlo, zhi) = (0, 1)
            (ylo, yhi), (xlo, xhi) = bounds
            if z_range is not None:
                raise ValueError("z ranges need the 'zy' view of 2-D fields")
        else:
            Z, X = shape
            Y = 1
            (zlo, zhi), (xlo, xhi) = bounds
            ylo, yhi = 0, 1
        if cfg.BAND:            # full-row bands (hip_band): one band column, x handled inside the kernel
            ntx, nty = 1, max(1, math.ceil(yhi / cfg.BTY))
        else:
            ntx = max(1, math.ceil((X if cfg.XB else xhi) / cfg.TX))
            nty = max(1, math.ceil(yhi / cfg.TY))
        nt = ntx * nty
        nz = max(0, zhi - zlo)
        # chunk length: aim at ~2 workgroups per CU (512 blocks), ZMIN..ZMAX planes per chunk (each chunk
        # re-reads 2·RZ halo planes). 7-point 1024³, 128×32 tiles: 64-plane chunks 1.536 ms vs 128-plane
        # 1.570 ms (profiles/r01_tune_cx_ab_1024.log); 512³ and 128×1024² slabs land on 64 by the target
        target = int(self.kernel.tuning.get('BLOCKS', os.environ.get('PSAD_MARCH_BLOCKS', cfg.BLK)))
        zc = self.kernel.tuning.get('ZC') or int(os.environ.get('PSAD_MARCH_ZC', 0)) or \
            min(nz, max(cfg.ZMIN, min(cfg.ZMAX, math.ceil(nz * nt / target))))
        explicit = self.kernel.tuning.get('ZC') or os.environ.get('PSAD_MARCH_ZC') or \
            'BLOCKS' in self.kernel.tuning or os.environ.get('PSAD_MARCH_BLOCKS')
        cus = _torch().cuda.get_device_properties(_torch().cuda.current_device()).multi_processor_count \
            if slots else 0
        # measured on the default WS tiles (one workgroup per CU, or the half-width tiles it picks for
        # x extents that pad less); with user tile / depth overrides that allow several partially filled
        # workgroups per CU it can pick an unbalanced grid (512³ D=3: 0.249 vs 0.188 ms), so those keep
        # the block-count target
        overridden = any(k in self.kernel.tuning for k in ('CX', 'NR', 'D', 'WX', 'NW'))
        # (not for the 2-D row ring, whose block-count target measured faster: 2-D varcoef 4096² fp32 adjoint 0.072 vs
        # 0.085 ms, profiles/r06_nl2d_zy.log)
        rows2d = ir.ndim == 2 and not cfg.ZSUM
        if slots and cfg.WS and nz and not explicit and (slots <= cus or not overridden) and not rows2d:
            ws = ws_geometry(ir, cfg)
            # workgroups that saturate HBM: ~64 KiB in flight per CU (one 256×16 fp32 ring of 4 planes)
            wsat = max(cus, math.ceil(cus * 65536 / (ws['D'] * ws['per_plane'] * 1024)))
            zc = self.quantized_chunk(nz, nt, slots, cfg.ZMIN, cfg.ZMAX, march_geometry(ir, cfg)['RZ'], wsat)
        zc = min(zc, nz) if nz else zc
        zc = max(zc, min(nz, 4 * max(1, march_geometry(ir, cfg)['RZ'])))
        nchunks = math.ceil(nz / zc) if nz else 0
        if nchunks:
            # equal chunks: same chunk count (same halo re-reads), no short tail chunk — 27-point fp16
            # 192×768² slab: 27 → 24 planes, 0.129 → 0.113 ms (profiles/r01_tune_zc_slab.log)
            zc = math.ceil(nz / nchunks)
        return dict(Z=Z, Y=Y, X=X, zlo=zlo, zhi=zhi, ylo=ylo, yhi=yhi, xlo=xlo, xhi=xhi, zc=zc, zstep=zc,
                    ntx=ntx, nty=nty, grid=nt * nchunks)

    def _plan_march(self, tensors, halo_list, shape, device, z_range, x_border=False, z_limits=None,
                    start_signal=False, halo_wait=False):
        torch = _torch()
        ir = self.ir
        ve = self._vec_elems()
        X = shape[-1]
        stencil = ir.stencil_fields
        by_name = {f.name: t for f, t in zip(ir.fields, tensors)}
        esize = 16 // ve

        def fits(v, step=None):
            step = v * esize if step is None else step
            return (step != v * esize or X % v == 0) and \
                all(by_name[f.name].data_ptr() % step == 0 for f in stencil) and \
                all(h.data_ptr() % step == 0 for h in halo_list if h is not None)
        bu = None
        dword_rows = (X * esize) % 4 == 0 and fits(ve, step=4) and all(t.data_ptr() % 4 == 0 for t in tensors)
        half_rows = esize == 2 and X % 2 == 1          # fp16 rows on half dwords: realigned in registers ('bo')
        if not fits(ve) and (dword_rows or half_rows) and not ir.has_index_dims and \
                int(np.prod(shape[1:])) * esize < 2 ** 31 - 1024 and os.environ.get('PSAD_BAND_UNALIGNED', '1') != '0':
            # rows whose pitch is not a multiple of 16 bytes on the row-band schedule: row-wise dword-aligned pieces,
            # a 16-byte row pitch in LDS, the partial last chunk stored as dwords (hip_band, 'bu')
            c = self._march_cfg(ve, shape, band=True)
            bu = c if c.BAND else None
        xm = False
        if bu is None and not fits(ve) and (X * esize) % 4 == 0 and fits(ve, step=4) and not ir.has_index_dims and \
                all(np.dtype(f.dtype.numpy_dtype).itemsize == esize for f in ir.fields) and \
                int(np.prod(shape[1:])) * esize < 2 ** 31 - 1024:       # (the loader's 32-bit offsets, below)
            # rows whose pitch is not a multiple of 16 bytes but of 4 (fp32 / fp64, fp16 with X even): the LDS-DMA
            # ring still takes 16-byte pieces (dword-aligned; the image in LDS keeps its layout) and zero-fills
            # past each row end (XM) — where the WS schedule applies
            probe = self._march_cfg(ve, shape, band=False)
            xm = bool(probe.WS) and probe.ZSUM and ws_geometry(ir, probe) is not None
        xo = False
        if not xm and not fits(ve) and esize == 2 and not ir.has_index_dims and os.environ.get('PSAD_XO', '1') != '0' and \
                all(np.dtype(f.dtype.numpy_dtype).itemsize == 2 for f in ir.fields) and \
                int(np.prod(shape[1:])) * 2 < 2 ** 31 - 1024:
            # fp16 rows starting on half dwords (X odd, or an odd-element base): the half-precision LDS-DMA ring
            # loads such rows one element early and shifts them back in LDS (XO) — 255³ fp16 instead of the
            # register-prefetch path
            probe = self._march_cfg(ve, shape, band=False)
            ws_p = ws_geometry(ir, probe) if probe.WS else None
            xo = ws_p is not None and ws_p['kind'] == 'h'
        if bu is not None:
            cfg = bu
        elif xm or xo:
            cfg = MarchConfig(**{**self._march_cfg(ve, shape, band=False).__dict__, 'XM': True,
                                 'XO': (1 if X % 2 else 2) if xo else 0})
        else:
            # widest plane-load vector the rows allow: 16 bytes (and the LDS-DMA loader) when the row pitch is a
            # multiple of 16 bytes, else 8 / 4 bytes (register-prefetch loads) before scalar ones — X = 262
            # fp32: 8-byte loads instead of 4-byte (profiles/r02_misaligned*.log)
            ve = next(v for v in (ve, ve // 2, ve // 4, 1) if v >= 1 and fits(v))
            if ve == 1 and ir.ndim == 2 and not halo_list and z_range is None and z_limits is None and \
                    not ir.has_index_dims:
                # 2-D rows of scalar loads: the one-thread-per-cell schedule streams them faster (4097² 5-point
                # 0.028 vs 0.046 ms, 4095×4094 0.027 vs 0.043; profiles/r02_misaligned.log)
                return self._plan_generic(tensors, shape, device)
            # the row-band schedule (hip_band): 16-byte pieces and stores on every field and halo, 32-bit plane offsets
            band_ok = ve == self._vec_elems() and all(t.data_ptr() % 16 == 0 for t in tensors) and \
                int(np.prod(shape[1:])) * esize < 2 ** 31 - 1024
            cfg = self._march_cfg(ve, shape, band=band_ok)
        if halo_list and ir.ndim == 2 and cfg.VIEW2D == 'yx':
            cfg = MarchConfig(**{**cfg.__dict__, 'VIEW2D': 'zy'})
        from .hip_emitter import ncomp
        if ir.has_index_dims and not cfg.ZSUM and not (cfg.WS and ws_geometry(ir, cfg)):
            if halo_list or z_range is not None or z_limits is not None:
                raise ValueError('vector-field kernels take halo planes / z ranges only in the zsum schedule')
            return self._plan_generic(tensors, shape, device)
        cmax = max([ncomp(f) for f in stencil] + [1])
        ws = ws_geometry(ir, cfg)
        if ws and int(np.prod(shape[1:])) * cmax * max(ws['esize'], ws.get('ssize', 0)) >= 2 ** 31 - 1024:
            # planes beyond the loader's 32-bit buffer offsets: register-prefetch form of the same schedule
            # (never with XM: its rows straddle, which only the loader's zero fill repairs)
            assert not cfg.XM
            if ir.has_index_dims and not cfg.ZSUM:
                # (the register-prefetch ring takes scalar fields only)
                if halo_list or z_range is not None or z_limits is not None:
                    raise ValueError('vector-field kernels beyond 32-bit plane offsets take no halo planes / z ranges')
                return self._plan_generic(tensors, shape, device)
            cfg = ws_fallback_config(cfg)
        xlo, xhi = ir.iteration_bounds(shape)[-1]
        if x_border and cfg.ZSUM and (xlo > 0 or xhi < shape[-1]) and \
                not (ir.ndim == 2 and cfg.VIEW2D == 'zy'):
            cfg = MarchConfig(**{**cfg.__dict__, 'XB': True})
        if cfg.BAND:
            # unmasked stores when every band row lies in [ylo, yhi) and the x range is whole rows
            g0 = self.march_launch_geometry(shape, cfg, z_range, z_limits=z_limits)
            if not (g0['ylo'] == 0 and g0['yhi'] == g0['nty'] * cfg.BTY and g0['xlo'] == 0 and g0['xhi'] == g0['X']) or \
                    g0['X'] % (16 // esize):                          # a partial last chunk per row
                cfg = MarchConfig(**{**cfg.__dict__, 'BMASK': True,
                                     'BXW': g0['xlo'] == 0 and g0['xhi'] == g0['X'] and not cfg.XB})
        if start_signal:
            cfg = MarchConfig(**{**cfg.__dict__, 'SIG': True})
        if halo_wait:
            if not ((cfg.BAND and not (cfg.BREG and shape[-1] % (16 // esize))) or ws_geometry(ir, cfg)):
                raise ValueError('a halo wait needs an LDS-DMA loader (band or WS schedule)')
            cfg = MarchConfig(**{**cfg.__dict__, 'HWAIT': True})
        variant = ('march', cfg)
        fn = self.function(variant, device)
        ws = ws_geometry(ir, cfg)
        slots = self._resident_slots(fn, ws['block'], device) if ws else None
        geo = self.march_launch_geometry(shape, cfg, z_range, slots=slots, z_limits=z_limits)
        grid = geo['grid'] if geo['yhi'] > geo['ylo'] and geo['xhi'] > geo['xlo'] else 0
        rz = march_geometry(ir, cfg)['RZ']
        plane = geo['Y'] * geo['X']
        for i, f in enumerate(stencil):
            for h in (halo_list[2 * i:2 * i + 2] if halo_list else ()):
                if h is not None and (not isinstance(h, torch.Tensor) or not h.is_contiguous() or
                                      h.numel() < rz * plane * ncomp(f) or h.dtype != by_name[f.name].dtype or
                                      h.device != by_name[f.name].device):
                    raise ValueError(f"halo for '{f.name}' must be a contiguous tensor of >= {rz} planes "
                                     "on the field's device")
        if max(geo['Z'], geo['Y'], geo['X']) >= 2 ** 31 or grid >= 2 ** 31:
            raise ValueError('field extent too large for the march schedule')
        statics = [int(geo[k]) for k in ('Z', 'Y', 'X', 'zlo', 'zhi', 'ylo', 'yhi', 'xlo', 'xhi', 'zc', 'zstep', 'ntx',
                                          'nty')]
        kinds = ['ptr'] * (len(tensors) + 2 * len(stencil)) + ['i32'] * len(statics)
        if cfg.SIG:
            kinds += ['ptr', 'u32']                     # the start signal: word and value, patched by the caller
            statics += [0, 0]
        if cfg.HWAIT:
            kinds += ['ptr', 'u32']                     # the halo wait: word and value, patched by the caller
            statics += [0, 0]
        kinds += [self._scalar_kind()] * len(ir.scalars)
        block = ws['block'] if ws else (band_geometry(cfg.BX, cfg.BTY, cfg.BAND, cfg.D, esize, cfg.BPAD, cfg.BREG, cfg.BFREE)['NT'] if cfg.BAND else
                                        cfg.NT)
        plan = _Plan(variant, fn, grid, kinds, len(tensors), 2 * len(stencil), statics, xb=cfg.XB, block=block)
        i = len(tensors) + 2 * len(stencil) + 13
        if cfg.SIG:
            plan.sig_offsets = (plan.offsets[i], plan.offsets[i + 1])
            i += 2
        if cfg.HWAIT:
            plan.hwait_offsets = (plan.offsets[i], plan.offsets[i + 1])
        return plan


class _Plane:
    """One component plane of an fzyx tensor, as the launch path sees a tensor: pointer, shape, strides,
    dtype, device (and the parent, kept alive for the duration of the call)."""
    __slots__ = ('parent', 'ptr', 'shape', 'strides', 'dtype', 'device', 'is_cuda')

    def __init__(self, parent, ptr, shape, strides):
        self.parent = parent
        self.ptr = ptr
        self.shape = shape
        self.strides = strides
        self.dtype = parent.dtype
        self.device = parent.device
        self.is_cuda = parent.is_cuda

    def data_ptr(self):
        return self.ptr

    def dim(self):
        return len(self.shape)

    def stride(self):
        return self.strides

    def numel(self):
        n = 1
        for v in self.shape:
            n *= v
        return n

    def element_size(self):
        return self.parent.element_size()

    def is_contiguous(self):
        expect = 1
        for n, st in zip(reversed(self.shape), reversed(self.strides)):
            if n != 1 and st != expect:
                return False
            expect *= n
        return True


def _align_class(p):
    """log2 of the largest power of two (≤ 32) dividing the address ``p`` (0 counts as 32-byte aligned)."""
    return min((p & -p).bit_length() - 1, 5) if p else 5


def _is_pair(z_range):
    return len(z_range) == 2 and all(isinstance(r, (tuple, list)) for r in z_range)


def _zkey(z_range):
    if z_range is None:
        return None
    return tuple(tuple(int(v) for v in r) for r in z_range) if _is_pair(z_range) else tuple(int(v) for v in z_range)


class _Plan:
    """A resolved launch: variant, function handle, grid and a struct that packs the argument
    buffer (pointers, then static extents, then scalars) at HIP_LAUNCH_PARAM_BUFFER alignment."""

    _CODES = {'ptr': ('Q', 8), 'i32': ('i', 4), 'u32': ('I', 4), 'i64': ('q', 8), 'f32': ('f', 4), 'f64': ('d', 8)}

    def __init__(self, variant, fn, grid, kinds, n_ptr, n_halo, statics, block=256, xb=False):
        import struct
        self.variant = variant
        self.fn = fn
        self.grid = grid
        self.block = block
        self.xb = xb                     # the launch also zeroes x outside the iteration bounds
        fmt, off = '<', 0
        self.kinds, self.offsets = list(kinds), []       # byte offset of every argument in the packed buffer
        for k in kinds:
            c, size = self._CODES[k]
            pad = (-off) % size
            fmt += 'x' * pad + c
            self.offsets.append(off + pad)
            off += pad + size
        fmt += 'x' * ((-off) % 8)
        self.struct = struct.Struct(fmt)
        self.n_ptr = n_ptr
        self.n_halo = n_halo
        self.statics = list(statics)
        self.sig_offsets = None          # (byte offset of the start-signal word, of its value): SIG launches
        self.hwait_offsets = None        # (byte offset of the halo-wait word, of its value): HWAIT launches

    def scalar_slots(self, n):
        """``(byte offset, is f64)`` of the last ``n`` arguments (the kernel's scalar parameters)."""
        return [(o, k == 'f64') for o, k in zip(self.offsets[len(self.offsets) - n:], self.kinds[len(self.kinds) - n:])] \
            if n else []

    def pack(self, ptrs, hptrs, scalars):
        return self.struct.pack(*ptrs, *(hptrs if hptrs else [0] * self.n_halo), *self.statics, *scalars)


_zero_border_fns = {}


def zero_border(t, bounds, ncomp=1, stream=None, x=True, zy=True):
    """Zero, in one launch on the current stream, every cell of the contiguous GPU tensor ``t`` outside the
    per-axis ``[lo, hi)`` ``bounds`` of its spatial axes (components, if any, last) — the border an
    interior-only kernel leaves to the reference's ``torch.zeros`` allocation. ``x=False`` leaves the x
    ends of the rows (written by an ``x_border`` launch), ``zy=False`` does only those."""
    import struct
    torch = _torch()
    from .hip_emitter import emit_zero_border
    nd = len(bounds)
    shape = [int(s) for s in t.shape[:nd]]
    bounds = [(int(a), int(b)) for a, b in bounds]
    if not x:
        bounds[-1] = (0, shape[-1])
    if not zy:
        bounds[:-1] = [(0, n) for n in shape[:-1]]
    while len(shape) < 3:
        shape.insert(0, 1)
        bounds.insert(0, (0, 1))
    (zlo, zhi), (ylo, yhi), (xlo, xhi) = bounds
    Z, Y, X = shape
    L = X * ncomp
    total = (Z - (zhi - zlo)) * Y * L + (zhi - zlo) * (Y - (yhi - ylo)) * L + \
        (zhi - zlo) * (yhi - ylo) * (L - (xhi - xlo) * ncomp)
    if total <= 0:
        return
    if not t.is_contiguous() or t.numel() != Z * Y * L:
        raise ValueError('zero_border needs a contiguous tensor of the kernel shape')
    device = t.device.index
    idx32 = Z * Y * L + 256 * 256 * 64 < 2 ** 31
    key = (t.element_size(), idx32, device)
    fn = _zero_border_fns.get(key)
    if fn is None:
        src, name = emit_zero_border(t.element_size(), idx32)
        fn = _zero_border_fns[key] = rt.load_function(rt.compile_hip(src), name, device)
    if stream is None:
        stream = torch._C._cuda_getCurrentRawStream(device)
    args = struct.pack('<Q9q', t.data_ptr(), Z, Y, L, zlo, zhi, ylo, yhi, xlo * ncomp, xhi * ncomp)
    rt.launch(fn, (min(math.ceil(total / 256), 256 * 64),), (256,), args, stream)
