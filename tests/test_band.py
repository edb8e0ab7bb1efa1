"""Row-band schedule (``backends/hip_band.py``): fp16 stencils on full-width bands of rows.

CPU part: eligibility (one fp16 stencil field, linear taps, radius 1), the (band height, rows per lane, depth)
choice and that the emitted kernels hiprtc-compile for gfx950. GPU part (``-m gpu``): forward and adjoint vs
the float64 oracle (fp16 tolerance 1e-3·max|ref|, tests/test_gpu_parity.py), ``None`` boundary handling
(interior-only stores, masked variant), ragged band counts, the z-slab launch pattern (halo planes read in place,
two-range face launches) bitwise equal to one full launch, chunk-length independence (bitwise), misaligned views
falling back to the zsum ring, and a two-output kernel."""
import numpy as np
import pytest
import sympy as sp

import pystencils_autodiff_amd as pa
from oracle import evaluate as OE
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from pystencils_autodiff_amd.backends.hip_band import band_choice, band_geometry, band_plans
from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel, default_march_config
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
from tests.conftest import abs_terms, assert_cells, assert_close_rel, n_terms

TOL16 = 1e-3


def _kernel(ac, bh='zeros', name='bandk', **tun):
    return StencilKernel(ac, boundary_handling=bh, function_name=name, target='gpu', gpu_indexing_params=tun)


def test_band_eligibility():
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    for ac in (op.forward_assignments, op.backward_assignments):
        plans = band_plans(HipStencilKernel(_kernel(ac)).ir)
        assert plans is not None and len(plans) == 1 and len(plans[0]['w']) == 27
    star = pa.AutoDiffOp(W.diffusion_7pt(dtype='float16'), boundary_handling='zeros')
    assert len(band_plans(HipStencilKernel(_kernel(star.forward_assignments)).ir)[0]['w']) == 7
    # fp32 storage fits (opt-in, BAND=R); fp64, a second field read pointwise, radius 2: not the band schedule
    f32 = pa.AutoDiffOp(W.stencil_27pt(dtype='float32'), boundary_handling='zeros')
    ir32 = HipStencilKernel(_kernel(f32.forward_assignments)).ir
    assert band_plans(ir32) is not None
    assert default_march_config(ir32, 4, (768, 768, 768)).BAND == 0           # measured slower: opt-in
    assert default_march_config(ir32, 4, (768, 768, 768), {'BAND': 4}).BAND == 4
    f64 = pa.AutoDiffOp(W.stencil_27pt(dtype='float64'), boundary_handling='zeros')
    assert band_plans(HipStencilKernel(_kernel(f64.forward_assignments)).ir) is None
    u, v, out = ps.fields('u, v, out: float16[3d]')
    two = ps.AssignmentCollection({out.center: u[1, 0, 0] + u[-1, 0, 0] * v.center})
    assert band_plans(HipStencilKernel(_kernel(two)).ir) is None
    wide = ps.AssignmentCollection({out.center: u[2, 0, 0] + u.center})
    assert band_plans(HipStencilKernel(_kernel(wide)).ir) is None


def test_band_choice_and_geometry():
    # rows of >= 96 chunks: 16-row bands of 2 rows per lane (one workgroup per CU; star stencils 1 plane in flight)
    assert band_choice(768) == (16, 2, 2) and band_choice(768, star=True) == (16, 2, 1)
    assert band_choice(768, wide16=False) == (8, 4, 2)
    assert band_choice(1024) == (8, 4, 2) and band_choice(768, 2)[1] == 2 and band_choice(512) == (8, 4, 2)
    assert band_choice(264) is None and band_choice(100) is None and band_choice(96) is None
    for X in (256, 512, 768, 1024, 640, 2048):
        c = band_choice(X)
        if c is None:
            continue
        TY, R, D = c
        g = band_geometry(X, TY, R, D)
        assert g['ntask'] % 64 == 0 and g['NCT'] <= 960 and D * g['NI'] <= 63
        assert g['lds_bytes'] <= (160 if (TY, R) == (16, 2) else 80) * 1024


@pytest.mark.parametrize('shape,expect,zc', [((768, 768, 768), 2, 48), ((1024, 1024, 1024), 4, 32),
                                             ((96, 768, 768), 4, 12), ((512, 512, 512), 4, 32), ((256, 256, 256), 4, 8),
                                             ((255, 255, 255), 4, 8), ((64, 256, 256), 0, 0), ((40, 40, 264), 0, 0),
                                             ((512, 1024, 1024), 4, 48)])
def test_band_default_selection(shape, expect, zc):
    """Box stencils: the band schedule with the longest chunk of the ladder that still fills one round of three
    workgroups per CU (BAND_ROUND_WG), both chunk ends peeled at that compile-time length (BTRIM=3)."""
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    cfg = default_march_config(HipStencilKernel(_kernel(op.forward_assignments)).ir, 8, shape)
    assert cfg.BAND == expect, cfg
    if expect:
        assert cfg.ZMIN == cfg.ZMAX == zc and cfg.BTRIM == 3, cfg
    # overrides of the zsum tile (or BAND=0) keep the zsum schedule
    cfg = default_march_config(HipStencilKernel(_kernel(op.forward_assignments)).ir, 8, shape, {'BAND': 0})
    assert cfg.BAND == 0


@pytest.mark.parametrize('shape,zc', [((512, 512, 512), 64), ((510, 510, 510), 64), ((511, 511, 511), 64),
                                      ((768, 768, 768), 8),
                                      ((1024, 1024, 1024), 8), ((256, 256, 256), 8)])
def test_band_default_selection_star(shape, zc):
    """fp16 7-point: 8-plane chunks, 64-plane ones on rows of <= 512 elements (>= 512 workgroups)."""
    op = pa.AutoDiffOp(W.diffusion_7pt(dtype='float16'), boundary_handling='zeros')
    cfg = default_march_config(HipStencilKernel(_kernel(op.forward_assignments)).ir, 8, shape)
    wide = shape[-1] == 768           # 16-row bands of 2 rows per lane, one plane in flight
    assert (cfg.BTY, cfg.BAND, cfg.D) == ((16, 2, 1) if wide else (8, 4, 2)), cfg
    assert cfg.ZMIN == cfg.ZMAX == zc and cfg.BPAD == 0, cfg
    assert cfg.BREG == shape[-1] % 2, cfg                      # odd rows: the register-staged padded image


@pytest.mark.parametrize('shape,band', [((512, 512, 512), True), ((768, 768, 768), False), ((1024, 1024, 1024), False),
                                        ((128, 1024, 1024), False)])
def test_band_default_selection_fp32_star(shape, band):
    """fp32 7-point: 8-row bands of 4 rows per lane, 16-plane chunks, on rows of <= 512 elements; zsum beyond."""
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    cfg = default_march_config(HipStencilKernel(_kernel(op.forward_assignments)).ir, 4, shape)
    assert (cfg.BAND > 0) == band, cfg
    if band:
        assert (cfg.BTY, cfg.BAND, cfg.D, cfg.ZMIN) == (8, 4, 2, 16), cfg


@pytest.mark.parametrize('builder,ve,shape,expect', [
    (W.stencil_27pt, 8, (512, 512, 520), (16, 2, 2)), (W.stencil_27pt, 8, (512, 512, 760), (16, 2, 2)),
    (W.stencil_27pt, 8, (512, 512, 1000), (16, 4, 1)), (lambda: W.diffusion_7pt(dtype='float16'), 8, (512, 512, 504),
                                                        (16, 2, 2)),
    (W.diffusion_7pt, 4, (512, 512, 520), (8, 2, 2)), (W.diffusion_7pt, 4, (512, 512, 1000), (4, 4, 2))])
def test_band_default_selection_idle_lanes(builder, ve, shape, expect):
    """Rows with no band height of whole compute waves take a band whose last compute wave holds idle lanes (not the
    zsum schedule), chunk lengths from the ladder (>= 768 workgroups), not the 16-row rule's 32 planes."""
    from pystencils_autodiff_amd.backends.hip_band import band_choice
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    ir = HipStencilKernel(_kernel(op.forward_assignments)).ir
    es = 16 // ve
    assert band_choice(shape[-1], 1, es) is None and band_choice(shape[-1], 1, es, idle=True) == expect
    cfg = default_march_config(ir, ve, shape)
    assert (cfg.BTY, cfg.BAND, cfg.D) == expect, cfg
    g = band_geometry(shape[-1], cfg.BTY, cfg.BAND, cfg.D, es, cfg.BPAD, cfg.BREG)
    assert g['ntask'] % 64 != 0 and g['NCT'] <= 960, g
    assert -(-shape[1] // cfg.BTY) * -(-shape[0] // cfg.ZMIN) >= 512, cfg


@pytest.mark.parametrize('builder,shape,expect', [
    (W.stencil_27pt, (512, 512, 576), (16, 2, 2, 16)), (W.stencil_27pt, (512, 512, 640), (16, 2, 2, 16)),
    (W.stencil_27pt, (512, 512, 320), (16, 2, 2, 16)), (W.stencil_27pt, (512, 512, 896), (8, 2, 3, 32)),
    (W.stencil_27pt, (1024, 1024, 1024), (16, 4, 1, 32)),
    (lambda: W.diffusion_7pt(dtype='float16'), (512, 512, 640), (16, 2, 2, 8))])
def test_band_default_selection_16_row_bands(builder, shape, expect):
    """fp16 rows whose whole-wave choices are 16-row bands of 2 rows per lane (ahead of 3 planes in flight), with
    ladder chunks — the 32-plane chunks stay with the 1024-wide box rule (16 rows, 4 per lane, one plane in flight)."""
    op = pa.AutoDiffOp(builder(), boundary_handling='zeros')
    cfg = default_march_config(HipStencilKernel(_kernel(op.forward_assignments)).ir, 8, shape)
    assert (cfg.BTY, cfg.BAND, cfg.D, cfg.ZMIN) == expect, cfg


def test_probe_knobs_are_not_tile_keys(monkeypatch):
    """Ablation knobs that give wrong results (``BABL``) and the removed probe knobs are rejected as tile parameters,
    through ``gpu_indexing_params`` and ``PSAD_MARCH`` alike; only ``hip_kernel.PROBE_KNOBS`` (set by probe scripts,
    never by the op) reaches the planner."""
    from pystencils_autodiff_amd.backends import hip_kernel as HK
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    ir = HipStencilKernel(_kernel(op.forward_assignments)).ir
    for key in ('BABL', 'BSHIFT', 'BDEAD', 'BPE', 'BSI', 'BPRIO', 'BLAUX', 'BSTAG', 'BWPE', 'BLDR', 'BMBR', 'BTB',
                'BFM', 'BLW'):
        with pytest.raises(ValueError, match='unknown tile parameter'):
            default_march_config(ir, 8, (768, 768, 768), {key: 1})
        with pytest.raises(ValueError, match='unknown tile parameter'):        # the kernel's gpu_indexing_params
            HipStencilKernel(_kernel(op.forward_assignments, **{key: 1}))._march_cfg(8, (768, 768, 768))
        monkeypatch.setenv('PSAD_MARCH', f'{key}=1')
        with pytest.raises(ValueError, match='unknown tile parameter'):
            default_march_config(ir, 8, (768, 768, 768))
        monkeypatch.delenv('PSAD_MARCH')
    assert default_march_config(ir, 8, (768, 768, 768)).BABL == 0
    monkeypatch.setitem(HK.PROBE_KNOBS, 'BABL', 2)
    assert default_march_config(ir, 8, (768, 768, 768)).BABL == 2


def test_band_sources_compile():
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    from pystencils_autodiff_amd.backends.hip_emitter import MarchConfig
    for ac in (pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros').backward_assignments,
               pa.AutoDiffOp(W.diffusion_7pt(dtype='float16'), boundary_handling='zeros').forward_assignments):
        hk = HipStencilKernel(_kernel(ac))
        cfg = default_march_config(hk.ir, 8, (32, 64, 256), {'BAND': 4})
        for c in (cfg, MarchConfig(**{**cfg.__dict__, 'BMASK': True}),
                  MarchConfig(**{**cfg.__dict__, 'BMASK': True, 'XB': True}),
                  MarchConfig(**{**cfg.__dict__, 'BTRIM': 1}), MarchConfig(**{**cfg.__dict__, 'BTRIM': 2}),
                  MarchConfig(**{**cfg.__dict__, 'BTRIM': 3, 'ZMIN': 16, 'ZMAX': 16}),
                  MarchConfig(**{**cfg.__dict__, 'BPAD': 1}), MarchConfig(**{**cfg.__dict__, 'BPAD': 1, 'BMASK': True}),
                  # the store cache-policy probe
                  MarchConfig(**{**cfg.__dict__, 'BMASK': True, 'BXW': True, 'BNT': 0}),
                  # the LDS handshake instead of plane barriers
                  MarchConfig(**{**cfg.__dict__, 'BFREE': 1}), MarchConfig(**{**cfg.__dict__, 'BFREE': 2, 'BMASK': True}),
                  MarchConfig(**{**cfg.__dict__, 'BFREE': 3, 'BTRIM': 3, 'ZMIN': 16, 'ZMAX': 16, 'BMASK': True})):
            src, kname = hk.source(('march', c))
            assert kname.endswith('_band') and 'band schedule' in src
            assert len(rt.compile_hip(src)) > 0


# ---------------------------------------------------------------------------------------------------------- GPU
def _torch():
    return pytest.importorskip('torch')


CASES = [('27pt', W.stencil_27pt), ('7pt_f16', lambda: W.diffusion_7pt(dtype='float16')),
         ('asym_f16', lambda: W.asym_7pt(dtype='float16')), ('asym_f32', W.asym_7pt),
         ('27pt_f32', lambda: W.stencil_27pt(dtype='float32'))]


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES, ids=lambda c: c[0])
@pytest.mark.parametrize('shape', [(11, 24, 256), (9, 21, 256), (7, 16, 768), (5, 12, 1024)])
@pytest.mark.parametrize('bh', ['zeros', None])
def test_band_vs_oracle(case, shape, bh):
    """Forward and adjoint sweeps on the band schedule vs the float64 oracle; Y not a multiple of the band height
    (ragged last band) and interior-only stores take the masked variant; rows whose pitch is not a multiple of 16
    bytes (``test_band_unaligned_vs_oracle``) load row-wise pieces and store a partial last chunk."""
    _band_vs_oracle(case, shape, bh)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES, ids=lambda c: c[0])
@pytest.mark.parametrize('shape', [(9, 21, 256), (7, 16, 768)])
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('knob', [{'BPAD': 1}, {'BPAD': 0}, {'BPAD': 1, 'BFREE': 1}, {'BPAD': 0, 'BFREE': 2},
                                  {'BPAD': 1, 'BFREE': 3}],
                         ids=['pad', 'dpp', 'pad-handshake', 'dpp-handshake4', 'pad-handshake5'])
def test_band_padded_rows_vs_oracle(case, shape, bh, knob):
    """Zero-padded LDS image rows (``BPAD=1``: row ends meet the zero pads, the x-edge dwords read from LDS) and the
    unpadded image (``BPAD=0``: wave-wide DPP plus boundary selects) vs the oracle, forward and adjoint, whole and
    masked stores; the same with the per-plane LDS handshake instead of the plane barriers (``BFREE``, deeper rings
    at 2 and 3)."""
    _band_vs_oracle(case, shape, bh, **knob)


def _band_vs_oracle(case, shape, bh, **extra):
    torch = _torch()
    op = pa.AutoDiffOp(case[1](), boundary_handling=bh)
    rng = np.random.default_rng(sum(shape))
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k0 = _kernel(ac, bh, f'band_{which}')
        dt = np.dtype(k0.ir.fields[0].dtype.numpy_dtype)
        choice = band_choice(shape[-1], 1, dt.itemsize) or band_choice(shape[-1], 1, dt.itemsize, idle=True)
        if choice is None:
            pytest.skip(f'no band geometry for rows of {shape[-1]} {dt}')
        k = _kernel(ac, bh, f'band_{which}', BAND=choice[1], **extra).compile()
        ins = {f.name: rng.uniform(-1, 1, shape).astype(dt) for f in k.ir.fields_read}
        ref = OE.evaluate(ac, {n: a.astype(np.float64) for n, a in ins.items()}, boundary_handling=bh)
        outs = {f.name: torch.zeros(shape, dtype=getattr(torch, dt.name), device='cuda') for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        cfg = k.last_variant[1]
        assert k.last_variant[0] == 'march' and cfg.BAND > 0, cfg
        assert all(getattr(cfg, key) == val for key, val in extra.items()), cfg
        whole = bh == 'zeros' and shape[1] % cfg.BTY == 0 and shape[2] % (16 // dt.itemsize) == 0
        assert cfg.BMASK == (not whole), cfg
        assert cfg.BXW == (cfg.BMASK and bh == 'zeros'), cfg          # x range = whole rows: no read-modify-write
        absr = abs_terms(ac, ins, bh)
        for n, t in outs.items():
            assert_close_rel(t.double().cpu().numpy(), ref[n], TOL16 if dt.itemsize == 2 else 1e-6,
                             f'{case[0]} {which} {n} {shape} {bh}')
            assert_cells(t.double().cpu().numpy(), ref[n], absr[n], n_terms(ac), dt, f'{case[0]} {which} {n} {shape} {bh}')


# rows whose chunk count has no band height of whole compute waves: the last compute wave holds idle lanes
IDLE = [('27pt', (9, 32, 520)), ('27pt', (7, 21, 504)), ('7pt_f16', (6, 16, 520)), ('asym_f16', (5, 19, 1000)),
        ('asym_f32', (6, 16, 520)), ('27pt_f32', (5, 11, 504)), ('27pt', (5, 16, 760))]


@pytest.mark.gpu
@pytest.mark.parametrize('case_shape', IDLE, ids=lambda c: f'{c[0]}-{c[1][2]}')
@pytest.mark.parametrize('bh', ['zeros', None])
def test_band_idle_lanes_vs_oracle(case_shape, bh):
    """Band geometries whose last compute wave holds idle lanes (rows of 63 / 65 / 95 / 125 chunks), forward and
    adjoint vs the oracle, whole and masked stores."""
    name, shape = case_shape
    test_band_vs_oracle(next(c for c in CASES if c[0] == name), shape, bh)


UNALIGNED = [('27pt', (7, 16, 766)), ('7pt_f16', (6, 13, 510)), ('27pt', (5, 9, 762)), ('asym_f16', (4, 8, 254)),
             ('27pt_f32', (5, 8, 765)), ('27pt', (6, 12, 767)), ('7pt_f16', (5, 9, 511)), ('27pt', (7, 8, 255)),
             ('27pt', (19, 9, 510)), ('7pt_f16', (21, 8, 511))]          # several z chunks


@pytest.mark.gpu
@pytest.mark.parametrize('case_shape', UNALIGNED, ids=lambda c: f'{c[0]}-{c[1][2]}')
@pytest.mark.parametrize('bh', ['zeros', None])
def test_band_unaligned_vs_oracle(case_shape, bh):
    """Rows whose pitch is not a multiple of 16 bytes on the band schedule: even fp16 rows (766, 510, 762, 254) and
    fp32 rows (765) load row-wise dword-aligned pieces and store a partial last chunk; fp16 rows on half dwords (767,
    511, 255) are loaded from the dword below and realigned in registers. Forward and adjoint vs the oracle."""
    name, shape = case_shape
    test_band_vs_oracle(next(c for c in CASES if c[0] == name), shape, bh)


@pytest.mark.gpu
@pytest.mark.parametrize('case_shape', UNALIGNED, ids=lambda c: f'{c[0]}-{c[1][2]}')
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('knob', [{'BZF': 0}, {'BREG': 1}, {'BFREE': 2}, {'BTAIL': 0}],
                         ids=['BZF0', 'BREG1', 'BFREE2', 'BTAIL0'])
def test_band_unaligned_variants_vs_oracle(case_shape, bh, knob):
    """Unaligned rows, forward and adjoint vs the oracle: ``BZF=0`` (no loader zero fill past each row end; the
    compute lanes of a row's last chunk zero its first element past X in registers) and ``BREG=1`` (a padded image
    filled through registers: row pieces read at the dword at or below them, realigned by v_alignbyte, cells past X
    zeroed, written with ds_write_b128)."""
    name, shape = case_shape
    _band_vs_oracle(next(c for c in CASES if c[0] == name), shape, bh, **knob)


@pytest.mark.gpu
@pytest.mark.parametrize('bh', ['zeros', None])
def test_band_zslab_launch_pattern_bitwise(bh):
    """z-slab sweep launches (interior z range, then both faces in one two-range launch reading the halo planes in
    place) == one full-domain launch, bitwise, on the band schedule."""
    torch = _torch()
    from pystencils_autodiff_amd.zslab import ZSlabOp
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling=bh)
    k = _kernel(op.forward_assignments, bh, 'bandz', BAND=4).compile()
    g = torch.Generator().manual_seed(3)
    Z = 30
    u = (torch.rand((Z, 40, 256), generator=g) * 2 - 1).half().cuda()
    full = torch.zeros_like(u)
    k(u=u, out=full)
    assert k.last_variant[1].BAND > 0
    kz = None if bh == 'zeros' else (1, Z - 1)
    outs = []
    for a, b in [(0, 11), (11, 19), (19, Z)]:
        sl = u[a:b].contiguous()
        out = torch.zeros_like(sl)
        lo = u[a - 1:a].contiguous() if a > 0 else None
        hi = u[b:b + 1].contiguous() if b < Z else None
        zl = None if kz is None else (max(0, kz[0] - a), min(b - a, kz[1] - a))
        inner, faces = ZSlabOp._launches(b - a, 1, zl or (0, b - a))
        if inner:
            k(u=sl, out=out, z_range=inner, z_limits=zl)
        ZSlabOp._launch_faces(k, {'u': (lo, hi)}, faces, zl, {'u': sl, 'out': out})
        assert k.last_variant[1].BAND > 0
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs), full)
    ref = OE.evaluate(op.forward_assignments, {'u': u.double().cpu().numpy()}, boundary_handling=bh)['out']
    assert_close_rel(full.double().cpu().numpy(), ref, TOL16)
    assert_cells(full.double().cpu().numpy(), ref, abs_terms(op.forward_assignments, {'u': u.double().cpu().numpy()},
                                                              bh)['out'], 27, np.float16, 'slab launches')


@pytest.mark.gpu
def test_band_chunk_length_and_band_height_bitwise():
    """Every output plane sees the same FMA sequence whatever the chunk length, band height (idle lanes on a 12-row
    band) or trimmed chunk-edge planes: results bitwise equal WITHIN each image layout. The layouts (padded image rows
    with the edge dwords from LDS, ``BPAD=1``; DPP across the whole wave with boundary selects, ``BPAD=0``) compile to
    different FMA contractions and differ by one fp16 ulp in ~3e-5 of the cells (DESIGN.md §4 band (7)): each
    layout's reference is checked element-wise against the oracle instead."""
    torch = _torch()
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    g = torch.Generator().manual_seed(11)
    u = (torch.rand((37, 48, 768), generator=g) * 2 - 1).half().cuda()
    common = ({}, {'ZMIN': 5, 'ZMAX': 5}, {'ZMIN': 16, 'ZMAX': 16}, {'ZMIN': 9, 'ZMAX': 9},
              {'BTY': 12},                      # 3 row groups x 96 chunks = 288 tasks on 320 lanes (idle lanes)
              # peeled chunk-edge planes (taps of outputs outside the chunk skipped): the same FMAs per stored cell
              {'BTRIM': 1}, {'BTRIM': 1, 'ZMIN': 1, 'ZMAX': 1}, {'BTRIM': 1, 'ZMIN': 16, 'ZMAX': 16},
              {'BTRIM': 2, 'ZMIN': 9, 'ZMAX': 9},
              {'BTRIM': 2, 'ZMIN': 2, 'ZMAX': 2},               # chunks of < 3 planes: the untrimmed loop
              # both chunk ends peeled with a compile-time chunk length (ragged chunks: the BTRIM=1 path)
              {'BTRIM': 3, 'ZMIN': 13, 'ZMAX': 13}, {'BTRIM': 3, 'ZMIN': 37, 'ZMAX': 37}, {'BTRIM': 3, 'ZMIN': 3, 'ZMAX': 3},
              # the LDS handshake instead of plane barriers: synchronisation only, the same FMAs
              {'BFREE': 1}, {'BFREE': 2, 'BTRIM': 3, 'ZMIN': 13, 'ZMAX': 13}, {'BFREE': 3, 'ZMIN': 5, 'ZMAX': 5},
              {'BFREE': 2, 'BTY': 12}, {'BFREE': 1, 'BTRIM': 1, 'ZMIN': 16, 'ZMAX': 16})
    layouts = {'BPAD=1': [{'BAND': 4, 'BPAD': 1, **t} for t in common],
               'BPAD=0': [{'BAND': 4, 'BPAD': 0, **t} for t in common]}
    ref64 = OE.evaluate(op.forward_assignments, {'u': u.double().cpu().numpy()}, boundary_handling='zeros')['out']
    absr = abs_terms(op.forward_assignments, {'u': u.double().cpu().numpy()}, 'zeros')['out']
    bad = []
    for layout, variants in layouts.items():
        res = []
        for tun in variants:
            k = _kernel(op.forward_assignments, 'zeros', 'bandc', **tun).compile()
            out = torch.full_like(u, float('nan'))
            k(u=u, out=out)
            cfg = k.last_variant[1]
            assert cfg.BAND == 4 and cfg.BPAD == tun['BPAD'], cfg
            res.append((tun, cfg, out))
        torch.cuda.synchronize()
        assert_cells(res[0][2].double().cpu().numpy(), ref64, absr, 27, np.float16, f'{layout} reference')
        for tun, cfg, r in res[1:]:
            if not torch.equal(r, res[0][2]):
                diff = (r.float() - res[0][2].float()).abs()
                where = torch.nonzero(diff > 0)[:6].tolist()
                bad.append(f'{layout} {tun}: {int((diff > 0).sum())} cells differ (max {float(diff.max()):.3g}, first '
                           f'(z, y, x) {where}), BTRIM={cfg.BTRIM} ZMIN={cfg.ZMIN}')
    assert not bad, '\n'.join(bad)


@pytest.mark.gpu
def test_band_misaligned_views_fall_back():
    """A field view whose base is not 16-byte aligned cannot take the band schedule's 16-byte pieces: the zsum
    half ring (XO rows) runs instead; the same kernel object on an aligned view takes the band schedule again."""
    torch = _torch()
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    k = _kernel(op.forward_assignments, 'zeros', 'bandm', BAND=4).compile()
    shape = (6, 16, 256)
    base = (torch.rand(int(np.prod(shape)) + 8) * 2 - 1).half().cuda()
    for off, band in ((1, False), (8, True)):
        u = base[off:off + int(np.prod(shape))].view(shape)
        out = torch.zeros(shape, dtype=torch.float16, device='cuda')
        k(u=u, out=out)
        torch.cuda.synchronize()
        assert (k.last_variant[1].BAND > 0) == band, k.last_variant
        ref = OE.evaluate(op.forward_assignments, {'u': u.double().cpu().numpy()}, boundary_handling='zeros')['out']
        assert_close_rel(out.double().cpu().numpy(), ref, TOL16, f'offset {off}')
        assert_cells(out.double().cpu().numpy(), ref, abs_terms(op.forward_assignments, {'u': u.double().cpu().numpy()})[
            'out'], 27, np.float16, f'offset {off}')


@pytest.mark.gpu
def test_band_two_outputs():
    """Two outputs from one stencil field (two z-partial-sum accumulator sets per cell, 2 rows per lane)."""
    torch = _torch()
    u, a, b = ps.fields('u, a, b: float16[3d]')
    ac = ps.AssignmentCollection({a.center: u[1, 0, 0] - 2 * u.center + u[0, -1, 1],
                                  b.center: sp.Float(0.25) * (u[0, 0, 1] + u[-1, 1, 0] + u[1, 1, 1])})
    k = _kernel(ac, 'zeros', 'band2', BAND=2).compile()
    shape = (10, 24, 256)
    x = np.random.default_rng(2).uniform(-1, 1, shape).astype(np.float16)
    outs = {n: torch.zeros(shape, dtype=torch.float16, device='cuda') for n in ('a', 'b')}
    k(u=torch.from_numpy(x).cuda(), **outs)
    torch.cuda.synchronize()
    assert k.last_variant[1].BAND == 2, k.last_variant
    ref = OE.evaluate(ac, {'u': x.astype(np.float64)}, boundary_handling='zeros')
    absr = abs_terms(ac, {'u': x.astype(np.float64)})
    for n in ('a', 'b'):
        assert_close_rel(outs[n].double().cpu().numpy(), ref[n], TOL16, n)
        assert_cells(outs[n].double().cpu().numpy(), ref[n], absr[n], n_terms(ac), np.float16, n)


@pytest.mark.gpu
@pytest.mark.parametrize('bh', ['zeros', None])
def test_band_through_the_op(bh, monkeypatch, shape=(12, 24, 256)):
    """The drop-in op (``create_tensorflow_op(backend='torch_native')``) on the band schedule (forced with
    ``PSAD_MARCH=BAND=4``): forward and adjoint vs the oracle; with ``None`` the op asks the kernel for the x ends of
    its rows (x_border, zeros) — the band kernel stores them as part of whole rows."""
    torch = _torch()
    monkeypatch.setenv('PSAD_MARCH', 'BAND=4')
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(7)
    u = rng.uniform(-1, 1, shape).astype(np.float16)
    d = rng.uniform(-1, 1, shape).astype(np.float16)
    ut = torch.from_numpy(u).cuda().requires_grad_(True)
    (out,) = fn.apply(ut)
    out.backward(torch.from_numpy(d).cuda())
    torch.cuda.synchronize()
    assert op.forward_ast_gpu.compile().last_variant[1].BAND == 4
    ref = OE.evaluate(op.forward_assignments, {'u': u.astype(np.float64)}, boundary_handling=bh)['out']
    assert_close_rel(out.detach().double().cpu().numpy(), ref, TOL16, 'forward')
    assert_cells(out.detach().double().cpu().numpy(), ref, abs_terms(op.forward_assignments, {'u': u}, bh)['out'], 27,
                 np.float16, 'forward')
    refb = OE.evaluate(op.backward_assignments, {'diffout': d.astype(np.float64)}, boundary_handling=bh)
    (gname,) = refb.keys()
    assert_close_rel(ut.grad.double().cpu().numpy(), refb[gname], TOL16, 'adjoint')
    assert_cells(ut.grad.double().cpu().numpy(), refb[gname], abs_terms(op.backward_assignments, {'diffout': d}, bh)[
        gname], 27, np.float16, 'adjoint')


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(6, 32, 1024), (5, 40, 1024)])
def test_band_16_row_bands_1024(shape):
    """The 1024-wide box-stencil geometry (16-row bands, 8 compute waves, one plane in flight) vs the oracle;
    Y = 40 leaves a ragged last band (masked stores)."""
    torch = _torch()
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    rng = np.random.default_rng(shape[1])
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = _kernel(ac, 'zeros', f'band16_{which}', BAND=4, BTY=16, D=1).compile()
        ins = {f.name: rng.uniform(-1, 1, shape).astype(np.float16) for f in k.ir.fields_read}
        ref = OE.evaluate(ac, {n: a.astype(np.float64) for n, a in ins.items()}, boundary_handling='zeros')
        outs = {f.name: torch.zeros(shape, dtype=torch.float16, device='cuda') for f in k.ir.fields_written}
        k(**{n: torch.from_numpy(a).cuda() for n, a in ins.items()}, **outs)
        torch.cuda.synchronize()
        cfg = k.last_variant[1]
        assert (cfg.BAND, cfg.BTY, cfg.D, cfg.BMASK) == (4, 16, 1, shape[1] % 16 != 0), cfg
        absr = abs_terms(ac, ins)
        for n, t in outs.items():
            assert_close_rel(t.double().cpu().numpy(), ref[n], TOL16, f'{which} {n} {shape}')
            assert_cells(t.double().cpu().numpy(), ref[n], absr[n], n_terms(ac), np.float16, f'{which} {n} {shape}')


@pytest.mark.gpu
def test_band_scalar_coefficient():
    """Tap weights that are kernel parameters (a sympy symbol, passed at launch) on the band schedule."""
    torch = _torch()
    u, out = ps.fields('u, out: float16[3d]')
    a = sp.Symbol('alpha')
    ac = ps.AssignmentCollection({out.center: u.center + a * (u[1, 0, 0] + u[-1, 0, 0] + u[0, 1, 0] + u[0, -1, 0] +
                                                              u[0, 0, 1] + u[0, 0, -1] - 6 * u.center)})
    k = _kernel(ac, 'zeros', 'bands', BAND=4).compile()
    shape = (9, 16, 256)
    x = np.random.default_rng(5).uniform(-1, 1, shape).astype(np.float16)
    res = torch.zeros(shape, dtype=torch.float16, device='cuda')
    k(u=torch.from_numpy(x).cuda(), out=res, alpha=0.15)
    torch.cuda.synchronize()
    assert k.last_variant[1].BAND == 4
    xs = x.astype(np.float64)
    acv = ps.AssignmentCollection({out.center: ac.main_assignments[0].rhs.subs(a, 0.15)})
    ref = OE.evaluate(acv, {'u': xs}, boundary_handling='zeros')['out']
    assert_close_rel(res.double().cpu().numpy(), ref, TOL16)
    assert_cells(res.double().cpu().numpy(), ref, abs_terms(acv, {'u': xs})['out'], n_terms(acv), np.float16)


@pytest.mark.gpu
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('shape', [(12, 23, 766), (10, 16, 510)])
def test_band_unaligned_rows_through_the_op(bh, shape, monkeypatch):
    """Rows whose pitch is not a multiple of 16 bytes through the drop-in op on the band schedule (the default for
    them): forward and adjoint vs the oracle, element-wise."""
    torch = _torch()
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling=bh)
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    rng = np.random.default_rng(17)
    u = rng.uniform(-1, 1, shape).astype(np.float16)
    d = rng.uniform(-1, 1, shape).astype(np.float16)
    monkeypatch.setenv('PSAD_MARCH', 'BAND=4')          # small domains: force the band schedule (BAND_MIN_WG)
    ut = torch.from_numpy(u).cuda().requires_grad_(True)
    (out,) = fn.apply(ut)
    out.backward(torch.from_numpy(d).cuda())
    torch.cuda.synchronize()
    cfg = op.forward_ast_gpu.compile().last_variant[1]
    assert cfg.BAND == 4 and cfg.BX == shape[2], cfg
    ref = OE.evaluate(op.forward_assignments, {'u': u.astype(np.float64)}, boundary_handling=bh)['out']
    refb = OE.evaluate(op.backward_assignments, {'diffout': d.astype(np.float64)}, boundary_handling=bh)
    (gname,) = refb.keys()
    assert_cells(out.detach().double().cpu().numpy(), ref, abs_terms(op.forward_assignments, {'u': u}, bh)['out'], 27,
                 np.float16, 'forward')
    assert_cells(ut.grad.double().cpu().numpy(), refb[gname],
                 abs_terms(op.backward_assignments, {'diffout': d}, bh)[gname], 27, np.float16, 'adjoint')


@pytest.mark.gpu
@pytest.mark.parametrize('off', [0, 1, 3])
@pytest.mark.parametrize('shape', [(5, 9, 511), (6, 11, 767)])
def test_band_half_dword_rows_any_base(shape, off):
    """fp16 rows of odd length on the band schedule from views whose first element sits on any half dword: the plane
    parity (the plane pointer's bit 1) and the row's own parity pick the realignment per row and plane; vs the oracle,
    element-wise, forward and adjoint."""
    torch = _torch()
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    n = int(np.prod(shape))
    rng = np.random.default_rng(off + shape[2])
    for which, ac in (('f', op.forward_assignments), ('b', op.backward_assignments)):
        k = _kernel(ac, 'zeros', f'bandodd_{which}', BAND=4).compile()
        (fin,) = [f.name for f in k.ir.fields_read]
        (fout,) = [f.name for f in k.ir.fields_written]
        base = torch.from_numpy(rng.uniform(-1, 1, n + 8).astype(np.float16)).cuda()
        u = base[off:off + n].view(shape)
        out = torch.zeros(shape, dtype=torch.float16, device='cuda')
        k(**{fin: u, fout: out})
        torch.cuda.synchronize()
        cfg = k.last_variant[1]
        assert cfg.BAND == 4 and cfg.BX == shape[2], cfg
        un = u.cpu().numpy()
        ref = OE.evaluate(ac, {fin: un.astype(np.float64)}, boundary_handling='zeros')[fout]
        assert_cells(out.double().cpu().numpy(), ref, abs_terms(ac, {fin: un}, 'zeros')[fout], 27, np.float16,
                     f'{which} offset {off}')
