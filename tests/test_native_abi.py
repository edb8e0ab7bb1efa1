"""The C-ABI library and the HIP emitter without a GPU.

* libpsad_hip.so loads and exports every symbol ``include/psad.h`` declares;
* every schedule's emitted source compiles for gfx950 through the library's
  hiprtc entry point (hiprtc needs no GPU), and the code object is an AMDGPU ELF;
* the launch-argument packing matches HIP_LAUNCH_PARAM_BUFFER alignment.
"""
import os
import re
import struct

import pytest

import pystencils_autodiff_amd as pa
from pystencils_autodiff_amd import ps
from pystencils_autodiff_amd import workloads as W
from pystencils_autodiff_amd.backends import hip_runtime as rt
from pystencils_autodiff_amd.backends.hip_emitter import MarchConfig

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


@pytest.fixture(scope='module', autouse=True)
def built():
    from pystencils_autodiff_amd.build import build
    build()


def test_library_exports_header_symbols():
    header = open(os.path.join(ROOT, 'include', 'psad.h')).read()
    declared = set(re.findall(r'\b(psad_[a-z0-9_]+)\s*\(', header))
    assert len(declared) >= 12
    lib = rt.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.psad_abi_version() == 3
    assert lib.psad_rtc_version() > 0
    assert lib.psad_error_string(1)


def test_native_libraries_built_from_these_sources():
    """Both native libraries carry the sha256 stamp of the sources they were built from (build.py), equal to the
    sources of this tree; the loaders refuse a stale one. On the GPU box this runs against the shipped .so files."""
    from pystencils_autodiff_amd import build
    assert build.embedded_hash(build.OUT) == build.source_hash(build.lib_sources())
    assert rt.lib().psad_source_hash().decode() == build.source_hash(build.lib_sources())
    assert build.embedded_hash(build.TORCH_OUT) == build.source_hash(build.torch_sources())
    import torch  # noqa: F401  (the extension resolves torch's symbols)
    from pystencils_autodiff_amd import _psad_torch
    assert _psad_torch.source_hash() == build.source_hash(build.torch_sources())
    with pytest.raises(rt.HipError, match='built from other sources'):
        rt._check_stamp('0123456789abcdef', 'lib', build.OUT)


def test_rtc_compile_error_is_reported():
    with pytest.raises(rt.HipError, match='hiprtc compilation failed'):
        rt.compile_hip('extern "C" __global__ void k() { this is not c++ }')


def _is_amdgpu_elf(code):
    return code[:4] == b'\x7fELF' and struct.unpack('<H', code[18:20])[0] == 224   # EM_AMDGPU


@pytest.mark.parametrize('builder,bh', [
    (W.diffusion_7pt, 'zeros'), (W.laplace_5pt, 'zeros'), (W.laplace_5pt, None), (W.stencil_27pt, 'zeros'),
    (lambda: W.diffusion_7pt(dtype='float64'), 'zeros'), (W.readme_op, None), (W.asym_7pt, None),
])
def test_all_schedules_compile_for_gfx950(builder, bh):
    op = pa.AutoDiffOp(builder(), boundary_handling=bh)
    for k in (op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()):
        variants = [k.primary_variant(), ('generic',)]
        if k.schedule() == 'march':
            variants.append(('march', MarchConfig(VE=1)))
        for v in variants:
            src, name = k.source(v)
            code = rt.compile_hip(src)
            assert _is_amdgpu_elf(code)
            assert name.encode() in code


def test_march_source_structure():
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    default = k.primary_variant()[1]
    assert default.ZSUM and 'zsum schedule' in k.code            # measured default for star stencils
    src, _ = k.source(('march', MarchConfig(CX=2, NR=2, VE=4)))   # the LDS-ring variant
    assert '__shared__' in src and '__syncthreads' in src
    assert 'XCD-aware' in src
    assert 'f32x4' in src                      # 16-byte plane loads
    # 7-point, NR=2 rows x CX=2 columns per thread, taps shared by the two rows read once:
    # per column 4 centre-column + 4 x-neighbour + 2 plane-above LDS taps; the plane below comes
    # from the register queue (lite ring: 2 LDS planes instead of 3)
    assert len(re.findall(r'const float t_u_', src)) == 20
    assert 'q_u_1_' in src


def test_zsum_eligibility():
    from pystencils_autodiff_amd.backends.hip_emitter import zsum_plan
    u, out = pa.ps.fields("u, out: float32[3d]")
    nonlinear = pa.ps.AssignmentCollection({out.center: u[1, 0, 0] * u[-1, 0, 0]})
    op = pa.AutoDiffOp(nonlinear, boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    assert zsum_plan(k.ir, MarchConfig()) is None
    assert not k.primary_variant()[1].ZSUM
    op27 = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    plan = zsum_plan(op27.forward_ast_gpu.ir, MarchConfig())
    assert sorted(plan[0]['lin']) == [-1, 0, 1] and all(len(plan[0]['lin'][dz]) == 9 for dz in (-1, 0, 1))
    assert plan[0]['rest'] == 0                                   # every centre-plane tap is a packed FMA too


def test_zsum_packed_variants_compile():
    op27 = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    k = op27.forward_ast_gpu.compile()
    default = k.primary_variant()[1]
    # measured default for fp16 box stencils: the half-precision ring (lanes own x-adjacent quads)
    from pystencils_autodiff_amd.backends.hip_emitter import ws_geometry
    assert default.ZSUM and default.WS and default.CX == 4 and ws_geometry(k.ir, default)['kind'] == 'h'
    for cfg in (MarchConfig(VE=8, CX=2, NR=4, ZSUM=True, PK=True),
                MarchConfig(VE=8, CX=2, WX=2, NR=4, ZSUM=True, PK=True, AR=True),
                MarchConfig(VE=8, CX=3, NR=2, ZSUM=True, PK=True)):       # odd CX: scalar fallback
        src, name = k.source(('march', cfg))
        assert ('f32x2 a0_' in src) == (cfg.PK and cfg.CX % 2 == 0)
        assert ('ds_read2_b32 %0' in src) == (cfg.AR and cfg.CX % 2 == 0)   # paired taps by inline asm
        code = rt.compile_hip(src)
        assert _is_amdgpu_elf(code) and name.encode() in code
    # every off-centre tap is one fused multiply-add into its accumulator
    src, _ = k.source(('march', MarchConfig(VE=8, CX=2, NR=1, ZSUM=True, PK=True)))
    assert re.search(r'a0_\d_p0_0 = a0_\d_p0_0 \+ \(', src)


def test_ws_loader_variants_compile():
    """Warp-specialised zsum (LDS-DMA loader wave): the measured default for star stencils in fp32 /
    fp64, counted vmcnt waits within the 6-bit counter, compiles for gfx950; fp16 storage reads the raw
    planes from a half-precision ring."""
    from pystencils_autodiff_amd.backends.hip_emitter import ws_geometry
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    k = op.forward_ast_gpu.compile()
    cfg = k._march_cfg(4, (1024, 1024, 1024))
    assert cfg.ZSUM and cfg.WS and cfg.D == 4 and (cfg.TX, cfg.TY) == (256, 16)
    ws = ws_geometry(k.ir, cfg)
    assert ws['block'] == 320 and ws['lds_bytes'] <= 160 * 1024
    for c in (cfg, MarchConfig(VE=4, CX=1, NR=3, ZSUM=True, WS=True, D=1),
              MarchConfig(VE=4, CX=2, WX=2, NR=2, ZSUM=True, WS=True, D=2, PK=True)):
        src, name = k.source(('march', c))
        assert '__builtin_amdgcn_raw_ptr_buffer_load_lds' in src and 'if (wave == 4)' in src
        waits = [int(v) for v in re.findall(r'vmcnt\((\d+)\)', src)]
        assert waits and max(waits) <= 63
        code = rt.compile_hip(src)
        assert _is_amdgpu_elf(code) and name.encode() in code
    two = pa.AutoDiffOp(W.asym_7pt(), boundary_handling='zeros').backward_ast_gpu
    assert ws_geometry(two.ir, MarchConfig(VE=4, CX=4, NR=8, ZSUM=True, WS=True, D=4))['D'] <= 4
    op27 = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')       # fp16 storage: half-precision ring
    k27 = op27.forward_ast_gpu.compile()
    c27 = MarchConfig(VE=8, CX=4, WX=1, NR=4, ZSUM=True, WS=True, D=3)
    ws = ws_geometry(k27.ir, c27)
    assert ws['kind'] == 'h' and ws['NS'] == 4 and ws['lds_type'] == '_Float16' and ws['lds_bytes'] <= 160 * 1024
    src, name = k27.source(('march', c27))
    assert '__builtin_amdgcn_raw_ptr_buffer_load_lds' in src and 'if (wave == 4)' in src and 'f16x4' in src
    assert _is_amdgpu_elf(rt.compile_hip(src))
    assert ws_geometry(k27.ir, MarchConfig(VE=8, CX=2, NR=4, ZSUM=True, WS=True)) is None    # lanes own quads
    assert ws_geometry(k27.ir, MarchConfig(VE=1, CX=2, NR=4, ZSUM=True, WS=True)) is None   # unaligned


def test_pack_args_alignment():
    buf = rt.pack_args([('ptr', 0x1000), ('i32', 7), ('i64', 9), ('f32', 1.5), ('f64', 2.0), ('i32', 3)])
    assert len(buf) % 8 == 0
    assert struct.unpack_from('<Q', buf, 0)[0] == 0x1000
    assert struct.unpack_from('<i', buf, 8)[0] == 7
    assert struct.unpack_from('<q', buf, 16)[0] == 9
    assert struct.unpack_from('<f', buf, 24)[0] == 1.5
    assert struct.unpack_from('<d', buf, 32)[0] == 2.0
    assert struct.unpack_from('<i', buf, 40)[0] == 3


def test_gpu_op_without_device_fails_loudly():
    torch = pytest.importorskip('torch')
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    with pytest.raises((RuntimeError, AssertionError, TypeError)):
        fn.apply(torch.zeros(4, 4, 4))


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(rt, '_lib', None)
    monkeypatch.setattr(rt, 'library_path', str(tmp_path / 'missing.so'))
    with pytest.raises(rt.HipError, match='missing'):
        rt.lib()


def test_unsupported_backends_raise():
    z, y, x = ps.fields("z, y, x: [20,30]")
    op = pa.AutoDiffOp(W.readme_op())
    with pytest.raises(NotImplementedError):
        op.create_tensorflow_op(backend='tensorflow_native')
    with pytest.raises(AssertionError):
        op.create_tensorflow_op(backend='jax')


def test_generic_schedule_variants_and_magic_division():
    """32-bit cell numbering with magic-number division (exact for every 32-bit numerator) and the
    contiguous-component variant whose grouped reads merge into wide loads."""
    import random
    from pystencils_autodiff_amd.backends.hip_emitter import emit_generic, magic_u32
    rng = random.Random(0)
    for d in [1, 2, 3, 7, 384, 1000, 1024, 65535, 12345677, 2 ** 31 - 1]:
        m, sh = magic_u32(d)
        for n in [0, 1, d - 1, d, d + 1, 2 ** 31 - 1, 2 ** 32 - 1] + [rng.randrange(2 ** 32) for _ in range(500)]:
            assert (((n * m) >> 32) + n) >> sh == n // d
    op = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling='zeros')
    ir = op.forward_ast_gpu.compile().ir
    for idx32 in (False, True):
        for contig in (False, True):
            src = emit_generic(ir, 'g', idx32=idx32, contig=contig)
            assert ('__umulhi' in src) == idx32 and ('st_u_3' in src.split('{', 1)[1]) == (not contig)
            assert _is_amdgpu_elf(rt.compile_hip(src))


def test_vector_field_zsum_compiles():
    """Vector fields take the zsum schedule (components interleaved in the plane image)."""
    from pystencils_autodiff_amd.backends.hip_emitter import march_geometry
    op = pa.AutoDiffOp(W.vector_laplace_7pt(), boundary_handling='zeros')
    for k in (op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()):
        assert k.schedule() == 'march'
        v = k.primary_variant()
        assert v[1].ZSUM
        g = march_geometry(k.ir, v[1])
        assert all(fg['C'] == 3 and fg['P'] == 3 * g['P'] for fg in g['FG'].values())
        assert _is_amdgpu_elf(rt.compile_hip(k.source(v)[0]))


def test_waves_per_workgroup_option():
    """NW (waves per workgroup) scales the block and the loaders' thread stride; WS keeps 4 + loader."""
    import pytest
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.backends.hip_emitter import MarchConfig, emit_zsum, ws_geometry
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    import pystencils_autodiff_amd as pa
    with pytest.raises(ValueError):
        MarchConfig(NW=3)
    with pytest.raises(ValueError):
        MarchConfig(NW=1, WX=2)
    op = pa.AutoDiffOp(W.stencil_27pt(), boundary_handling='zeros')
    k = StencilKernel(op.forward_assignments, boundary_handling='zeros', function_name='nw', target='gpu',
                      gpu_indexing_params={'NW': 1}).compile()
    cfg = k._march_cfg(k._vec_elems(), (64, 64, 256))
    assert cfg.NW == 1 and cfg.WX == 1 and cfg.NT == 64 and cfg.TY == cfg.NR
    src = emit_zsum(k.ir, 'nw_zsum', cfg)
    assert '__launch_bounds__(64)' in src and 'tid + k * 64' in src and 'tid + k * 256' not in src
    assert ws_geometry(k.ir, MarchConfig(VE=4, WS=True, ZSUM=True, NW=2, WX=1)) is None


def test_quantized_chunk_model():
    """WS chunk count: power-of-two cubes / 1024² slabs keep 128-plane chunks; 768³ avoids a short last round."""
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel
    q = HipStencilKernel.quantized_chunk
    assert q(1024, 256, 256, 32, 128, 1, 256) == 128
    assert q(512, 64, 256, 32, 128, 1, 256) == 128
    assert q(128, 256, 256, 32, 128, 1, 256) == 128
    assert q(768, 144, 256, 32, 128, 1, 256) == 110
    assert q(5, 7, 256, 32, 128, 1, 256) == 5


def test_rccl_entry_points_report_errors_without_gpu():
    """The RCCL halo entry points fail with a described code (never abort) when librccl is missing.
    Run in a fresh interpreter: ``psad_rccl_open`` keeps the first library a process opened, so an
    earlier test that loaded the real librccl would make the failure path unobservable here."""
    import subprocess
    import sys
    code = r"""
import ctypes, sys
sys.path.insert(0, %r)
from pystencils_autodiff_amd.backends import hip_runtime as rt
L = rt.lib()
rc = L.psad_rccl_open(b'/nonexistent/librccl.so')
assert rc == 20100, rc
assert b'RCCL' in L.psad_error_string(rc)
uid = ctypes.create_string_buffer(128)
assert L.psad_rccl_unique_id(uid) == 20100
comm = ctypes.c_void_p()
assert L.psad_rccl_comm_init(uid, 1, 0, ctypes.byref(comm)) == 20100
vp = ctypes.c_void_p
z = (vp * 1)(0)
n = (ctypes.c_size_t * 1)(0)
assert L.psad_halo_exchange(None, 1, z, z, z, z, n, -1, -1, None) == 20100
print('ok')
""" % ROOT
    proc = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
    assert proc.returncode == 0 and 'ok' in proc.stdout, proc.stdout + proc.stderr