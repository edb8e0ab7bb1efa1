"""ISA audit of the LDS-DMA schedules on the CPU: at no ``s_barrier`` of the compute waves may an LDS read still be
outstanding (a read sunk past the barrier races the loader wave's DMA refill of that ring slot — the round-4 band race,
DESIGN.md §4). Compiles the kernels with hiprtc for gfx950 and walks the disassembly's control-flow graph
(``scripts/probes/barrier_audit.py``); no GPU needed."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scripts', 'probes'))

OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'

CASES = [('diffusion7', (1024, 1024, 1024), {}),                        # headline: WS zsum
         ('stencil27', (768, 768, 768), {}),                            # config 5: row bands
         ('diffusion7_f16', (768, 768, 768), {}),                       # fp16 star row bands
         ('varcoef', (512, 512, 512), {}),                              # nonlinear: LDS-DMA plane ring
         ('varcoef', (512, 512, 512), {'WS': 1, 'NW': 8, 'CX': 4, 'NR': 1, 'D': 3})]


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason='llvm-objdump not in this image')
@pytest.mark.parametrize('which', ['forward', 'backward'])
@pytest.mark.parametrize('workload,shape,tun', CASES, ids=[f'{c[0]}-{c[1][0]}-{len(c[2])}' for c in CASES])
def test_no_lds_read_outstanding_at_any_barrier(workload, shape, tun, which):
    import barrier_audit as B
    text, cfg = B.disassemble(workload, shape, tun, which)
    assert cfg.WS or cfg.BAND, f'{workload}: expected an LDS-DMA schedule, got {cfg}'
    res = B.audit(B.parse(text))
    assert res, 'no s_barrier found'
    bad = {i: n for i, n in res.items() if n}
    assert not bad, f'{workload} {which}: LDS reads outstanding at {len(bad)} barrier(s): {bad}'


HANDSHAKE = [('stencil27', (768, 768, 768), {'BFREE': 2}), ('diffusion7_f16', (768, 768, 768), {'BFREE': 1}),
             ('stencil27', (64, 64, 512), {'BFREE': 3, 'BAND': 4}), ('diffusion7_f16', (64, 64, 1024), {'BFREE': 2, 'BAND': 2})]


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason='llvm-objdump not in this image')
@pytest.mark.parametrize('which', ['forward', 'backward'])
@pytest.mark.parametrize('workload,shape,tun', HANDSHAKE, ids=[f'{c[0]}-{c[1][2]}-{c[2]["BFREE"]}' for c in HANDSHAKE])
def test_band_handshake_releases_after_reads(workload, shape, tun, which):
    """The band's LDS handshake (``BFREE``, no plane barriers): at every ``ds_write`` — a compute wave's release word,
    the loader's published-plane word or its zero fill — no ``ds_read`` is outstanding on any path, and the handshake
    words are LDS operations (``ds_``), not flat ones (a flat access would also wait on the wave's stores)."""
    import barrier_audit as B
    text, cfg = B.disassemble(workload, shape, tun, which)
    assert cfg.BAND and cfg.BFREE == tun['BFREE'], cfg
    ins = B.parse(text)
    assert not [op for _, op, _, _ in ins if op.startswith('flat_')], 'flat memory operations in the band kernel'
    res = B.audit(ins, ('ds_write',))
    assert len(res) >= 6, f'expected release / publish writes, found {len(res)}'
    bad = {i: n for i, n in res.items() if n}
    assert not bad, f'{workload} {which}: LDS reads outstanding at {len(bad)} ds_write(s): {bad}'
    assert B.polls(ins), 'no acquire poll (ds_read_b32 -> v_readfirstlane_b32) found'
