"""ISA audit of the LDS-DMA ring barriers: LDS reads still outstanding at an ``s_barrier``.

A compute wave that passes barrier j with a ``ds_read`` of ring slot s still in flight races the loader wave, which
refills slot s by LDS-DMA right after that barrier (the DMA writes are invisible to the compiler). This prints, for
every ``s_barrier`` of a kernel, the worst number of ``ds_read`` instructions not yet covered by an
``s_waitcnt lgkmcnt`` on any path reaching it (a dataflow fixed point over the kernel's basic blocks, so the
loops' back edges count). Exit status 1 if any barrier has one.

With the band schedule's LDS handshake (``BFREE``: no plane barriers) the same dataflow checks the two halves of
the handshake instead: at every ``ds_write`` (a compute wave's release word, the loader's published-plane word and
zero fill) no ``ds_read`` may be outstanding — a release issued before the plane's reads returned would let the
loader refill the slot under them — and on every path the plane reads between two releases (poll reads, a
``ds_read_b32`` whose value goes through ``v_readfirstlane``, not counted) are the same count, so no read crossed a
release into another plane step. (A read hoisted above its own step's poll is excluded at the source: a memory
clobber follows the poll; the compiler may place the poll loops out of line, so program order says nothing here.)

python scripts/probes/barrier_audit.py <workload> <Z,Y,X> [KEY=VAL,...] [forward|backward]   (no GPU needed)
python scripts/probes/barrier_audit.py --isa kernel.s
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LLVM = '/opt/rocm/lib/llvm/bin'


def disassemble(workload, shape, tun, which):
    sys.path.insert(0, ROOT)
    from pystencils_autodiff_amd import AutoDiffOp, workloads as W
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    from pystencils_autodiff_amd.backends.hip_kernel import HipStencilKernel, default_march_config
    from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel
    wl = {'stencil27': W.stencil_27pt, 'diffusion7': W.diffusion_7pt,
          'diffusion7_f16': lambda: W.diffusion_7pt(dtype='float16'), 'varcoef': W.varcoef_diffusion_7pt,
          'varcoef_f16': lambda: W.varcoef_diffusion_7pt(dtype='float16')}[workload]
    op = AutoDiffOp(wl(), boundary_handling='zeros')
    asg = op.forward_assignments if which == 'forward' else op.backward_assignments
    k = StencilKernel(asg, boundary_handling='zeros', function_name='audit', target='gpu', gpu_indexing_params=tun)
    hk = HipStencilKernel(k)
    cfg = default_march_config(hk.ir, hk._vec_elems(), shape, tun)
    code = rt.compile_hip(hk.source(('march', cfg))[0])
    path = f'/tmp/barrier_audit_{os.getpid()}.co'
    with open(path, 'wb') as fh:
        fh.write(code)
    try:
        return subprocess.run([f'{LLVM}/llvm-objdump', '-d', '--mcpu=gfx950', path], capture_output=True,
                              text=True, check=True).stdout, cfg
    finally:
        os.remove(path)


def parse(text):
    """[(address, opcode, operands, branch target address or None)] of the first kernel in the listing."""
    ins = []
    for line in text.splitlines():
        m = re.match(r'^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):', line)
        if not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = re.search(r'<\S+\+0x([0-9a-f]+)>', line)
        ins.append((addr, op, args, int(t.group(1), 16) if t and op.startswith(('s_cbranch', 's_branch')) else None))
    return ins


def audit(ins, at=('s_barrier',)):
    """Worst outstanding ds_read count at each instruction whose opcode starts with one of ``at``: {index: count}."""
    base = ins[0][0] if ins else 0
    index = {a - base: i for i, (a, _, _, _) in enumerate(ins)}
    # successors of each instruction
    succ = []
    for i, (a, op, args, tgt) in enumerate(ins):
        s = []
        if op in ('s_endpgm',):
            pass
        elif op == 's_branch':
            s.append(index.get(tgt))
        else:
            if i + 1 < len(ins):
                s.append(i + 1)
            if tgt is not None:
                s.append(index.get(tgt))
        succ.append([j for j in s if j is not None])
    CAP = 64
    state = [None] * len(ins)      # (lgkm ops outstanding, of which ds_read) on entry, max over paths
    state[0] = (0, 0)
    work = [0]
    while work:
        i = work.pop()
        tot, rd = state[i]
        _, op, args, _ = ins[i]
        if op.startswith('ds_read') or op.startswith('ds_'):
            tot, rd = min(CAP, tot + 1), min(CAP, rd + (1 if op.startswith('ds_read') else 0))
        elif op.startswith(('s_load', 's_buffer_load')):
            tot = min(CAP, tot + 1)
        elif op == 's_waitcnt':
            m = re.search(r'lgkmcnt\((\d+)\)', args)
            if m:
                n = int(m.group(1))
                tot, rd = min(tot, n), min(rd, n)
        for j in succ[i]:
            new = (tot, rd) if state[j] is None else (max(state[j][0], tot), max(state[j][1], rd))
            if new != state[j]:
                state[j] = new
                work.append(j)
    return {i: state[i][1] for i, (_, op, _, _) in enumerate(ins) if op.startswith(at) and state[i] is not None}


def polls(ins):
    """Indices of the acquire polls: a ds_read_b32 whose destination is read by a v_readfirstlane_b32 within the next
    few instructions (the wave-uniform read of the loader's published-plane word)."""
    out = []
    for i, (_, op, args, _) in enumerate(ins):
        if op != 'ds_read_b32':
            continue
        dst = args.split(',')[0].strip()
        for j in range(i + 1, min(i + 6, len(ins))):
            if ins[j][1] == 'v_readfirstlane_b32' and dst in ins[j][2].split(',')[1:][0]:
                out.append(i)
                break
    return out


def release_intervals(ins, poll_reads):
    """(min, max) plane reads since the previous ds_write on any path reaching each ds_write."""
    base = ins[0][0] if ins else 0
    index = {a - base: i for i, (a, _, _, _) in enumerate(ins)}
    succ = []
    for i, (a, op, args, tgt) in enumerate(ins):
        s = []
        if op == 's_branch':
            s.append(index.get(tgt))
        elif op != 's_endpgm':
            if i + 1 < len(ins):
                s.append(i + 1)
            if tgt is not None:
                s.append(index.get(tgt))
        succ.append([j for j in s if j is not None])
    state = [None] * len(ins)
    state[0] = (0, 0)
    work = [0]
    out = {}
    while work:
        i = work.pop()
        lo, hi = state[i]
        op = ins[i][1]
        if op.startswith('ds_write'):
            out[i] = (lo, hi)
            lo = hi = 0
        elif op.startswith('ds_read') and i not in poll_reads:
            lo, hi = min(lo + 1, 999), min(hi + 1, 999)
        for j in succ[i]:
            new = (lo, hi) if state[j] is None else (min(state[j][0], lo), max(state[j][1], hi))
            if new != state[j]:
                state[j] = new
                work.append(j)
    return out


def main():
    if sys.argv[1] == '--isa':
        text, cfg = open(sys.argv[2]).read(), None
    else:
        tun = {}
        if len(sys.argv) > 3 and sys.argv[3]:
            for kv in sys.argv[3].split(','):
                k, v = kv.split('=')
                tun[k] = int(v)
        which = sys.argv[4] if len(sys.argv) > 4 else 'forward'
        text, cfg = disassemble(sys.argv[1], tuple(int(v) for v in sys.argv[2].split(',')), tun, which)
    ins = parse(text)
    res = audit(ins)
    if cfg is not None and getattr(cfg, 'BFREE', 0):
        wr = audit(ins, ('ds_write',))
        bad = sum(1 for v in wr.values() if v > 0)
        ps = polls(ins)
        iv = release_intervals(ins, set(ps))
        counts = sorted({v for lo_hi in iv.values() for v in lo_hi})
        print(f'  handshake: {len(wr)} ds_write, {bad} with a ds_read outstanding on the worst path; {len(ps)} acquire '
              f'polls; plane reads between releases on any path: {counts}')
        print(f'{" ".join(sys.argv[1:])} [band, LDS handshake]: {"FAIL" if bad else "ok"}')
        sys.exit(1 if bad else 0)
    bad = 0
    bars = sorted(res)
    for k, i in enumerate(bars):
        # LDS reads laid out between this barrier and the next one (a read sunk below the next barrier would move
        # from one plane step's segment into the next: the peeled steps of a kernel all show the same count)
        nxt = bars[k + 1] if k + 1 < len(bars) else len(ins)
        seg = sum(1 for j in range(i + 1, nxt) if ins[j][1].startswith('ds_read'))
        print(f'  s_barrier at +0x{ins[i][0] - ins[0][0]:x}: {res[i]} ds_read outstanding on the worst path, '
              f'{seg} ds_read before the next barrier')
        bad += res[i] > 0
    tag = f'{cfg.BAND and "band" or ("WS" if cfg.WS else "march")}' if cfg else 'isa'
    print(f'{" ".join(sys.argv[1:])} [{tag}]: {len(res)} barriers, {bad} with LDS reads in flight')
    sys.exit(1 if bad else 0)


if __name__ == '__main__':
    main()
