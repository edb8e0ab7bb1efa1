"""Benchmark: Mcells/s forward+backward, 3-D 7-point fp32 1024³ (BASELINE.json metric).

One step = one forward sweep + one TF-MAD adjoint sweep of the 7-point diffusion op
``out = u + 0.1·(Σ₆ u[nb] − 6u)`` (boundary 'zeros') through the drop-in API
(``AutoDiffOp(...).create_tensorflow_op(backend='torch_native')`` → ``Op.apply`` +
``out.backward``), inputs resident in HBM. N>1: the 1024³ domain is split into z-slabs
(``zslab.py``) with an RCCL halo exchange per sweep — strong scaling, total work fixed.

``--workload stencil27_f16`` runs BASELINE config 5 instead (27-point anisotropic stencil, fp16 storage,
768³ by default) through the same path, at 1 GPU or as 8 z-slabs; the default stays the headline.

Run: ``python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W] [--edge E]``; N>1 via
``torch.distributed.run --nproc-per-node N``.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md), GB/s

# the BASELINE configs bench.py can run: builder, storage dtype, default cube edge, algorithmic bytes per cell
# and sweep (distinct fields read + written), labels
WORKLOADS = {
    'diffusion7_f32': dict(builder='diffusion_7pt', dtype='float32', edge=1024, bytes=8, label='3D 7-point fp32',
                           dtype_tag='f32',
                           desc='3D 7-point diffusion out=u+0.1*(sum6 u[nb]-6u), boundary zeros, fp32'),
    'stencil27_f16': dict(builder='stencil_27pt', dtype='float16', edge=768, bytes=4, label='3D 27-point fp16',
                          dtype_tag='f16 storage, f32 arithmetic',
                          desc='3D 27-point anisotropic stencil (27 distinct weights), boundary zeros, fp16 storage '
                               'with fp32 arithmetic (BASELINE config 5)'),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    # 10 warmup steps (28 ms at 1024³) cover the power-management transient a sustained HBM-bound load
    # first causes (dispatches 0-9 of the kernel trace run up to 4 % slower, profiles/r02g_bench_dispatches.txt)
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--workload', default='diffusion7_f32', choices=sorted(WORKLOADS),
                   help='diffusion7_f32 (default, the headline) or stencil27_f16 (BASELINE config 5)')
    p.add_argument('--secondary', default='stencil27_f16', choices=sorted(WORKLOADS) + ['none'],
                   help='a second BASELINE workload timed in the same run, reported under "secondary" '
                        '(default: config 5, stencil27_f16 768^3; none to skip)')
    p.add_argument('--secondary-edge', type=int, default=None, help='cube edge of the secondary workload')
    p.add_argument('--edge', type=int, default=None,
                   help='cube edge (default: the workload\'s BASELINE size, 1024 / 768)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--cpu-seconds', type=float, default=12.0, help='budget of the CPU baseline sample')
    p.add_argument('--kernel-only', action='store_true', help='also time the raw kernel loop')
    return p.parse_args()


def cpu_model():
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or 'unknown'


def cpu_baseline(budget_s, workload='diffusion7_f32', edge=1024):
    """The oracle's C restatement of the reference CPU kernel on bounded slabs of the workload: first with
    ONE thread — the reference's default (``create_kernel`` without ``cpu_openmp``, ``_autodiff.py:487-489``),
    reported as ``value`` — then with OpenMP over this process's cores (``cpu_openmp=True``)."""
    import numpy as np
    from oracle import cref
    build_dir = os.path.join(ROOT, 'oracle', 'build_native')
    lib = cref.load(build_dir=build_dir, march='native')
    # OpenMP threads: the CPUs this process may run on (sched_getaffinity), capped by OMP_NUM_THREADS where the
    # job sets it — the GPU box exports OMP_NUM_THREADS=16, its CPU share per GPU, while sched_getaffinity there
    # lists every CPU of the host (256); the cap is reported with the figure
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get('OMP_NUM_THREADS', '0'))
    mt = min(omp, affinity) if omp > 0 else affinity
    cap = (f'OMP_NUM_THREADS={omp} (the job\'s CPU share) of {affinity} CPUs in sched_getaffinity' if 0 < omp < affinity
           else f'sched_getaffinity: {affinity} CPUs')
    w27 = workload == 'stencil27_f16'
    if w27:
        from pystencils_autodiff_amd import workloads as W
        wf = np.asarray(W.WEIGHTS_27PT, dtype=np.float32)
        wb = wf[::-1].copy()                     # the TF-MAD adjoint: the same stencil with flipped offsets
    dt = np.float16 if w27 else np.float32

    def run(threads, planes, budget):
        got = lib.set_threads(threads)
        shape = (planes, edge, edge)
        rng = np.random.default_rng(0)
        u = rng.uniform(0, 1, shape).astype(dt)
        d = rng.uniform(-1, 1, shape).astype(dt)
        if w27:
            sweeps = (lambda: lib.stencil27_f16(u, wf), lambda: lib.stencil27_f16(d, wb))
        else:
            out, du = np.empty_like(u), np.empty_like(u)
            sweeps = (lambda: lib.diffusion7_f32(u, 0.1, out), lambda: lib.diffusion7_f32(d, 0.1, du))
        sweeps[0]()                              # warm-up (first touch, thread pool)
        reps, t0 = 0, time.perf_counter()
        while True:
            sweeps[0]()                          # forward sweep
            sweeps[1]()                          # adjoint sweep
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget or reps >= 5000:
                break
        return got, reps, el, round(reps * u.size / el / 1e6, 2)

    p1, pm = (16, 64) if not w27 else (16, 48)
    t1, reps1, el1, v1 = run(1, p1, budget_s / 2)
    tm, repsm, elm, vm = run(mt, pm, budget_s / 2)
    model = cpu_model()
    kind = 'fp16 27-point (F16C conversions, fp32 arithmetic)' if w27 else 'fp32 7-point'
    return {'value': v1, 'unit': 'Mcells/s', 'cores': t1, 'kind': 'port',
            'sample': f'{reps1} fwd+bwd sweeps of a {p1}x{edge}x{edge} {kind} slab of the {edge}^3 workload in '
                      f'{el1:.1f} s, 1 thread (the reference default: no cpu_openmp); oracle/stencil_ref.c '
                      f'(pystencils CPU loop nest restated), gcc -O3 -march=native -fopenmp; host CPU {model}',
            'threads_1': {'value': v1, 'threads': t1, 'sweeps': reps1, 'seconds': round(el1, 2),
                          'sample': f'{p1}x{edge}x{edge}'},
            'threads_mt': {'value': vm, 'threads': tm, 'sweeps': repsm, 'seconds': round(elm, 2),
                           'sample': f'{pm}x{edge}x{edge}', 'cpu_openmp': True, 'threads_rule': cap},
            'cpu_model': model, 'cpus_available': affinity}


def load_traffic(workload, kernel):
    """HBM bytes per launch of ``kernel`` from the committed PMC summary (profiles/traffic.json):
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled (gfx950 wide-read correction). Returns
    (bytes, the entry: its source, the git commit it was collected at, the sha of the kernels it measured)."""
    path = os.path.join(ROOT, 'profiles', 'traffic.json')
    try:
        with open(path) as fh:
            entry = json.load(fh).get(workload) or {}
    except (OSError, ValueError):
        return None, {}
    k = entry.get('kernels', {}).get(kernel)
    return (k['total'] if k else None), entry


def kernel_sha(*kernels):
    """16 hex digits of sha256 over the HIP sources of the launches that ran (the emitted kernels, the exact code
    the PMC passes of profiles/traffic.json measured when its ``kernel_sha16`` is the same)."""
    import hashlib
    h = hashlib.sha256()
    for k in kernels:
        h.update(k.source(k.last_variant)[0].encode() if k.last_variant else b'?')
    return h.hexdigest()[:16]


def _sig(x, n=4):
    """``x`` to ``n`` significant digits (a fraction of the peak stays readable at small N=2 rehearsal sizes)."""
    return float(f'{x:.{n}g}')


def roofline(name, r, world):
    """The line's ``roofline`` object: ``achieved`` = algorithmic bytes of one step (forward + adjoint sweep over the
    whole domain) ÷ the step time (barrier-bracketed, max over ranks) ÷ GPUs, so ``frac`` is the
    step-level figure; ``frac_fwd`` / ``frac_bwd`` are each sweep on its own (algorithmic bytes of one launch over
    this rank's slab ÷ its HIP-event time on the launch stream). ``traffic``: HBM bytes per launch from the committed
    PMC passes for this exact launch shape (full domain at N=1), else null (no slab-shaped entry)."""
    wl = WORKLOADS[name]
    n, zl = r['n'], r['zl']
    key = f'{name}_{n}^3' if world == 1 else f'{name}_{zl}x{n}^2_slab'
    tf, entry = load_traffic(key, r['kname'])
    tb, _ = load_traffic(key, r['kname'].replace('_forward_', '_backward_'))
    traffic = tf + tb if tf is not None and tb is not None else None      # per step, like ``achieved``
    src = entry.get('source')
    if src and entry.get('git_head'):
        src = (f'{src}; collected at commit {entry["git_head"]} — the kernel sha (traffic_kernel_sha16 vs kernel_sha16), '
               f'not the commit, ties the PMC passes to the kernels benched here')
    match = entry.get('kernel_sha16') == r['ksha'] if entry.get('kernel_sha16') else None
    return {'bound': 'hbm', 'achieved': round(r['achieved'], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': _sig(r['achieved'] / HBM_PEAK_GBS),
            'frac_fwd': _sig(r['achieved_fwd'] / HBM_PEAK_GBS),
            'frac_bwd': _sig(r['achieved_bwd'] / HBM_PEAK_GBS),
            'achieved_fwd': round(r['achieved_fwd'], 1), 'achieved_bwd': round(r['achieved_bwd'], 1),
            'traffic': traffic, 'traffic_fwd_launch': tf,
            'traffic_source': src or f'no PMC entry for the launch shape {key}',
            'kernel_sha16': r['ksha'], 'traffic_kernel_sha16': entry.get('kernel_sha16'),
            'traffic_measured_these_kernels': match,
            'kernel': f'{r["kname"]} + its adjoint (step: both sweeps, {2 * wl["bytes"]} B per cell)',
            'bytes_per_launch': r['bytes_fwd'], 'bytes_per_step': 2 * wl['bytes'] * r['cells']}


def run_workload(name, edge, args, world, rank, distributed, extras, warmup=None):
    """Warmup, then EXACTLY ``args.steps`` timed fwd+bwd steps of workload ``name`` through the drop-in path
    (1 GPU: the op; N GPUs: this rank's z-slab through ``ZSlabOp.autograd_function()``), bracketed by barrier +
    synchronize, max over ranks. Returns the figures of the JSON line."""
    import torch
    import torch.distributed as dist

    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import ZSlabOp, slab_bounds
    wl = WORKLOADS[name]
    n = edge or wl['edge']
    tdtype = getattr(torch, wl['dtype'])
    bytes_per_cell = wl['bytes']
    lo, hi = slab_bounds(n, world, rank)
    zl = hi - lo
    # the op named after the workload: its kernels (<name>_forward_gpu_zsum, ...) stay apart in rocprof traces
    op = pa.AutoDiffOp(getattr(W, wl['builder'])(), name, boundary_handling='zeros')
    fn = op.create_tensorflow_op(use_cuda=True, backend='torch_native')
    fwd_k = op.forward_ast_gpu.compile()
    bwd_k = op.backward_ast_gpu.compile()

    g = torch.Generator(device='cuda').manual_seed(0 + rank)
    u = torch.rand((zl, n, n), generator=g, device='cuda', dtype=torch.float32).to(tdtype)
    g1 = torch.Generator(device='cuda').manual_seed(1000 + rank)
    d = (torch.rand((zl, n, n), generator=g1, device='cuda', dtype=torch.float32) * 2 - 1).to(tdtype)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    ev = []
    # every N times the same autograd engine mode: the backward runs in this thread. At N>1 torch's autograd
    # device thread doubles the host cost of every HIP / RCCL call of a slab sweep
    # (scripts/probes/slab_step.py ... sweeps: 95 vs 52 us per sweep), which at 8 ranks is what the GPU
    # would wait on; same work, same autograd graph. N=1 also reports the default engine (below).
    torch.autograd.set_multithreading_enabled(False)

    if distributed:
        # the same drop-in contract over this rank's slab: Function.apply + backward, with the
        # RCCL halo exchange inside the forward and the backward (zslab.py)
        zop = ZSlabOp(op, use_cuda=True)
        fn = zop.autograd_function()
        zop.connect(u.device)       # setup, not a step: the RCCL communicator exists before warmup
        zop.warm_exchange(u=u, diffout=d)   # and RCCL's peer connections (set up on first use)
    # setup, not a step: the 1024^3 kernel variants compiled (hiprtc) and loaded, and the output and
    # gradient blocks reserved in torch's caching allocator, before warmup
    scratch = [torch.empty_like(u), torch.empty_like(u)]
    fwd_k.prepare(u=u, out=scratch[0])
    bwd_k.prepare(diffout=d, diffu=scratch[1])
    del scratch
    # and a first backward with an explicit gradient (its lazy imports in autograd._make_grads cost ~40 ms)
    # run on a 1-element tensor (measured by a round-2 probe)
    probe = torch.zeros(1, device=u.device, requires_grad=True)
    (probe * 2).backward(torch.ones_like(probe))
    del probe
    uu = u.requires_grad_(True)

    def step(record):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e2 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        (o,) = fn.apply(uu)
        e1.record(stream)
        o.backward(d)
        e2.record(stream)
        uu.grad = None
        if record:
            ev.append((e0, e1, e2))

    # (the secondary 27-point sweep gets >= 60 warmup steps and at least 0.5 s of them: its first dispatches after the
    # 1024^3 run land in a power-management transient, profiles/r02_power_transient_27pt.txt; alone with 10 warmup
    # steps config 5 measured 0.760 ms per step, with 300 0.704, profiles/r05_b27_warmup.log)
    i = 0
    if warmup is None:
        for i in range(1, args.warmup + 1):        # the line's contract: exactly W warmup steps
            step(False)
    else:
        # blocks of 8 steps until both the count and the time are reached; at N>1 the ranks agree after each block
        # (every step exchanges halos, so all ranks must run the same number of steps)
        t_warm = time.perf_counter()
        while True:
            for _ in range(8):
                step(False)
                i += 1
            torch.cuda.synchronize()
            more = i < warmup or time.perf_counter() - t_warm < 0.5
            if distributed:
                flag = torch.tensor([1.0 if more else 0.0], device='cuda')
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                more = flag.item() > 0
            if not more:
                break
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    fwd_ms = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    bwd_ms = sum(b.elapsed_time(c) for _, b, c in ev) / len(ev)
    if os.environ.get('PSAD_BENCH_ADDR'):
        # where the sweeps' streams sit (probe of the per-process fwd / bwd split): inputs, and the output /
        # gradient blocks the caching allocator hands the op (the same block every step)
        (o,) = fn.apply(uu)
        o.backward(d)
        torch.cuda.synchronize()
        print(json.dumps({'workload': name, 'rank': rank, 'u': hex(u.data_ptr()), 'diffout': hex(d.data_ptr()),
                          'out': hex(o.data_ptr()), 'diffu': hex(uu.grad.data_ptr()), 'fwd_ms': round(fwd_ms, 4),
                          'bwd_ms': round(bwd_ms, 4),
                          'fwd_each': [round(a.elapsed_time(b), 4) for a, b, _ in ev],
                          'bwd_each': [round(b.elapsed_time(c), 4) for _, b, c in ev]}), file=sys.stderr)
        del o
        uu.grad = None
    cells_total = n ** 3
    value = cells_total * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # algorithmic bytes of one sweep (forward or adjoint) over this rank's slab; per sweep from its HIP-event time,
    # per step (both sweeps, the line's roofline) from the barrier-bracketed clock, max over ranks, per GPU
    bytes_fwd = bytes_per_cell * zl * n * n
    achieved_fwd = bytes_fwd / (fwd_ms * 1e-3) / 1e9
    achieved_bwd = bytes_fwd / (bwd_ms * 1e-3) / 1e9
    achieved = 2 * bytes_per_cell * cells_total / world / (ms_per_step * 1e-3) / 1e9
    result_extra = {}
    if extras and not distributed:
        # the same step with torch's default engine (backward on its device thread; the op's backward is
        # the C++ node, so no Python runs there)
        torch.autograd.set_multithreading_enabled(True)
        for _ in range(3):
            step(False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(False)
        torch.cuda.synchronize()
        result_extra['value_default_engine'] = round(cells_total * args.steps / (time.perf_counter() - t1) / 1e6, 1)
        torch.autograd.set_multithreading_enabled(False)
    if extras and args.kernel_only and not distributed:
        out = torch.empty_like(u)
        du = torch.empty_like(u)
        for _ in range(2):
            fwd_k(u=u.detach(), out=out)
            bwd_k(diffout=d, diffu=du)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            fwd_k(u=u.detach(), out=out)
            bwd_k(diffout=d, diffu=du)
        torch.cuda.synchronize()
        kt = time.perf_counter() - t1
        result_extra['kernel_only_mcells_s'] = round(cells_total * args.steps / kt / 1e6, 1)

    zop_keep = zop if distributed else None
    kname = fwd_k.source(fwd_k.last_variant)[1] if fwd_k.last_variant else fwd_k.name
    out = dict(n=n, zl=zl, value=value, ms_per_step=ms_per_step, fwd_ms=fwd_ms, bwd_ms=bwd_ms, achieved=achieved,
               ksha=kernel_sha(fwd_k, bwd_k), warmup_steps=i,
               achieved_fwd=achieved_fwd, achieved_bwd=achieved_bwd, bytes_fwd=bytes_fwd, kname=kname,
               cells=cells_total, extra=result_extra, zop=zop_keep)
    del uu, u, d, fn, op
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    distributed = world > 1
    if args.gpus != world and distributed:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if distributed:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        backend = os.environ.get('PSAD_DIST_BACKEND', 'nccl')   # nccl = RCCL; gloo only to rehearse on 1 GPU
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
        else:
            dist.init_process_group(backend)

    primary = run_workload(args.workload, args.edge, args, world, rank, distributed, extras=True)
    secondary = None
    if args.secondary != 'none' and args.secondary != args.workload:
        # BASELINE config 5 measured in the same run (the driver's scaling runs call bench.py with its default
        # workload only): same path, same timing rules, its own barrier + max-over-ranks clock
        secondary = run_workload(args.secondary, args.secondary_edge, args, world, rank, distributed, extras=False,
                                 warmup=max(args.warmup, 60))
    n = primary['n']
    wl = WORKLOADS[args.workload]
    value, ms_per_step, fwd_ms, bwd_ms = (primary[k] for k in ('value', 'ms_per_step', 'fwd_ms', 'bwd_ms'))
    achieved, cells_total = primary['achieved'], primary['cells']
    result_extra = primary['extra']
    zop = primary['zop']
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # after the timed loop, at every N (north_star: the CPU path "in the same run"); the other ranks
        # wait at the barrier below
        try:
            cpu = cpu_baseline(args.cpu_seconds, args.workload, n)
        except Exception as exc:  # noqa: BLE001 - report, don't fail the GPU bench
            cpu = {'value': None, 'unit': 'Mcells/s', 'cores': None, 'kind': 'port', 'sample': f'failed: {exc}'}
    if distributed:
        dist.barrier()
    if rank == 0:
        res = {
            'metric': f'Mcells/s forward+backward, {wl["label"]} {n}^3',
            'value': round(value, 1),
            'unit': 'Mcells/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_per_step, 4),
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': wl['dtype_tag'],
            'data': 'synthetic: u~U(0,1), diffout~U(-1,1) (torch generator seeds 0/1000+rank)',
            'config': {'workload': f'{wl["desc"]}, {n}^3 forward + TF-MAD adjoint per step',
                       'name': args.workload,
                       'cells': cells_total, 'decomposition': f'z-slab x{world}' if world > 1 else 'single GPU',
                       'path': ('AutoDiffOp.create_tensorflow_op(backend=torch_native) apply+backward' if world == 1
                                else 'ZSlabOp(AutoDiffOp).autograd_function() apply+backward, RCCL halo exchange')
                       + ', autograd engine single-threaded (set_multithreading_enabled(False)) at every N'},
            'fwd_ms': round(fwd_ms, 4),
            'bwd_ms': round(bwd_ms, 4),
            'hbm_roofline_frac_step': round(achieved / HBM_PEAK_GBS, 4),
            'roofline': roofline(args.workload, primary, world),
            'cpu_baseline': cpu,
        }
        if secondary is not None:
            w2 = WORKLOADS[args.secondary]
            n2 = secondary['n']
            res['secondary'] = {
                'metric': f'Mcells/s forward+backward, {w2["label"]} {n2}^3', 'name': args.secondary,
                'value': round(secondary['value'], 1), 'unit': 'Mcells/s', 'n_gpus': world, 'steps': args.steps,
                'warmup': secondary['warmup_steps'], 'ms_per_step': round(secondary['ms_per_step'], 4),
                'fwd_ms': round(secondary['fwd_ms'], 4), 'bwd_ms': round(secondary['bwd_ms'], 4),
                'dtype': w2['dtype_tag'], 'cells': secondary['cells'],
                'decomposition': f'z-slab x{world}' if world > 1 else 'single GPU',
                'hbm_roofline_frac_step': round(secondary['achieved'] / HBM_PEAK_GBS, 4),
                'roofline': roofline(args.secondary, secondary, world)}
        res.update(result_extra)
        print(json.dumps(res))
    if distributed:
        for r in (primary, secondary):
            if r is not None and r['zop'] is not None:
                r['zop'].close()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
