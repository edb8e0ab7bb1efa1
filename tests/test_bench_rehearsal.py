"""End-to-end rehearsal of ``bench.py`` at N>1 on the one GPU of a test box.

The driver runs ``torch.distributed.run --nproc-per-node N bench.py --gpus N`` on a whole node; nothing
of that path (rendezvous, slab split, ZSlabOp Function, barrier + max-over-ranks timing, the JSON line)
may first execute there. Two ranks share cuda:0 over ``gloo`` (RCCL refuses two ranks on one device);
the launcher is a fresh child process, never an exec of this (GPU-initialised) interpreter.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('nproc,workload', [(2, 'diffusion7_f32'), (2, 'stencil27_f16')])
def test_bench_two_ranks_end_to_end(nproc, workload):
    env = dict(os.environ, PSAD_DIST_BACKEND='gloo', HSA_ENABLE_IPC_MODE_LEGACY='0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(ROOT, 'bench.py'), '--gpus', str(nproc), '--edge', '128', '--steps', '3', '--warmup', '1',
           '--workload', workload, '--cpu-seconds', '1', '--secondary-edge', '96']
    t0 = time.perf_counter()
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    assert proc.returncode == 0, proc.stdout[-3000:] + proc.stderr[-3000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, proc.stdout
    res = json.loads(lines[0])
    assert res['n_gpus'] == nproc
    assert res['config']['decomposition'] == f'z-slab x{nproc}'
    assert res['steps'] == 3 and res['value'] > 0
    assert res['ms_per_step'] * res['steps'] / 1e3 <= wall
    assert res['value'] == pytest.approx(128 ** 3 * 3 / (res['ms_per_step'] * 3 / 1e3) / 1e6, rel=1e-3)
    assert res['config']['name'] == workload
    assert res['metric'].endswith('128^3') and ('27-point fp16' in res['metric']) == (workload == 'stencil27_f16')
    rl = res['roofline']
    bpc = 8 if workload == 'diffusion7_f32' else 4
    assert rl['bytes_per_launch'] == bpc * 64 * 128 * 128 and rl['bytes_per_step'] == 2 * bpc * 128 ** 3
    # frac is the step-level figure: both sweeps' algorithmic bytes / ms_per_step / (N x peak)
    step_frac = 2 * bpc * 128 ** 3 / (res['ms_per_step'] * 1e-3) / 1e9 / (rl['peak'] * nproc)
    assert rl['frac'] == pytest.approx(step_frac, rel=1e-2) and rl['frac_fwd'] > 0 and rl['frac_bwd'] > 0
    assert rl['traffic'] is None            # no PMC entry for a slab-shaped launch: never the 1-GPU figure
    # rank 0 times the CPU path after the timed loop at every N (north_star: "in the same run")
    if workload == 'diffusion7_f32':            # config 5 timed in the same run (the driver's scaling runs)
        sec = res['secondary']
        assert sec['name'] == 'stencil27_f16' and sec['n_gpus'] == nproc and sec['value'] > 0
        assert sec['decomposition'] == f'z-slab x{nproc}' and sec['cells'] == 96 ** 3
    else:
        assert 'secondary' not in res
    cpu = res['cpu_baseline']
    assert cpu is not None and cpu['value'] > 0 and cpu['cores'] == 1 and cpu['kind'] == 'port', cpu
