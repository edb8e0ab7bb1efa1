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


@pytest.mark.parametrize('nproc', [2])
def test_bench_two_ranks_end_to_end(nproc):
    env = dict(os.environ, PSAD_DIST_BACKEND='gloo', HSA_ENABLE_IPC_MODE_LEGACY='0')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(ROOT, 'bench.py'), '--gpus', str(nproc), '--edge', '128', '--steps', '3', '--warmup', '1']
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
    assert res['cpu_baseline'] is None          # rank 0 times the CPU only at N=1
