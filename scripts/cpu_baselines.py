"""CPU baselines of the BASELINE configs on the GPU box's host: the oracle's C restatement of the
reference CPU loop nest (oracle/stencil_ref.c, gcc -O3 -march=native -fopenmp), 1 thread (the reference
default) and all threads of the box (OMP_NUM_THREADS, cpu_openmp=True), on bounded slabs of each
config. One JSON line per (config, threads). Run: python scripts/cpu_baselines.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(name, shape, seconds):
    import numpy as np
    from oracle import cref
    from pystencils_autodiff_amd import workloads as W
    lib = cref.load(build_dir=os.path.join(ROOT, 'oracle', 'build_native'), march='native')
    rng = np.random.default_rng(0)
    if name.startswith('stencil27'):
        u = rng.uniform(0, 1, shape).astype(np.float16)
        d = rng.uniform(-1, 1, shape).astype(np.float16)
        w = np.asarray(W.WEIGHTS_27PT, dtype=np.float32)
        wb = w.reshape(3, 3, 3)[::-1, ::-1, ::-1].reshape(-1).copy()    # adjoint: flipped taps
        sweep = (lambda: lib.stencil27_f16(u, w), lambda: lib.stencil27_f16(d, wb))
    else:
        u = rng.uniform(0, 1, shape).astype(np.float32)
        d = rng.uniform(-1, 1, shape).astype(np.float32)
        out, du = np.empty_like(u), np.empty_like(u)
        sweep = (lambda: lib.diffusion7_f32(u, 0.1, out), lambda: lib.diffusion7_f32(d, 0.1, du))
    sweep[0]()
    reps, t0 = 0, time.perf_counter()
    while True:
        sweep[0]()
        sweep[1]()
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    cells = reps * int(np.prod(shape))
    print(json.dumps({'config': name, 'sample_shape': list(shape), 'threads': int(os.environ['OMP_NUM_THREADS']),
                      'fwd_bwd_sweeps': reps, 'seconds': round(el, 2), 'mcells_per_s': round(cells / el / 1e6, 1)}))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        child(sys.argv[2], tuple(int(v) for v in sys.argv[3].split(',')), float(sys.argv[4]))
        return
    mt = int(os.environ.get('OMP_NUM_THREADS', '0')) or len(os.sched_getaffinity(0))
    cfgs = [('diffusion7_f32_512^3', '32,512,512'), ('diffusion7_f32_1024^3', '16,1024,1024'),
            ('stencil27_f16_768^3', '16,768,768')]
    for name, shape in cfgs:
        for threads in (1, mt):
            env = dict(os.environ, OMP_NUM_THREADS=str(threads))
            subprocess.run([sys.executable, __file__, 'child', name, shape, '6' if threads == 1 else '4'],
                           env=env, check=True)


if __name__ == '__main__':
    main()
