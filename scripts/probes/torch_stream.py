"""torch's own streaming kernels over a config's bytes (the memory-pattern ceiling a sweep is compared with):
``out = u * c`` (one read + one write of the field) and ``copy_``, fp16 and fp32, HIP events, settled.

python scripts/probes/torch_stream.py N [N ...]      (N^3 fields)
"""
import sys
import time

import torch


def timeit(fn, n=50):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    for n in [int(v) for v in sys.argv[1:]] or [768]:
        for dt in (torch.float16, torch.float32):
            u = torch.rand((n, n, n), device='cuda').to(dt)
            out = torch.empty_like(u)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.5:
                torch.mul(u, 0.5, out=out)
            nbytes = 2 * u.numel() * u.element_size()
            for name, fn in (('mul', lambda: torch.mul(u, 0.5, out=out)), ('copy_', lambda: out.copy_(u))):
                ms = min(timeit(fn) for _ in range(3))
                print(f'{n}^3 {str(dt):14s} {name:6s} {ms:.4f} ms  {nbytes / ms / 1e9:.3f} TB/s', flush=True)


if __name__ == '__main__':
    main()
