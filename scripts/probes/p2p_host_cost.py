"""Host cost of the halo-exchange call pattern on the RCCL backend, measured with world_size 1
(send/recv to self): batch_isend_irecv of two 4 MiB faces each way + wait(), and the same inside
a zslab-shaped step (interior launch, exchange, face launch)."""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    n = 1024
    t = torch.rand((8, n, n), device='cuda')
    lo = torch.empty((1, n, n), device='cuda')
    hi = torch.empty((1, n, n), device='cuda')

    def exchange():
        ops = [dist.P2POp(dist.isend, t[:1], 0), dist.P2POp(dist.irecv, lo, 0),
               dist.P2POp(dist.isend, t[-1:], 0), dist.P2POp(dist.irecv, hi, 0)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()

    for _ in range(20):
        exchange()
    torch.cuda.synchronize()
    for reps in (200,):
        t0 = time.perf_counter()
        for _ in range(reps):
            exchange()
        host = (time.perf_counter() - t0) / reps * 1e6
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps * 1e6
        print(f'exchange: host {host:.1f} us per call, wall incl. GPU {wall:.1f} us per call')
    assert torch.equal(lo[0], t[0]) and torch.equal(hi[0], t[-1])
    import sys
    sys.path.insert(0, '.')
    from pystencils_autodiff_amd.zslab import RcclHalo
    halo = RcclHalo(loopback=True)
    plane = n * n * 4
    planes = [(t.data_ptr(), lo.data_ptr(), t.data_ptr() + 7 * plane, hi.data_ptr(), plane)]
    cur = torch.cuda.current_stream()

    def exchange_c():
        halo.stream.wait_stream(cur)
        halo.exchange(planes, 0, 0)
        cur.wait_stream(halo.stream)
    lo.zero_()
    hi.zero_()
    for _ in range(20):
        exchange_c()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        exchange_c()
    host = (time.perf_counter() - t0) / 200 * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 200 * 1e6
    print(f'psad_halo_exchange (+2 stream waits): host {host:.1f} us per call, wall incl. GPU {wall:.1f} us per call')
    assert torch.equal(lo[0], t[0]) and torch.equal(hi[0], t[-1])
    halo.close()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
