"""Z-slab decomposition with halo exchange (world_size 2 and 3, gloo).

CPU: the C kernels on ghosted copies. GPU (marked): two gloo ranks share cuda:0 and run the
HIP march kernel with halo planes read in place and the interior/boundary z-range split —
the same code path the RCCL bench runs on 8 GPUs.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _dtype(builder_name):
    return np.float16 if builder_name == 'stencil_27pt' else np.float32


class _GlooHalo:
    """Stand-in for zslab.RcclHalo with RcclHalo's exchange contract (device pointers, peers, its own
    stream) carried over gloo through host staging: drives ZSlabOp._sweep_rccl — peers, face
    pointers, stream order, the two-range face launch — with 2-3 real ranks on one GPU, which RCCL
    itself refuses."""
    loopback = False

    def __init__(self):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = torch.device('cuda', torch.cuda.current_device())
        self.stream = torch.cuda.Stream()
        self.ev_faces, self.ev_halos = torch.cuda.Event(), torch.cuda.Event()

    def exchange(self, planes, peer_lo, peer_hi):
        from pystencils_autodiff_amd.backends import hip_runtime as rt
        L, s = rt.lib(), self.stream.cuda_stream

        def stage_out(ptr, n):
            t = torch.empty(n, dtype=torch.uint8, device=self.device)
            rt._check(L.psad_memcpy_d2d_async(t.data_ptr(), ptr, n, s), 'stage')
            return t
        self.stream.synchronize()          # the faces are final (the caller made this stream wait)
        ops, recvs = [], []
        for send_lo, recv_lo, send_hi, recv_hi, n in planes:
            for peer, snd, rcv in ((peer_lo, send_lo, recv_lo), (peer_hi, send_hi, recv_hi)):
                if peer < 0:
                    continue
                out = stage_out(snd, n)
                self.stream.synchronize()
                ops.append(dist.P2POp(dist.isend, out.cpu(), peer))
                buf = torch.empty(n, dtype=torch.uint8)
                ops.append(dist.P2POp(dist.irecv, buf, peer))
                recvs.append((buf, rcv, n))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for buf, rcv, n in recvs:
            d = buf.to(self.device)
            torch.cuda.current_stream().synchronize()
            rt._check(L.psad_memcpy_d2d_async(rcv, d.data_ptr(), n, s), 'unstage')
        self.stream.synchronize()

    def close(self):
        pass


def _worker(rank, world, port, shape, builder_name, use_cuda, result_dir, opts=None):
    opts = opts or {}
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import ZSlabOp, slab_bounds
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        builder = getattr(W, builder_name)
        op = pa.AutoDiffOp(builder(), boundary_handling=opts.get('bh', 'zeros'),
                           diff_fields_prefix=opts.get('prefix', 'diff'))
        rng = np.random.default_rng(0)
        dt = _dtype(builder_name)
        u = rng.uniform(0, 1, shape).astype(dt)
        d = rng.uniform(-1, 1, shape).astype(dt)
        lo, hi = slab_bounds(shape[0], world, rank)
        dev = 'cuda' if use_cuda else 'cpu'
        ul = torch.from_numpy(u[lo:hi].copy()).to(dev)
        dl = torch.from_numpy(d[lo:hi].copy()).to(dev)
        out = torch.zeros_like(ul)
        du = torch.zeros_like(ul)
        z = ZSlabOp(op, use_cuda=use_cuda)
        if os.environ.get('PSAD_TEST_EMULATED_RCCL'):
            z._halo = _GlooHalo()
            # the setup exchange bench.py runs before its timed loop: real peers, per-rank slab shapes
            # (remainder planes) and receive buffers the sweeps below then reuse
            z.warm_exchange(**{'u': ul, op.adjoint_name(op.forward_output_fields[0]): dl})
        if os.environ.get('PSAD_TEST_ZSLAB_AUTOGRAD'):
            fn = z.autograd_function()
            uu = ul.clone().requires_grad_(True)
            (o,) = fn.apply(uu)
            o.backward(dl)
            out.copy_(o.detach())
            du.copy_(uu.grad)
        else:
            p = opts.get('prefix', 'diff')
            z.fwd(u=ul, out=out)
            z.bwd(**{p + 'out': dl, p + 'u': du})
        if use_cuda:
            torch.cuda.synchronize()
        np.save(os.path.join(result_dir, f'out_{rank}.npy'), out.cpu().numpy())
        np.save(os.path.join(result_dir, f'du_{rank}.npy'), du.cpu().numpy())
    finally:
        dist.destroy_process_group()


def _run(world, shape, builder_name, use_cuda, tmp_path, **opts):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, shape, builder_name, use_cuda, str(tmp_path), opts), nprocs=world,
             join=True)
    out = np.concatenate([np.load(tmp_path / f'out_{r}.npy') for r in range(world)])
    du = np.concatenate([np.load(tmp_path / f'du_{r}.npy') for r in range(world)])
    from oracle import stencils as S
    taps = {'diffusion_7pt': S.taps_diffusion_7pt(), 'asym_7pt': S.taps_asym_7pt(),
            'stencil_27pt': S.taps_27pt()}[builder_name]
    rng = np.random.default_rng(0)
    dt = _dtype(builder_name)
    u = rng.uniform(0, 1, shape).astype(dt)
    d = rng.uniform(-1, 1, shape).astype(dt)
    ref_out, ref_du = S.linear_stencil(u, taps), S.linear_stencil(d, S.flip(taps))
    if opts.get('bh', 'zeros') is None:
        # interior-only kernels (_autodiff.py:485-486,518-519): interior cells read only in-domain
        # neighbours, so they equal the 'zeros' values; the radius-1 border keeps torch.zeros
        ref_out, ref_du = _interior(ref_out, 1), _interior(ref_du, 1)
    return out, du, ref_out, ref_du


def _interior(a, g):
    b = np.zeros_like(a)
    sl = tuple(slice(g, n - g) for n in a.shape)
    b[sl] = a[sl]
    return b


@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('world,shape', [(2, (10, 9, 12)), (3, (13, 6, 7))])
@pytest.mark.parametrize('builder_name', ['asym_7pt', 'diffusion_7pt'])
def test_zslab_gloo_cpu(world, shape, builder_name, bh, tmp_path):
    from tests.conftest import assert_close_rel
    out, du, ref_out, ref_du = _run(world, shape, builder_name, False, tmp_path, bh=bh)
    assert_close_rel(out, ref_out, 1e-6, 'out')
    assert_close_rel(du, ref_du, 1e-6, 'diffu')


@pytest.mark.parametrize('bh,prefix', [('zeros', 'diff'), ('zeros', 'grad'), (None, 'grad')])
def test_zslab_autograd_function_gloo_cpu(tmp_path, monkeypatch, bh, prefix):
    """The slab Function with the reference's own keyword surface: a non-default ``diff_fields_prefix``
    (adjoint names from the op's field map, ``_autodiff.py:81-84``) and the default boundary (None)."""
    from tests.conftest import assert_close_rel
    monkeypatch.setenv('PSAD_TEST_ZSLAB_AUTOGRAD', '1')
    out, du, ref_out, ref_du = _run(2, (11, 8, 9), 'asym_7pt', False, tmp_path, bh=bh, prefix=prefix)
    assert_close_rel(out, ref_out, 1e-6, 'out')
    assert_close_rel(du, ref_du, 1e-6, 'diffu')


def test_zslab_none_mode_thin_edge_slabs(tmp_path):
    """boundary_handling=None with 4 ranks on 6 planes: the edge ranks hold a single global-border plane
    plus one interior plane, the inner ranks read both neighbours' faces."""
    from tests.conftest import assert_close_rel
    out, du, ref_out, ref_du = _run(4, (7, 6, 9), 'diffusion_7pt', False, tmp_path, bh=None)
    assert_close_rel(out, ref_out, 1e-6, 'out')
    assert_close_rel(du, ref_du, 1e-6, 'diffu')


def test_slab_bounds_cover_domain():
    from pystencils_autodiff_amd.zslab import slab_bounds
    for n in (1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            b = [slab_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h - lo for lo, h in b) - min(h - lo for lo, h in b) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize('bh', ['zeros', None])
@pytest.mark.parametrize('world,shape', [(2, (24, 40, 64)), (3, (19, 33, 70))])
@pytest.mark.parametrize('builder_name', ['asym_7pt', 'diffusion_7pt'])
def test_zslab_gloo_gpu_halo_path(world, shape, builder_name, bh, tmp_path):
    from tests.conftest import assert_close_rel
    out, du, ref_out, ref_du = _run(world, shape, builder_name, True, tmp_path, bh=bh)
    assert_close_rel(out, ref_out, 1e-6, 'out')
    assert_close_rel(du, ref_du, 1e-6, 'diffu')


@pytest.mark.gpu
def test_rccl_c_abi_self_exchange():
    """psad_halo_exchange through a one-rank RCCL communicator, both faces sent to itself: the
    receive buffers hold the slab's own first / last planes (pointer math, group, stream)."""
    import ctypes
    import sys
    sys.path.insert(0, ROOT)
    from pystencils_autodiff_amd.zslab import RcclHalo
    halo = RcclHalo(loopback=True)
    try:
        t = torch.rand((7, 33, 40), device='cuda')
        v = torch.rand((7, 33, 40), device='cuda')
        bufs = [torch.full((2, 33, 40), -1.0, device='cuda') for _ in range(4)]
        nb = 2 * 33 * 40 * 4
        plane = 33 * 40 * 4
        halo.stream.wait_stream(torch.cuda.current_stream())
        halo.exchange([(t.data_ptr(), bufs[0].data_ptr(), t.data_ptr() + 5 * plane, bufs[1].data_ptr(), nb),
                       (v.data_ptr(), bufs[2].data_ptr(), v.data_ptr() + 5 * plane, bufs[3].data_ptr(), nb)], 0, 0)
        halo.stream.synchronize()
        assert torch.equal(bufs[0], t[:2]) and torch.equal(bufs[1], t[-2:])
        assert torch.equal(bufs[2], v[:2]) and torch.equal(bufs[3], v[-2:])
        assert ctypes is not None
    finally:
        halo.close()


@pytest.mark.gpu
@pytest.mark.parametrize('builder_name,shape', [('asym_7pt', (12, 40, 70)), ('diffusion_7pt', (3, 17, 64)),
                                                ('diffusion_7pt', (2, 9, 64)), ('diffusion_7pt', (1, 9, 64)),
                                                ('stencil_27pt', (9, 24, 80))])
def test_zslab_rccl_loopback_sweep(builder_name, shape):
    """The RCCL sweep (faces out on the halo stream, interior launch, wait, one two-range face launch)
    on one GPU with a loopback communicator: equals the stencil with a periodic z boundary."""
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from oracle import stencils as S
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp
    from tests.conftest import assert_close_rel
    op = pa.AutoDiffOp(getattr(W, builder_name)(), boundary_handling='zeros')
    taps = {'diffusion_7pt': S.taps_diffusion_7pt(), 'asym_7pt': S.taps_asym_7pt(),
            'stencil_27pt': S.taps_27pt()}[builder_name]
    dt = np.float16 if builder_name == 'stencil_27pt' else np.float32
    tol = 1e-3 if dt == np.float16 else 1e-6
    rng = np.random.default_rng(5)
    u = rng.uniform(0, 1, shape).astype(dt)
    d = rng.uniform(-1, 1, shape).astype(dt)
    z = ZSlabOp(op, use_cuda=True)
    z._halo = RcclHalo(loopback=True)
    try:
        tu, td = torch.from_numpy(u).cuda(), torch.from_numpy(d).cuda()
        out, du = torch.empty_like(tu), torch.empty_like(td)
        z.warm_exchange(u=tu, diffout=td)      # setup exchange: the sweeps reuse its receive buffers
        for which, kw in (('forward', dict(u=tu, out=out)), ('backward', dict(diffout=td, diffu=du))):
            k = z.kernels[which]
            z._sweep_rccl(k, z._halo, k.ir.stencil_fields, 1, kw)
        torch.cuda.synchronize()

        def periodic(a, tp):
            a64 = a.astype(np.float64)
            ext = np.concatenate([a64[-1:], a64, a64[:1]])
            return S.linear_stencil(ext, tp)[1:-1]
        assert_close_rel(out.cpu().numpy().astype(np.float64), periodic(u, taps), tol, 'out')
        assert_close_rel(du.cpu().numpy().astype(np.float64), periodic(d, S.flip(taps)), tol, 'diffu')
    finally:
        z.close()


@pytest.mark.gpu
@pytest.mark.parametrize('world,shape,bh', [(2, (24, 40, 64), 'zeros'), (3, (19, 33, 70), 'zeros'),
                                            (3, (7, 9, 64), 'zeros'), (3, (19, 33, 70), None),
                                            (3, (7, 9, 64), None)])
@pytest.mark.parametrize('builder_name', ['asym_7pt', 'stencil_27pt'])
def test_zslab_rccl_sweep_emulated_ranks(world, shape, builder_name, bh, tmp_path, monkeypatch):
    """ZSlabOp's RCCL sweep with 2-3 ranks on one GPU, the exchange carried by _GlooHalo (after the
    setup exchange bench.py runs, ``warm_exchange``), both boundary modes."""
    from tests.conftest import assert_close_rel
    monkeypatch.setenv('PSAD_TEST_EMULATED_RCCL', '1')
    out, du, ref_out, ref_du = _run(world, shape, builder_name, True, tmp_path, bh=bh)
    tol = 1e-3 if builder_name == 'stencil_27pt' else 1e-6
    assert_close_rel(out, ref_out, tol, 'out')
    assert_close_rel(du, ref_du, tol, 'diffu')


def _rccl_agreement_worker(rank, world, port, result_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    if rank == 1:   # this rank cannot open librccl; rank 0 can
        os.environ['PSAD_RCCL_LIBRARY'] = '/nonexistent/librccl.so'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from pystencils_autodiff_amd.zslab import RcclHalo, RcclUnavailable
        try:
            RcclHalo()
            outcome = 'constructed'
        except RcclUnavailable:
            outcome = 'unavailable'
        with open(os.path.join(result_dir, f'rccl_{rank}.txt'), 'w') as fh:
            fh.write(outcome)
    finally:
        dist.destroy_process_group()


def test_rccl_open_failure_is_agreed_by_every_rank(tmp_path):
    """A rank that cannot open librccl makes EVERY rank raise RcclUnavailable before the unique-id
    broadcast (none is left waiting in a collective); ZSlabOp then uses batch_isend_irecv."""
    pytest.importorskip('pystencils_autodiff_amd.backends.hip_runtime')
    from pystencils_autodiff_amd.backends import hip_runtime as rt
    try:
        rt.lib()
    except Exception as exc:  # noqa: BLE001
        pytest.skip(f'libpsad_hip.so not built: {exc}')
    mp.spawn(_rccl_agreement_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f'rccl_{r}.txt').read() for r in range(2)] == ['unavailable', 'unavailable']


# --- fzyx (SoA) vector fields: one face pair and one halo pair per component ----------------------------------

def _vector_ac(layout):
    """Two coupled components, asymmetric along z (a swapped lower / upper halo shows) and one product term (the
    adjoint then reads the forward input too: two stencil fields exchanged per backward sweep)."""
    import sys
    sys.path.insert(0, ROOT)
    from pystencils_autodiff_amd import ps
    u, out = ps.fields("u(2), out(2): float32[3d]", layout=layout)
    return ps.AssignmentCollection([
        ps.Assignment(out.center(0), u[-1, 0, 0](1) - 0.5 * u[1, 0, 0](0) + 0.25 * u[0, 1, 0](0) + 0.1 * u[0, 0, -1](1)),
        ps.Assignment(out.center(1), 0.75 * u[1, 0, 0](1) + u[-1, 0, 0](0) * u[0, 0, 0](1))])


def _vector_data(shape):
    rng = np.random.default_rng(11)
    return (rng.uniform(-1, 1, shape + (2,)).astype(np.float32), rng.uniform(-1, 1, shape + (2,)).astype(np.float32))


def _vector_worker(rank, world, port, shape, layout, bh, mode, use_cuda, result_dir):
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd.zslab import ZSlabOp, slab_bounds
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        op = pa.AutoDiffOp(_vector_ac(layout), boundary_handling=bh)
        u, d = _vector_data(shape)
        lo, hi = slab_bounds(shape[0], world, rank)
        dev = 'cuda' if use_cuda else 'cpu'

        def slab(a):
            t = torch.from_numpy(a[lo:hi].copy()).to(dev)
            return t.permute(3, 0, 1, 2).contiguous().permute(1, 2, 3, 0) if layout == 'fzyx' else t
        ul, dl = slab(u), slab(d)
        z = ZSlabOp(op, use_cuda=use_cuda)
        if mode == 'rccl':
            z._halo = _GlooHalo()
            z.warm_exchange(u=ul, diffout=dl)
        if mode == 'autograd':
            fn = z.autograd_function()
            uu = ul.clone().requires_grad_(True)
            (o,) = fn.apply(uu)
            o.backward(dl)
            out, du = o.detach(), uu.grad
        else:
            fk, bk = z.kernels['forward'], z.kernels['backward']
            out = z._alloc(fk, 'out', ul, ul.dtype, False)
            du = z._alloc(bk, 'diffu', ul, ul.dtype, 'diffu' in {r.field.name for r in bk.ir.reads})
            z.fwd(u=ul, out=out)
            bw = {'u': ul, 'diffout': dl, 'diffu': du}
            z.bwd(**{n: v for n, v in bw.items() if n in {f.name for f in bk.ir.fields}})
        if use_cuda:
            torch.cuda.synchronize()
        soa = [tuple(t.stride()) == (t.shape[1] * t.shape[2], t.shape[2], 1, t.shape[0] * t.shape[1] * t.shape[2])
               for t in (out, du)]
        np.save(os.path.join(result_dir, f'out_{rank}.npy'), out.cpu().numpy())
        np.save(os.path.join(result_dir, f'du_{rank}.npy'), du.cpu().numpy())
        np.save(os.path.join(result_dir, f'soa_{rank}.npy'), np.array(soa))
    finally:
        dist.destroy_process_group()


def _run_vector(world, shape, layout, bh, mode, use_cuda, tmp_path):
    mp.spawn(_vector_worker, args=(world, _free_port(), shape, layout, bh, mode, use_cuda, str(tmp_path)),
             nprocs=world, join=True)
    out = np.concatenate([np.load(tmp_path / f'out_{r}.npy') for r in range(world)])
    du = np.concatenate([np.load(tmp_path / f'du_{r}.npy') for r in range(world)])
    soa = [bool(v) for r in range(world) for v in np.load(tmp_path / f'soa_{r}.npy')]
    import pystencils_autodiff_amd as pa
    from oracle import evaluate as OE
    op = pa.AutoDiffOp(_vector_ac(layout), boundary_handling=bh)
    u, d = _vector_data(shape)
    ref = OE.evaluate(op.forward_assignments, {'u': u}, boundary_handling=bh)['out']
    refb = OE.evaluate(op.backward_assignments, {'u': u, 'diffout': d}, boundary_handling=bh)['diffu']
    return out, du, ref, refb, soa


@pytest.mark.parametrize('world,shape,bh,mode', [(2, (9, 6, 7), 'zeros', 'sweep'), (3, (10, 5, 8), None, 'sweep'),
                                                 (2, (8, 6, 5), 'zeros', 'autograd'), (2, (9, 7, 6), None, 'autograd')])
def test_zslab_fzyx_vector_gloo_cpu(world, shape, bh, mode, tmp_path):
    """z-slabs of an fzyx vector field (C kernels on ghosted copies): forward and adjoint vs the oracle on the
    undivided field, results in fzyx order."""
    from tests.conftest import assert_close_rel
    out, du, ref, refb, soa = _run_vector(world, shape, 'fzyx', bh, mode, False, tmp_path)
    assert_close_rel(out, ref, 1e-6, 'out')
    assert_close_rel(du, refb, 1e-6, 'diffu')
    assert all(soa)


@pytest.mark.gpu
@pytest.mark.parametrize('world,shape,bh,mode', [(2, (12, 20, 64), 'zeros', 'sweep'), (3, (13, 17, 70), None, 'sweep'),
                                                 (2, (12, 20, 64), 'zeros', 'rccl'), (3, (13, 17, 70), None, 'rccl'),
                                                 (2, (10, 9, 64), 'zeros', 'autograd'),
                                                 (3, (11, 9, 40), None, 'autograd')])
def test_zslab_fzyx_vector_gpu(world, shape, bh, mode, tmp_path):
    """z-slabs of an fzyx 2-component field on the HIP kernels (ranks sharing one GPU): one face pair per component
    exchanged, one halo pair per component field read by the march kernels; the torch exchange ('sweep',
    'autograd') and the RCCL sweep's exchange contract ('rccl', carried by _GlooHalo)."""
    from tests.conftest import assert_close_rel
    out, du, ref, refb, soa = _run_vector(world, shape, 'fzyx', bh, mode, True, tmp_path)
    assert_close_rel(out, ref, 1e-6, 'out')
    assert_close_rel(du, refb, 1e-6, 'diffu')
    assert all(soa)


# --- BASELINE configs 4 and 5 in their 8-way z-slab form, full size, 8 ranks sharing one GPU -------------------

def _hash_unit(idx, seed, xp):
    """A counter-based hash of the global cell index → [0, 1) (24 bits), identical in torch (on the GPU, per
    slab) and numpy (the oracle's 3-plane neighbourhoods): no rank ever holds the global field."""
    h = idx * 2654435761 + seed * 40503
    h = (h ^ (h >> 16)) & 0x7FFFFFFF
    h = h * 0x45D9F3B
    h = (h ^ (h >> 16)) & 0x7FFFFFFF
    h = h * 0x45D9F3B
    h = (h ^ (h >> 16)) & 0xFFFFFF
    return h.to(xp.float64) / float(1 << 24) if hasattr(h, 'to') else h.astype(xp.float64) / float(1 << 24)


def _synth_planes(z0, z1, Y, X, seed, dtype, signed):
    """numpy: planes [z0, z1) of the synthetic field, rounded to the storage dtype (float64 values)."""
    idx = np.arange(z0 * Y * X, z1 * Y * X, dtype=np.int64)
    v = _hash_unit(idx, seed, np)
    v = 2 * v - 1 if signed else v
    return v.astype(dtype).astype(np.float64).reshape(z1 - z0, Y, X)


def _full_size_worker(rank, world, port, builder_name, edge, result_dir):
    import json
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import ZSlabOp, slab_bounds
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dt = torch.float16 if builder_name == 'stencil_27pt' else torch.float32
        lo, hi = slab_bounds(edge, world, rank)
        idx = torch.arange(lo * edge * edge, hi * edge * edge, dtype=torch.int64, device='cuda')
        ul = _hash_unit(idx, 1, torch).to(dt).view(hi - lo, edge, edge)
        dl = (2 * _hash_unit(idx, 2, torch) - 1).to(dt).view(hi - lo, edge, edge)
        del idx
        op = pa.AutoDiffOp(getattr(W, builder_name)(), boundary_handling='zeros')
        z = ZSlabOp(op, use_cuda=True)
        z._halo = _GlooHalo()                 # RcclHalo's contract, carried over gloo (RCCL: one rank per GPU)
        z.warm_exchange(u=ul, diffout=dl)
        fn = z.autograd_function()
        uu = ul.clone().requires_grad_(True)
        (o,) = fn.apply(uu)
        o.backward(dl)
        torch.cuda.synchronize()
        du = uu.grad
        for name, t in (('out', o.detach()), ('du', du)):
            np.save(os.path.join(result_dir, f'{name}_{rank}.npy'),
                    torch.stack([t[0], t[-1]]).float().cpu().numpy())
        # the global adjoint identity <A u, d> = <u, A^T d> over every cell of every slab
        dots = torch.stack([(o.detach().double() * dl.double()).sum(), (ul.double() * du.double()).sum(),
                            o.detach().double().abs().sum(), torch.isfinite(o.detach()).all().double(),
                            torch.isfinite(du).all().double()]).cpu()
        dist.all_reduce(dots)
        if rank == 0:
            with open(os.path.join(result_dir, 'dots.json'), 'w') as fh:
                json.dump([float(v) for v in dots], fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize('builder_name,edge', [('diffusion_7pt', 1024), ('stencil_27pt', 768)],
                         ids=['config4_7pt_f32_1024', 'config5_27pt_f16_768'])
def test_zslab_full_size_eight_ranks_emulated(builder_name, edge, tmp_path):
    """BASELINE configs 4 and 5 as configured: the full 1024³ fp32 7-point / 768³ fp16 27-point domain split
    into 8 z-slabs (128 / 96 planes), 8 ranks sharing one GPU, each driving ``ZSlabOp.autograd_function()``
    apply + backward with the RCCL sweep (faces on the halo stream, interior launch, two-range face launch),
    the exchange carried by ``_GlooHalo``. Every rank's first and last planes of the output and of the
    gradient — both global faces and all 14 slab-boundary planes — vs the float64 oracle on their 3-plane
    neighbourhoods, and the global adjoint identity over all cells."""
    import json
    world = 8
    from oracle import stencils as S
    from pystencils_autodiff_amd.zslab import slab_bounds
    from tests.conftest import assert_cells, assert_close_rel
    mp.spawn(_full_size_worker, args=(world, _free_port(), builder_name, edge, str(tmp_path)), nprocs=world,
             join=True)
    f16 = builder_name == 'stencil_27pt'
    dt = np.float16 if f16 else np.float32
    taps = S.taps_27pt() if f16 else S.taps_diffusion_7pt()
    tol = 1e-3 if f16 else 1e-6

    def ref_plane(p, seed, signed, tp):
        """(the oracle's plane p, Σ|w·u| per cell: the same stencil with |w| on |u|)"""
        a, b = max(0, p - 1), min(edge, p + 2)
        block = np.zeros((3, edge, edge))
        block[a - (p - 1):b - (p - 1)] = _synth_planes(a, b, edge, edge, seed, dt, signed)
        absw = {o: abs(w) for o, w in tp.items()}
        return S.linear_stencil(block, tp)[1], S.linear_stencil(np.abs(block), absw)[1]
    for r in range(world):
        lo, hi = slab_bounds(edge, world, r)
        assert hi - lo == edge // world
        out, du = np.load(tmp_path / f'out_{r}.npy'), np.load(tmp_path / f'du_{r}.npy')
        for k, p in enumerate((lo, hi - 1)):
            for got, (ref, absr), name in ((out[k], ref_plane(p, 1, False, taps), 'out'),
                                           (du[k], ref_plane(p, 2, True, S.flip(taps)), 'diffu')):
                assert_close_rel(got, ref, tol, f'rank {r} {name} plane {p}')
                # element-wise: the north star's relative error plus the fp32 sum bound (+ half an fp16 ulp)
                assert_cells(got, ref, absr, len(taps), dt, f'rank {r} {name} plane {p}')
    ad, ua, mass, fin_o, fin_d = json.load(open(tmp_path / 'dots.json'))
    assert fin_o == world and fin_d == world
    assert mass > 0
    assert abs(ad - ua) <= (5e-3 if f16 else 1e-5) * max(abs(ad), abs(ua)), (ad, ua)


@pytest.mark.gpu
def test_zslab_native_plan_on_two_streams(monkeypatch):
    """One native slab plan applied from two compute streams: the signal-memory ordering
    (``hipStreamWriteValue32`` of a sweep counter, the halo stream waiting for ``>=``) holds only while one stream
    writes the counter, so the plan keeps it for the stream it first ran on and a sweep enqueued on another stream
    orders through event record + wait. Results bitwise equal on both streams, the second stream's two sweeps on the
    event path, the first stream back on the signals afterwards."""
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import _psad_torch
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp
    monkeypatch.delenv('PSAD_SLAB_SYNC', raising=False)
    monkeypatch.setenv('PSAD_NATIVE_SLAB', '1')
    op = pa.AutoDiffOp(W.diffusion_7pt(), boundary_handling='zeros')
    g = torch.Generator().manual_seed(9)
    tu = torch.rand((16, 40, 128), generator=g).cuda()
    td = (torch.rand((16, 40, 128), generator=g) * 2 - 1).cuda()
    z = ZSlabOp(op, use_cuda=True)
    z._halo = RcclHalo(loopback=True)
    try:
        z.warm_exchange(u=tu, diffout=td)
        fn = z.autograd_function()

        def step():
            uu = tu.clone().requires_grad_(True)
            (o,) = fn.apply(uu)
            assert 'CppNode' in o.grad_fn.name(), o.grad_fn.name()
            o.backward(td)
            return o.detach().clone(), uu.grad.clone()
        ref = step()
        torch.cuda.synchronize()
        n0 = _psad_torch.num_event_sweeps()
        s2 = torch.cuda.Stream()
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            other = step()
        torch.cuda.current_stream().wait_stream(s2)
        n1 = _psad_torch.num_event_sweeps()
        again = step()
        torch.cuda.synchronize()
        assert n1 - n0 == 2, (n0, n1)
        assert _psad_torch.num_event_sweeps() == n1
        for a, b in ((ref, other), (ref, again)):
            assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    finally:
        z.close()


@pytest.mark.gpu
@pytest.mark.parametrize('face_wait', ['0', '1'], ids=['faces-halo-stream', 'faces-wait-in-kernel'])
@pytest.mark.parametrize('builder_name,shape', [('asym_7pt', (12, 40, 70)), ('diffusion_7pt', (2, 9, 64)),
                                                ('stencil_27pt', (9, 24, 80)), ('stencil_27pt', (96, 64, 256)),
                                                ('diffusion_7pt', (40, 64, 256))])
def test_zslab_native_node_loopback(builder_name, shape, face_wait, monkeypatch):
    """The slab Function through the native node (``_psad_torch.apply_slab``: RCCL group, stream events, interior
    and face launches in C++) on a loopback communicator: the periodic-z oracle, and bitwise the Python Function's
    sweeps (``PSAD_NATIVE_SLAB=0``) on the same inputs; a second call reuses the plan. ``face_wait``: the face
    launches on the halo stream behind the exchange, or (``PSAD_SLAB_FACE_WAIT=1``) on the compute stream behind the
    interior with their loader waves waiting in-kernel for the halo stream's word (schedules with an LDS-DMA loader)."""
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from oracle import stencils as S
    from pystencils_autodiff_amd import _psad_torch
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import RcclHalo, ZSlabOp
    from tests.conftest import assert_close_rel
    op = pa.AutoDiffOp(getattr(W, builder_name)(), boundary_handling='zeros')
    taps = {'diffusion_7pt': S.taps_diffusion_7pt(), 'asym_7pt': S.taps_asym_7pt(),
            'stencil_27pt': S.taps_27pt()}[builder_name]
    dt = np.float16 if builder_name == 'stencil_27pt' else np.float32
    tol = 1e-3 if dt == np.float16 else 1e-6
    rng = np.random.default_rng(6)
    u = rng.uniform(0, 1, shape).astype(dt)
    d = rng.uniform(-1, 1, shape).astype(dt)
    monkeypatch.setenv('PSAD_SLAB_FACE_WAIT', face_wait)
    z = ZSlabOp(op, use_cuda=True)
    z._halo = RcclHalo(loopback=True)
    try:
        tu, td = torch.from_numpy(u).cuda(), torch.from_numpy(d).cuda()
        z.warm_exchange(u=tu, diffout=td)
        fn = z.autograd_function()
        n0 = _psad_torch.num_slab_plans()
        s0 = _psad_torch.num_start_signal_sweeps()
        w0 = _psad_torch.num_face_wait_sweeps()
        res = []
        for native in ('1', '1', '0'):
            monkeypatch.setenv('PSAD_NATIVE_SLAB', native)
            uu = tu.clone().requires_grad_(True)
            (o,) = fn.apply(uu)
            assert ('CppNode' in o.grad_fn.name()) == (native == '1'), o.grad_fn.name()
            o.backward(td)
            torch.cuda.synchronize()
            res.append((o.detach().clone(), uu.grad.clone()))
        assert _psad_torch.num_slab_plans() == n0 + 1
        # slabs with interior planes: each native sweep's interior launch wrote the halo stream's signal itself (no
        # stream-memory write kernel on the compute queue); a slab of faces only keeps hipStreamWriteValue32
        assert _psad_torch.num_start_signal_sweeps() - s0 == (4 if shape[0] > 2 else 0)
        if face_wait == '0' or shape[0] <= 2:
            assert _psad_torch.num_face_wait_sweeps() == w0
        elif shape[2] >= 256:
            # rows wide enough for an LDS-DMA loader (row bands, the WS rings; narrower rows take register-prefetch
            # tiles, whose faces stay on the halo stream): every native sweep's faces waited in-kernel
            assert _psad_torch.num_face_wait_sweeps() - w0 == 4
        assert torch.equal(res[0][0], res[2][0]) and torch.equal(res[0][1], res[2][1])
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])

        def periodic(a, tp):
            a64 = a.astype(np.float64)
            ext = np.concatenate([a64[-1:], a64, a64[:1]])
            return S.linear_stencil(ext, tp)[1:-1]
        assert_close_rel(res[0][0].cpu().numpy(), periodic(u, taps), tol, 'out')
        assert_close_rel(res[0][1].cpu().numpy(), periodic(d, S.flip(taps)), tol, 'diffu')
    finally:
        z.close()


def _worker_varcoef(rank, world, port, shape, use_cuda, result_dir):
    """Two input fields and a nonlinear stencil on z-slabs: the halos of u and k (forward) and of u, k and diffout
    (adjoint) exchanged; this rank's slabs of out / diffu / diffk saved."""
    import sys
    sys.path.insert(0, ROOT)
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    from pystencils_autodiff_amd.zslab import ZSlabOp, slab_bounds
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    try:
        op = pa.AutoDiffOp(W.varcoef_diffusion_7pt(), boundary_handling='zeros')
        u, k, d = _varcoef_inputs(shape)
        lo, hi = slab_bounds(shape[0], world, rank)
        dev = 'cuda' if use_cuda else 'cpu'
        ul, kl, dl = (torch.from_numpy(a[lo:hi].copy()).to(dev) for a in (u, k, d))
        out, du, dk = (torch.zeros_like(ul) for _ in range(3))
        z = ZSlabOp(op, use_cuda=use_cuda)
        z.fwd(u=ul, k=kl, out=out)
        z.bwd(u=ul, k=kl, diffout=dl, diffu=du, diffk=dk)
        if use_cuda:
            torch.cuda.synchronize()
        for n, t in (('out', out), ('du', du), ('dk', dk)):
            np.save(os.path.join(result_dir, f'{n}_{rank}.npy'), t.cpu().numpy())
    finally:
        dist.destroy_process_group()


def _varcoef_inputs(shape):
    rng = np.random.default_rng(4)
    return (rng.uniform(-1, 1, shape).astype(np.float32), rng.uniform(0.1, 1.1, shape).astype(np.float32),
            rng.uniform(-1, 1, shape).astype(np.float32))


def _run_varcoef(world, shape, use_cuda, tmp_path):
    from oracle import evaluate as OE
    from tests.conftest import assert_close_rel
    import pystencils_autodiff_amd as pa
    from pystencils_autodiff_amd import workloads as W
    port = _free_port()
    mp.spawn(_worker_varcoef, args=(world, port, shape, use_cuda, str(tmp_path)), nprocs=world, join=True)
    got = {n: np.concatenate([np.load(tmp_path / f'{n}_{r}.npy') for r in range(world)]) for n in ('out', 'du', 'dk')}
    op = pa.AutoDiffOp(W.varcoef_diffusion_7pt(), boundary_handling='zeros')
    u, k, d = (a.astype(np.float64) for a in _varcoef_inputs(shape))
    ref = {**OE.evaluate(op.forward_assignments, {'u': u, 'k': k}),
           **OE.evaluate(op.backward_assignments, {'u': u, 'k': k, 'diffout': d})}
    assert_close_rel(got['out'], ref['out'], 1e-6, 'out')
    assert_close_rel(got['du'], ref['diffu'], 1e-6, 'diffu')
    assert_close_rel(got['dk'], ref['diffk'], 1e-6, 'diffk')


@pytest.mark.parametrize('world,shape', [(2, (10, 9, 12)), (3, (13, 6, 8))])
def test_zslab_two_input_nonlinear_gloo_cpu(world, shape, tmp_path):
    _run_varcoef(world, shape, False, tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize('world,shape', [(2, (24, 40, 64)), (3, (19, 33, 72))])
def test_zslab_two_input_nonlinear_gloo_gpu(world, shape, tmp_path):
    """The plane ring (LDS-DMA form at these widths) with halo planes of two / three fields across ranks."""
    _run_varcoef(world, shape, True, tmp_path)
