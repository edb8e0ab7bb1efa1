"""Z-slab domain decomposition of a stencil op across ranks, halo exchange over RCCL.

The reference has no multi-device execution at all; this is
the MI355X layer's scale-out for the 3-D configs (BASELINE configs 4 and 5):

* axis 0 of every field is split into contiguous slabs, rank ``k`` of ``P``
  owning planes ``[k·Z/P, (k+1)·Z/P)`` (remainder spread over the first ranks);
* one exchange step per sweep: each stencil field sends its first / last
  ``RZ`` planes to rank ``k-1`` / ``k+1`` and receives their boundary planes as
  halos — point-to-point over xGMI, neighbours talk over their own link, nothing
  here is a ring collective. On GPUs with the ``nccl`` (= RCCL) process group the
  exchange is ONE ``ncclGroupStart; ncclSend/ncclRecv…; ncclGroupEnd`` on a
  dedicated stream through the C ABI (``psad_halo_exchange``, a communicator of
  its own, :class:`RcclHalo`); ``torch.distributed.batch_isend_irecv`` (~80 µs
  of host time per exchange) remains the path for ``gloo`` and for
  ``PSAD_HALO=torch``. Rank 0's lower and rank ``P-1``'s upper
  halos stay absent, which the kernel reads as zeros — the ``'zeros'``
  boundary of the undivided domain;
* the exchange overlaps the interior planes: the march kernel first writes
  planes ``[RZ, Zl-RZ)`` (no halo needed) while the faces are in flight, then,
  after the receive completes, the ``RZ`` planes at each end (one launch for both
  faces: a two-range ``z_range``). The halo planes
  are read by the kernel in place from the receive buffers (no ghosted copy of
  the slab).

On the CPU (``gloo``) the same exchange runs and the C kernel evaluates a
ghosted copy — used by the multi-process tests.

fzyx (SoA) vector fields: every component is a C-contiguous spatial array of its own, and the GPU kernels
bind each as a scalar field (``kernel_ir.split_soa``). A slab of such a field therefore exchanges one face
pair PER COMPONENT (each face contiguous, in the same RCCL group) and hands the kernel one halo pair per
component field (``u__c0``, ``u__c1``, …).
"""
import ctypes
import glob
import itertools
import os

import torch
import torch.distributed as dist

__all__ = ['slab_bounds', 'ZSlabOp', 'exchange_halos', 'RcclHalo', 'RcclUnavailable']


def rccl_library_path():
    """torch's bundled librccl (the copy its process group already loaded), else the ROCm one."""
    cands = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so*')))
    cands += sorted(glob.glob('/opt/rocm/lib/librccl.so*'))
    return os.environ.get('PSAD_RCCL_LIBRARY') or (cands[0] if cands else 'librccl.so.1')


class RcclUnavailable(RuntimeError):
    """Raised on every rank alike when the C-ABI RCCL communicator cannot be set up; the sweep then
    uses ``torch.distributed.batch_isend_irecv`` on the same ``nccl`` (= RCCL) process group."""


class RcclHalo:
    """An RCCL communicator of its own over ``group`` for the slab-face exchange, and the stream the
    exchange runs on. Construction is collective (``ncclCommInitRank`` on every rank)."""

    def __init__(self, group=None, device=None, loopback=False):
        """``loopback=True``: a one-rank communicator without ``torch.distributed`` whose exchange
        sends both faces to itself — the slab then sees its own far faces as halos, a periodic z
        boundary; it exercises the whole RCCL path on one GPU (tests)."""
        from .backends import hip_runtime as rt
        self._rt = rt
        L = rt.lib()
        opened = L.psad_rccl_open(rccl_library_path().encode())
        self.loopback = loopback
        self.rank = 0 if loopback else dist.get_rank(group)
        self.world = 1 if loopback else dist.get_world_size(group)
        if not loopback:
            # every rank agrees before the collective setup below: a rank that could not open librccl
            # must not leave the others waiting in the unique-id broadcast
            if dist.get_backend(group) == 'gloo':
                dev = torch.device('cpu')
            else:
                dev = torch.device('cuda', torch.cuda.current_device()) if device is None else device
            flag = torch.tensor([0 if opened == 0 else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
            if int(flag.item()):
                raise RcclUnavailable('librccl could not be opened on at least one rank'
                                      + (f' ({rt.lib().psad_rccl_error_string(opened).decode()})' if opened else ''))
        else:
            rt._check(opened, 'opening librccl')
        uid = ctypes.create_string_buffer(128)
        status = 0
        if self.rank == 0:
            status = L.psad_rccl_unique_id(uid)
        # rank 0 sends (status, id): a failed ncclGetUniqueId makes every rank raise alike instead of
        # leaving the others waiting for an id that never comes
        obj = [(status, uid.raw) if self.rank == 0 else None]
        if not loopback:
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
        status, uid_raw = obj[0]
        if status:
            raise RcclUnavailable(f'ncclGetUniqueId failed on rank 0 ({L.psad_error_string(status).decode()})')
        self.device = torch.device('cuda', torch.cuda.current_device()) if device is None else device
        with torch.cuda.device(self.device):
            comm = ctypes.c_void_p()
            rt._check(L.psad_rccl_comm_init(uid_raw, self.world, self.rank, ctypes.byref(comm)), 'ncclCommInitRank')
            self.comm = comm
            # (a high-priority stream for the exchange measured slower: 0.74 vs 0.42 ms per 128×1024² fp32
            # loopback step, profiles/r03p_slab_variants.log)
            self.stream = torch.cuda.Stream(device=self.device)
            # reused stream-order events (Stream.wait_stream would create two per sweep)
            self.ev_faces = torch.cuda.Event()
            self.ev_halos = torch.cuda.Event()
        self._arrays = {}
        self._exchange = L.psad_halo_exchange
        self._stream_handle = self.stream.cuda_stream

    def exchange(self, planes, peer_lo, peer_hi):
        """``planes`` = [(send_lo, recv_lo, send_hi, recv_hi, nbytes)] (device pointers, 0 for an
        absent side); enqueued on :attr:`stream`, which the caller orders against its own."""
        n = len(planes)
        bufs = self._arrays.get(n)
        if bufs is None:           # argument arrays reused across sweeps (ctypes construction is not free)
            bufs = self._arrays[n] = ([(ctypes.c_void_p * n)() for _ in range(4)], (ctypes.c_size_t * n)())
        arrs, sizes = bufs
        for i, (a, b, c, d, nb) in enumerate(planes):
            arrs[0][i], arrs[1][i], arrs[2][i], arrs[3][i], sizes[i] = a, b, c, d, nb
        rc = self._exchange(self.comm, n, arrs[0], arrs[1], arrs[2], arrs[3], sizes, peer_lo, peer_hi,
                            self._stream_handle)
        if rc:
            self._rt._check(rc, 'RCCL halo exchange')

    def close(self):
        if self.comm:
            self._rt._check(self._rt.lib().psad_rccl_comm_destroy(self.comm), 'ncclCommDestroy')
            self.comm = None


def slab_bounds(n, world, rank):
    """``[lo, hi)`` of axis 0 owned by ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def exchange_halos(t, rz, group=None, bufs=None):
    """Send the first/last ``rz`` planes of ``t`` to the lower/upper neighbour and receive theirs.

    Returns ``(works, lo_halo, hi_halo)``; halos are ``None`` at the global boundary. The
    receive buffers may be passed in (``bufs=(lo, hi)``) to avoid reallocation.
    """
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if rz == 0 or world == 1:
        return [], None, None
    if t.shape[0] < rz:
        raise ValueError(f"slab of {t.shape[0]} planes is thinner than the stencil radius {rz}")
    plane_shape = (rz,) + tuple(t.shape[1:])
    lo = hi = None
    ops = []
    peer = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    if rank > 0:
        lo = bufs[0] if bufs is not None and bufs[0] is not None else torch.empty(plane_shape, dtype=t.dtype,
                                                                                 device=t.device)
        ops.append(dist.P2POp(dist.isend, t[:rz].contiguous(), peer(rank - 1), group))
        ops.append(dist.P2POp(dist.irecv, lo, peer(rank - 1), group))
    if rank < world - 1:
        hi = bufs[1] if bufs is not None and bufs[1] is not None else torch.empty(plane_shape, dtype=t.dtype,
                                                                                 device=t.device)
        ops.append(dist.P2POp(dist.isend, t[-rz:].contiguous(), peer(rank + 1), group))
        ops.append(dist.P2POp(dist.irecv, hi, peer(rank + 1), group))
    if ops and t.is_cuda and dist.get_backend(group) == 'gloo':
        # gloo moves host memory only: stage through the CPU (tests / debugging, not the RCCL path)
        staged = [dist.P2POp(op.op, op.tensor.cpu() if op.op is dist.isend else torch.empty_like(op.tensor, device='cpu'),
                             op.peer, op.group) for op in ops]
        for w in dist.batch_isend_irecv(staged):
            w.wait()
        for op, st in zip(ops, staged):
            if op.op is dist.irecv:
                op.tensor.copy_(st.tensor)
        return [], lo, hi
    works = dist.batch_isend_irecv(ops) if ops else []
    return works, lo, hi


class ZSlabOp:
    """Run the forward / backward kernels of an ``AutoDiffOp`` on this rank's z-slab.

    ``fwd(**fields)`` / ``bwd(**fields)`` take the local slabs by field name (outputs
    preallocated, written in place) plus scalars, exchange the halos of every stencil field,
    and launch with interior / boundary overlap.

    Both boundary modes of the reference (``_autodiff.py:479-542``): ``'zeros'`` (every cell written,
    zero reads outside the global domain) and ``None`` (only the global interior ``[g, Z-g)`` of axis
    0 — and ``[g, N-g)`` of the others — is written; the untouched border keeps what the caller
    allocated). Interior-only slabs need their place in the global domain: ``z_offset`` / ``global_z``,
    else gathered once from every rank's slab extent (collective, on the first sweep).
    """

    def __init__(self, autodiff_op, use_cuda=True, group=None, z_offset=None, global_z=None):
        self.op = autodiff_op
        self.use_cuda = use_cuda
        self.group = group
        target = 'gpu' if use_cuda else 'cpu'
        self.kernels = {'forward': getattr(autodiff_op, f'forward_ast_{target}'),
                        'backward': getattr(autodiff_op, f'backward_ast_{target}')}
        for k in self.kernels.values():
            if k.ir.ndim != 3 and k.ir.ndim != 2:
                raise ValueError('z-slab decomposition needs 2-D or 3-D fields')
            if k.ir.periodic:
                # a periodic lattice needs a wrap-around exchange between the first and last rank (and the
                # kernels' own wrapped reads disabled along z): not built
                raise NotImplementedError("z-slab decomposition of boundary_handling='periodic' kernels")
        self._span = {} if z_offset is None or global_z is None else None
        self._fixed_span = None if self._span is not None else (int(z_offset), int(global_z))
        self._bufs = {}
        self._halo = None
        self._no_rccl = False
        self._meta = {}

    def _rccl(self, device):
        """The RCCL exchange path (GPU, ``nccl`` process group, ``PSAD_HALO`` not ``torch``)."""
        if not (self.use_cuda and dist.is_initialized() and dist.get_backend(self.group) == 'nccl'
                and os.environ.get('PSAD_HALO', 'rccl') == 'rccl'):
            return None
        if self._halo is None:
            if self._no_rccl:
                return None
            try:
                self._halo = RcclHalo(self.group, device)
            except RcclUnavailable as exc:
                import sys
                print(f'zslab: {exc}; halo exchange falls back to torch.distributed.batch_isend_irecv',
                      file=sys.stderr)
                self._no_rccl = True
                return None
        return self._halo

    def connect(self, device=None):
        """Create the RCCL halo communicator now (collective: every rank calls it) instead of in the
        first sweep — setup kept out of a timed loop. A no-op off the ``nccl`` process group."""
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            self._rccl(device if device is not None else torch.device('cuda', torch.cuda.current_device()))

    def close(self):
        """Destroy the halo communicator (collective, before ``destroy_process_group``)."""
        if self._halo is not None:
            self._halo.close()
            self._halo = None

    @staticmethod
    def _units(f, t):
        """The exchange units of stencil field ``f``'s slab ``t`` as ``[(halo name, tensor)]``: the slab itself, or
        for an fzyx (SoA) field one C-contiguous component array per component under the kernels' component field
        names (``Field.component_field``, ``kernel_ir.split_soa``)."""
        if not f.is_soa:
            return [(f.name, t)]
        sdim = t.dim() - f.index_dimensions
        return [(f.component_field(idx).name, t[(Ellipsis,) + idx])
                for idx in itertools.product(*[range(int(n)) for n in t.shape[sdim:]])]

    @staticmethod
    def _layout(f, t):
        """``t`` in the memory order the kernels expect for field ``f``: C order, or fzyx (components-first) for
        an SoA field — copied only if it is not already."""
        if not f.is_soa:
            return t.contiguous()
        sdim = t.dim() - f.index_dimensions
        from .backends._torch_native import _soa_empty
        want = _soa_empty(tuple(t.shape), sdim, torch.empty, t.dtype, 'meta').stride()
        if tuple(t.stride()) == tuple(want):
            return t
        out = _soa_empty(tuple(t.shape), sdim, torch.empty, t.dtype, t.device)
        out.copy_(t)
        return out

    def _radius(self, kernel, field):
        return max([abs(r.offsets[0]) for r in kernel.ir.reads if r.field.name == field.name] + [0])

    def span(self, zl):
        """``(z_offset, global_z)`` of a local slab of ``zl`` planes: given at construction, else the
        slab extents of all ranks gathered once (collective), else the slab alone (no process group)."""
        if self._fixed_span is not None:
            return self._fixed_span
        got = self._span.get(zl)
        if got is None:
            if dist.is_initialized() and dist.get_world_size(self.group) > 1:
                sizes = [None] * dist.get_world_size(self.group)
                dist.all_gather_object(sizes, int(zl), group=self.group)
                r = dist.get_rank(self.group)
                got = (sum(sizes[:r]), sum(sizes))
            else:
                got = (0, int(zl))
            self._span[zl] = got
        return got

    def z_limits(self, kernel, zl):
        """Local ``[lo, hi)`` of the planes this rank writes: all of them under ``'zeros'``, the part of
        the global interior ``[g, Z-g)`` under ``boundary_handling=None``."""
        ir = kernel.ir
        if ir.zeros or ir.ghost_layers == 0:
            return 0, zl
        z0, Z = self.span(zl)
        g = ir.ghost_layers
        lo, hi = max(0, g - z0), min(zl, Z - g - z0)
        return (lo, hi) if hi > lo else (0, 0)

    def fwd(self, **kwargs):
        return self._sweep('forward', kwargs)

    def bwd(self, **kwargs):
        return self._sweep('backward', kwargs)

    @staticmethod
    def _launches(zl, rz, lim):
        """The interior range (no halo read) and the face ranges (read halos) of a split sweep,
        restricted to the written planes ``lim``: ``(interior or None, [face ranges])``."""
        lo, hi = lim

        def clip(a, b):
            a, b = max(a, lo), min(b, hi)
            return (a, b) if b > a else None
        if zl <= 2 * rz:
            return None, [r for r in [clip(0, zl)] if r]
        inner = clip(rz, zl - rz)
        faces = [r for r in (clip(0, rz), clip(zl - rz, zl)) if r]
        return inner, faces

    @staticmethod
    def _launch_faces(compiled, halos, faces, zlim, kwargs):
        if len(faces) == 2 and faces[0][1] - faces[0][0] == faces[1][1] - faces[1][0]:
            compiled(halos=halos, z_range=tuple(faces), z_limits=zlim, **kwargs)   # both faces in one launch
        else:
            for f in faces:
                compiled(halos=halos, z_range=f, z_limits=zlim, **kwargs)

    def _sweep(self, which, kwargs):
        meta = self._meta.get(which)
        if meta is None:
            k = self.kernels[which]
            meta = self._meta[which] = (k, k.ir.stencil_fields,
                                        max([self._radius(k, f) for f in k.ir.stencil_fields] + [0]))
        k, stencil, rz = meta
        ir = k.ir
        ref = kwargs[ir.fields_written[0].name]
        zl = ref.shape[0]
        zlim = self.z_limits(k, zl)
        split = rz > 0 and dist.is_initialized() and dist.get_world_size(self.group) > 1
        halo = None
        if rz > 0 and self._halo is not None:
            halo = self._halo                         # created by _rccl, or preset (loopback / emulation tests)
        elif split:
            halo = self._rccl(ref.device)
        if halo is not None:
            self._sweep_rccl(k, halo, stencil, rz, kwargs, zlim)
            return
        pending, halos = [], {}
        for f in stencil:
            # the GPU kernels take one halo pair per fzyx component; the CPU path ghosts whole slabs
            for name, t in (self._units(f, kwargs[f.name]) if self.use_cuda else [(f.name, kwargs[f.name])]):
                key = (which, name, rz, t.dtype, tuple(t.shape[1:]), t.device)
                works, lo, hi = exchange_halos(t, rz, self.group, self._bufs.get(key))
                self._bufs[key] = (lo, hi)
                pending += works
                halos[name] = (lo, hi)
        # interior-only kernels always take the limits (their own bounds would skip the slab's end planes)
        kz = None if (ir.zeros or ir.ghost_layers == 0) else zlim
        if self.use_cuda:
            compiled = k.compile()
            if split:
                inner, faces = self._launches(zl, rz, zlim)
                if inner:
                    compiled(z_range=inner, z_limits=kz, **kwargs)   # interior overlaps the exchange
                for w in pending:
                    w.wait()                                          # current stream waits on RCCL
                self._launch_faces(compiled, halos, faces, kz, kwargs)
            elif zlim[1] > zlim[0]:
                compiled(halos=halos, z_limits=kz, **kwargs)
            return
        # CPU / gloo: evaluate a ghosted copy with the C kernel; under boundary_handling=None the copy
        # carries g >= rz planes per side so that its own interior covers every local plane
        for w in pending:
            w.wait()
        pad = rz if (ir.zeros or ir.ghost_layers == 0) else max(rz, ir.ghost_layers)
        ghosted = dict(kwargs)
        outs = {f.name: kwargs[f.name] for f in ir.fields_written}
        read_names = {r.field.name for r in ir.reads}

        def zeros(n, t):
            return torch.zeros((n,) + tuple(t.shape[1:]), dtype=t.dtype)
        for f in ir.fields:
            t = kwargs[f.name]
            if not pad:
                continue
            if f in stencil:
                lo, hi = halos[f.name]
                ghosted[f.name] = torch.cat([zeros(pad - rz, t), lo if lo is not None else zeros(rz, t), t,
                                             hi if hi is not None else zeros(rz, t), zeros(pad - rz, t)])
            elif f.name in outs and f.name not in read_names:
                ghosted[f.name] = zeros(zl + 2 * pad, t)
            else:
                ghosted[f.name] = torch.cat([zeros(pad, t), t, zeros(pad, t)])
        k.compile()(**ghosted)
        a, b = zlim
        for name, t in outs.items():
            if pad and b > a:
                t[a:b].copy_(ghosted[name][pad + a:pad + b])

    @staticmethod
    def _peers(halo):
        if halo.loopback:
            return 0, 0
        return (halo.rank - 1 if halo.rank > 0 else -1), (halo.rank + 1 if halo.rank < halo.world - 1 else -1)

    def _face_planes(self, halo, named, rz):
        """Send / receive pointers of the RZ boundary planes of each ``(name, slab)`` and the receive
        buffers (cached per field, dtype, shape, device) as ``{name: (lo, hi)}`` halos."""
        peer_lo, peer_hi = self._peers(halo)
        planes, halos = [], {}
        for name, t in named:
            if t.shape[0] < rz:
                raise ValueError(f"slab of {t.shape[0]} planes is thinner than the stencil radius {rz}")
            if not t.is_contiguous():
                raise ValueError(f"slab of '{name}' must be contiguous for the RCCL face exchange")
            lo, hi, nbytes, last_off = self._recv_bufs(halo, name, rz, tuple(t.shape), t.dtype, t.device)
            first = t.data_ptr()
            last = first + last_off
            if halo.loopback:
                # RCCL pairs a peer's sends and receives in issue order: swap the faces so that, as
                # with real neighbours, the lower halo receives the far (upper) face — periodic z
                first, last = last, first
            planes.append((first, lo.data_ptr() if lo is not None else 0, last,
                           hi.data_ptr() if hi is not None else 0, nbytes))
            t.record_stream(halo.stream)
            halos[name] = (lo, hi)
        return planes, halos

    def _recv_bufs(self, halo, name, rz, shape, dtype, device):
        """The receive buffers of field ``name``'s halos (cached per field, radius, dtype, shape, device: the
        forward and the adjoint sweep may read a field at different radii), its face bytes and the byte offset
        of its last ``rz`` planes."""
        peer_lo, peer_hi = self._peers(halo)
        key = ('rccl', name, rz, dtype, tuple(shape), device)
        bufs = self._bufs.get(key)
        if bufs is None:
            hshape = (rz,) + tuple(shape[1:])
            esize = torch.empty((), dtype=dtype).element_size()
            plane = esize
            for n in shape[1:]:
                plane *= int(n)
            bufs = (torch.empty(hshape, dtype=dtype, device=device) if peer_lo >= 0 else None,
                    torch.empty(hshape, dtype=dtype, device=device) if peer_hi >= 0 else None,
                    rz * plane, (int(shape[0]) - rz) * plane)
            self._bufs[key] = bufs
        return bufs

    def warm_exchange(self, **slabs):
        """One face exchange of the given slabs (``name=tensor``, stencil field names) with no compute:
        RCCL sets up its peer connections on first use, so this keeps that out of a timed loop and
        leaves the receive buffers allocated. Collective; a no-op without an RCCL communicator."""
        halo = self._halo
        if halo is None or not slabs:
            return
        cur = torch.cuda.current_stream(halo.device)
        halo.ev_faces.record(cur)
        halo.stream.wait_event(halo.ev_faces)
        for which in ('forward', 'backward'):      # each with its own kernel's radius, as its sweep does
            k = self.kernels.get(which)
            if k is None:
                continue
            named = [u for f in k.ir.stencil_fields if f.name in slabs for u in self._units(f, slabs[f.name])]
            rz = max([self._radius(k, f) for f in k.ir.stencil_fields] + [0])
            if named and rz:
                planes, _ = self._face_planes(halo, named, rz)
                halo.exchange(planes, *self._peers(halo))
        halo.stream.synchronize()

    def _sweep_rccl(self, k, halo, stencil, rz, kwargs, zlim=None):
        """Faces out on the halo stream (one RCCL group for every stencil field) while the interior
        planes run on the caller's stream; then the two face ranges in one launch."""
        peer_lo, peer_hi = self._peers(halo)
        cur = torch.cuda.current_stream(halo.device)
        halo.ev_faces.record(cur)
        halo.stream.wait_event(halo.ev_faces)         # the faces are final; the last sweep's reads are done
        planes, halos = self._face_planes(halo, [u for f in stencil for u in self._units(f, kwargs[f.name])], rz)
        halo.exchange(planes, peer_lo, peer_hi)
        compiled = k.compile()
        zl = kwargs[k.ir.fields_written[0].name].shape[0]
        zlim = (0, zl) if zlim is None else zlim
        kz = None if (k.ir.zeros or k.ir.ghost_layers == 0) else zlim
        inner, faces = self._launches(zl, rz, zlim)
        if inner:
            compiled(z_range=inner, z_limits=kz, **kwargs)  # interior overlaps the exchange
        halo.ev_halos.record(halo.stream)
        cur.wait_event(halo.ev_halos)
        self._launch_faces(compiled, halos, faces, kz, kwargs)

    def _alloc(self, kernel, name, like, dtype, read):
        """An output / gradient slab of field ``name`` (the spatial shape of ``like``, the field's components; fzyx
        fields components-first): zeros when the kernel accumulates into it or (CPU) leaves a border; under
        ``boundary_handling=None`` on the GPU uninitialised plus one zero fill of the planes, rows and columns the
        kernel does not write (the reference's ``torch.zeros`` values)."""
        from .backends._torch_native import _soa_components, _soa_empty
        ir = kernel.ir
        sdim = ir.ndim
        f = next((g for g in ir.fields if g.name == name), None)
        comps = tuple(int(n) for n in f.index_shape) if f is not None and f.index_dimensions else ()
        shape = tuple(like.shape[:sdim]) + comps
        soa = f is not None and f.is_soa
        zero = read or (not ir.zeros and ir.ghost_layers and not like.is_cuda)
        factory = torch.zeros if zero else torch.empty
        t = _soa_empty(shape, sdim, factory, dtype, like.device) if soa else \
            factory(shape, dtype=dtype, device=like.device)
        if not zero and not ir.zeros and ir.ghost_layers:
            from .backends.hip_kernel import zero_border
            bounds = ir.iteration_bounds(tuple(like.shape[:sdim]))
            bounds[0] = self.z_limits(kernel, like.shape[0])
            ncomp = 1
            for n in comps:
                ncomp *= n
            for p in (_soa_components(t, sdim) if soa else [t]):
                zero_border(p, bounds, 1 if soa else ncomp)
        return t

    def autograd_function(self):
        """A ``torch.autograd.Function`` over this rank's slabs with the drop-in op's contract:
        ``apply(*slabs)`` in ``forward_input_fields`` order returns the output slabs (tuple, in
        ``forward_output_fields`` order); ``backward`` exchanges the gradient halos and returns the
        input gradients. Scalars come from ``class_kwargs``. Adjoint names follow the op's field map
        / ``diff_fields_prefix`` like the single-device op (``_torch_native.py:96-100``)."""
        op = self.op
        zop = self
        fwd_inputs = list(op.forward_input_fields)
        fwd_outputs = list(op.forward_output_fields)
        fk, bk = self.kernels['forward'], self.kernels['backward']
        fwd_names = {f.name for f in fk.ir.fields}
        fwd_read = {r.field.name for r in fk.ir.reads}
        bwd_names = {f.name for f in bk.ir.fields}
        bwd_outputs = [f.name for f in op.backward_output_fields]
        bwd_read = {r.field.name for r in bk.ir.reads}        # accumulated adjoints start from zeros
        adj = {f.name: op.adjoint_name(f) for f in fwd_inputs + fwd_outputs}
        bwd_field = {f.name: f for f in bk.ir.fields}

        def tdtype(f):
            return getattr(torch, f.dtype.numpy_dtype.name)

        class ZSlabFunction(torch.autograd.Function):
            class_kwargs = {}

            @staticmethod
            def forward(ctx, *slabs):
                kw = {f.name: zop._layout(f, t) for f, t in zip(fwd_inputs, slabs) if f.name in fwd_names}
                kw.update({s.name: ZSlabFunction.class_kwargs[s.name] for s in fk.ir.scalars})
                outs = [zop._alloc(fk, f.name, slabs[0], tdtype(f), f.name in fwd_read) for f in fwd_outputs]
                kw.update({f.name: t for f, t in zip(fwd_outputs, outs)})
                zop.fwd(**kw)
                saved = [n for n in [f.name for f in fwd_inputs + fwd_outputs] if n in bwd_names and n in kw]
                ctx.saved_names = saved
                ctx.save_for_backward(*[kw[n] for n in saved])
                ctx.n_inputs = len(slabs)
                return tuple(outs)

            @staticmethod
            def backward(ctx, *grads):
                kw = dict(zip(ctx.saved_names, ctx.saved_tensors))
                kw.update({s.name: ZSlabFunction.class_kwargs[s.name] for s in bk.ir.scalars})
                like = next(g for g in grads if g is not None)
                for f, g in zip(fwd_outputs, grads):
                    a = adj[f.name]
                    if a in bwd_names:
                        kw[a] = zop._layout(bwd_field[a], g) if g is not None else \
                            zop._alloc(bk, a, like, tdtype(f), True)
                res = {}
                for name in bwd_outputs:
                    res[name] = zop._alloc(bk, name, like, like.dtype, name in bwd_read)
                    kw[name] = res[name]
                zop.bwd(**kw)
                return tuple(res.get(adj[f.name]) for f in fwd_inputs[:ctx.n_inputs])

        native = _NativeSlab(self, fwd_inputs, fwd_outputs, fwd_read, bwd_outputs, bwd_read, adj, tdtype)
        function_apply = torch.autograd.Function.apply.__func__

        def apply(cls, *args, **kwargs):
            """``apply(*slabs)``: through the native slab node (``_psad_torch``: the whole sweep — RCCL group,
            stream events, interior and face launches — without Python) when the call fits its plan, else the
            Python Function above (same launches, same results)."""
            if not kwargs:
                outs = native(args, cls.class_kwargs)
                if outs is not None:
                    return outs
            return function_apply(cls, *args, **kwargs)
        ZSlabFunction.apply = classmethod(apply)
        ZSlabFunction.__name__ = f"{op.op_name}_zslab"
        return ZSlabFunction


class _NativeSlab:
    """The slab Function's forward and backward sweeps as one C++ autograd node (``_psad_torch.apply_slab``,
    ``csrc/psad_torch.cpp`` "z-slab sweeps"). A plan per input signature (shapes, dtypes, device) holds, for
    each sweep, the interior and face launches (argument templates resolved by the kernels' own ``prepare``
    on stand-in pointers, the receive buffers' halo pointers baked in) and the RCCL exchange (receive
    buffers, bytes, peers, the communicator and halo stream of :class:`RcclHalo`). Calls it cannot express take
    the Python Function: no RCCL communicator (gloo, the emulated-rank tests' stand-in), an interior-only
    (``boundary_handling=None``) kernel, a stencil radius of 0, inputs that are not contiguous 32-byte-aligned
    device tensors."""

    def __init__(self, zop, fwd_inputs, fwd_outputs, fwd_read, bwd_outputs, bwd_read, adj, tdtype):
        self.zop = zop
        self.fwd_inputs, self.fwd_outputs = fwd_inputs, fwd_outputs
        self.fwd_read, self.bwd_outputs, self.bwd_read = fwd_read, bwd_outputs, bwd_read
        self.adj, self.tdtype = adj, tdtype
        self.plans = {}
        self.keep = []                      # receive buffers the plans point at

    def __call__(self, args, class_kwargs):
        from .backends._torch_native import native_module
        zop = self.zop
        halo = zop._halo
        if not isinstance(halo, RcclHalo) or native_module() is None or os.environ.get('PSAD_NATIVE_SLAB', '1') == '0':
            return None
        if len(args) != len(self.fwd_inputs) or not args or not all(isinstance(a, torch.Tensor) for a in args):
            return None
        names = sorted({s.name for k in zop.kernels.values() for s in k.ir.scalars})
        try:
            scal = [float(class_kwargs[n]) for n in names]
        except (KeyError, TypeError, ValueError):
            return None
        a0 = args[0]
        # per-call conditions (checked on every call, never cached: a later call of the same signature may meet them)
        for a in args:
            if not a.is_cuda or not a.is_contiguous() or a.data_ptr() % 32 or a.device != a0.device or \
                    tuple(a.shape) != tuple(a0.shape):
                return None
        key = (tuple(a0.shape), tuple(a.dtype for a in args), a0.device)
        pid = self.plans.get(key)
        if pid is None:
            try:
                pid = self._build(args, names, halo)
            except (TypeError, ValueError):
                pid = None
            self.plans[key] = -1 if pid is None else pid     # -1: the signature itself does not fit a plan
        if pid is None or pid < 0:
            return None
        outs = native_module().apply_slab(pid, list(args), scal)
        return None if outs is None else tuple(outs)

    def _build(self, args, scalar_names, halo):
        import struct

        from .backends._torch_native import _SCALAR_TYPE, native_module
        from .backends.hip_kernel import _Plane
        zop = self.zop
        fk, bk = zop.kernels['forward'], zop.kernels['backward']
        for k in (fk, bk):
            if not (k.ir.zeros or k.ir.ghost_layers == 0):
                return None                 # interior-only kernels: border fills and global z limits
            if any(f.is_soa for f in k.ir.fields):
                return None                 # fzyx vector fields: per-component halos and strided slabs
        for a in args:
            if not a.is_cuda or not a.is_contiguous() or a.data_ptr() % 32 or a.device != args[0].device or \
                    str(a.dtype).replace('torch.', '') not in _SCALAR_TYPE or tuple(a.shape) != tuple(args[0].shape):
                return None
        dev = args[0].device
        shape = tuple(int(n) for n in args[0].shape)
        zl = shape[0]
        seeds, fake = {}, [0]

        def stand_in(dtype):
            if dtype not in seeds:
                seeds[dtype] = torch.empty(1, dtype=dtype, device=dev)
            st, acc = [], 1
            for n in reversed(shape):
                st.insert(0, acc)
                acc *= n
            fake[0] += 1
            return _Plane(seeds[dtype], fake[0] << 40, shape, tuple(st))

        scal = {n: 1.0 for n in scalar_names}

        def sweep(which, kw, table):
            k = zop.kernels[which]
            _, stencil, rz = zop._meta.get(which) or (None, k.ir.stencil_fields,
                                                      max([zop._radius(k, f) for f in k.ir.stencil_fields] + [0]))
            if rz == 0:
                return None
            compiled = k.compile()
            inner, faces = zop._launches(zl, rz, (0, zl))
            halos, ex_slot, ex_off, rlo, rhi, nbytes = {}, [], [], [], [], []
            for f in stencil:
                if f.name not in kw:
                    return None
                lo, hi, nb, last = zop._recv_bufs(halo, f.name, rz, shape, self.tdtype(f), dev)
                self.keep.append((lo, hi))
                halos[f.name] = (lo, hi)
                ex_slot.append(table.index(f.name))
                ex_off.append(last)
                rlo.append(lo.data_ptr() if lo is not None else 0)
                rhi.append(hi.data_ptr() if hi is not None else 0)
                nbytes.append(nb)

            def resolve(**extra):
                try:
                    prep = compiled.prepare(**kw, **scal, **extra)
                except ValueError:
                    if not extra.get('halo_wait'):
                        raise
                    return None                 # no LDS-DMA loader to wait in: the faces stay on the halo stream
                if prep is None:
                    return None
                fn, grid, block, packed, xb, _ = prep
                fnames = [f[0] for f in compiled._field_specs()]
                if grid == 0 or xb or any(n not in table for n in fnames):
                    return None
                if list(struct.unpack_from(f'<{len(fnames)}Q', packed)) != [kw[n].data_ptr() for n in fnames]:
                    return None
                sn = [sc.name for sc in compiled.ir.scalars]
                slots = [[off, int(f64), scalar_names.index(n)]
                         for (off, f64), n in zip(compiled.last_plan.scalar_slots(len(sn)), sn)]
                pl = compiled.last_plan
                sig = list(pl.sig_offsets or (-1, -1)) + list(pl.hwait_offsets or (-1, -1))
                return (int(fn), int(grid), int(block), bytes(packed), [table.index(n) for n in fnames], slots, sig)
            # the interior launch signals its own start (the halo stream's exchange waits for it): no stream-memory
            # write kernel on the compute queue (csrc/psad_torch.cpp run_sweep)
            inner_l = resolve(z_range=inner, start_signal=True) if inner else None
            if inner and inner_l is None:
                return None
            def face_launches(**extra):
                if len(faces) == 2 and faces[0][1] - faces[0][0] == faces[1][1] - faces[1][0]:
                    return [resolve(halos=halos, z_range=tuple(faces), **extra)]
                return [resolve(halos=halos, z_range=f, **extra) for f in faces]
            # the face launches with a halo wait in their loader (they may then run on the compute stream behind the
            # interior, csrc/psad_torch.cpp run_sweep), or as before where the schedule has no LDS-DMA loader
            face_l = face_launches(halo_wait=True) if inner_l is not None else [None]
            if any(f is None for f in face_l):
                face_l = face_launches()
            if any(f is None for f in face_l):
                return None
            peer_lo, peer_hi = zop._peers(halo)
            ex = (ex_slot, ex_off, rlo, rhi, nbytes, peer_lo, peer_hi, bool(halo.loopback))
            return inner_l, face_l, ex

        def allocs(outs, read, kw):
            shapes, dtypes, zero, names = [], [], [], []
            for f in outs:
                dt = self.tdtype(f)
                if str(dt).replace('torch.', '') not in _SCALAR_TYPE:
                    return None
                kw[f.name] = stand_in(dt)
                shapes.append(list(shape))
                dtypes.append(_SCALAR_TYPE[str(dt).replace('torch.', '')])
                zero.append(f.name in read)
                names.append(f.name)
            return shapes, dtypes, zero, names
        fwd_names = {f.name for f in fk.ir.fields}
        kw = {}
        in_names = [f.name for f in self.fwd_inputs]
        for name, a in zip(in_names, args):
            kw[name] = stand_in(a.dtype)
        fo = allocs(self.fwd_outputs, self.fwd_read, kw)
        if fo is None:
            return None
        fwd_table = in_names + fo[3]
        fkw = {n: v for n, v in kw.items() if n in fwd_names}
        fs = sweep('forward', fkw, fwd_table)
        if fs is None:
            return None
        bwd_names = {f.name for f in bk.ir.fields}
        saved = [n for n in in_names + fo[3] if n in bwd_names]
        bkw = {n: kw[n] for n in saved}
        grad_names = []
        for i, f in enumerate(self.fwd_outputs):
            a = self.adj[f.name]
            grad_names.append(a if a in bwd_names else f'\0grad{i}')
            if a in bwd_names:
                bkw[a] = stand_in(self.tdtype(f))
        bo_fields = [next(g for g in bk.ir.fields if g.name == n) for n in self.bwd_outputs]
        bo = allocs(bo_fields, self.bwd_read, bkw)
        if bo is None:
            return None
        bwd_table = saved + grad_names + bo[3]
        bs = sweep('backward', {n: v for n, v in bkw.items() if n in bwd_names}, bwd_table)
        if bs is None:
            return None
        grad_of_input = [bwd_table.index(self.adj[n], len(saved) + len(grad_names))
                         if self.adj.get(n) in bo[3] else -1 for n in in_names]
        return native_module().register_slab_plan(
            'zslab', dev.index, [list(a.shape) for a in args],
            [_SCALAR_TYPE[str(a.dtype).replace('torch.', '')] for a in args],
            fo[0], fo[1], fo[2], fs[0], fs[1], fs[2], [fwd_table.index(n) for n in saved],
            bo[0], bo[1], bo[2], bs[0], bs[1], bs[2], grad_of_input, len(scalar_names),
            int(halo.comm.value), int(halo._stream_handle))
