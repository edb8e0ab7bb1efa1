"""``backend='torch_native'``: an ``AutoDiffOp`` as a ``torch.autograd.Function``.

Same contract as the reference's ``backends/_torch_native.py:10-142``:

* ``Op.apply(*inputs)`` takes the forward input tensors positionally in
  ``autodiff_obj.forward_input_fields`` order (sorted by name) and returns a
  **tuple** of outputs in ``forward_output_fields`` order (``:58-59,88``);
  ``Op.call(**named)`` returns a single tensor when there is one output
  (``:120-124``); scalar parameters come from ``Op.class_kwargs`` (``:41,45``).
* inputs are moved to the op's device and made contiguous (``:47-52``);
  backward asserts gradient shapes / element strides / device (``:101-105``).
* class attributes ``class_kwargs, kernel, ast, parameters, forward_parameters,
  forward_ast, backward_ast, num_regs, code`` (``:126-140``).

Differences, all deliberate: kernels run on torch's current HIP stream
(not the legacy default stream); outputs every cell of which the kernel writes
are allocated with ``torch.empty`` (the reference memsets with ``torch.zeros``,
an extra HBM pass); with ``boundary_handling=None`` only the untouched border slabs
are zero-filled (``_allocator``); only tensors the backward kernel reads are saved on
``ctx``; gradients are returned in forward-input order with ``None`` for
constant fields; native errors raise ``RuntimeError`` instead of ``exit()``.
On ``use_cuda=True`` there is no CPU fallback: a missing HIP extension raises.
"""
import hashlib

import sympy as sp

__all__ = ['create_autograd_function', 'numpy_dtype_to_torch']


def numpy_dtype_to_torch(dtype):
    """``backends/_pytorch.py:95-97``."""
    import torch
    return getattr(torch, str(dtype))


class _Parameter:
    def __init__(self, name, field=None):
        self.symbol = sp.Symbol(name)
        self.field = field
        self.is_field_parameter = field is not None

    def __repr__(self):
        return f"Parameter({self.symbol.name})"


class TorchModule:
    """The pair of compiled kernels an op uses (stands in for the reference's ``TorchModule``)."""

    def __init__(self, module_name, kernels):
        self.module_name = module_name
        self.kernels = [k for k in kernels if k is not None]
        self.kernel_wrappers = [_Wrapper(k) for k in self.kernels]

    @property
    def code(self):
        return '\n'.join(k.compile().code for k in self.kernels)

    def compile(self):
        for k in self.kernels:
            k.compile().build() if k.target == 'gpu' else k.compile()
        return self

    def __str__(self):
        return self.code


class _Wrapper:
    def __init__(self, kernel):
        self.function_name = 'call_' + kernel.function_name
        self._kernel = kernel

    def get_parameters(self):
        return [_Parameter(p.symbol.name, p.field) for p in self._kernel.get_parameters()]


def _components_complete(kernel, field_name=None):
    """Every component of the given vector output (all outputs if None) is assigned."""
    import itertools
    for f in kernel.ir.fields_written:
        if field_name is not None and f.name != field_name:
            continue
        if f.index_dimensions:
            written = {tuple(idx) for fld, _, idx, _ in kernel.ir.stores if fld.name == f.name}
            if written != set(itertools.product(*[range(int(n)) for n in f.index_shape])):
                return False
    return True


def _full_write(kernel, field_name=None):
    """True if the kernel writes every cell of its outputs (no untouched border) and, for the given output
    (all outputs if None), every component of a vector field — else the output keeps the reference's
    ``torch.zeros`` allocation (``_torch_native.py:64,108``)."""
    if not (kernel.ir.zeros or kernel.ir.periodic or kernel.ir.ghost_layers == 0):
        return False
    return _components_complete(kernel, field_name)


# CPU: below this many elements one memset is cheaper than 2·ndim border fills
BORDER_ZERO_MIN = 1 << 22
# GPU: zero the border with one hiprtc kernel (hip_kernel.zero_border) instead of a full memset
BORDER_KERNEL = True


def _soa_empty(shape, sdim, factory, dtype, device):
    """A tensor of ``shape`` (spatial axes, then component axes) in fzyx (SoA) memory order: allocated
    components-first and viewed with the component axes last."""
    import torch
    nidx = len(shape) - sdim
    t = factory(tuple(shape[sdim:]) + tuple(shape[:sdim]), dtype=dtype, device=device)
    return t.permute(*range(nidx, nidx + sdim), *range(nidx)) if nidx else t


def _soa_components(t, sdim):
    """The C-contiguous per-component views of an fzyx tensor."""
    import itertools
    return [t[(Ellipsis,) + idx] for idx in itertools.product(*[range(int(n)) for n in t.shape[sdim:]])]


def _allocator(kernel, field_name, read_names=()):
    """How an output is allocated: ``torch.empty`` when the kernel writes all of it; for an interior-only
    kernel (``boundary_handling=None``, the reference's default) that assigns every component at offset 0,
    ``torch.empty`` plus zero fills of the untouched border slabs — the reference's ``torch.zeros``
    values without a memset pass over the whole field; otherwise ``torch.zeros``. fzyx (SoA) outputs are
    allocated components-first (``_soa_empty``)."""
    import torch
    ir = kernel.ir
    sdim = ir.ndim
    soa = any(f.name == field_name and f.is_soa for f in ir.fields_written)

    def plain(factory):
        if not soa:
            return factory

        def alloc(shape, dtype, device):
            return _soa_empty(shape, sdim, factory, dtype, device)
        return alloc
    if field_name in read_names:
        return plain(torch.zeros)
    if _full_write(kernel, field_name):
        return plain(torch.empty)
    if not _components_complete(kernel, field_name) or \
            any(any(o != 0 for o in off) for fld, off, _, _ in ir.stores if fld.name == field_name):
        return plain(torch.zeros)

    ncomp = 1
    for f in ir.fields_written:
        if f.name == field_name:
            for n in (f.index_shape if f.index_dimensions else ()):
                ncomp *= int(n)

    def alloc(shape, dtype, device, pending=None):
        t = _soa_empty(shape, sdim, torch.empty, dtype, device) if soa else \
            torch.empty(shape, dtype=dtype, device=device)
        parts = _soa_components(t, sdim) if soa else [t]
        per = 1 if soa else ncomp
        if t.is_cuda:
            if not BORDER_KERNEL:
                return t.zero_()
            from .hip_kernel import zero_border
            bounds = ir.iteration_bounds(tuple(shape[:sdim]))
            # the x ends of the interior rows are left to the kernel's x_border stores (or, if its launch
            # cannot, to a second fill after it: ``pending``)
            for p in parts:
                zero_border(p, bounds, per, x=pending is None)
                if pending is not None:
                    pending.append(lambda p=p: zero_border(p, bounds, per, zy=False))
            return t
        if t.numel() < BORDER_ZERO_MIN:
            return t.zero_()
        for d, (lo, hi) in enumerate(ir.iteration_bounds(tuple(shape[:sdim]))):
            n = int(shape[d])
            if lo > 0:
                t.narrow(d, 0, min(lo, n)).zero_()
            if hi < n:
                t.narrow(d, hi, n - hi).zero_()
        return t
    alloc.border = True
    return alloc


def _border_kw(alloc, pending):
    return {'pending': pending} if getattr(alloc, 'border', False) else {}


def _launch(call, kwargs, pending):
    """Launch; when outputs have a zeroed border (``_allocator``), ask the kernel to store the x ends of
    its rows too (``x_border``) and fill them separately only if its schedule cannot."""
    if not pending:
        call(**kwargs)
    elif not call(x_border=True, **kwargs):
        for fill in pending:
            fill()


_native = None


def native_module():
    """The ``_psad_torch`` extension (``csrc/psad_torch.cpp``): the op's autograd node in C++. Raises if it
    has not been built, like ``libpsad_hip.so``; ``PSAD_NATIVE_AUTOGRAD=0`` selects the Python Function."""
    global _native
    if _native is None:
        import os
        if os.environ.get('PSAD_NATIVE_AUTOGRAD', '1') == '0':
            _native = False
        else:
            import torch  # (the extension resolves torch's symbols from the loaded libraries)
            try:
                from .. import _psad_torch
            except ImportError as exc:
                if torch.cuda.is_available():
                    raise ImportError(f"{exc}: build the extension with `python -m pystencils_autodiff_amd.build`") \
                        from exc
                # no GPU here: nothing launches, ops are only built (hiprtc) — the Python Function will do
                _psad_torch = False
            if _psad_torch:
                from .hip_runtime import HipError, _check_stamp
                if not hasattr(_psad_torch, 'source_hash'):
                    raise HipError(f'{_psad_torch.__file__} predates the source stamp (a stale build): rebuild with '
                                   '`python -m pystencils_autodiff_amd.build`')
                _check_stamp(_psad_torch.source_hash(), 'torch', _psad_torch.__file__)
            _native = _psad_torch
    return _native or None


# c10::ScalarType codes of the dtypes the kernels take
_SCALAR_TYPE = {'float16': 5, 'float32': 6, 'float64': 7}


class _NativePath:
    """The forward + adjoint launches of one op as a C++ ``torch::autograd::Function`` (``_psad_torch``):
    the backward then runs on torch's autograd device thread without Python (no GIL hand-off), the forward
    without the Python Function's bookkeeping. One native plan per input signature (input shapes, dtypes,
    device), resolved by the kernels' own ``prepare`` on the first call; the scalar parameters are patched into
    the argument buffers per call (their byte offsets are part of the plan). Ops the plan
    cannot express take the Python Function: fzyx fields, outputs with a zero border larger than
    ``BORDER_ZERO_MIN`` (the border kernel beats a memset there), no backward kernel, inputs that are
    not contiguous 32-byte-aligned device tensors."""

    def __init__(self, spec):
        self.spec = spec
        self.plans = {}

    def _kind(self, alloc, shape):
        import torch
        if alloc is torch.empty:
            return False
        if alloc is torch.zeros:
            return True
        if getattr(alloc, 'border', False):
            n = 1
            for s in shape:
                n *= int(s)
            return True if n < BORDER_ZERO_MIN else None
        return None

    def __call__(self, args):
        import torch
        s = self.spec
        if len(args) != len(s['fwd_inputs']) or not args or not isinstance(args[0], torch.Tensor):
            return None
        try:
            scal = tuple(s['class_kwargs'][n] for n in s['scalar_names'])
        except KeyError:
            return None
        a0 = args[0]
        # per-call conditions (the C++ side checks them again): such a call takes the Python Function without
        # marking its signature as one the plan cannot express
        for a in args:
            if not isinstance(a, torch.Tensor) or not a.is_cuda or not a.is_contiguous() or a.data_ptr() % 32 \
                    or a.device != a0.device:
                return None
        key = (tuple(a0.shape), a0.dtype, a0.device)
        pid = self.plans.get(key)
        if pid is None:
            pid = self._build(args, scal)
            # a signature the plan cannot express is remembered as such (-1): later calls go straight to the
            # Python Function instead of resolving stand-in launches again
            self.plans[key] = -1 if pid is None else pid
        if pid is None or pid < 0:
            return None
        try:
            scal = [float(v) for v in scal]
        except (TypeError, ValueError):
            return None
        outs = native_module().apply(pid, list(args), scal)
        return None if outs is None else tuple(outs)

    def _build(self, args, scal):
        import struct

        import torch
        s = self.spec
        for a in args:
            if not isinstance(a, torch.Tensor) or not a.is_cuda or not a.is_contiguous() or a.data_ptr() % 32 \
                    or a.device != args[0].device or str(a.dtype).replace('torch.', '') not in _SCALAR_TYPE:
                return None
        dev = args[0].device
        scalars = dict(zip(s['scalar_names'], scal))
        from .hip_kernel import _Plane
        seeds = {}
        fake = [0]

        def stand_in(shape, dtype):
            # a C-contiguous, 256-byte-aligned pointer record: plans depend on shapes, dtypes and alignment
            # only, so no output- or gradient-sized buffer is allocated to resolve them
            if dtype not in seeds:
                seeds[dtype] = torch.empty(1, dtype=dtype, device=dev)
            strides, acc = [], 1
            for n in reversed(shape):
                strides.insert(0, acc)
                acc *= int(n)
            fake[0] += 1
            return _Plane(seeds[dtype], fake[0] << 40, tuple(int(n) for n in shape), tuple(strides))

        def alloc_specs(outs, like_shape, kw):
            shapes, dtypes, zero, names = [], [], [], []
            for name, dtype, fixed, alloc, sdim, ishape in outs:
                shape = tuple(fixed) if fixed is not None else tuple(like_shape[:sdim]) + tuple(ishape)
                z = self._kind(alloc, shape)
                if z is None or str(dtype).replace('torch.', '') not in _SCALAR_TYPE:
                    return None
                kw[name] = stand_in(shape, dtype)
                shapes.append(list(shape))
                dtypes.append(_SCALAR_TYPE[str(dtype).replace('torch.', '')])
                zero.append(z)
                names.append(name)
            return shapes, dtypes, zero, names

        def resolve(call, kw, table):
            prep = call.prepare(**{n: v for n, v in kw.items()})
            if prep is None:
                return None
            fn, grid, block, packed, xb, _ = prep
            names = [f[0] for f in call._field_specs()]
            if grid == 0 or xb or len(packed) < 8 * len(names) or any(n not in table for n in names):
                return None
            if list(struct.unpack_from(f'<{len(names)}Q', packed)) != [kw[n].data_ptr() for n in names]:
                return None                     # pointer slots are not the leading 8-byte arguments
            snames = [sc.name for sc in call.ir.scalars]
            slots = [[off, int(f64), s['scalar_names'].index(n)]
                     for (off, f64), n in zip(call.last_plan.scalar_slots(len(snames)), snames)]
            if len(slots) != len(snames):
                return None
            return int(fn), int(grid), int(block), bytes(packed), [table.index(n) for n in names], slots

        fwd_call, bwd_call = s['fwd_call'], s['bwd_call']
        if getattr(fwd_call, '_soa', None) or getattr(bwd_call, '_soa', None):
            return None
        kw = dict(scalars)
        in_names = [f.name for f in s['fwd_inputs']]
        for name, a in zip(in_names, args):
            kw[name] = a
        fo = alloc_specs(s['fwd_out'], tuple(args[0].shape), kw)
        if fo is None:
            return None
        fwd_table = in_names + fo[3]
        try:
            fl = resolve(fwd_call, kw, fwd_table)
        except (TypeError, ValueError):
            return None
        if fl is None:
            return None
        saved_names = [n for n in s['saved_fwd'] if n in kw]
        bkw = dict(scalars)
        for n in saved_names:
            bkw[n] = kw[n]
        grad_names = []
        for i, (aname, dtype, fixed, strides, fname) in enumerate(s['grad_specs']):
            g = stand_in(kw[fname].shape, kw[fname].dtype)
            grad_names.append(aname if aname is not None else f'\0grad{i}')
            if aname is not None:
                bkw[aname] = g
        bo = alloc_specs(s['bwd_out'], tuple(kw[s['fwd_out'][0][0]].shape), bkw)
        if bo is None:
            return None
        bwd_table = saved_names + grad_names + bo[3]
        try:
            bl = resolve(bwd_call, bkw, bwd_table)
        except (TypeError, ValueError):
            return None
        if bl is None:
            return None
        grad_of_input = [bwd_table.index(a, len(saved_names) + len(grad_names)) if a is not None and a in bo[3]
                         else -1 for a in s['in_adj']]
        return native_module().register_plan(
            s['op_name'], dev.index, [list(a.shape) for a in args],
            [_SCALAR_TYPE[str(a.dtype).replace('torch.', '')] for a in args],
            fo[0], fo[1], fo[2], *fl[:4], fl[4], fl[5], [fwd_table.index(n) for n in saved_names],
            bo[0], bo[1], bo[2], *bl[:4], bl[4], bl[5], grad_of_input, len(s['scalar_names']))


def create_autograd_function(autodiff_obj, use_cuda, op_name=None):
    import torch

    if use_cuda:
        forward_kernel = autodiff_obj.forward_ast_gpu
        backward_kernel = autodiff_obj.backward_ast_gpu if autodiff_obj.backward_output_fields else None
    else:
        forward_kernel = autodiff_obj.forward_ast_cpu
        backward_kernel = autodiff_obj.backward_ast_cpu if autodiff_obj.backward_output_fields else None

    if not op_name:
        digest = hashlib.md5((forward_kernel.compile().code + str(autodiff_obj) +
                              str(autodiff_obj.constant_fields)).encode()).hexdigest()
        op_name = f"{autodiff_obj.op_name}_{digest}"
    module = TorchModule(op_name, [forward_kernel, backward_kernel])
    module.compile()

    fwd_inputs = list(autodiff_obj.forward_input_fields)
    fwd_outputs = list(autodiff_obj.forward_output_fields)
    bwd_outputs = list(autodiff_obj.backward_output_fields) if backward_kernel else []
    bwd_inputs = list(autodiff_obj.backward_input_fields) if backward_kernel else []
    # adjoint of output i <-> grad_outputs[i]; match by name like the reference's prefixing
    prefix = getattr(autodiff_obj, 'diff_fields_prefix', 'diff')
    field_map = getattr(autodiff_obj, '_backward_field_map', None) or {}
    adj_of = {}
    for f in fwd_outputs + fwd_inputs:
        a = field_map.get(f)
        if a is None:
            cand = [g for g in bwd_inputs + bwd_outputs if g.name == prefix + f.name]
            a = cand[0] if cand else None
        adj_of[f.name] = a
    fwd_kernel_fields = {f.name for f in forward_kernel.ir.fields}
    bwd_kernel_fields = {f.name for f in backward_kernel.ir.fields} if backward_kernel else set()
    class_kwargs = dict()

    # everything that does not depend on the call's tensors is resolved once here
    def _tdtype(field):
        return numpy_dtype_to_torch(field.dtype.numpy_dtype)

    def _fixed(field):
        return tuple(int(x) for x in field.shape) if field.has_fixed_shape else None

    fwd_call = forward_kernel.compile()
    bwd_call = backward_kernel.compile() if backward_kernel else None
    fwd_in = [(i, f.name) for i, f in enumerate(fwd_inputs) if f.name in fwd_kernel_fields]
    def _index_shape(field):
        return tuple(int(n) for n in field.index_shape) if field.index_dimensions else ()

    fwd_reads = {r.field.name for r in forward_kernel.ir.reads}
    fwd_out = [(f.name, _tdtype(f), _fixed(f), _allocator(forward_kernel, f.name, fwd_reads),
                f.spatial_dimensions, _index_shape(f)) for f in fwd_outputs]
    fwd_scalars = [s.name for s in forward_kernel.ir.scalars]
    saved_fwd = [n for n in [f.name for f in fwd_inputs] + [f.name for f in fwd_outputs] if n in bwd_kernel_fields]
    if backward_kernel:
        bwd_reads = {r.field.name for r in backward_kernel.ir.reads}
        bwd_scalars = [s.name for s in backward_kernel.ir.scalars]
        grad_specs = []
        for f in fwd_outputs:
            a = adj_of[f.name]
            grad_specs.append((a.name if a is not None and a.name in bwd_kernel_fields else None, _tdtype(f),
                               _fixed(a) if a is not None else None,
                               tuple(a.strides) if a is not None and a.has_fixed_shape else None, f.name))
        bwd_out = [(f.name, _tdtype(f), _fixed(f), _allocator(backward_kernel, f.name, bwd_reads),
                    f.spatial_dimensions, _index_shape(f)) for f in bwd_outputs]
        in_adj = [adj_of[f.name].name if adj_of.get(f.name) is not None else None for f in fwd_inputs]

    soa_fields = {f.name: f.spatial_dimensions for f in fwd_inputs + fwd_outputs if f.is_soa}

    def _to_device(t, name=None):
        """On the op's device, C-contiguous — or, for an fzyx (SoA) field, in fzyx order."""
        if not isinstance(t, torch.Tensor):
            return t
        if use_cuda:
            if not t.is_cuda:
                t = t.cuda()
        elif t.is_cuda:
            t = t.cpu()
        sdim = soa_fields.get(name)
        if sdim is not None and t.dim() > sdim:
            from ..ps.field import _soa_strides
            if tuple(t.stride()) != _soa_strides(tuple(t.shape), t.dim() - sdim):
                t = _soa_empty(tuple(t.shape), sdim, torch.empty, t.dtype, t.device).copy_(t)
            return t
        return t if t.is_contiguous() else t.contiguous()

    def forward(ctx, *args):
        args = [_to_device(a, fwd_inputs[i].name if i < len(fwd_inputs) else None) for i, a in enumerate(args)]
        first = next((a for a in args if isinstance(a, torch.Tensor)), None)
        if first is None:
            raise ValueError(f"{op_name}: at least one input tensor is required")
        kwargs = {}
        for i, name in fwd_in:
            if i < len(args):
                kwargs[name] = args[i]
        for name in fwd_scalars:
            if name not in class_kwargs:
                raise TypeError(f"{op_name}: scalar parameter '{name}' missing: set {op_name}.class_kwargs['{name}']")
            kwargs[name] = class_kwargs[name]
        outputs = []
        pending = []
        for name, dtype, fixed, alloc, sdim, ishape in fwd_out:
            # variable-size outputs: the first input's spatial extent plus the output's own index shape (the
            # reference takes the first input's whole shape, _torch_native.py:66-72)
            t = alloc(fixed if fixed is not None else tuple(first.shape[:sdim]) + ishape, dtype=dtype,
                      device=first.device, **_border_kw(alloc, pending))
            kwargs[name] = t
            outputs.append(t)
        _launch(fwd_call, kwargs, pending)
        ctx.saved_names = [n for n in saved_fwd if n in kwargs]
        ctx.save_for_backward(*[kwargs[n] for n in ctx.saved_names])
        ctx.scalars = dict(class_kwargs)
        ctx.n_inputs = len(args)
        ctx.like_shape = first.shape
        ctx.like_device = first.device
        return tuple(outputs)

    def backward(ctx, *grad_outputs):
        if backward_kernel is None:
            return tuple(None for _ in range(ctx.n_inputs))
        kwargs = {n: ctx.scalars[n] for n in bwd_scalars}
        for n, t in zip(ctx.saved_names, ctx.saved_tensors):
            kwargs[n] = t
        like = None
        for g, (aname, dtype, fixed, strides, fname) in zip(grad_outputs, grad_specs):
            if g is None:
                shape = fixed if fixed is not None else ctx.like_shape
                g = _soa_empty(shape, soa_fields[fname], torch.zeros, dtype, ctx.like_device) \
                    if fname in soa_fields and len(shape) > soa_fields[fname] else \
                    torch.zeros(shape, dtype=dtype, device=ctx.like_device)
            g = _to_device(g, fname)
            assert g.is_cuda == use_cuda, ("Some of the tensors where on the wrong device. "
                                           f"Op was compiled for CUDA: {str(use_cuda)}")
            if fixed is not None:
                assert tuple(g.shape) == fixed, f"gradient of {fname} has shape {tuple(g.shape)}"
                assert tuple(g.stride()) == strides, f"gradient of {fname} has strides {g.stride()}"
            if aname is not None:
                kwargs[aname] = g
            like = g if like is None else like
        result = {}
        pending = []
        for name, dtype, fixed, alloc, sdim, ishape in bwd_out:
            t = alloc(fixed if fixed is not None else tuple(like.shape[:sdim]) + ishape, dtype=dtype,
                      device=like.device, **_border_kw(alloc, pending))
            result[name] = t
            kwargs[name] = t
        _launch(bwd_call, kwargs, pending)
        return tuple(result.get(a) if a is not None else None for a in in_adj[:ctx.n_inputs]) + \
            (None,) * max(0, ctx.n_inputs - len(in_adj))

    def call(cls, **kwargs):
        rtn = cls.apply(*[kwargs[p.symbol.name] for p in cls.forward_parameters])
        if len(rtn) == 1:
            rtn = rtn[0]
        return rtn

    native = None
    if use_cuda and backward_kernel is not None and not soa_fields and native_module() is not None:
        native = _NativePath({
            'op_name': op_name, 'fwd_inputs': fwd_inputs, 'fwd_out': fwd_out, 'bwd_out': bwd_out,
            'grad_specs': grad_specs, 'saved_fwd': saved_fwd, 'in_adj': in_adj, 'class_kwargs': class_kwargs,
            'scalar_names': sorted(set(fwd_scalars) | set(bwd_scalars)), 'fwd_call': fwd_call, 'bwd_call': bwd_call})
    function_apply = torch.autograd.Function.apply.__func__

    def apply(cls, *args, **kwargs):
        """``Op.apply(*inputs)``: through the native autograd node when the call fits its plan, else the
        Python Function (same kernels, same results)."""
        if native is not None and not kwargs:
            outs = native(args)
            if outs is not None:
                return outs
        return function_apply(cls, *args, **kwargs)

    parameters = module.kernel_wrappers[0].get_parameters()
    cls = type(op_name, (torch.autograd.Function,), {
        'forward': staticmethod(forward),
        'backward': staticmethod(backward),
        'call': classmethod(call),
        'apply': classmethod(apply),
    })
    cls.class_kwargs = class_kwargs
    cls.kernel = forward_kernel
    cls.ast = module
    cls.parameters = parameters
    cls.forward_parameters = [p for p in parameters if p.symbol.name in [f.name for f in fwd_inputs]]
    cls.forward_ast = forward_kernel
    cls.backward_ast = backward_kernel
    cls.num_regs = None
    cls.code = module.code
    cls.autodiff_op = autodiff_obj
    return cls
