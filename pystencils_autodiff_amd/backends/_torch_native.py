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
an extra HBM pass) — ``boundary_handling=None`` keeps ``torch.zeros`` because the
border is not written; only tensors the backward kernel reads are saved on
``ctx``; gradients are returned in forward-input order with ``None`` for
constant fields; native errors raise ``RuntimeError`` instead of ``exit()``.
On ``use_cuda=True`` there is no CPU fallback: a missing HIP extension raises.
"""
import hashlib
from collections import OrderedDict

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


def _full_write(kernel):
    """True if the kernel writes every cell of its outputs (no untouched border)."""
    return kernel.ir.zeros or kernel.ir.ghost_layers == 0


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
    prefix = 'diff'
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
    device_kind = 'cuda' if use_cuda else 'cpu'

    def _to_device(t):
        if not isinstance(t, torch.Tensor):
            return t
        t = t.cuda() if use_cuda else t.cpu()
        return t.contiguous()

    def _alloc(field, like, full):
        dtype = numpy_dtype_to_torch(field.dtype.numpy_dtype)
        shape = tuple(int(s) for s in field.shape) if field.has_fixed_shape else tuple(like.shape)
        alloc = torch.empty if full else torch.zeros
        return alloc(shape, dtype=dtype, device=like.device)

    def forward(ctx, *args):
        args = [_to_device(a) for a in args]
        kwargs = dict(class_kwargs)
        first = next((a for a in args if isinstance(a, torch.Tensor)), None)
        if first is None:
            raise ValueError(f"{op_name}: at least one input tensor is required")
        for i, f in enumerate(fwd_inputs):
            if i < len(args) and f.name in fwd_kernel_fields:
                kwargs[f.name] = args[i]
        full = _full_write(forward_kernel)
        outputs = OrderedDict()
        for f in fwd_outputs:
            if f.name not in kwargs:
                kwargs[f.name] = _alloc(f, first, full)
            outputs[f.name] = kwargs[f.name]
        forward_kernel(**{k: v for k, v in kwargs.items()
                          if k in fwd_kernel_fields or k in {s.name for s in forward_kernel.ir.scalars}})
        # keep what the backward kernel reads: forward inputs / outputs and scalars
        saved_names = [n for n in list(kwargs) if n in bwd_kernel_fields and isinstance(kwargs[n], torch.Tensor)]
        ctx.saved_names = saved_names
        ctx.scalars = {k: v for k, v in kwargs.items() if not isinstance(v, torch.Tensor)}
        ctx.save_for_backward(*[kwargs[n] for n in saved_names])
        ctx.n_inputs = len(args)
        return tuple(outputs.values())

    def backward(ctx, *grad_outputs):
        if backward_kernel is None:
            return tuple(None for _ in range(ctx.n_inputs))
        grads = []
        for g, f in zip(grad_outputs, fwd_outputs):
            if g is None:
                a = adj_of[f.name]
                like = ctx.saved_tensors[0] if ctx.saved_tensors else None
                shape = tuple(int(s) for s in a.shape) if a is not None and a.has_fixed_shape else \
                    (tuple(like.shape) if like is not None else None)
                g = torch.zeros(shape, dtype=numpy_dtype_to_torch(f.dtype.numpy_dtype),
                                device=device_kind if like is None else like.device)
            grads.append(g.contiguous().cuda() if use_cuda else g.contiguous().cpu())
        for g, f in zip(grads, fwd_outputs):
            a = adj_of[f.name]
            if a is None:
                continue
            if a.has_fixed_shape:
                assert tuple(a.shape) == tuple(g.shape), f"gradient of {f.name} has shape {tuple(g.shape)}"
                assert tuple(a.strides) == tuple(g.stride()), f"gradient of {f.name} has strides {g.stride()}"
            assert g.is_cuda == use_cuda, ("Some of the tensors where on the wrong device. "
                                           f"Op was compiled for CUDA: {str(use_cuda)}")
        kwargs = dict(ctx.scalars)
        for n, t in zip(ctx.saved_names, ctx.saved_tensors):
            kwargs[n] = t
        for g, f in zip(grads, fwd_outputs):
            a = adj_of[f.name]
            if a is not None and a.name in bwd_kernel_fields:
                kwargs[a.name] = g
        full = _full_write(backward_kernel)
        like = grads[0]
        result = OrderedDict()
        for f in bwd_outputs:
            # time-constant fields accumulate into their adjoint: start from zeros
            accum = f.name in {r.field.name for r in backward_kernel.ir.reads}
            result[f.name] = _alloc(f, like, full and not accum)
            kwargs[f.name] = result[f.name]
        backward_kernel(**{k: v for k, v in kwargs.items()
                           if k in bwd_kernel_fields or k in {s.name for s in backward_kernel.ir.scalars}})
        out = []
        for i in range(ctx.n_inputs):
            f = fwd_inputs[i] if i < len(fwd_inputs) else None
            a = adj_of.get(f.name) if f is not None else None
            out.append(result.get(a.name) if a is not None else None)
        return tuple(out)

    def call(cls, **kwargs):
        rtn = cls.apply(*[kwargs[p.symbol.name] for p in cls.forward_parameters])
        if len(rtn) == 1:
            rtn = rtn[0]
        return rtn

    parameters = module.kernel_wrappers[0].get_parameters()
    cls = type(op_name, (torch.autograd.Function,), {
        'forward': staticmethod(forward),
        'backward': staticmethod(backward),
        'call': classmethod(call),
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
