"""Reverse-mode differentiation of stencil assignment collections.

This module restates the reference's symbolic AD core
(``src/pystencils_autodiff/_autodiff.py``) on top of the
``pystencils_autodiff_amd.ps`` front-end:

* ``tf_mad_backward`` — "transposed forward-mode" adjoint
  (``_autodiff.py:21-173``): for every forward assignment ``out[w] = f(...)``
  and every non-constant read field ``F``::

      diffF[0] += sum_{ra in accesses of F} ∂f/∂ra · diffout[-ra.offsets - w]

  i.e. the adjoint is again a *gather* with flipped stencil offsets, every cell
  of ``diffF`` written by exactly one thread. Faithful quirks kept for parity:
  the partial derivative is evaluated at the forward cell's own neighbourhood
  (exact only for linear stencils, ``_autodiff.py:102-109``); time-constant
  fields accumulate per forward assignment (``:110-113``); the vector-field
  branch keeps only the last component's assignment (``:125-152``).
* ``transposed_backward`` — classic transposed adjoint (``_autodiff.py:354-437``),
  a scatter, only valid where writes stay exclusive.
* ``AutoDiffOp`` — the operator object (``_autodiff.py:209-709``) with the same
  constructor, properties, field orderings (sorted by ``str``) and
  ``create_tensorflow_op(backend='torch_native')`` entry point; the kernels it
  hands out are MI355X HIP kernels (``backends/``) instead of pystencils ASTs.
"""
import collections
from enum import Enum
from typing import List

import numpy as np
import sympy as sp

from ._adjoint_field import AdjointField
from .backends import AVAILABLE_BACKENDS
from .ps import Assignment, AssignmentCollection, Field
from .ps.simp import sympy_cse_on_assignment_list

__all__ = ['AutoDiffOp', 'AutoDiffBoundaryHandling', 'DiffModes', 'create_backward_assignments',
           'get_jacobian_of_assignments', 'AutoDiffAstPair', 'has_exclusive_writes']

DEFAULT_OP_NAME = "autodiffop"


class AutoDiffBoundaryHandling(str, Enum):
    """In-kernel boundary handling (``_autodiff.py:176-197``).

    ``None``: interior cells only (a stencil-radius wide border is not written).
    ``'zeros'``: out-of-domain reads are 0, every cell is written, forward and backward.
    ``'valid'``: not implemented by the reference either (``_autodiff.py:246-247``).
    ``'periodic'``: (extension, not in the reference) reads and offset writes wrap around the domain,
    every cell is written — the lattice Boltzmann step's periodic lattice (``lbm/``) without ghost layers.
    """
    NONE = None
    ZEROS = 'zeros'
    VALID = 'valid'
    PERIODIC = 'periodic'


class DiffModes(str, Enum):
    """Backward differentiation mode (``_autodiff.py:200-206``)."""
    TRANSPOSED = 'transposed'
    TF_MAD = 'transposed-forward'


def _is_constant(field, constant_fields):
    return field in constant_fields or field.name in constant_fields


def _flatten_forward(forward_assignments):
    """Main assignments with all subexpressions substituted (``_autodiff.py:35-45``)."""
    ac = forward_assignments
    if hasattr(ac, 'new_without_subexpressions'):
        ac = ac.new_without_subexpressions()
    if hasattr(ac, 'main_assignments'):
        ac = ac.main_assignments
    return AssignmentCollection(list(ac), [])


def _finish_backward(backward_list, do_cse):
    """CSE (errors swallowed like ``_autodiff.py:158-163``), then split main/subexpressions."""
    if do_cse:
        try:
            backward_list = sympy_cse_on_assignment_list(backward_list)
        except Exception:  # noqa: BLE001 - the reference ignores CSE failures too
            pass
    main = [a for a in backward_list if isinstance(a.lhs, Field.Access)]
    subs = [a for a in backward_list if not isinstance(a.lhs, Field.Access)]
    return AssignmentCollection(main, subs)


def tf_mad_backward(forward_assignments, diff_fields_prefix='diff', constant_fields=(),
                    time_constant_fields=None, do_cse=True):
    """TF-MAD adjoint. Returns ``(backward_collection, info)`` where ``info`` holds the
    forward read/write accesses and fields in the reference's (``str``-sorted) order."""
    forward = _flatten_forward(forward_assignments)
    reads = sorted((s for s in forward.free_symbols if isinstance(s, Field.Access)), key=str)
    writes = [a.lhs for a in forward.main_assignments]
    if not writes or not all(isinstance(w, Field.Access) for w in writes):
        raise AssertionError("Please check if your assignments are a AssignmentCollection or main_assignments only")
    read_fields = sorted({a.field for a in reads}, key=str)
    write_fields = sorted({w.field for w in writes}, key=str)

    adj_read = {f: AdjointField(f, diff_fields_prefix) for f in read_fields
                if not _is_constant(f, constant_fields)}
    adj_write = {f: AdjointField(f, diff_fields_prefix) for f in write_fields}
    time_const = time_constant_fields

    contributions = collections.OrderedDict()   # adjoint lhs -> list of rhs terms

    def add(lhs, rhs):
        contributions.setdefault(lhs, []).append(rhs)

    for fa in forward.main_assignments:
        out_adj = adj_write[fa.lhs.field]
        w_off, w_idx = fa.lhs.offsets, fa.lhs.index
        for F in read_fields:
            if _is_constant(F, constant_fields):
                continue
            dF = adj_read[F]
            accumulate = time_const is not None and F in time_const
            if dF.index_dimensions == 0:
                total = 0
                for ra in reads:
                    if ra.field != F:
                        continue
                    flipped = tuple(-o - w for o, w in zip(ra.offsets, w_off))
                    total += sp.diff(fa.rhs, ra) * out_adj[flipped](*w_idx)
                add(dF.center, dF.center + total if accumulate else total)
            elif dF.index_dimensions == 1:
                per_index = {}
                for ra in reads:
                    if ra.field != F:
                        continue
                    # the reference flips against the FIRST write access and drops the write index
                    flipped = tuple(-o - w for o, w in zip(ra.offsets, writes[0].offsets))
                    per_index[ra.index[0]] = per_index.get(ra.index[0], 0) + \
                        sp.diff(fa.rhs, ra) * out_adj[flipped]
                last = None
                for idx, s in per_index.items():
                    lhs = dF.center.at_index(idx)
                    last = (lhs, lhs + s if accumulate else s)
                if last is None:
                    raise UnboundLocalError("vector-field adjoint without contributions")
                # quirk kept for parity: only the last component is stored (``_autodiff.py:149-152``)
                add(*last)
            else:
                raise NotImplementedError()

    backward = [Assignment(lhs, sp.Add(*terms)) for lhs, terms in contributions.items()]
    backward = _finish_backward(backward, do_cse)
    if not has_exclusive_writes(backward):
        raise AssertionError("Backward assignments don't have exclusive writes!")
    info = dict(forward_read_accesses=reads, forward_write_accesses=sorted(writes, key=str),
                forward_input_fields=read_fields, forward_output_fields=write_fields,
                backward_field_map={**adj_read, **adj_write})
    return backward, info


def transposed_backward(forward_assignments, diff_fields_prefix='diff', constant_fields=(),
                        time_constant_fields=None, do_cse=True):
    """Classic transposed adjoint (``_autodiff.py:354-437``): ``diffF[ra] = (∂f/∂ra)ᵀ · diffout``."""
    forward = _flatten_forward(forward_assignments)
    reads = [s for s in forward.free_symbols if isinstance(s, Field.Access)]
    writes = [a.lhs for a in forward.main_assignments]
    if not all(isinstance(w, Field.Access) for w in writes):
        raise AssertionError("Please assure that you only assign to fields in your main_assignments!")
    read_fields = {a.field for a in reads}
    write_fields = {w.field for w in writes}
    adj_read = {f: AdjointField(f, diff_fields_prefix) for f in read_fields}
    adj_write = {f: AdjointField(f, diff_fields_prefix) for f in write_fields}
    adj_write_acc = sp.Matrix([adj_write[w.field][w.offsets](*w.index) for w in writes])
    rhs_vec = sp.Matrix([a.rhs for a in forward.main_assignments])

    backward = []
    for ra in reads:
        if _is_constant(ra.field, constant_fields):
            continue
        lhs = adj_read[ra.field][ra.offsets](*ra.index)
        rhs = (rhs_vec.diff(ra).T * adj_write_acc)[0, 0]
        if time_constant_fields is not None and ra.field in time_constant_fields:
            backward.append(Assignment(lhs, lhs + rhs))
        else:
            backward.append(Assignment(lhs, rhs))
    backward = _finish_backward(backward, do_cse)
    if not has_exclusive_writes(backward):
        raise AssertionError("Backward assignments don't have exclusive writes. "
                             "You should consider using 'transposed-forward' mode for resolving those conflicts")
    # the reference lists the fields in set order (``_autodiff.py:430-431``: hash-seed dependent across
    # processes); sorted by ``str`` here, the TF-MAD mode's order, so positional arguments are stable
    out_fields = sorted(write_fields, key=str)
    in_fields = sorted(read_fields, key=str)
    field_map = {**adj_read, **adj_write}
    info = dict(forward_read_accesses=reads, forward_write_accesses=writes,
                forward_input_fields=in_fields, forward_output_fields=out_fields,
                backward_field_map=field_map,
                backward_input_fields=[field_map[f] for f in out_fields],
                backward_output_fields=[field_map[f] for f in in_fields])
    return backward, info


def has_exclusive_writes(assignment_collection):
    """Each (field, index) written at most once (``_autodiff.py:759-779``)."""
    seen = set()
    for a in assignment_collection.main_assignments:
        if not isinstance(a.lhs, Field.Access):
            continue
        key = (a.lhs.field, a.lhs.index)
        if key in seen:
            return False
        seen.add(key)
    return True


_has_exclusive_writes = has_exclusive_writes


def get_jacobian_of_assignments(assignments, diff_variables):
    """Jacobian of the main assignments' right-hand sides (``_autodiff.py:782-798``)."""
    if hasattr(assignments, 'main_assignments'):
        assignments = assignments.main_assignments
    return sp.Matrix([a.rhs for a in assignments]).jacobian(diff_variables)


class AutoDiffOp:
    """Forward + adjoint stencil operator (reference ``_autodiff.py:209``)."""

    def __init__(self,
                 forward_assignments: List[Assignment],
                 op_name: str = DEFAULT_OP_NAME,
                 boundary_handling: AutoDiffBoundaryHandling = None,
                 time_constant_fields: List[Field] = None,
                 constant_fields: List[Field] = (),
                 diff_fields_prefix='diff',
                 do_common_subexpression_elimination=True,
                 diff_mode=DiffModes.TF_MAD,
                 backward_assignments=None,
                 **kwargs):
        diff_mode = DiffModes(diff_mode)
        if 'target' in kwargs:
            assert kwargs['target'].lower() in ['cpu', 'gpu'], "AutoDiffOp always supports both cpu and gpu"
            del kwargs['target']
        kwargs.pop('no_chaching', None)   # accepted (and ignored) by the reference too

        main = [a for a in forward_assignments if isinstance(a.lhs, Field.Access)]
        subs = [a for a in forward_assignments if not isinstance(a.lhs, Field.Access)]
        forward = AssignmentCollection(main, subs)

        if boundary_handling is not None:
            boundary_handling = AutoDiffBoundaryHandling(boundary_handling)
        if boundary_handling == AutoDiffBoundaryHandling.VALID:
            raise NotImplementedError('there seems to be still a bug with valid. -> Use "zeros"')
        if boundary_handling == AutoDiffBoundaryHandling.NONE:
            boundary_handling = None

        self._forward_assignments = forward
        self._constant_fields = list(constant_fields) + ['indexVector']
        self._time_constant_fields = time_constant_fields
        self._kwargs = kwargs
        self.op_name = op_name
        self._diff_fields_prefix = diff_fields_prefix
        self._do_common_subexpression_elimination = do_common_subexpression_elimination
        self._boundary_handling = boundary_handling
        self._diff_mode = diff_mode
        self._kernels = {}
        self._forward_read_accesses = None
        self._forward_write_accesses = None
        self._backward_field_map = None

        if backward_assignments:
            self._backward_assignments = backward_assignments
            self._forward_input_fields = sorted(forward.free_fields, key=str)
            self._forward_output_fields = sorted(forward.bound_fields, key=str)
            self._backward_input_fields = sorted(backward_assignments.free_fields, key=str)
            self._backward_output_fields = sorted(backward_assignments.bound_fields, key=str)
        elif diff_mode == DiffModes.TRANSPOSED:
            backward, info = transposed_backward(forward, diff_fields_prefix, self._constant_fields,
                                                 time_constant_fields, do_common_subexpression_elimination)
            self._backward_assignments = backward
            self._forward_read_accesses = info['forward_read_accesses']
            self._forward_write_accesses = info['forward_write_accesses']
            self._forward_input_fields = info['forward_input_fields']
            self._forward_output_fields = info['forward_output_fields']
            self._backward_field_map = info['backward_field_map']
            self._backward_input_fields = info['backward_input_fields']
            self._backward_output_fields = info['backward_output_fields']
        else:
            backward, info = tf_mad_backward(forward, diff_fields_prefix, self._constant_fields,
                                             time_constant_fields, do_common_subexpression_elimination)
            self._backward_assignments = backward
            self._forward_read_accesses = info['forward_read_accesses']
            self._forward_write_accesses = info['forward_write_accesses']
            self._backward_field_map = info['backward_field_map']
            # the reference re-derives the orderings from the collections (``_autodiff.py:289-294``)
            self._forward_input_fields = sorted(forward.free_fields, key=str)
            self._forward_output_fields = sorted(forward.bound_fields, key=str)
            self._backward_input_fields = sorted(backward.free_fields, key=str)
            self._backward_output_fields = sorted(backward.bound_fields, key=str)

    # -- identity / printing --------------------------------------------------------------------
    def __hash__(self):
        return hash((str(self.forward_assignments), str(self.backward_assignments), str(self.constant_fields)))

    def __repr__(self):
        fwd = str(self.forward_assignments).replace('\n', '\n    ').rstrip()
        bwd = str(self.backward_assignments).replace('\n', '\n    ').rstrip()
        return f"Forward:\n    {fwd}\nBackward:\n    {bwd}\n"

    def __str__(self):
        return self.__repr__()

    def __getstate__(self):
        return {'forward_assignments': self.forward_assignments,
                'backward_assignments': self.backward_assignments,
                'kwargs': self._kwargs,
                'boundary_handling': self._boundary_handling,
                'op_name': self.op_name}

    def __setstate__(self, state):
        self.__init__(state['forward_assignments'], op_name=state.get('op_name', DEFAULT_OP_NAME),
                      boundary_handling=state.get('boundary_handling'),
                      backward_assignments=state['backward_assignments'], **state['kwargs'])

    # -- assignments & fields -------------------------------------------------------------------
    @property
    def forward_assignments(self):
        return self._forward_assignments

    @property
    def backward_assignments(self):
        return self._backward_assignments

    @property
    def boundary_handling(self):
        return self._boundary_handling

    def jacobian(self):
        return get_jacobian_of_assignments(self._forward_assignments, self._forward_read_accesses)

    @property
    def forward_write_accesses(self):
        return self._forward_write_accesses

    @property
    def forward_read_accesses(self):
        return self._forward_read_accesses

    @property
    def backward_write_accesses(self):
        return [a.lhs for a in self.backward_assignments.main_assignments]

    @property
    def backward_read_accesses(self):
        return [a for a in self.backward_assignments.free_symbols if isinstance(a, Field.Access)]

    @property
    def forward_input_fields(self):
        return self._forward_input_fields

    @property
    def forward_output_fields(self):
        return self._forward_output_fields

    @property
    def backward_input_fields(self):
        return self._backward_input_fields

    @property
    def backward_output_fields(self):
        return self._backward_output_fields

    @property
    def backward_fields(self):
        return self._backward_output_fields + self._backward_input_fields

    @property
    def forward_fields(self):
        return self._forward_output_fields + self._forward_input_fields

    @property
    def constant_fields(self):
        return self._constant_fields

    @property
    def diff_fields_prefix(self):
        return self._diff_fields_prefix

    def adjoint_name(self, field):
        """Name of the adjoint of a forward field: the field map the adjoint derivation built
        (``_autodiff.py:81-84``), else ``<diff_fields_prefix><name>`` (user-given backward assignments)."""
        fmap = self._backward_field_map or {}
        a = fmap.get(field)
        return a.name if a is not None else self._diff_fields_prefix + field.name

    @property
    def time_constant_fields(self):
        return self._time_constant_fields

    # -- kernels (MI355X HIP on 'gpu', C on 'cpu') ----------------------------------------------
    def _kernel(self, which, target):
        key = (which, target)
        if key not in self._kernels:
            from .backends.kernel_ir import StencilKernel
            ac = self._forward_assignments if which == 'forward' else self._backward_assignments
            assert ac, 'No backward assignments!'
            self._kernels[key] = StencilKernel(ac, boundary_handling=self._boundary_handling,
                                               function_name=f"{self.op_name}_{which}_{target}",
                                               target=target, **self._kwargs)
        return self._kernels[key]

    @property
    def forward_ast_gpu(self):
        return self._kernel('forward', 'gpu')

    @property
    def backward_ast_gpu(self):
        return self._kernel('backward', 'gpu')

    @property
    def forward_ast_cpu(self):
        return self._kernel('forward', 'cpu')

    @property
    def backward_ast_cpu(self):
        return self._kernel('backward', 'cpu')

    @property
    def forward_kernel_gpu(self):
        return self.forward_ast_gpu.compile()

    @property
    def backward_kernel_gpu(self):
        return self.backward_ast_gpu.compile()

    @property
    def forward_kernel_cpu(self):
        return self.forward_ast_cpu.compile()

    @property
    def backward_kernel_cpu(self):
        return self.backward_ast_cpu.compile()

    def _create_kernel(self, which, target='cpu', data_type=None, iteration_slice=None, ghost_layers=None,
                       **kwargs):
        """``ps.create_kernel(assignments, *args, **kwargs).compile()`` (``_autodiff.py:592-598``): a
        compiled kernel of this op's forward / backward assignments with pystencils' defaults — interior
        only unless ``ghost_layers=0`` (then out-of-domain reads are zeros, the only defined meaning);
        ``iteration_slice`` (slices — strided too — / ints per axis, absolute coordinates) restricts the cells written,
        as in pystencils (ghost layers are then ignored; reads leaving the domain read zeros)."""
        from .backends.kernel_ir import StencilKernel
        ac = self._forward_assignments if which == 'forward' else self._backward_assignments
        if ghost_layers not in (None, 0) and iteration_slice is None:
            # pystencils' explicit ghost layers: k per axis, or (lower, upper) per axis -> iterate [lo, N - hi); the
            # stencil's reads then stay inside the array for a radius up to the layer count, as pystencils' do
            ndim = ac.main_assignments[0].lhs.field.spatial_dimensions
            gl = [(int(ghost_layers), int(ghost_layers))] * ndim if isinstance(ghost_layers, (int, np.integer)) \
                else [(int(g), int(g)) if isinstance(g, (int, np.integer)) else (int(g[0]), int(g[1]))
                      for g in ghost_layers]
            if len(gl) != ndim:
                raise ValueError(f'ghost_layers {ghost_layers}: one entry per spatial axis ({ndim})')
            if len(set(gl)) == 1 and gl[0][0] == gl[0][1]:
                # the same k layers on every side, at least the stencil's own (pystencils' required ghost layers):
                # the interior-only kernel of boundary_handling=None with k layers — the tuned schedules, not the
                # one-thread-per-cell slice kernel (ghost_layers=1 on a radius-1 stencil is the default's cells)
                k = StencilKernel(ac, boundary_handling=None, function_name=f"{self.op_name}_{which}_{target}_custom",
                                  target=target, data_type=data_type, **{**self._kwargs, **kwargs})
                if gl[0][0] >= k.ir.ghost_layers:
                    k.ir.ghost_layers = gl[0][0]
                    return k.compile()
            iteration_slice = tuple(slice(lo, -hi if hi else None) for lo, hi in gl)
        bh = 'zeros' if ghost_layers == 0 else None
        return StencilKernel(ac, boundary_handling=bh, function_name=f"{self.op_name}_{which}_{target}_custom",
                             target=target, data_type=data_type, iteration_slice=iteration_slice,
                             **{**self._kwargs, **kwargs}).compile()

    def create_forward_kernel(self, *args, **kwargs):
        return self._create_kernel('forward', *args, **kwargs)

    def create_backward_kernel(self, *args, **kwargs):
        return self._create_kernel('backward', *args, **kwargs)

    def get_forward_kernel(self, is_gpu):
        return self.forward_kernel_gpu if is_gpu else self.forward_kernel_cpu

    def get_backward_kernel(self, is_gpu):
        return self.backward_kernel_gpu if is_gpu else self.backward_kernel_cpu

    # -- framework ops --------------------------------------------------------------------------
    def create_torch_op(self, *args, **kwargs):
        return self.create_tensorflow_op(*args, backend='torch_native', **kwargs)

    def create_tensorflow_op(self, inputfield_tensor_dict={}, forward_loop=None, backward_loop=None,  # noqa: B006
                             use_cuda=True, backend='tensorflow'):
        """Build the framework operator (``_autodiff.py:611-709``).

        Only ``backend='torch_native'`` is provided by the MI355X layer: it returns a
        ``torch.autograd.Function`` subclass whose kernels are HIP (``use_cuda=True``) or
        C (``use_cuda=False``). The TensorFlow backends and the python-loop ``'torch'``
        backend are out of scope and raise ``NotImplementedError``.
        """
        backend = backend.lower()
        assert backend in AVAILABLE_BACKENDS, \
            f"\"{backend}\" is not a valid backend. Available backends: {AVAILABLE_BACKENDS}"
        for f in inputfield_tensor_dict.keys():
            if isinstance(f, Field) and f not in self._forward_input_fields:
                f_adjoint = AdjointField(f)
                self._forward_input_fields.append(f)
                self._backward_output_fields.append(f_adjoint)
                if self._backward_field_map is not None:
                    self._backward_field_map[f] = f_adjoint
        if backend == 'torch':
            # the reference's python-loop backend (backends/_pytorch.py:18-85) runs the same kernels on
            # tensors given up front (and is a legacy, instance-method autograd.Function current torch
            # rejects); here it is the native Function, on the device of those tensors
            if forward_loop is not None or backward_loop is not None:
                raise NotImplementedError("custom forward_loop / backward_loop callables are not supported; "
                                          "the operator runs the generated kernels")
            tensors = [t for t in inputfield_tensor_dict.values() if hasattr(t, 'is_cuda')]
            use_cuda = bool(tensors) and all(t.is_cuda for t in tensors)
            backend = 'torch_native'
        if backend == 'torch_native':
            from .backends import _torch_native
            return _torch_native.create_autograd_function(
                self, use_cuda, op_name=self.op_name if self.op_name != DEFAULT_OP_NAME else None)
        raise NotImplementedError(f"backend '{backend}' is not provided by the MI355X execution layer; "
                                  "use backend='torch_native'")


def create_backward_assignments(forward_assignments, diff_fields_prefix="diff", time_constant_fields=[],  # noqa: B006
                                constant_fields=[], diff_mode=DiffModes.TF_MAD,  # noqa: B006
                                do_common_sub_expression_elimination=True):
    """Backward assignments of ``forward_assignments`` (``_autodiff.py:712-729``)."""
    op = AutoDiffOp(forward_assignments, diff_fields_prefix=diff_fields_prefix,
                    time_constant_fields=time_constant_fields, constant_fields=constant_fields,
                    diff_mode=diff_mode, do_common_subexpression_elimination=do_common_sub_expression_elimination)
    return op.backward_assignments


class AutoDiffAstPair:
    """Forward/backward kernel pair (``_autodiff.py:732-756``)."""

    def __init__(self, forward_ast, backward_ast, compilation_target='cpu'):
        self.forward_ast = forward_ast
        self.backward_ast = backward_ast
        self._target = compilation_target
        self._forward_kernel = self.forward_ast.compile()
        self._backward_kernel = None

    def backward(self, *args, **kwargs):
        if not self._backward_kernel:
            self._backward_kernel = self.backward_ast.compile()
        return self._backward_kernel(*args, **kwargs)

    def forward(self, *args, **kwargs):
        return self._forward_kernel(*args, **kwargs)

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)
