"""Lowering of an assignment collection into a stencil kernel description.

This is the MI355X layer's replacement for ``pystencils.create_kernel``
([ext], called from ``_autodiff.py:479-542``): it fixes the semantics the
reference's generated kernels have, independent of how they are scheduled:

* iteration space = the common spatial shape of all fields, C layout,
  coordinate 0 slowest;
* ``boundary_handling='zeros'`` (``transformations.py:12-36`` +
  ``ghost_layers=0``): every cell is written; a read outside the domain yields
  exactly 0 (``ConditionalFieldAccess`` atoms are recognised and stripped —
  the zero-filled halo load realises them);
* ``boundary_handling=None`` (``ghost_layers=None``): only the interior
  ``[g, N-g)`` of every axis is written, ``g`` = largest ``|offset|`` of any
  access (pystencils' ``required_ghost_layers`` rule), the border keeps what the
  caller allocated (zeros in the torch op);
* statements are evaluated in order: subexpressions, then main assignments;
  free non-field symbols become scalar kernel parameters (sorted by name).

``StencilKernel`` keeps pystencils' ``KernelFunction`` surface the reference
touches (``function_name``, ``fields_accessed``, ``fields_read``,
``fields_written``, ``get_parameters()``, ``compile()``) and picks the
schedule the HIP emitter prints (``hip_emitter.py``).
"""
import hashlib
import itertools
from dataclasses import dataclass, field as dc_field
from functools import cached_property
from typing import Dict, List, Optional, Tuple

import numpy as np
import sympy as sp

from ..ps import AssignmentCollection, Field
from ..ps.conditional import ConditionalFieldAccess

__all__ = ['StencilKernel', 'KernelIR', 'lower', 'Parameter']


def _c_ident(s):
    out = ''.join(ch if ch.isalnum() else '_' for ch in str(s))
    return out if not out[:1].isdigit() else '_' + out


def _offset_tag(offsets):
    return '_'.join(f"m{-o}" if o < 0 else str(o) for o in offsets)


@dataclass(frozen=True)
class ReadAccess:
    field: Field
    offsets: Tuple[int, ...]
    index: Tuple[int, ...]

    @property
    def var(self):
        tag = _offset_tag(self.offsets)
        idx = ('_i' + '_'.join(str(i) for i in self.index)) if self.index else ''
        return f"v_{_c_ident(self.field.name)}_{tag}{idx}"


@dataclass
class KernelIR:
    ndim: int
    fields: List[Field]                    # pointer-argument order (sorted by name)
    fields_read: List[Field]
    fields_written: List[Field]
    reads: List[ReadAccess]                # unique reads, sorted
    scalars: List[sp.Symbol]               # scalar parameters, sorted by name
    subexpressions: List[Tuple[sp.Symbol, sp.Expr]]
    stores: List[Tuple[Field, Tuple[int, ...], Tuple[int, ...], sp.Expr]]  # field, lhs offsets, index, rhs
    zeros: bool                            # zero-padded reads, full iteration space
    ghost_layers: int                      # interior-only iteration when not zeros
    radius: Tuple[int, ...]                # per-axis max |read offset|
    compute_dtype: np.dtype
    symbol_names: Dict[sp.Symbol, str] = dc_field(default_factory=dict)
    periodic: bool = False                 # reads / offset writes wrap around, full iteration space
    islice: Optional[Tuple] = None         # pystencils' iteration_slice: per-axis (start, stop)
    isteps: Optional[Tuple] = None         # ... and its per-axis steps (None: all 1)

    @cached_property
    def pointwise(self):
        return all(all(o == 0 for o in r.offsets) for r in self.reads) and \
            all(all(o == 0 for o in s[1]) for s in self.stores)

    @cached_property
    def has_index_dims(self):
        return any(f.index_dimensions > 0 for f in self.fields)

    @cached_property
    def stencil_fields(self):
        """Read fields with at least one non-zero offset (they need halo data)."""
        return sorted({r.field for r in self.reads if any(o != 0 for o in r.offsets)}, key=lambda f: f.name)

    @cached_property
    def point_fields(self):
        st = set(self.stencil_fields)
        return sorted({r.field for r in self.reads if r.field not in st}, key=lambda f: f.name)

    def iteration_bounds(self, shape):
        """Per-axis [lo, hi) of the cells this kernel writes."""
        if self.islice is not None:
            # strided slices: [lo, lo + count) numbers the cells the kernel writes, cell k at lo + k·step
            out = []
            steps = self.isteps or (1,) * len(self.islice)
            for (a, b), s, n in zip(self.islice, steps, shape):
                lo, hi, _ = slice(a, b, s).indices(int(n))
                out.append((lo, lo + len(range(lo, hi, s))))
            return out
        g = 0 if self.zeros or self.periodic else self.ghost_layers
        return [(g, max(g, int(n) - g)) for n in shape]


def normalize_slice(iteration_slice, ndim):
    """``iteration_slice`` (a slice / int per spatial axis, e.g. ``make_slice[1:-1, 2]`` or ``make_slice[::2, 1::3]``)
    as ``(((start, stop), …), steps or None)``; missing trailing axes are whole. Steps are positive (pystencils'
    ``create_kernel`` iterates ``start, start + step, … < stop``)."""
    items = iteration_slice if isinstance(iteration_slice, tuple) else (iteration_slice,)
    if len(items) > ndim:
        raise ValueError(f'iteration_slice {iteration_slice} has more axes than the {ndim}-d kernel')
    out, steps = [], []
    for it in list(items) + [slice(None)] * (ndim - len(items)):
        if isinstance(it, slice):
            step = 1 if it.step is None else int(it.step)
            if step < 1:
                raise NotImplementedError(f'iteration_slice with step {it.step}: positive steps only')
            out.append((it.start, it.stop))
            steps.append(step)
        elif isinstance(it, (int, np.integer)):
            i = int(it)
            out.append((i, i + 1 if i != -1 else None))
            steps.append(1)
        else:
            raise TypeError(f'iteration_slice entry {it!r}: a slice or an int')
    return tuple(out), (tuple(steps) if any(s != 1 for s in steps) else None)


def _strip_conditionals(expr):
    if not expr.has(ConditionalFieldAccess):
        return expr, False
    return expr.replace(lambda e: isinstance(e, ConditionalFieldAccess), lambda e: e.args[0]), True


def lower(assignments, boundary_handling=None, data_type=None):
    """Build the ``KernelIR`` of an assignment collection."""
    if not isinstance(assignments, AssignmentCollection):
        assignments = AssignmentCollection(list(assignments), [])
    zeros = boundary_handling is not None and str(getattr(boundary_handling, 'value', boundary_handling)) \
        in ('zeros', 'valid')
    periodic = boundary_handling is not None and str(getattr(boundary_handling, 'value', boundary_handling)) \
        == 'periodic'

    subexpressions, stores = [], []
    had_conditionals = False
    ordered = list(assignments.subexpressions) + list(assignments.main_assignments)
    for a in ordered:
        rhs, had = _strip_conditionals(a.rhs)
        had_conditionals |= had
        if isinstance(a.lhs, Field.Access):
            stores.append((a.lhs.field, tuple(a.lhs.offsets), tuple(a.lhs.index), rhs))
        else:
            subexpressions.append((a.lhs, rhs))
    zeros = zeros or had_conditionals
    if periodic and had_conditionals:
        raise ValueError("periodic boundary handling of assignments with conditional (zero-padded) reads")
    if not stores:
        raise ValueError('kernel without field writes')

    reads = set()
    scalars = set()
    bound = {s for s, _ in subexpressions}
    all_accesses = []
    for _, rhs in subexpressions:
        for s in rhs.free_symbols:
            if isinstance(s, Field.Access):
                reads.add(ReadAccess(s.field, tuple(s.offsets), tuple(s.index)))
                all_accesses.append(s.offsets)
            elif s not in bound:
                scalars.add(s)
    for _, _, _, rhs in stores:
        for s in rhs.free_symbols:
            if isinstance(s, Field.Access):
                reads.add(ReadAccess(s.field, tuple(s.offsets), tuple(s.index)))
                all_accesses.append(s.offsets)
            elif s not in bound:
                scalars.add(s)
    all_accesses += [s[1] for s in stores]

    fields_written = sorted({s[0] for s in stores}, key=lambda f: f.name)
    fields_read = sorted({r.field for r in reads}, key=lambda f: f.name)
    fields = sorted(set(fields_written) | set(fields_read), key=lambda f: f.name)
    names = [f.name for f in fields]
    if len(set(names)) != len(names):
        raise ValueError(f"two different fields share a name: {names}")
    ndims = {f.spatial_dimensions for f in fields}
    if len(ndims) != 1:
        raise ValueError(f"all fields of a kernel must have the same number of spatial dimensions, got {ndims}")
    ndim = ndims.pop()
    fixed = [tuple(int(s) for s in f.spatial_shape) for f in fields if f.has_fixed_shape]
    if fixed and any(s != fixed[0] for s in fixed):
        raise ValueError(f"fields of one kernel must share their spatial shape, got {fixed}")

    radius = tuple(max([abs(int(r.offsets[d])) for r in reads] + [0]) for d in range(ndim))
    ghost_layers = max([max([abs(int(o)) for o in offs] + [0]) for offs in all_accesses] + [0])
    if zeros or periodic or ghost_layers == 0:
        # components of a vector output that no assignment writes are the zeros of the reference's
        # torch.zeros allocation (_torch_native.py:61-73); with every cell written they become zero
        # stores, so the output is allocated uninitialised and written in one pass (no memset sweep)
        read_names = {r.field.name for r in reads}
        for f in fields_written:
            if not f.index_dimensions or f.name in read_names:
                continue
            mine = [st for st in stores if st[0] == f]
            offs = {st[1] for st in mine}
            written = {st[2] for st in mine}
            if len(offs) == 1:
                off = next(iter(offs))
                for idx in itertools.product(*[range(int(n)) for n in f.index_shape]):
                    if idx not in written:
                        stores.append((f, off, idx, sp.Integer(0)))

    dtypes = {f.dtype.numpy_dtype for f in fields}
    if data_type is not None:
        from ..ps.data_types import create_type
        compute = create_type(data_type).numpy_dtype
    elif np.dtype('float64') in dtypes:
        compute = np.dtype('float64')
    else:
        compute = np.dtype('float32')          # float32 and float16 storage compute in float32
    for f in fields:
        if not f.dtype.is_float:
            raise NotImplementedError(f"field '{f.name}' has non-floating dtype {f.dtype}")

    reads = sorted(reads, key=lambda r: (r.field.name, r.offsets, r.index))
    scalars = sorted(scalars, key=lambda s: s.name)
    ir = KernelIR(ndim=ndim, fields=fields, fields_read=fields_read, fields_written=fields_written,
                  reads=reads, scalars=scalars, subexpressions=subexpressions, stores=stores, zeros=zeros,
                  ghost_layers=ghost_layers, radius=radius, compute_dtype=compute, periodic=periodic)
    sym = {}
    for r in reads:
        acc = Field.Access(r.field, r.offsets, r.index)
        sym[acc] = r.var
    for s in scalars:
        sym[s] = f"p_{_c_ident(s.name)}"
    for i, (s, _) in enumerate(subexpressions):
        sym[s] = f"s{i}_{_c_ident(s.name)}"
    ir.symbol_names = sym
    return ir


def split_soa(ir):
    """The GPU view of a kernel with fzyx (SoA) vector fields: every component of such a field becomes a
    scalar field of its own (``Field.component_field``), so each component plane is a C-contiguous array
    and the stencil schedules (``zsum``, ``march``, ``pointwise``) run unchanged on it — a component read
    ``u[o](k)`` is a scalar read ``u__ck[o]``. Returns ``(ir, components)`` with ``components`` =
    ``{field name: [(component field, index), ...]}`` (empty, and ``ir`` itself, without SoA fields).
    The split happens after ``lower``, so components completed with zero stores are kept as stores."""
    soa = [f for f in ir.fields if f.is_soa]
    if not soa:
        return ir, {}
    comps, sub = {}, {}
    for f in soa:
        comps[f.name] = [(f.component_field(idx), idx)
                         for idx in itertools.product(*[range(int(n)) for n in f.index_shape])]
    cf = {(name, idx): c for name, lst in comps.items() for c, idx in lst}

    def acc(field, offsets, idx):
        return Field.Access(cf[(field.name, tuple(idx))], tuple(offsets))
    for r in ir.reads:
        if r.field.is_soa:
            sub[Field.Access(r.field, r.offsets, r.index)] = acc(r.field, r.offsets, r.index)
    subexpressions = [(s, e.xreplace(sub)) for s, e in ir.subexpressions]
    stores = []
    for f, offs, idx, rhs in ir.stores:
        lhs = acc(f, offs, idx) if f.is_soa else Field.Access(f, offs, idx)
        stores.append((lhs, rhs.xreplace(sub)))
    from ..ps import Assignment
    ac = AssignmentCollection([Assignment(lhs, rhs) for lhs, rhs in stores],
                              [Assignment(s, e) for s, e in subexpressions])
    out = lower(ac, 'zeros' if ir.zeros else ('periodic' if ir.periodic else None), np.dtype(ir.compute_dtype).name)
    if not out.zeros and not out.periodic and out.ghost_layers != ir.ghost_layers:
        raise AssertionError('SoA split changed the iteration space')
    return out, comps


class Parameter:
    """Kernel parameter (mirrors pystencils ``KernelFunction.Parameter``: ``.symbol.name``)."""

    def __init__(self, symbol, field=None):
        self.symbol = symbol
        self.field = field
        self.is_field_parameter = field is not None

    @property
    def field_name(self):
        return self.field.name if self.field is not None else None

    def __repr__(self):
        return f"Parameter({self.symbol.name})"


class StencilKernel:
    """One forward or backward kernel of an ``AutoDiffOp`` for one target ('gpu' / 'cpu')."""

    def __init__(self, assignments, boundary_handling=None, function_name='kernel', target='gpu',
                 data_type=None, cpu_openmp=False, gpu_indexing_params=None, iteration_slice=None, **kwargs):
        self.assignments = assignments
        self.boundary_handling = boundary_handling
        self.function_name = function_name
        self.target = target
        if iteration_slice is not None:
            # pystencils' create_kernel(iteration_slice=...): iterate over this rectangular subset of the field
            # (absolute cell coordinates, ghost layers ignored); cells outside it are not touched. A read that
            # leaves the domain reads zero here (pystencils reads out of bounds); the one-thread-per-cell schedule
            self.ir = lower(assignments, 'zeros', data_type)
            self.ir.islice, self.ir.isteps = normalize_slice(iteration_slice, self.ir.ndim)
        else:
            self.ir = lower(assignments, boundary_handling, data_type)
        self.cpu_openmp = cpu_openmp
        self.tuning = dict(gpu_indexing_params or {})
        self.extra_kwargs = kwargs
        self._compiled = None

    # pystencils KernelFunction-like surface -----------------------------------------------------
    @property
    def fields_accessed(self):
        return set(self.ir.fields)

    @property
    def fields_read(self):
        return set(self.ir.fields_read)

    @property
    def fields_written(self):
        return set(self.ir.fields_written)

    @property
    def backend(self):
        return 'hip' if self.target == 'gpu' else 'c'

    def get_parameters(self):
        params = [Parameter(sp.Symbol(f.name), f) for f in self.ir.fields]
        params += [Parameter(s) for s in self.ir.scalars]
        return params

    @property
    def code(self):
        return self.compile().code

    @property
    def hash(self):
        return hashlib.sha256(self.code.encode()).hexdigest()[:16]

    def compile(self):
        if self._compiled is None:
            if self.target == 'gpu':
                from .hip_kernel import HipStencilKernel
                self._compiled = HipStencilKernel(self)
            else:
                from .cpu_kernel import CpuStencilKernel
                self._compiled = CpuStencilKernel(self)
        return self._compiled

    def __call__(self, **kwargs):
        return self.compile()(**kwargs)

    def __str__(self):
        return self.code
