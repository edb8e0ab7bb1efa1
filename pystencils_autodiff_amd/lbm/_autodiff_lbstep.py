"""Differentiable lattice Boltzmann time stepping (reference ``lbm/_autodiff_lbstep.py``).

``AutoDiffLatticeBoltzmannStep`` keeps the reference's constructor, field guessing and naming
(``_autodiff_lbstep.py:27-66,142-160``) but is not an lbmpy ``LatticeBoltzmannStep`` subclass (lbmpy is
absent): it owns its pdf arrays (the field's memory layout, lbmpy's default ``fzyx`` = one C-contiguous
plane per component) and runs the time loop the reference's ``run`` / ``run_backward`` drive through
lbmpy (``:336-398``) directly on the HIP kernels of an ``AutoDiffOp`` built with
``boundary_handling='periodic'``: the kernels wrap their reads (and the adjoint its writes) around the
lattice, so there are no ghost layers, no per-step ghost sync (lbmpy's ``_sync_src``) and no adjoint
fold-back — one kernel launch per step in each direction:

    forward step:  dst = stream-pull-collide(src)                      → swap
    adjoint step:  diffsrc = transposed kernel(diffdst, recorded src)  → swap
                   (scatter to x − c_i: for a fixed component i, x ↦ x − c_i is a bijection of the
                   periodic lattice, so every (component, cell) is written exactly once, no zero fill)

Deliberate deviations, each because the reference's behaviour is not a gradient:
* the adjoint is the ``DiffModes.TRANSPOSED`` form (``_autodiff.py:354-437``), not TF-MAD. TF-MAD
  evaluates ∂f/∂src at the unshifted cell (``_autodiff.py:102-109``), exact only for linear stencils, and
  its vector-field branch keeps only the last component's assignment (``_autodiff.py:138-152``); the
  collision is nonlinear and all components are needed.
* the backward of T steps needs each step's src state (the collision Jacobian depends on it): the forward
  records them (``record=True`` / the timestep op: T + 1 arrays, written in turn, no copies); the
  reference's ``run_backward`` re-uses whatever the arrays hold.

Rules made by ``create_lb_update_rule`` run on the lattice schedule (``_lattice_kernels``: one forward and one
adjoint kernel written for the lattice, any pdf strides, the op's internal states in the row-interleaved
``[z][y][q][x]`` layout) — which also carries no-slip walls (``set_boundary_including_adjoint``,
``_autodiff_lbstep.py:162-187``; half-way bounce-back fused into the pull, obstacle cells keep their state).
Other rules run on the ``AutoDiffOp`` kernels (periodic, no walls).
"""
import os

import numpy as np
import sympy as sp

from .. import ps
from ..autodiff import AutoDiffOp
from ._lattice_kernels import LatticeKernels, fix_cells, neighbour_mask
from ._method import LBStencil
from .boundaries import (AdjointBoundaryCondition, AdjointNoSlip, Boundary, BoundaryHandling, LBMethodView,  # noqa: F401
                         NoSlip, link_form)

__all__ = ['AutoDiffLatticeBoltzmannStep', 'PdfFieldNotDetectedException', 'SimulationResultsTensors']


class PdfFieldNotDetectedException(Exception):
    pass


class SimulationResultsTensors:
    """Same record as the reference (``_autodiff_lbstep.py:19-24``)."""

    def __init__(self, input_pdf_tensor, output_pdf_tensor, output_density_tensor, output_velocity_tensor):
        self.input_pdf_tensor = input_pdf_tensor
        self.output_pdf_tensor = output_pdf_tensor
        self.output_density_tensor = output_density_tensor
        self.output_velocity_tensor = output_velocity_tensor


def _lattice_sweeps(step, which, launches, force=None, dforce=None):
    """The lattice kernels over ``launches`` (tensor tuples of ``LatticeKernels.forward`` / ``adjoint``) on the
    current stream: one launch plan per distinct (shapes, strides) — the first, middle and last steps — and only
    the pointers packed per launch. ``force`` (a per-cell force field): bound to every launch; ``dforce``: the
    adjoint launches add their force adjoints into it."""
    K = step._lattice_kernels()
    mask = step._flag_arg()
    ids = step._ids_arg()
    cells = step._cells_arg()
    om = step._omega_of()
    mptr = (mask.data_ptr() if mask is not None else 0, ids.data_ptr() if ids is not None else 0)
    if force is not None:
        mptr += (force.data_ptr(),) + ((dforce.data_ptr(),) if which == 'adj' else ())
    stream = _torch()._C._cuda_getCurrentRawStream(launches[0][0].device.index)
    rho = K.rho_buffer(launches[0][0]) if which == 'adj' and K.link_pass else None
    if rho is not None:
        mptr += (rho.data_ptr(),)
    plans = {}
    for ts in launches:
        sig = tuple(t.stride() for t in ts)
        plan = plans.get(sig)
        if plan is None:
            plan = plans[sig] = K.plan(which, list(ts), mask, om, ids, force, dforce if which == 'adj' else None)
        plan(tuple(t.data_ptr() for t in ts) + mptr, stream, om)
        # link-program walls (HIP): the fix-up kernels over the cells next to them
        K.fix_launch(which, list(ts), mask, om, ids, force, dforce if which == 'adj' else None, cells, stream)
        if rho is not None:
            # the second pass of density-weighted walls (and, on the CPU, link programs) on this launch's output
            K.rho_pass(ts[2], mask, rho, ts[0], ids, stream)


def _plain_force_field(force, D):
    """The force FIELD when the rule's force is exactly ``F(x)[a]`` per axis a (one field of D components read at
    the cell itself), else None."""
    if force is None:
        return None
    comps = [sp.sympify(v) for v in force]
    if len(comps) != D or not all(isinstance(c, ps.Field.Access) for c in comps):
        return None
    fields = {c.field for c in comps}
    if len(fields) != 1:
        return None
    (F,) = fields
    if F.index_dimensions != 1 or int(F.index_shape[0]) != D:
        return None
    for a, c in enumerate(comps):
        if tuple(int(o) for o in c.offsets) != (0,) * D or tuple(int(i) for i in c.index) != (a,):
            return None
    return F


def _guess_src_dst_field_from_update_rule(update_rule, src_hint, dst_hint):
    """``_autodiff_lbstep.py:27-46``: a string hint means "find the one ≥9-component field"."""
    src_candidates = dst_candidates = None
    if isinstance(src_hint, str):
        src_candidates = [f for f in update_rule.free_fields if f.index_dimensions == 1 and f.index_shape[0] >= 9]
        if len(src_candidates) != 1:
            raise PdfFieldNotDetectedException(
                'Could not guess source PDF field from update rule.' +
                'Please specify the field explicitly in the constructor of AutoDiffLatticeBoltzmannStep!')
    if isinstance(dst_hint, str):
        dst_candidates = [f for f in update_rule.bound_fields if f.index_dimensions == 1 and f.index_shape[0] >= 9]
        if len(dst_candidates) != 1:
            raise PdfFieldNotDetectedException(
                'Could not guess temporary PDF field from update rule.' +
                'Please specify the field explicitly in the constructor of AutoDiffLatticeBoltzmannStep!')
    src = src_hint if isinstance(src_hint, ps.Field) else src_candidates[0]
    dst = dst_hint if isinstance(dst_hint, ps.Field) else dst_candidates[0]
    return src, dst


def _torch():
    import torch
    return torch


class AutoDiffLatticeBoltzmannStep:
    """Forward and adjoint lattice Boltzmann time steps on one periodic domain.

    ``update_rule``: a stream-pull-collide ``AssignmentCollection`` (``lbm.create_lb_update_rule``), its pdf
    fields found as in the reference. ``domain_size``: the spatial extent (without ghost layers).
    ``relaxation_rate`` sets the value of the rule's free scalar (``omega``) unless given as
    ``kernel_params``. ``target``: ``'gpu'`` (HIP kernels on torch tensors) or ``'cpu'`` (the C kernels on
    numpy arrays)."""

    def __init__(self, update_rule, src_pdf_field='', tmp_pdf_field='', time_constant_fields=(), *args,
                 constant_fields=(), domain_size=None, relaxation_rate=None, target='gpu', kernel_params=None,
                 device=None, **method_parameters):
        if args:
            raise TypeError('positional lbmpy LatticeBoltzmannStep arguments are not supported: pass keywords')
        src, tmp = _guess_src_dst_field_from_update_rule(update_rule, src_pdf_field, tmp_pdf_field)
        self.pdf_field = src
        self.temporary_field = tmp
        self._pdf_arr_name = src.name
        self._tmp_arr_name = tmp.name
        self._target = str(target).lower()
        if self._target not in ('gpu', 'cpu'):
            raise ValueError("target must be 'gpu' or 'cpu'")
        self._gpu = self._target == 'gpu'
        self._update_rule = update_rule
        self.method = getattr(update_rule, 'stencil', None) or LBStencil(
            {(2, 9): 'D2Q9', (3, 19): 'D3Q19', (3, 27): 'D3Q27'}[(src.spatial_dimensions, int(src.index_shape[0]))])
        if domain_size is None:
            if not src.has_fixed_shape:
                raise ValueError('domain_size is required for variable-size pdf fields')
            domain_size = tuple(int(s) for s in src.spatial_shape)
        self.domain_size = tuple(int(s) for s in domain_size)
        if len(self.domain_size) != src.spatial_dimensions or min(self.domain_size) < 2:
            raise ValueError(f'domain_size {self.domain_size} does not fit the {src.spatial_dimensions}-D pdf field')
        # periodic kernels (wrapped reads, every cell written) and the transposed adjoint — for the rules of
        # ``create_lb_update_rule`` written through the collision's structure (``create_lb_adjoint_rule``)
        backward = None
        # (a force term that depends on the pdfs — Guo's, through u — is not in that structure: the generic
        # transposed derivation then; the 'simple' term is a constant and changes no derivative)
        from ._method import force_is_field
        if getattr(update_rule, 'stencil', None) is not None and not time_constant_fields and \
                getattr(update_rule, 'force_model', None) in (None, 'simple') and \
                not force_is_field(getattr(update_rule, 'force', None)):
            from ._method import create_lb_adjoint_rule
            backward = create_lb_adjoint_rule(update_rule)
        # the rule's AutoDiffOp (its kernels are the schedule for rules the lattice kernels do not take, and its
        # transposed derivation — tens of seconds of sympy for a D3Q19 force-field rule — is only needed then):
        # built on first use
        self._autodiff_op = None
        self._autodiff_args = dict(forward_assignments=update_rule, op_name='LBM', boundary_handling='periodic',
                                   diff_mode='transposed', time_constant_fields=list(time_constant_fields) or None,
                                   constant_fields=list(constant_fields), backward_assignments=backward)
        self._diff_prefix = 'diff'
        # the op's forward input fields (the fields the rule reads, sorted by name — transposed_backward's order)
        read = {a.field for asg in update_rule.all_assignments for a in sp.sympify(asg.rhs).atoms(ps.Field.Access)}
        self._additional_fields = [f for f in sorted(read, key=str) if f not in (src, tmp)]
        scalars = sorted({s for a in update_rule.all_assignments for s in a.rhs.free_symbols
                          if isinstance(s, sp.Symbol) and not isinstance(s, ps.Field.Access)}
                         - {a.lhs for a in update_rule.subexpressions}, key=str)
        self.kernel_params = dict(kernel_params or {})
        for s in scalars:
            if s.name not in self.kernel_params:
                if relaxation_rate is None:
                    raise ValueError(f"scalar '{s.name}' of the update rule needs a value (relaxation_rate / "
                                     f"kernel_params)")
                self.kernel_params[s.name] = float(relaxation_rate)
        self._device = device
        self._arrays = {}
        self._records = None
        # the lattice schedule for the rules of create_lb_update_rule (SRT, stream_pull_collide); walls need it
        rr = getattr(update_rule, 'relaxation_rate', None)
        self._omega_of = (lambda: float(self.kernel_params[rr.name])) if isinstance(rr, sp.Symbol) else \
            ((lambda v=rr: float(v)) if rr is not None else None)
        # (PSAD_LBM_LATTICE=0: the AutoDiffOp kernels instead — tests of that path, A/B probes)
        force = getattr(update_rule, 'force', None)
        # a per-cell force read as F(x)[a] (the field's centre, component a, for every axis): the lattice kernels
        # take the field as an array and accumulate its adjoint; any other force expression runs on the AutoDiffOp
        # kernels
        self._force_field = _plain_force_field(force, src.spatial_dimensions)
        if self._force_field is not None:
            self._lattice_force = (getattr(update_rule, 'force_model', None), None)
        else:
            self._lattice_force = (getattr(update_rule, 'force_model', None),
                                   None if force is None else tuple(float(v) for v in force)) \
                if force is None or all(sp.sympify(v).is_number for v in force) else None
        extras_ok = not self._additional_fields or (self._force_field is not None and
                                                    self._additional_fields == [self._force_field])
        # TRT: the odd rate from the magic number (a function of the ω argument) or a constant
        self._lattice_trt = None
        trt_ok = True
        if getattr(update_rule, 'method', 'srt') == 'trt':
            if getattr(update_rule, 'magic_number', None) is not None:
                self._lattice_trt = ('magic', float(update_rule.magic_number))
            elif sp.sympify(update_rule.relaxation_rate_odd).is_number:
                self._lattice_trt = ('rate', float(update_rule.relaxation_rate_odd))
            else:
                trt_ok = False                      # a symbolic odd rate: the AutoDiffOp kernels
        # MRT: the relaxation matrix A = ω P_ω + C (groups relaxing with the rule's ω / with constant rates)
        self._lattice_mrt = None
        if getattr(update_rule, 'method', 'srt') == 'mrt':
            from ._method import MRT_GROUPS, mrt_relaxation_matrices
            P = mrt_relaxation_matrices(update_rule.stencil)
            Qn = update_rule.stencil.Q
            Pw = [[0.0] * Qn for _ in range(Qn)]
            Cm = [[0.0] * Qn for _ in range(Qn)]
            om = sp.sympify(update_rule.relaxation_rate)
            for grp in MRT_GROUPS:
                r = sp.sympify(update_rule.mrt_rates[grp])
                if r == om:
                    tgt, scale = Pw, 1.0
                elif r.is_number:
                    tgt, scale = Cm, float(r)
                else:
                    trt_ok = False                  # a symbolic rate other than ω: the AutoDiffOp kernels
                    break
                for i in range(Qn):
                    for k in range(Qn):
                        tgt[i][k] += scale * float(P[grp][i][k])
            else:
                self._lattice_mrt = (Pw, Cm)
        self._lattice = {} if (getattr(update_rule, 'stencil', None) is not None and not time_constant_fields
                               and self._lattice_force is not None
                               and os.environ.get('PSAD_LBM_LATTICE', '1') != '0'
                               and extras_ok and trt_ok and self._omega_of is not None
                               and np.dtype(src.dtype.numpy_dtype) in (np.float32, np.float64)
                               and (self._force_field is None or
                                    self._force_field.dtype.numpy_dtype == src.dtype.numpy_dtype)) else None
        self._boundary = BoundaryHandling(self.domain_size, on_change=self._flags_changed)
        # the lb_method the boundaries see: the stencil plus the rule's compressibility (FixedDensity reads it)
        self._bc_method = LBMethodView(self.method, getattr(update_rule, 'compressible', False))
        self._adjoint_boundary_conditions = {}
        self._flag_dev = None
        self._ids_dev = None

    @property
    def _autodiff(self):
        if self._autodiff_op is None:
            self._autodiff_op = AutoDiffOp(**self._autodiff_args)
        return self._autodiff_op

    def _adjoint_name(self, field):
        """The adjoint array name of an additional input field (the op's field map once it exists; the AdjointField
        naming ``diff<name>`` before, which is what that map holds)."""
        if self._autodiff_op is not None:
            return self._autodiff_op.adjoint_name(field)
        return self._diff_prefix + field.name

    # -- reference-named properties ----------------------------------------------------------------
    @property
    def backward_pdf_array_name(self):
        return "diff" + self._tmp_arr_name

    @property
    def _backward_tmp_array_name(self):
        return "diff" + self._pdf_arr_name

    @property
    def forward_assignments(self):
        return self._autodiff.forward_assignments

    @property
    def backward_assignments(self):
        return self._autodiff.backward_assignments

    @property
    def lb_method(self):
        return self.method

    @property
    def autodiff_op(self):
        return self._autodiff

    # -- arrays ------------------------------------------------------------------------------------
    def _alloc(self, zero=True):
        """A pdf array in the field's memory layout, spatial axes first in the returned view (``zero=False``:
        uninitialised, for arrays a kernel writes completely)."""
        Q = int(self.pdf_field.index_shape[0])
        dims = list(self.domain_size)
        dt = self.pdf_field.dtype.numpy_dtype
        if self._gpu:
            torch = _torch()
            tdt = getattr(torch, np.dtype(dt).name)
            dev = self._device or torch.device('cuda', torch.cuda.current_device())
            new = torch.zeros if zero else torch.empty
            if self.pdf_field.is_soa:
                return new([Q] + dims, dtype=tdt, device=dev).permute(*range(1, len(dims) + 1), 0)
            return new(dims + [Q], dtype=tdt, device=dev)
        new = np.zeros if zero else np.empty
        if self.pdf_field.is_soa:
            return np.moveaxis(new([Q] + dims, dtype=dt), 0, -1)
        return new(dims + [Q], dtype=dt)

    def empty_pdfs(self):
        """An uninitialised pdf tensor in the step's memory layout (``[*domain_size, q]`` view; for ``fzyx``
        one contiguous plane per component) — inputs in this layout enter the timestep op without a copy."""
        return self._alloc(zero=False)

    def _as_layout(self, t):
        """``t`` itself if it has the step's memory layout, else a copy in it."""
        ref = self._array(self._pdf_arr_name)
        if tuple(t.shape) == tuple(ref.shape) and tuple(t.stride()) == tuple(ref.stride()) and t.dtype == ref.dtype:
            return t
        out = self._alloc(zero=False)
        out.copy_(t)
        return out

    def _internal_states(self, n):
        """``n`` states only the time-step op sees, in the row-interleaved layout (lattice schedule), as views
        of one allocation."""
        if n <= 0:
            return []
        torch = _torch()
        dev = self._device or torch.device('cuda', torch.cuda.current_device())
        Q = int(self.pdf_field.index_shape[0])
        dims = list(self.domain_size)
        base = torch.empty([n] + dims[:-1] + [Q, dims[-1]],
                           dtype=getattr(torch, np.dtype(self.pdf_field.dtype.numpy_dtype).name), device=dev)
        return list(base.transpose(-1, -2).unbind(0))

    def _lattice_input_ok(self, t):
        """A tensor the lattice kernels take as it is: ``[*domain, q]`` of the pdf dtype on the step's device."""
        ref = self._array(self._pdf_arr_name)
        return tuple(t.shape) == tuple(ref.shape) and t.dtype == ref.dtype and t.device == ref.device

    def _array(self, name):
        if name not in self._arrays:
            self._arrays[name] = self._alloc()
        return self._arrays[name]

    @property
    def pdf_array(self):
        """The current pdfs (``[*domain_size, q]``)."""
        return self._array(self._pdf_arr_name)

    def set_pdfs(self, pdfs):
        self._array(self._pdf_arr_name)[...] = pdfs
        self._records = None

    # -- boundaries (``_autodiff_lbstep.py:162-187``) --------------------------------------------------
    @property
    def boundary_handling(self):
        """The obstacle flags (``BoundaryHandling.set_boundary``); forward and adjoint read the same flags."""
        return self._boundary

    @property
    def backward_boundary_handling(self):
        return self._boundary

    def set_boundary_including_adjoint(self, boundary_condition, slice_obj=None, mask_callback=None, mask_array=None,
                                       adjoint_boundary_condition=None):
        """Set ``boundary_condition`` (a ``Boundary``: ``NoSlip``, ``UBB``, ``FixedDensity``, or any boundary whose
        link reads only the fluid cell's own pdfs, ``boundaries.link_form``) on the selected cells for the forward
        AND the adjoint steps (the reference's signature; the adjoint condition defaults to
        ``AdjointBoundaryCondition(bc)``, derived from the forward link by AD)."""
        if not isinstance(boundary_condition, Boundary) or \
                isinstance(boundary_condition, (AdjointNoSlip, AdjointBoundaryCondition)):
            raise NotImplementedError(f'boundary {boundary_condition!r}: needs a forward Boundary object')
        if self._lattice is None:
            raise NotImplementedError('walls need the lattice schedule (a create_lb_update_rule rule without '
                                      'time-constant or additional fields)')
        if adjoint_boundary_condition is None:
            adjoint_boundary_condition = self._adjoint_boundary_conditions.setdefault(
                boundary_condition, AdjointBoundaryCondition(
                    boundary_condition, time_constant_fields=list(self._autodiff_args['time_constant_fields'] or []),
                    constant_fields=list(self._autodiff_args['constant_fields'] or []) + ['indexVector']))
        elif not isinstance(adjoint_boundary_condition, (AdjointNoSlip, AdjointBoundaryCondition)):
            raise NotImplementedError(f'adjoint boundary {adjoint_boundary_condition!r}')
        link_form(boundary_condition, adjoint_boundary_condition, self._bc_method)   # the kernels' form, or raise
        self._boundary.set_boundary(boundary_condition, slice_obj, mask_callback=mask_callback, mask_array=mask_array,
                                    adjoint=adjoint_boundary_condition)

    def _flags_changed(self):
        self._flag_dev = None
        self._ids_dev = None
        self._links_cached = None
        self._records = None

    def _flag_arg(self):
        """The cells' neighbour masks for the wall kernels (computed once per flag change), None without walls."""
        if not self._boundary.has_walls:
            return None
        if self._flag_dev is None:
            if self._gpu:
                torch = _torch()
                dev = self._device or torch.device('cuda', torch.cuda.current_device())
                fix = self._fix_mask()
                self._flag_dev = neighbour_mask(torch.from_numpy(self._boundary.flags.copy()).to(dev), self.method,
                                                torch, fix=fix)
                self._cells_dev = None if fix is None else \
                    torch.from_numpy(np.flatnonzero(fix.ravel()).astype(np.int32)).to(dev)
            else:
                self._flag_dev = neighbour_mask(self._boundary.flags, self.method, np)
        return self._flag_dev

    def _fix_mask(self):
        """The fluid cells next to link-program walls (``FIX_BIT``: the HIP fix-up kernels' list), None if no
        boundary is a link program."""
        progs = self._programs()
        if progs is None:
            return None
        return fix_cells(self._boundary.flags, self.method, [k for k, p in enumerate(progs) if p is not None])

    def _cells_arg(self):
        """The fix-up kernels' cell list (int32 on the device), None without link programs (or on the CPU)."""
        if not self._gpu or self._flag_arg() is None:
            return None
        return getattr(self, '_cells_dev', None)

    def _links(self):
        """The wall kernels' link tables (None: every wall a plain bounce-back, or no walls), derived once per
        boundary change (``link_form`` differentiates each boundary's sympy link: not per step)."""
        return self._link_data()[0]

    def _programs(self):
        """The link programs of the walls the fused form does not take (None if there are none)."""
        return self._link_data()[1]

    def _link_data(self):
        cached = getattr(self, '_links_cached', None)
        if cached is None:
            cached = self._links_cached = (self._boundary.link_tables(self._bc_method) if self._boundary.has_walls
                                           else (None, None))
        return cached

    def _ids_arg(self):
        """The cells' wall ids for kernels with link tables (the flag array on the kernels' device), else None."""
        if self._links() is None:
            return None
        if getattr(self, '_ids_dev', None) is None:
            if self._gpu:
                torch = _torch()
                dev = self._device or torch.device('cuda', torch.cuda.current_device())
                self._ids_dev = torch.from_numpy(self._boundary.flags.copy()).to(dev)
            else:
                self._ids_dev = np.ascontiguousarray(self._boundary.flags)
        return self._ids_dev

    def _lattice_kernels(self):
        walls = self._boundary.has_walls
        links, programs = self._link_data()
        k = self._lattice.get((walls, links, programs))
        if k is None:
            k = self._lattice[(walls, links, programs)] = LatticeKernels(
                self.method, getattr(self._update_rule, 'compressible', False), self.pdf_field.dtype.numpy_dtype,
                walls, self._target, links, *self._lattice_force, force_field=self._force_field is not None,
                trt=self._lattice_trt, programs=programs, mrt=self._lattice_mrt)
        return k

    # -- kernels -----------------------------------------------------------------------------------
    def _kernels(self):
        op = self._autodiff
        if self._gpu:
            return op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
        return op.forward_ast_cpu.compile(), op.backward_ast_cpu.compile()

    def _fwd(self, src, dst, extra):
        if self._lattice is not None:
            return self._lattice_kernels().forward(src, dst, self._omega_of(), self._flag_arg(), ids=self._ids_arg(),
                                                   force=self._force_arg(extra), cells=self._cells_arg())
        kf, _ = self._kernels()
        kf(**{self._pdf_arr_name: src, self._tmp_arr_name: dst}, **extra, **self.kernel_params)

    def _force_arg(self, extra):
        """The per-cell force array of the lattice kernels (None without a force field)."""
        if self._force_field is None:
            return None
        try:
            return extra[self._force_field.name]
        except (KeyError, TypeError):
            raise ValueError(f"the update rule reads the force field '{self._force_field.name}': pass its array "
                             "(extra={name: array})") from None

    def _bwd(self, src, diffdst, diffsrc, extra, extra_adj):
        if self._lattice is not None:
            dforce = None
            if self._force_field is not None:
                name = self._adjoint_name(self._force_field)
                if name not in (extra_adj or {}):
                    raise ValueError(f"the force field's adjoint '{name}' needs an array (extra_adj), accumulated into")
                dforce = extra_adj[name]
            return self._lattice_kernels().adjoint(src, diffdst, diffsrc, self._omega_of(), self._flag_arg(),
                                                   ids=self._ids_arg(), force=self._force_arg(extra), dforce=dforce,
                                                   cells=self._cells_arg())
        _, kb = self._kernels()
        kb(**{self._pdf_arr_name: src, 'diff' + self._tmp_arr_name: diffdst, 'diff' + self._pdf_arr_name: diffsrc},
           **extra, **extra_adj, **self.kernel_params)

    # -- time loops --------------------------------------------------------------------------------
    def time_step(self, extra=None):
        """One forward step on the owned arrays: stream-pull-collide, swap. While recording, the step writes
        into a fresh array and its src stays as the record (no copies)."""
        a = self._array(self._pdf_arr_name)
        if self._records is not None:
            self._records.append(a)
            b = self._alloc(zero=False)
            self._fwd(a, b, extra or {})
            self._arrays[self._pdf_arr_name] = b
            return
        b = self._array(self._tmp_arr_name)
        self._fwd(a, b, extra or {})
        self._arrays[self._pdf_arr_name], self._arrays[self._tmp_arr_name] = b, a

    def run(self, time_steps, record=False, extra=None):
        """``time_steps`` forward steps; ``record=True`` keeps each step's src state for ``run_backward``
        (T + 1 pdf arrays live until the backward has consumed them)."""
        self._records = [] if record else None
        for _ in range(int(time_steps)):
            self.time_step(extra)

    def backward_time_step(self, src_state, extra=None, extra_adj=None):
        """One adjoint step: diffsrc = Kᵀ(diffdst) with the collision Jacobian at ``src_state``."""
        g_dst = self._array(self.backward_pdf_array_name)
        g_src = self._array(self._backward_tmp_array_name)
        self._bwd(src_state, g_dst, g_src, extra or {}, extra_adj or {})
        self._arrays[self.backward_pdf_array_name], self._arrays[self._backward_tmp_array_name] = g_src, g_dst

    def set_adjoint_pdfs(self, grad):
        """The adjoint of the current (final) pdfs."""
        self._array(self.backward_pdf_array_name)[...] = grad

    @property
    def adjoint_pdf_array(self):
        return self._array(self.backward_pdf_array_name)

    def run_backward(self, time_steps, extra=None, extra_adj=None):
        """``time_steps`` adjoint steps in reverse over the states the last ``run(..., record=True)`` kept;
        the result is ``adjoint_pdf_array`` (gradient w.r.t. the pdfs before that run)."""
        if self._records is None or len(self._records) < int(time_steps):
            raise RuntimeError('run_backward needs the states of a preceding run(time_steps, record=True)')
        for t in range(int(time_steps)):
            self.backward_time_step(self._records[-1 - t], extra, extra_adj)
        self._records = self._records[:len(self._records) - int(time_steps)]

    # -- torch ops ---------------------------------------------------------------------------------
    def create_timestep_op(self, num_time_steps, input_field_to_tensor_dict=None, backend='torch_native'):
        """A ``torch.autograd.Function`` for ``num_time_steps`` steps: ``Op.apply(pdfs)`` with the interior
        pdfs (``[*domain_size, q]``) returns the pdfs after the steps; its backward runs the adjoint steps
        in reverse over the recorded states (``_autodiff_lbstep.py:189-247``; the reference's
        ``torch_native`` backend ignores the loops and differentiates one kernel launch)."""
        if str(backend).lower() not in ('torch_native', 'torch'):
            raise NotImplementedError(f"backend '{backend}': only the torch backends are built")
        extras = list(self._additional_fields)
        known = {self.pdf_field.name} | {f.name for f in extras}
        unknown = [getattr(f, 'name', f) for f in (input_field_to_tensor_dict or {}) if getattr(f, 'name', f) not in known]
        if unknown:
            raise ValueError(f'input fields {unknown} are not read by the update rule (inputs: {sorted(known)})')
        torch = _torch()
        step = self
        T = int(num_time_steps)
        adj = {f.name: self._adjoint_name(f) for f in extras}

        class LbmTimesteps(torch.autograd.Function):
            @staticmethod
            def forward(ctx, pdfs, *xs):
                if len(xs) != len(extras):
                    raise TypeError(f'{LbmTimesteps.__name__}.apply(pdfs, {", ".join(f.name for f in extras)}): '
                                    f'{1 + len(xs)} tensors given')
                # additional input fields (a per-cell force): constant over the steps, bound to every launch
                ex = {f.name: step._field_layout(f, x.detach()) for f, x in zip(extras, xs)}
                ctx.extras = ex
                if not step._gpu:
                    ex = {n: x.cpu().numpy() for n, x in ex.items()}
                    ctx.extras = ex
                    step.set_pdfs(pdfs.detach().cpu().numpy())
                    step.run(T, record=True, extra=ex)
                    ctx.records = step._records
                    step._records = None
                    return torch.from_numpy(step.pdf_array.copy())
                # states on fresh arrays: the input is the first state (the lattice kernels read any strides;
                # the AutoDiffOp kernels need the field's layout — ``empty_pdfs`` — or get a copy), the output, in
                # the field's layout, the last; the lattice schedule keeps the states between in the
                # row-interleaved layout, all in one allocation (no copies either way)
                lattice = step._lattice is not None
                x0 = pdfs.detach()
                x0 = x0 if lattice and step._lattice_input_ok(x0) else step._as_layout(x0)
                if lattice:
                    states = [x0] + step._internal_states(T - 1) + [step._alloc(zero=False)]
                    _lattice_sweeps(step, 'fwd', [(states[t], states[t + 1]) for t in range(T)],
                                    step._force_arg(ex))
                else:
                    states = [x0]
                    for t in range(T):
                        out = step._alloc(zero=False)
                        step._fwd(states[-1], out, ex)
                        states.append(out)
                # state 0 may be the caller's tensor: keep it through save_for_backward, so that an in-place
                # change between forward and backward raises (version counter) instead of skewing the adjoint
                ctx.input_is_state0 = states[0].data_ptr() == pdfs.data_ptr()
                ctx.save_for_backward(pdfs if ctx.input_is_state0 else None)
                ctx.records = states[1:-1] if ctx.input_is_state0 else states[:-1]
                return states[-1]

            @staticmethod
            def backward(ctx, grad):
                ex = ctx.extras
                ctx.extras = None
                if not step._gpu:
                    step._records = ctx.records
                    step.set_adjoint_pdfs(grad.detach().cpu().numpy())
                    acc = {n: np.zeros_like(x) for n, x in ex.items()}
                    for t in range(T):
                        # each step's adjoint of the additional fields into a zeroed array, summed over the steps
                        tmp = {adj[n]: np.zeros_like(x) for n, x in ex.items()}
                        step.backward_time_step(step._records[-1 - t], ex, tmp)
                        for n in acc:
                            acc[n] += tmp[adj[n]]
                    step._records = step._records[:len(step._records) - T]
                    ctx.records = None
                    return (torch.from_numpy(step.adjoint_pdf_array.copy()),
                            *[torch.from_numpy(acc[f.name]) for f in extras])
                lattice = step._lattice is not None
                g = grad if lattice and step._lattice_input_ok(grad) else step._as_layout(grad)
                x0 = ctx.saved_tensors[0].detach() if ctx.input_is_state0 else None
                records = ([x0 if lattice and step._lattice_input_ok(x0) else step._as_layout(x0)]
                           if ctx.input_is_state0 else []) + list(ctx.records)
                ctx.records = None
                if lattice:
                    # adjoints of states T-1 .. 1 alternate between two row-interleaved arrays; the gradient
                    # (adjoint of state 0) leaves in the field's layout
                    ping = step._internal_states(min(2, T - 1))
                    out = step._alloc(zero=False)
                    cur, launches = g, []
                    for t in reversed(range(T)):
                        nxt = out if t == 0 else ping[(T - 1 - t) % 2]
                        launches.append((records[t], cur, nxt))
                        cur = nxt
                    if step._force_field is None:
                        _lattice_sweeps(step, 'adj', launches)
                        return out
                    # the force adjoint: every step's adjoint launch adds its share into one zeroed array
                    F = step._force_arg(ex)
                    dF = torch.zeros_like(F)
                    _lattice_sweeps(step, 'adj', launches, F, dF)
                    return out, dF
                cur = g
                acc = {n: torch.zeros_like(x) for n, x in ex.items()}
                for t in reversed(range(T)):
                    nxt = step._alloc(zero=False)
                    tmp = {adj[n]: torch.zeros_like(x) for n, x in ex.items()}
                    step._bwd(records[t], cur, nxt, ex, tmp)
                    for n in acc:
                        acc[n] += tmp[adj[n]]
                    cur = nxt
                return (cur, *[acc[f.name] for f in extras]) if extras else cur

        LbmTimesteps.num_time_steps = T
        LbmTimesteps.lb_step = self
        return LbmTimesteps

    def _field_layout(self, f, t):
        """An additional input tensor in field ``f``'s memory layout (fzyx: components-first) on the step's side."""
        if not self._gpu:
            return t
        if f.index_dimensions and f.is_soa:
            from ..zslab import ZSlabOp
            return ZSlabOp._layout(f, t)
        return t.contiguous()

    def _pdf_io_field(self):
        """The pdf field of the macroscopic ops, in the step's pdf layout (fzyx pdfs enter without a copy)."""
        return ps.fields(f"pdfs({self.method.Q}): {np.dtype(self.pdf_field.dtype.numpy_dtype).name}"
                         f"[{len(self.domain_size)}D]", layout='fzyx' if self.pdf_field.is_soa else None)

    def create_end_to_end_op(self, num_time_steps, velocity_input_tensor, density_input_tensor,
                             additional_fields_to_tensor_map=None, force_input_tensor=None, backend='torch_native',
                             num_times_steps_without_save=0, **kernel_compilation_kwargs):
        """Equilibrium from (ρ, u) → ``num_time_steps`` steps → (ρ, u), differentiable end to end
        (``_autodiff_lbstep.py:310-334``, there TensorFlow only): the setter op, the time-step ops in groups of
        ``num_times_steps_without_save + 1`` steps, the getter op, evaluated on the given tensors (torch
        autograd records the chain). Returns ``SimulationResultsTensors``."""
        if str(backend).lower() not in ('torch_native', 'torch'):
            raise NotImplementedError(f"backend '{backend}': only the torch backends are built")
        from ._method import force_is_field
        given = {getattr(f, 'name', f): t for f, t in dict(additional_fields_to_tensor_map or {}).items()}
        force = getattr(self._update_rule, 'force', None)
        if force_input_tensor is not None:
            if not force_is_field(force):
                raise ValueError('force_input_tensor given, but the update rule has no force field')
            (ff,) = {a.field for v in force for a in sp.sympify(v).atoms(ps.Field.Access)}
            given[ff.name] = force_input_tensor
        missing = [f.name for f in self._additional_fields if f.name not in given]
        if missing:
            raise ValueError(f'tensors for the update rule\'s additional input fields {missing} are needed '
                             '(additional_fields_to_tensor_map / force_input_tensor)')
        xs = [given[f.name] for f in self._additional_fields]
        setter = self._e2e_ops.get('setter') if hasattr(self, '_e2e_ops') else None
        if setter is None:
            self._e2e_ops = {'setter': self.create_macroscopic_setter_op(backend, **kernel_compilation_kwargs),
                             'getter': self.create_macroscopic_getter_op(backend, **kernel_compilation_kwargs)}
        ops = self._e2e_ops
        group = int(num_times_steps_without_save) + 1
        step_op = self.create_timestep_op(group, backend=backend)
        (input_pdf,) = ops['setter'].apply(density_input_tensor, velocity_input_tensor)
        out = input_pdf
        for _ in range(int(num_time_steps) // group):
            out = step_op.apply(out, *xs)
        rho, vel = self._apply_getter(ops['getter'], out, given)
        return SimulationResultsTensors(input_pdf, out, rho, vel)

    def _macroscopic_fields(self):
        dt = self.pdf_field.dtype.numpy_dtype
        D = len(self.domain_size)
        return ps.fields(f"rho, vel({D}): {np.dtype(dt).name}[{D}D]")

    def _apply_getter(self, getter, pdfs, given):
        """The getter on ``pdfs`` (and, with a per-cell Guo force, the force tensor: its inputs in the op's order)."""
        names = [f.name for f in getter.autodiff_op.forward_input_fields]
        pdf = self._pdf_io_field().name
        return getter.apply(*[pdfs if n == pdf else given[n] for n in names])

    def create_macroscopic_getter_op(self, backend='torch_native', **kernel_compilation_kwargs):
        """ρ and u from pdfs as a differentiable op (``_autodiff_lbstep.py:249-280``): ``Op.apply(pdfs)`` →
        ``(rho, vel)`` (a per-cell Guo force: its field is an input too, in the op's ``forward_input_fields``
        order)."""
        from ._method import macroscopic_getter
        rho, vel = self._macroscopic_fields()
        pdf = self._pdf_io_field()
        ac = macroscopic_getter(self.method, pdf, rho, vel, getattr(self._update_rule, 'compressible', False),
                                getattr(self._update_rule, 'force_model', None), getattr(self._update_rule, 'force', None))
        op = AutoDiffOp(ac, 'LBM_GetMacroscopicValues', diff_mode='transposed', **kernel_compilation_kwargs)
        return op.create_tensorflow_op(use_cuda=self._gpu, backend=backend)

    def create_macroscopic_setter_op(self, backend='torch_native', **kernel_compilation_kwargs):
        """pdfs = feq(ρ, u) as a differentiable op (``_autodiff_lbstep.py:282-308``): ``Op.apply(rho, vel)``."""
        from ._method import equilibrium_setter
        rho, vel = self._macroscopic_fields()
        pdf = self._pdf_io_field()
        ac = equilibrium_setter(self.method, pdf, rho, vel, getattr(self._update_rule, 'compressible', False))
        op = AutoDiffOp(ac, 'LBM_SetMacroscopicValues', diff_mode='transposed', **kernel_compilation_kwargs)
        return op.create_tensorflow_op(use_cuda=self._gpu, backend=backend)
