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
Only periodic lattices are built (lbmpy's boundary handling / ``AdjointBoundaryCondition``,
``adjoint_boundaryconditions.py``, needs lbmpy's flag fields).
"""
import numpy as np
import sympy as sp

from .. import ps
from ..autodiff import AutoDiffOp
from ._method import LBStencil

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
        if getattr(update_rule, 'stencil', None) is not None and not time_constant_fields:
            from ._method import create_lb_adjoint_rule
            backward = create_lb_adjoint_rule(update_rule)
        self._autodiff = AutoDiffOp(update_rule, 'LBM', boundary_handling='periodic', diff_mode='transposed',
                                    time_constant_fields=list(time_constant_fields) or None,
                                    constant_fields=list(constant_fields), backward_assignments=backward)
        self._additional_fields = [f for f in self._autodiff.forward_input_fields if f not in (src, tmp)]
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

    # -- kernels -----------------------------------------------------------------------------------
    def _kernels(self):
        op = self._autodiff
        if self._gpu:
            return op.forward_ast_gpu.compile(), op.backward_ast_gpu.compile()
        return op.forward_ast_cpu.compile(), op.backward_ast_cpu.compile()

    def _fwd(self, src, dst, extra):
        kf, _ = self._kernels()
        kf(**{self._pdf_arr_name: src, self._tmp_arr_name: dst}, **extra, **self.kernel_params)

    def _bwd(self, src, diffdst, diffsrc, extra, extra_adj):
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
        extra_inputs = [f for f in (input_field_to_tensor_dict or {}) if f not in (self.pdf_field, self.pdf_field.name)]
        if extra_inputs or self._additional_fields:
            # the kernels would need those fields bound per step (and their adjoints accumulated): not built
            raise NotImplementedError('timestep op over update rules with additional input fields '
                                      f'({[getattr(f, "name", f) for f in extra_inputs or self._additional_fields]})')
        torch = _torch()
        step = self
        T = int(num_time_steps)

        class LbmTimesteps(torch.autograd.Function):
            @staticmethod
            def forward(ctx, pdfs):
                if not step._gpu:
                    step.set_pdfs(pdfs.detach().cpu().numpy())
                    step.run(T, record=True)
                    ctx.records = step._records
                    step._records = None
                    return torch.from_numpy(step.pdf_array.copy())
                # states on fresh arrays in the field's layout: the input is the first state when it has
                # that layout already (``empty_pdfs``), the output is the last — no copies
                states = [step._as_layout(pdfs.detach())]
                for _ in range(T):
                    out = step._alloc(zero=False)
                    step._fwd(states[-1], out, {})
                    states.append(out)
                # state 0 may be the caller's tensor: keep it through save_for_backward, so that an in-place
                # change between forward and backward raises (version counter) instead of skewing the adjoint
                ctx.input_is_state0 = states[0].data_ptr() == pdfs.data_ptr()
                ctx.save_for_backward(pdfs if ctx.input_is_state0 else None)
                ctx.records = states[1:-1] if ctx.input_is_state0 else states[:-1]
                return states[-1]

            @staticmethod
            def backward(ctx, grad):
                if not step._gpu:
                    step._records = ctx.records
                    step.set_adjoint_pdfs(grad.detach().cpu().numpy())
                    step.run_backward(T)
                    ctx.records = None
                    return torch.from_numpy(step.adjoint_pdf_array.copy())
                g = step._as_layout(grad)
                records = ([step._as_layout(ctx.saved_tensors[0].detach())] if ctx.input_is_state0 else []) + \
                    list(ctx.records)
                cur, spare = g, None                # cur: adjoint of state t + 1 (never written when it is g)
                for t in reversed(range(T)):
                    nxt = spare if spare is not None else step._alloc(zero=False)
                    step._bwd(records[t], cur, nxt, {}, {})
                    spare = cur if cur is not g else None
                    cur = nxt
                ctx.records = None
                return cur

        LbmTimesteps.num_time_steps = T
        LbmTimesteps.lb_step = self
        return LbmTimesteps

    def _macroscopic_fields(self):
        dt = self.pdf_field.dtype.numpy_dtype
        D = len(self.domain_size)
        return ps.fields(f"rho, vel({D}): {np.dtype(dt).name}[{D}D]")

    def create_macroscopic_getter_op(self, backend='torch_native', **kernel_compilation_kwargs):
        """ρ and u from pdfs as a differentiable op (``_autodiff_lbstep.py:249-280``): ``Op.apply(pdfs)`` →
        ``(rho, vel)``."""
        from ._method import macroscopic_getter
        rho, vel = self._macroscopic_fields()
        pdf = ps.fields(f"pdfs({self.method.Q}): {np.dtype(self.pdf_field.dtype.numpy_dtype).name}"
                        f"[{len(self.domain_size)}D]")
        ac = macroscopic_getter(self.method, pdf, rho, vel, getattr(self._update_rule, 'compressible', False))
        op = AutoDiffOp(ac, 'LBM_GetMacroscopicValues', diff_mode='transposed', **kernel_compilation_kwargs)
        return op.create_tensorflow_op(use_cuda=self._gpu, backend=backend)

    def create_macroscopic_setter_op(self, backend='torch_native', **kernel_compilation_kwargs):
        """pdfs = feq(ρ, u) as a differentiable op (``_autodiff_lbstep.py:282-308``): ``Op.apply(rho, vel)``."""
        from ._method import equilibrium_setter
        rho, vel = self._macroscopic_fields()
        pdf = ps.fields(f"pdfs({self.method.Q}): {np.dtype(self.pdf_field.dtype.numpy_dtype).name}"
                        f"[{len(self.domain_size)}D]")
        ac = equilibrium_setter(self.method, pdf, rho, vel, getattr(self._update_rule, 'compressible', False))
        op = AutoDiffOp(ac, 'LBM_SetMacroscopicValues', diff_mode='transposed', **kernel_compilation_kwargs)
        return op.create_tensorflow_op(use_cuda=self._gpu, backend=backend)
