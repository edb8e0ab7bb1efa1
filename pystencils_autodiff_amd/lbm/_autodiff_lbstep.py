"""Differentiable lattice Boltzmann time stepping (reference ``lbm/_autodiff_lbstep.py``).

``AutoDiffLatticeBoltzmannStep`` keeps the reference's constructor, field guessing and naming
(``_autodiff_lbstep.py:27-66,142-160``) but is not an lbmpy ``LatticeBoltzmannStep`` subclass (lbmpy is
absent): it owns its two pdf arrays (``src`` / ``tmp``, one periodic ghost layer per side, the field's
memory layout) and runs the time loop the reference's ``run`` / ``run_backward`` drive through lbmpy
(``:336-398``) directly on the HIP kernels of an ``AutoDiffOp``:

    forward step:  periodic ghost sync of src → stream-pull-collide kernel (interior cells) → swap
    adjoint step:  zero the border of diffsrc → transposed kernel (reads diffdst and the RECORDED src of
                   that step, scatters to diffsrc at x − c_i) → fold ghost contributions back onto the
                   periodic images (the adjoint of the sync) → swap

Deliberate deviations, each because the reference's behaviour is not a gradient:
* the adjoint is the ``DiffModes.TRANSPOSED`` form (``_autodiff.py:354-437``), not TF-MAD. TF-MAD
  evaluates ∂f/∂src at the unshifted cell (``_autodiff.py:102-109``), exact only for linear stencils, and
  its vector-field branch keeps only the last component's assignment (``_autodiff.py:138-152``); the
  collision is nonlinear and all components are needed. For pull streaming each component is read at ONE
  offset, so the transposed (scatter) adjoint still writes every (component, cell) exactly once.
* the backward of T steps needs each step's src state (the collision Jacobian depends on it): the forward
  records them (``record=True`` / the timestep op); the reference's ``run_backward`` re-uses whatever the
  arrays hold.
Only periodic domains are built (lbmpy's boundary handling / ``AdjointBoundaryCondition``,
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
            domain_size = tuple(int(s) - 2 for s in src.spatial_shape)
        self.domain_size = tuple(int(s) for s in domain_size)
        if len(self.domain_size) != src.spatial_dimensions or min(self.domain_size) < 2:
            raise ValueError(f'domain_size {self.domain_size} does not fit the {src.spatial_dimensions}-D pdf field')
        # interior-only kernels (ghost layer 1, ``boundary_handling=None``) and the transposed adjoint
        self._autodiff = AutoDiffOp(update_rule, 'LBM', boundary_handling=None, diff_mode='transposed',
                                    time_constant_fields=list(time_constant_fields) or None,
                                    constant_fields=list(constant_fields))
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
    def _alloc(self):
        """A padded pdf array in the field's memory layout: spatial axes first in the returned view."""
        Q = int(self.pdf_field.index_shape[0])
        padded = [s + 2 for s in self.domain_size]
        dt = self.pdf_field.dtype.numpy_dtype
        if self._gpu:
            torch = _torch()
            tdt = getattr(torch, np.dtype(dt).name)
            dev = self._device or torch.device('cuda', torch.cuda.current_device())
            if self.pdf_field.is_soa:
                return torch.zeros([Q] + padded, dtype=tdt, device=dev).permute(*range(1, len(padded) + 1), 0)
            return torch.zeros(padded + [Q], dtype=tdt, device=dev)
        if self.pdf_field.is_soa:
            return np.moveaxis(np.zeros([Q] + padded, dtype=dt), 0, -1)
        return np.zeros(padded + [Q], dtype=dt)

    def _array(self, name):
        if name not in self._arrays:
            self._arrays[name] = self._alloc()
        return self._arrays[name]

    @property
    def pdf_array(self):
        """Interior view of the current pdfs (``[*domain_size, q]``)."""
        return self._interior(self._array(self._pdf_arr_name))

    def set_pdfs(self, pdfs):
        a = self._array(self._pdf_arr_name)
        self._interior(a)[...] = pdfs
        self._records = None

    def _interior(self, a):
        return a[tuple(slice(1, -1) for _ in self.domain_size)]

    def _slab(self, a, axis, i):
        return a[tuple(i if d == axis else slice(None) for d in range(len(self.domain_size)))]

    def _sync(self, a):
        """Periodic ghost layers, axis by axis (the corner ghosts come out right): the reference's
        ``_sync_src`` periodic communication."""
        for d, n in enumerate(self.domain_size):
            self._slab(a, d, 0)[...] = self._slab(a, d, n)
            self._slab(a, d, n + 1)[...] = self._slab(a, d, 1)

    def _sync_adjoint(self, g):
        """Adjoint of ``_sync``: ghost contributions are added to the interior cells they were copied from
        (axes in reverse order), then the ghosts are cleared."""
        for d in reversed(range(len(self.domain_size))):
            n = self.domain_size[d]
            self._slab(g, d, n)[...] += self._slab(g, d, 0)
            self._slab(g, d, 1)[...] += self._slab(g, d, n + 1)
            self._slab(g, d, 0)[...] = 0
            self._slab(g, d, n + 1)[...] = 0

    def _clear_border(self, g):
        """Cells the transposed kernel may leave unwritten: the two outermost layers on each side (for
        |c| ≤ 1 a component is written at x = y − c for interior y only)."""
        for d, n in enumerate(self.domain_size):
            for i in (0, 1, n, n + 1):
                self._slab(g, d, i)[...] = 0

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
        """One forward step on the owned arrays: sync, stream-pull-collide, swap."""
        a, b = self._array(self._pdf_arr_name), self._array(self._tmp_arr_name)
        self._sync(a)
        if self._records is not None:
            self._records.append(a.clone() if self._gpu else a.copy())
        self._fwd(a, b, extra or {})
        self._arrays[self._pdf_arr_name], self._arrays[self._tmp_arr_name] = b, a

    def run(self, time_steps, record=False, extra=None):
        """``time_steps`` forward steps; ``record=True`` keeps each step's src state for ``run_backward``."""
        self._records = [] if record else None
        for _ in range(int(time_steps)):
            self.time_step(extra)

    def backward_time_step(self, src_state, extra=None, extra_adj=None):
        """One adjoint step: diffsrc = Sᵀ Kᵀ(diffdst) with the collision Jacobian at ``src_state``."""
        g_dst = self._array(self.backward_pdf_array_name)
        g_src = self._array(self._backward_tmp_array_name)
        self._clear_border(g_src)
        self._bwd(src_state, g_dst, g_src, extra or {}, extra_adj or {})
        self._sync_adjoint(g_src)
        self._arrays[self.backward_pdf_array_name], self._arrays[self._backward_tmp_array_name] = g_src, g_dst

    def set_adjoint_pdfs(self, grad):
        """The adjoint of the current (final) pdfs, interior values; the ghost layer stays zero."""
        g = self._array(self.backward_pdf_array_name)
        g[...] = 0
        self._interior(g)[...] = grad

    @property
    def adjoint_pdf_array(self):
        return self._interior(self._array(self.backward_pdf_array_name))

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
        torch = _torch()
        step = self
        T = int(num_time_steps)

        class LbmTimesteps(torch.autograd.Function):
            @staticmethod
            def forward(ctx, pdfs):
                if step._gpu and not pdfs.is_cuda:
                    pdfs = pdfs.cuda()
                step.set_pdfs(pdfs.detach() if step._gpu else pdfs.detach().cpu().numpy())
                step.run(T, record=True)
                ctx.records = step._records
                step._records = None
                out = step.pdf_array
                return out.clone() if step._gpu else torch.from_numpy(out.copy())

            @staticmethod
            def backward(ctx, grad):
                step._records = ctx.records
                step.set_adjoint_pdfs(grad if step._gpu else grad.detach().cpu().numpy())
                step.run_backward(T)
                ctx.records = None
                g = step.adjoint_pdf_array
                return g.clone() if step._gpu else torch.from_numpy(g.copy())

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
