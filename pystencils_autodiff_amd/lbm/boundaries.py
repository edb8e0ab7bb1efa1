"""No-slip walls for ``AutoDiffLatticeBoltzmannStep`` and their adjoints (reference
``/root/reference/src/pystencils_autodiff/lbm/adjoint_boundaryconditions.py:7-72``, lbmpy's ``NoSlip`` [ext]).

lbmpy describes a boundary by an object that prints assignments for lbmpy's boundary-handling kernels over
index lists of boundary links, and the reference derives the adjoint object from it
(``AdjointBoundaryCondition``: TF-MAD of the forward boundary's assignments) or spells it out
(``AdjointNoSlip``: ``pdf(dir) = pdf[neighbour](inv_dir)``, the forward copy transposed). Here the boundary
objects name the condition and the cells it covers are a flag array; the lattice kernels
(``_lattice_kernels``) fuse the half-way bounce-back into the pull and its transpose into the adjoint scatter,
so there is no separate boundary kernel, no index list and no sync step. Only no-slip is built.
"""
import numpy as np

__all__ = ['NoSlip', 'AdjointNoSlip', 'AdjointBoundaryCondition', 'BoundaryHandling', 'make_slice']


class _MakeSlice:
    """``make_slice[:, 0]`` → ``(slice(None), 0)`` (pystencils' ``make_slice`` [ext])."""

    def __getitem__(self, item):
        return item


make_slice = _MakeSlice()


class NoSlip:
    """Half-way simple bounce-back at obstacle cells (lbmpy ``NoSlip`` [ext]): zero velocity at the wall."""

    def __init__(self, name=None):
        self.name = name or 'NoSlip'

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, NoSlip) and self.name == other.name

    def __repr__(self):
        return f'NoSlip({self.name!r})'


class AdjointNoSlip:
    """The adjoint of ``NoSlip`` (``adjoint_boundaryconditions.py:49-72``): applied by the adjoint kernel."""

    def __init__(self, name=None):
        self.name = name or 'AdjointNoSlip'

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, AdjointNoSlip) and self.name == other.name


class AdjointBoundaryCondition:
    """The adjoint of a forward boundary condition (``adjoint_boundaryconditions.py:7-46``). Built for
    ``NoSlip`` only (its transpose is fused into the adjoint lattice kernel)."""

    def __init__(self, forward_boundary_condition, time_constant_fields=(), constant_fields=()):
        if not isinstance(forward_boundary_condition, NoSlip):
            raise NotImplementedError(f'adjoint of {forward_boundary_condition!r}: only NoSlip is built')
        self.name = 'Adjoint' + forward_boundary_condition.name
        self._forward_condition = forward_boundary_condition
        self._time_constant_fields = list(time_constant_fields or [])
        self._constant_fields = list(constant_fields or [])

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, AdjointBoundaryCondition) and self._forward_condition == other._forward_condition


class BoundaryHandling:
    """The obstacle flags of one lattice (``uint8``, one per cell, 1 = no-slip obstacle) and lbmpy's
    ``set_boundary`` surface over them. The forward and the adjoint kernels read the same flags, so the
    forward handling and the ``backward_boundary_handling`` of the step are this one object."""

    def __init__(self, domain_size, on_change=None):
        self.domain_size = tuple(int(n) for n in domain_size)
        self.flags = np.zeros(self.domain_size, np.uint8)
        self._on_change = on_change
        self.conditions = {}
        self._has_walls = False

    @property
    def has_walls(self):
        """Any obstacle cell (kept up to date by ``set_boundary``: the kernels ask once per launch)."""
        return self._has_walls

    def set_boundary(self, boundary_obj, slice_obj=None, mask_callback=None, mask_array=None, **_):
        """Mark cells as ``boundary_obj`` (``NoSlip``; ``AdjointNoSlip`` / ``AdjointBoundaryCondition(NoSlip)``
        or ``'domain'`` to clear them): the cells of ``slice_obj`` (domain coordinates, default all), narrowed
        by ``mask_callback(*midpoints)`` (cell-midpoint coordinate arrays of the region, axis 0 first) or a
        boolean ``mask_array`` (the region's or the domain's shape)."""
        if boundary_obj == 'domain':
            value = 0
        elif isinstance(boundary_obj, (NoSlip, AdjointNoSlip, AdjointBoundaryCondition)):
            value = 1
        else:
            raise NotImplementedError(f'boundary {boundary_obj!r}: only NoSlip walls are built')
        if slice_obj is None:
            slice_obj = tuple(slice(None) for _ in self.domain_size)
        elif not isinstance(slice_obj, tuple):
            slice_obj = (slice_obj,)
        region = self.flags[slice_obj]
        grids = np.meshgrid(*[np.arange(n, dtype=np.float64)[s] + 0.5 if isinstance(s, slice) else
                              np.asarray([s % n + 0.5]) for s, n in
                              zip(slice_obj + (slice(None),) * (len(self.domain_size) - len(slice_obj)),
                                  self.domain_size)], indexing='ij')
        mask = np.ones(grids[0].shape, bool)
        if mask_callback is not None:
            mask &= np.asarray(mask_callback(*grids), bool).reshape(mask.shape)
        if mask_array is not None:
            m = np.asarray(mask_array, bool)
            if m.shape == self.domain_size and region.shape != self.domain_size:
                m = m[slice_obj]
            mask &= m.reshape(mask.shape)
        sub = self.flags[slice_obj]
        sub = np.where(mask.reshape(sub.shape), np.uint8(value), sub)
        self.flags[slice_obj] = sub
        self._has_walls = bool(self.flags.any())
        if value:
            self.conditions[boundary_obj] = True
        if self._on_change is not None:
            self._on_change()
