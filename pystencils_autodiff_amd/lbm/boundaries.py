"""Walls for ``AutoDiffLatticeBoltzmannStep`` and their adjoints (reference
``/root/reference/src/pystencils_autodiff/lbm/adjoint_boundaryconditions.py:7-72``, lbmpy's ``NoSlip`` / ``UBB``
[ext]).

lbmpy describes a boundary by an object whose ``__call__(pdf_field, direction, lb_method)`` prints the assignment
of one boundary LINK — from the fluid cell ``x`` in direction ``d`` into the wall cell ``x + c_d`` — for lbmpy's
boundary kernels, which run over index lists before the streaming step writes the wall cell's incoming population:

    NoSlip:  pdf[c_d](ī_d) ← pdf(d)                                 (half-way bounce-back)
    UBB:     pdf[c_d](ī_d) ← pdf(d) − 6 w_d (c_d · u_wall)           (velocity bounce-back, 2/c_s² = 6)

and the reference derives the adjoint object from it (``AdjointBoundaryCondition``: the backward assignments of the
forward link, ``adjoint_boundaryconditions.py:24-37``) or spells one out (``AdjointNoSlip``: ``pdf(d) ←
pdf[c_d](ī_d)``, the forward copy transposed, ``:49-72``).

Here the boundary objects print the same link assignments in this package's ``ps`` front-end, and the lattice
kernels (``_lattice_kernels``) fuse every link of the form ``f_in = α·f_out + β`` (α, β constants per object and
direction) into the pull — ``f_j(x) = α·src_ī(x) + β`` where ``x − c_j`` is a wall cell — and the adjoint link into
the adjoint scatter. ``link_coefficients`` reads (α, β) off the forward assignment and the adjoint coefficient off
the adjoint object's assignment, so any boundary object of that form works (``NoSlip``, ``UBB``, user subclasses
of ``Boundary``). ``AdjointBoundaryCondition`` derives the adjoint link with the transposed-mode AD of this package
(``DiffModes.TRANSPOSED``): the reference's TF-MAD call reads the adjoint of an offset write at the mirrored offset and
at component 0 (``_autodiff.py:120-151``, the quirk its own ``AdjointNoSlip`` docstring calls "bug-safe" to avoid),
which is not the gradient; the transposed form is what ``AdjointNoSlip`` spells out, for any affine link. The cells
a boundary covers are a flag array (one id per boundary object): no index list, no separate boundary kernel.

UBB: lbmpy multiplies the velocity term by the fluid cell's density ρ(x) = Σ_k pdf(k) for one of its two method
families (the ``compressible`` branch differs between lbmpy versions): ``UBB(u, density_weighted=True)`` prints that
link, ``pdf[c_d](ī_d) ← pdf(d) − 6 w_d (c_d · u) ρ(x)`` — affine in ALL the cell's pdfs. The lattice kernels fuse it
too: the forward adds ``βρ·ρ(x)`` (ρ from the cell's own pre-streaming pdfs, loaded on cells next to a wall), the
adjoint scatters ``γ v`` as for any link and adds the density term ``Σ_j γρ_j v_j`` to every component of the cell in
a second pass (``lbm_adj_rho``; those entries are written by other threads in the first). Links of any other form
(a pressure / outflow condition, a nonlinear link) raise.
"""
import numpy as np
import sympy as sp

__all__ = ['Boundary', 'NoSlip', 'UBB', 'AdjointNoSlip', 'AdjointBoundaryCondition', 'BoundaryHandling',
           'make_slice', 'link_coefficients']


class _MakeSlice:
    """``make_slice[:, 0]`` → ``(slice(None), 0)`` (pystencils' ``make_slice`` [ext])."""

    def __getitem__(self, item):
        return item


make_slice = _MakeSlice()


def _directions(lb_method):
    st = getattr(lb_method, 'stencil', lb_method)
    return st


class Boundary:
    """lbmpy's boundary surface (``lbmpy.boundaries.boundaryconditions.Boundary`` [ext]): a name, equality by
    name, and ``__call__(pdf_field, direction, lb_method)`` → the link assignment(s) for direction index
    ``direction`` (lbmpy passes a direction symbol evaluated over index lists; the lattice kernels here are printed
    per direction, so it is a concrete index)."""

    def __init__(self, name=None):
        self._name = name

    @property
    def name(self):
        return self._name if self._name is not None else type(self).__name__

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        raise NotImplementedError

    def __hash__(self):
        return hash((type(self).__name__, self.name))

    def __eq__(self, other):
        return type(other) is type(self) and self.name == other.name

    def __repr__(self):
        return f'{type(self).__name__}({self.name!r})'


class NoSlip(Boundary):
    """Half-way simple bounce-back (lbmpy ``NoSlip`` [ext]): zero velocity at the wall."""

    def __init__(self, name=None):
        super().__init__(name if name is not None else 'NoSlip')

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        st = _directions(lb_method)
        c = st.directions[direction]
        from .. import ps
        return [ps.Assignment(pdf_field[c](st.inverse_direction_index(direction)), pdf_field(direction))]


class UBB(Boundary):
    """Velocity bounce-back (lbmpy ``UBB`` [ext]): a wall moving with ``velocity`` (one component per spatial axis,
    axis 0 first), e.g. the lid of a lid-driven cavity: ``pdf[c_d](ī_d) ← pdf(d) − 6 w_d (c_d · u)``;
    ``density_weighted=True``: lbmpy's compressible form, the velocity term times the fluid cell's density
    ``ρ = Σ_k pdf(k)`` (a subexpression, as lbmpy prints it)."""

    def __init__(self, velocity, name=None, density_weighted=False):
        super().__init__(name if name is not None else 'UBB')
        self.velocity = tuple(velocity)
        self.density_weighted = bool(density_weighted)

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        st = _directions(lb_method)
        c = st.directions[direction]
        if len(self.velocity) != len(c):
            raise ValueError(f'UBB velocity {self.velocity} has not one component per axis of {st.name}')
        vel_term = 6 * st.weights[direction] * sum(ci * sp.sympify(ui) for ci, ui in zip(c, self.velocity) if ci)
        from .. import ps
        link = pdf_field[c](st.inverse_direction_index(direction))
        if self.density_weighted:
            rho = sp.Symbol('rho')
            return [ps.Assignment(rho, sum(pdf_field(k) for k in range(st.Q))),
                    ps.Assignment(link, pdf_field(direction) - vel_term * rho)]
        return [ps.Assignment(link, pdf_field(direction) - vel_term)]

    def __hash__(self):
        return hash(('UBB', self.name, self.velocity, self.density_weighted))

    def __eq__(self, other):
        return isinstance(other, UBB) and self.name == other.name and self.velocity == other.velocity and \
            self.density_weighted == other.density_weighted

    def __repr__(self):
        return f'UBB({self.velocity!r}, {self.name!r}' + (', density_weighted=True)' if self.density_weighted else ')')


class AdjointNoSlip(Boundary):
    """The adjoint of ``NoSlip`` spelled out (``adjoint_boundaryconditions.py:49-72``):
    ``pdf(d) ← pdf[c_d](ī_d)``, the forward copy transposed."""

    def __init__(self, name=None):
        super().__init__(name if name is not None else 'AdjointNoSlip')

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        st = _directions(lb_method)
        c = st.directions[direction]
        from .. import ps
        return [ps.Assignment(pdf_field(direction), pdf_field[c](st.inverse_direction_index(direction)))]


class AdjointBoundaryCondition(Boundary):
    """The adjoint of a forward boundary condition (``adjoint_boundaryconditions.py:7-46``): the backward
    assignments of the forward link (transposed-mode AD, see the module docstring), on the adjoint pdf field
    (an ``AdjointField``, or a field named ``diff<name>`` like the reference's heuristic)."""

    def __init__(self, forward_boundary_condition, time_constant_fields=(), constant_fields=()):
        if not isinstance(forward_boundary_condition, Boundary) or \
                isinstance(forward_boundary_condition, (AdjointBoundaryCondition, AdjointNoSlip)):
            raise NotImplementedError(f'adjoint of {forward_boundary_condition!r}: needs a forward Boundary')
        super().__init__('Adjoint' + forward_boundary_condition.name)
        self._forward_condition = forward_boundary_condition
        self._time_constant_fields = list(time_constant_fields or [])
        self._constant_fields = list(constant_fields or [])

    @property
    def forward_condition(self):
        return self._forward_condition

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        from .. import ps
        from .._adjoint_field import AdjointField
        from ..autodiff import DiffModes, create_backward_assignments
        if not isinstance(pdf_field, AdjointField) and pdf_field.name.startswith('diff'):
            forward_field = pdf_field.new_field_with_different_name(pdf_field.name[len('diff'):])
            pdf_field = AdjointField(forward_field)
        if not isinstance(pdf_field, AdjointField):
            raise TypeError(f'{pdf_field} should be an AdjointField to use AdjointBoundaryCondition')
        forward_field = pdf_field.corresponding_forward_field
        fwd = self._forward_condition(forward_field, direction, lb_method, **kwargs)
        bwd = create_backward_assignments(ps.AssignmentCollection(list(fwd)), diff_fields_prefix=pdf_field.name_prefix,
                                          time_constant_fields=self._time_constant_fields,
                                          constant_fields=self._constant_fields, diff_mode=DiffModes.TRANSPOSED)
        assert bwd.all_assignments, ('Must have a at least one read field in forward boundary to have an meaningful '
                                     'adjoint boundary condition')
        return bwd

    def __hash__(self):
        return hash(('Adjoint', hash(self._forward_condition)))

    def __eq__(self, other):
        return isinstance(other, AdjointBoundaryCondition) and self._forward_condition == other._forward_condition


def _affine(expr, var):
    """(α, β) with ``expr = α·var + β`` (numbers), else None."""
    expr = sp.expand(sp.sympify(expr))
    a = sp.diff(expr, var)
    b = sp.expand(expr - a * var)
    if a.free_symbols or b.free_symbols:
        return None
    return float(a), float(b)


def _inline(assignments, lhs):
    """The right-hand side of the assignment to ``lhs`` with the list's symbol assignments substituted."""
    sym = [a for a in assignments if isinstance(a.lhs, sp.Symbol) and not hasattr(a.lhs, 'field')]
    main = [a for a in assignments if a.lhs == lhs]
    if len(main) != 1:
        return None
    rhs = main[0].rhs
    for a in reversed(sym):
        rhs = rhs.subs(a.lhs, a.rhs)
    return rhs


def link_coefficients(forward_bc, adjoint_bc, lb_method):
    """Per direction ``d`` of ``lb_method``'s stencil: ``(α, β, γ, βρ, γρ)`` with the forward link
    ``f_{ī_d}(x + c_d) = α·f_d(x) + βρ·Σ_k f_k(x) + β`` and the adjoint link
    ``g_k(x) += (γ δ_kd + γρ)·g_{ī_d}(x + c_d)`` — the form the lattice kernels fuse (βρ = γρ = 0: a link in one pdf;
    nonzero: a density-weighted link). Raises ``NotImplementedError`` for a boundary of another form."""
    from .. import ps
    from .._adjoint_field import AdjointField
    st = _directions(lb_method)
    f = ps.fields(f'__pdf({st.Q}): [{st.D}D]')
    g = AdjointField(f)
    out = []
    for d in range(st.Q):
        c = st.directions[d]
        if not any(c):
            out.append((1.0, 0.0, 1.0, 0.0, 0.0))
            continue
        inv = st.inverse_direction_index(d)
        fwd = list(forward_bc(f, d, lb_method))
        rhs = _inline(fwd, f[c](inv))
        if rhs is None or any(a.lhs != f[c](inv) and hasattr(a.lhs, 'field') for a in fwd):
            raise NotImplementedError(f'{forward_bc!r}: the lattice kernels fuse one link assignment '
                                      f'pdf[c_d](inv_d) <- alpha*pdf(d) + beta (+ beta_rho*rho) per direction, got {fwd}')
        coef = [_affine(sp.diff(rhs, f(k)) * f(k), f(k)) for k in range(st.Q)]
        const = sp.expand(rhs - sum(sp.diff(rhs, f(k)) * f(k) for k in range(st.Q)))
        if any(ck is None for ck in coef) or const.free_symbols or \
                any(sp.diff(rhs, f(k)).free_symbols for k in range(st.Q)):
            raise NotImplementedError(f'{forward_bc!r}: link {fwd} is not affine in the cell\'s pdfs with constant '
                                      'coefficients')
        a_k = [ck[0] for ck in coef]
        others = [a_k[k] for k in range(st.Q) if k != d]
        if max(others) - min(others) > 1e-15 * max(1.0, max(abs(v) for v in others)):
            raise NotImplementedError(f'{forward_bc!r}: link {fwd} weights the other pdfs unequally (only a density '
                                      'term Σ_k pdf(k) is fused)')
        br = others[0]
        alpha, beta = a_k[d] - br, float(const)
        bwd = adjoint_bc(g, d, lb_method)
        allb = list(getattr(bwd, 'all_assignments', bwd))
        gk = []
        for k in range(st.Q):
            r = _inline(allb, g(k))
            if r is None:
                gk.append(0.0)
                continue
            gb = _affine(r, g[c](inv))
            if gb is None or gb[1] != 0:
                raise NotImplementedError(f'{adjoint_bc!r}: adjoint link of pdf({k}) is not linear in '
                                          f'diffpdf[c_d](inv_d): {r}')
            gk.append(gb[0])
        if any(hasattr(a.lhs, 'field') and a.lhs not in [g(k) for k in range(st.Q)] for a in allb):
            raise NotImplementedError(f'{adjoint_bc!r}: adjoint assignments beyond diffpdf(k) <- gamma_k * '
                                      f'diffpdf[c_d](inv_d): {allb}')
        gothers = [gk[k] for k in range(st.Q) if k != d]
        if max(gothers) - min(gothers) > 1e-15 * max(1.0, max(abs(v) for v in gothers)):
            raise NotImplementedError(f'{adjoint_bc!r}: adjoint link weights the pdfs unequally')
        gr = gothers[0]
        out.append((alpha, beta, gk[d] - gr, br, gr))
    return tuple(out)


class BoundaryHandling:
    """The wall flags of one lattice (``uint8``, one per cell: 0 = fluid, k ≥ 1 = the k-th boundary object set)
    and lbmpy's ``set_boundary`` surface over them. The forward and the adjoint kernels read the same flags, so the
    forward handling and the ``backward_boundary_handling`` of the step are this one object; each boundary object
    keeps the adjoint condition it was set with."""

    def __init__(self, domain_size, on_change=None):
        self.domain_size = tuple(int(n) for n in domain_size)
        self.flags = np.zeros(self.domain_size, np.uint8)
        self._on_change = on_change
        self.conditions = {}            # forward boundary object -> flag id
        self.adjoints = {}              # flag id -> adjoint boundary object
        self._has_walls = False

    @property
    def has_walls(self):
        """Any wall cell (kept up to date by ``set_boundary``: the kernels ask once per launch)."""
        return self._has_walls

    def objects(self):
        """Forward boundary objects by flag id (index 0: fluid, None)."""
        out = [None] * (max(self.conditions.values(), default=0) + 1)
        for obj, k in self.conditions.items():
            out[k] = obj
        return out

    def flag_id(self, boundary_obj, adjoint=None):
        """The flag id of ``boundary_obj`` (allocated on first use; adjoints count as their forward condition)."""
        if isinstance(boundary_obj, AdjointBoundaryCondition):
            boundary_obj = boundary_obj.forward_condition
        elif isinstance(boundary_obj, AdjointNoSlip):
            boundary_obj = NoSlip()
        k = self.conditions.get(boundary_obj)
        if k is None:
            k = len(self.conditions) + 1
            if k > 255:
                raise ValueError('more than 255 boundary objects on one lattice')
            self.conditions[boundary_obj] = k
        if adjoint is not None:
            self.adjoints[k] = adjoint
        elif k not in self.adjoints:
            self.adjoints[k] = AdjointNoSlip() if isinstance(boundary_obj, NoSlip) else \
                AdjointBoundaryCondition(boundary_obj)
        return k

    def set_boundary(self, boundary_obj, slice_obj=None, mask_callback=None, mask_array=None, adjoint=None, **_):
        """Mark cells as ``boundary_obj`` (a ``Boundary``; its adjoint object, or ``'domain'`` to clear them): the
        cells of ``slice_obj`` (domain coordinates, default all), narrowed by ``mask_callback(*midpoints)``
        (cell-midpoint coordinate arrays of the region, axis 0 first) or a boolean ``mask_array`` (the region's or
        the domain's shape)."""
        if boundary_obj == 'domain':
            value = 0
        elif isinstance(boundary_obj, Boundary):
            value = self.flag_id(boundary_obj, adjoint)
        else:
            raise NotImplementedError(f'boundary {boundary_obj!r}: not a Boundary object')
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
        if self._on_change is not None:
            self._on_change()

    def link_tables(self, lb_method):
        """Per flag id ≥ 1: the ``link_coefficients`` of its (forward, adjoint) boundary pair, as a tuple, or None
        when every id is a plain bounce-back (α = γ = 1, β = 0: the kernels' fast path, no id loads)."""
        objs = self.objects()
        tables = [None]
        plain = True
        for k in range(1, len(objs)):
            obj = objs[k]
            t = link_coefficients(obj, self.adjoints[k], lb_method)
            plain &= all(a == 1.0 and b == 0.0 and g == 1.0 and br == 0.0 and gr == 0.0 for a, b, g, br, gr in t)
            tables.append(t)
        if plain:
            return None
        st = _directions(lb_method)
        tables[0] = tuple((1.0, 0.0, 1.0, 0.0, 0.0) for _ in range(st.Q))
        return tuple(tables)
