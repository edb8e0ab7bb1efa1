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
a second pass (``lbm_adj_rho``; those entries are written by other threads in the first).

Links of any other form that read only the fluid cell's own pdfs — lbmpy's ``FixedDensity`` (a pressure boundary,
quadratic in the cell's velocity), a link that weights another population of the cell, any user link of that
kind — are LINK PROGRAMS (``link_program``): the forward value and its Jacobian row ``∂f_in/∂pdf(k)`` (read off
the adjoint object's assignments) printed as C per (wall id, direction) and compiled into the same lattice kernels:
the forward evaluates the link from the cell's own pre-streaming pdfs, the adjoint accumulates ``Σ_j J_jk v_j`` per
component k of the cell and adds it in the second pass. A link that reads another cell or another field raises.
"""
import numpy as np
import sympy as sp

__all__ = ['Boundary', 'NoSlip', 'UBB', 'FixedDensity', 'AdjointNoSlip', 'AdjointBoundaryCondition',
           'BoundaryHandling', 'LBMethodView', 'make_slice', 'link_coefficients', 'link_program', 'link_form']


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


class FixedDensity(Boundary):
    """lbmpy's ``FixedDensity`` [ext] — a pressure boundary by anti-bounce-back with the symmetric part of the
    equilibrium: ``pdf[c_d](ī_d) ← 2 feq_sym_d − pdf(d)`` with ``feq_sym_d = w_d ρ_w (1 + 4.5 (c_d·u)² − 1.5 u²)``
    (compressible) or ``w_d (ρ_w + 4.5 (c_d·u)² − 1.5 u²)`` (incompressible). lbmpy prints the equilibrium's
    subexpressions of the fluid cell's own pdfs with the density symbol replaced by the prescribed density, so the
    velocity is ``u = Σ_k c_k pdf(k) / ρ_w`` (compressible) or ``Σ_k c_k pdf(k)``. ``compressible``: the method's
    (None: read from ``lb_method.compressible``, which ``AutoDiffLatticeBoltzmannStep`` passes). Nonlinear in the
    cell's pdfs: a link program (parity with lbmpy itself unpinned, lbmpy absent)."""

    def __init__(self, density, name=None, compressible=None):
        super().__init__(name if name is not None else 'FixedDensity')
        self.density = density
        self.compressible = compressible

    def __call__(self, pdf_field, direction, lb_method, **kwargs):
        st = _directions(lb_method)
        comp = self.compressible if self.compressible is not None else getattr(lb_method, 'compressible', None)
        if comp is None:
            raise ValueError('FixedDensity: the method\'s compressibility is unknown (pass compressible=)')
        c = st.directions[direction]
        from .. import ps
        rho_w = sp.sympify(self.density)
        us = sp.symbols(f'fd_u_:{st.D}')
        sub = []
        for a in range(st.D):
            m = sum(st.directions[k][a] * pdf_field(k) for k in range(st.Q) if st.directions[k][a])
            sub.append(ps.Assignment(us[a], m / rho_w if comp else m))
        cu = sum(ci * ua for ci, ua in zip(c, us) if ci)
        usq = sum(ua * ua for ua in us)
        poly = sp.Rational(9, 2) * cu * cu - sp.Rational(3, 2) * usq
        w = sp.sympify(st.weights[direction])
        feq_sym = w * rho_w * (1 + poly) if comp else w * (rho_w + poly)
        link = pdf_field[c](st.inverse_direction_index(direction))
        return sub + [ps.Assignment(link, 2 * feq_sym - pdf_field(direction))]

    def program(self, lb_method):
        """The link program (``link_program``'s form, adjoint = the derivative) written out: per direction d with
        u = m/ρ_w (m = Σ_k c_k c_k-th pdf; incompressible u = m), ``L_d = 2 w_d ρ_w (1 + 4.5 (c_d·u)² − 1.5 u²) − c_d``
        and ``∂L_d/∂c_k = 2 w_d (9 (c_d·u)(c_d·c_k) − 3 u·c_k) − δ_dk`` (the same in both families). Equal to the
        general derivation (``tests/test_lbm.py::test_lbm_link_program_paths_agree``), at a fraction of its sympy
        time (a D3Q19 program: milliseconds instead of seconds)."""
        st = _directions(lb_method)
        comp = self.compressible if self.compressible is not None else getattr(lb_method, 'compressible', None)
        if comp is None:
            raise ValueError('FixedDensity: the method\'s compressibility is unknown (pass compressible=)')
        dens = sp.sympify(self.density)
        if not dens.is_number:
            # a symbolic wall density (a trained or scheduled pressure) is not a constant of the compiled link
            # program; the general derivation refuses free symbols the same way (link_program)
            raise NotImplementedError(f'FixedDensity({self.density!r}): the lattice kernels take a numeric wall '
                                      'density (a symbol would have to be a kernel parameter)')
        rw = float(dens)
        pr = _c_printer()
        D, Q = st.D, st.Q
        dirs = [tuple(int(v) for v in c) for c in st.directions]
        mom = []
        for a in range(D):
            t = ' '.join(('+ ' if dirs[k][a] > 0 else '- ') + f'c{k}' for k in range(Q) if dirs[k][a])
            t = t[2:] if t.startswith('+ ') else t
            mom.append(f'({t}) / (T){rw!r}' if comp else f'({t})')
        ulines = tuple(f'const T fu{a} = {mom[a]};' for a in range(D))
        usq = ' + '.join(f'fu{a} * fu{a}' for a in range(D))
        out = []
        for d in range(Q):
            c = dirs[d]
            if not any(c):
                out.append(None)
                continue
            w = pr.doprint(sp.sympify(st.weights[d]))
            cu = ' + '.join(f'{"" if v > 0 else "-"}fu{a}' for a, v in enumerate(c) if v)
            lines = ulines + (f'const T fcu = {cu};', f'const T fusq = {usq};')
            sym = f'(T){rw!r} * ((T)1 + (T)4.5 * fcu * fcu - (T)1.5 * fusq)' if comp else \
                f'((T){rw!r} + (T)4.5 * fcu * fcu - (T)1.5 * fusq)'
            val = f'(T)2 * {w} * {sym} - c{d}'
            rows = []
            for k in range(Q):
                cc = sum(x * y for x, y in zip(c, dirs[k]))
                uc = ' + '.join(f'{"" if v > 0 else "-"}fu{a}' for a, v in enumerate(dirs[k]) if v)
                terms = []
                if cc:
                    terms.append(f'(T){9 * cc} * fcu')
                if uc:
                    terms.append(f'(T)-3 * ({uc})')
                e = f'(T)2 * {w} * (' + ' + '.join(terms) + ')' if terms else None
                if k == d:
                    e = f'{e} - (T)1' if e else '(T)-1'
                if e is not None:
                    rows.append((k, lines, e))
            out.append((lines, val, tuple(rows)))
        return tuple(out)

    def __hash__(self):
        return hash(('FixedDensity', self.name, str(self.density), self.compressible))

    def __eq__(self, other):
        return isinstance(other, FixedDensity) and self.name == other.name and \
            sp.sympify(self.density) == sp.sympify(other.density) and self.compressible == other.compressible

    def __repr__(self):
        return f'FixedDensity({self.density!r}, {self.name!r})'


class LBMethodView:
    """The ``lb_method`` a boundary sees (lbmpy passes its method object): the stencil's attributes plus the rule's
    ``compressible`` flag (``FixedDensity`` needs it)."""

    def __init__(self, stencil, compressible):
        self.stencil = stencil
        self.compressible = bool(compressible)

    def __getattr__(self, name):
        return getattr(self.__dict__['stencil'], name)

    @property
    def dim(self):
        return self.stencil.D


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


def _c_printer():
    """sympy → C for the link programs: constants as casts to the kernels' compute type ``T``, small integer powers
    as products (no ``pow`` on the device)."""
    from sympy.printing.c import C99CodePrinter

    class P(C99CodePrinter):
        def _print_Float(self, e):
            return f'(T){float(e)!r}'

        def _print_Rational(self, e):
            return f'((T){int(e.p)} / (T){int(e.q)})'

        def _print_Integer(self, e):
            return f'(T){int(e)}'

        def _print_Pow(self, e):
            b, x = e.args
            if x.is_Integer and 1 <= int(x) <= 4:
                return '(' + ' * '.join([self.parenthesize(b, 100)] * int(x)) + ')'
            if x.is_Integer and -4 <= int(x) <= -1:
                return '((T)1 / (' + ' * '.join([self.parenthesize(b, 100)] * -int(x)) + '))'
            raise NotImplementedError(f'link program: power {e}')
    return P()


def _program_code(exprs):
    """(temporaries, expressions) as C: ``const T lt_k = …;`` lines (common subexpressions) and one expression per
    input, in the cell's own pdfs ``c0 … c{Q-1}``."""
    pr = _c_printer()
    tmp = sp.numbered_symbols('lt_')
    reps, red = sp.cse([sp.sympify(e) for e in exprs], symbols=tmp)
    lines = tuple(f'const T {pr.doprint(a)} = {pr.doprint(b)};' for a, b in reps)
    return lines, tuple(pr.doprint(e) for e in red)


def link_program(forward_bc, adjoint_bc, lb_method):
    """Per direction ``d`` of the stencil, for a link that reads only the fluid cell's own pdfs: ``None`` (the rest
    population) or ``(lines, value, jac)`` — C source of the forward link value ``f_{ī_d}(x + c_d) = L_d(pdf(x))``
    (``lines``: temporaries, ``value``: an expression in ``c0 … c{Q-1}``, the cell's own pre-streaming pdfs) and of
    the adjoint link's Jacobian row ``((k, lines_k, J_dk), …)`` read off the adjoint object's assignments
    ``diffpdf(k) ← J_dk · diffpdf[c_d](ī_d)`` (J_dk may depend on the cell's pdfs; zero entries left out).
    Raises ``NotImplementedError`` for a link that reads another cell or another field."""
    from .. import ps
    from .._adjoint_field import AdjointField
    st = _directions(lb_method)
    f = ps.fields(f'__pdf({st.Q}): [{st.D}D]')
    g = AdjointField(f)
    cs = sp.symbols(f'c0:{st.Q}')
    own = {f(k): cs[k] for k in range(st.Q)}
    # (a program reads only the cell's pdfs: the adjoint object's constant / time-constant fields change nothing)
    derived = isinstance(adjoint_bc, AdjointBoundaryCondition) and adjoint_bc.forward_condition == forward_bc and \
        type(adjoint_bc) is AdjointBoundaryCondition
    if derived and callable(getattr(forward_bc, 'program', None)):
        return forward_bc.program(lb_method)          # written out by the boundary (FixedDensity)
    out = []
    for d in range(st.Q):
        c = st.directions[d]
        if not any(c):
            out.append(None)
            continue
        inv = st.inverse_direction_index(d)
        fwd = list(forward_bc(f, d, lb_method))
        if any(hasattr(a.lhs, 'field') and a.lhs != f[c](inv) for a in fwd):
            raise NotImplementedError(f'{forward_bc!r}: a link writes one population of the wall cell, got {fwd}')
        rhs = _inline(fwd, f[c](inv))
        if rhs is None:
            raise NotImplementedError(f'{forward_bc!r}: no link assignment to pdf[c_d](inv_d) in {fwd}')
        rhs = sp.sympify(rhs)
        bad = [a for a in rhs.atoms(ps.Field.Access) if a not in own]
        if bad or (rhs.free_symbols - set(rhs.atoms(ps.Field.Access))):
            raise NotImplementedError(f'{forward_bc!r}: the lattice kernels take links of the fluid cell\'s own pdfs '
                                      f'and constants, got {rhs}')
        value = rhs.xreplace(own)
        lines, (val,) = _program_code([value])
        if derived:
            # the adjoint object is the transposed derivative of this link (AdjointBoundaryCondition): its Jacobian
            # row straight from the forward expression (what the transposed AD prints, without its cost per link)
            rows = []
            try:                                    # polynomial links (FixedDensity: quadratic): fast derivatives
                poly = sp.Poly(value, *cs)
                grads = [poly.diff(ck).as_expr() for ck in cs]
            except sp.PolynomialError:
                grads = [sp.diff(value, ck) for ck in cs]
            pr = _c_printer()
            for k, jk in enumerate(grads):
                if jk != 0:
                    rows.append((k, (), pr.doprint(jk)))
            out.append((lines, val, tuple(rows)))
            continue
        bwd = adjoint_bc(g, d, lb_method)
        allb = list(getattr(bwd, 'all_assignments', bwd))
        if any(hasattr(a.lhs, 'field') and a.lhs not in [g(k) for k in range(st.Q)] for a in allb):
            raise NotImplementedError(f'{adjoint_bc!r}: adjoint assignments beyond diffpdf(k) <- J_k * '
                                      f'diffpdf[c_d](inv_d): {allb}')
        jac = []
        gv = sp.Symbol('__gv')
        for k in range(st.Q):
            r = _inline(allb, g(k))
            if r is None:
                continue
            r = sp.expand(sp.sympify(r).xreplace({g[c](inv): gv}))
            jk = sp.diff(r, gv)
            if sp.expand(r - jk * gv) != 0:
                raise NotImplementedError(f'{adjoint_bc!r}: adjoint link of pdf({k}) is not linear in '
                                          f'diffpdf[c_d](inv_d): {r}')
            if any(a not in own for a in jk.atoms(ps.Field.Access)):
                raise NotImplementedError(f'{adjoint_bc!r}: adjoint coefficient of pdf({k}) reads {jk}')
            jk = sp.expand(jk.xreplace(own))
            if jk != 0:
                jac.append((k, jk))
        jrows = []
        for k, jk in jac:
            jl, (je,) = _program_code([jk])
            jrows.append((k, jl, je))
        out.append((lines, val, tuple(jrows)))
    return tuple(out)


_FORMS = {}


def link_form(forward_bc, adjoint_bc, lb_method):
    """``('affine', link_coefficients(...))`` — the fused (α, β, γ, βρ, γρ) form — or ``('program',
    link_program(...))``; raises ``NotImplementedError`` for a link neither takes. Memoised per (boundary pair,
    stencil, compressibility): a D3Q19 ``FixedDensity`` program takes seconds of sympy."""
    st = _directions(lb_method)
    key = (forward_bc, adjoint_bc, type(adjoint_bc), getattr(st, 'name', None), st.Q,
           getattr(lb_method, 'compressible', None))
    try:
        hit = _FORMS.get(key)
    except TypeError:                       # an unhashable user boundary: no memo
        key, hit = None, None
    if hit is not None:
        return hit
    try:
        res = 'affine', link_coefficients(forward_bc, adjoint_bc, lb_method)
    except NotImplementedError:
        res = 'program', link_program(forward_bc, adjoint_bc, lb_method)
    if key is not None:
        _FORMS[key] = res
    return res


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
        """``(tables, programs)``. ``tables``: per flag id ≥ 1 the ``link_coefficients`` of its (forward, adjoint)
        boundary pair, or None when every id is a plain bounce-back (α = γ = 1, β = 0: the kernels' fast path, no id
        loads). ``programs``: None, or per flag id the ``link_program`` of a boundary the fused form does not take
        (None for the others; its table row is all zeros, so the fused path contributes nothing)."""
        objs = self.objects()
        st = _directions(lb_method)
        zero = tuple((0.0, 0.0, 0.0, 0.0, 0.0) for _ in range(st.Q))
        tables, programs = [None], [None]
        plain = True
        for k in range(1, len(objs)):
            kind, t = link_form(objs[k], self.adjoints[k], lb_method)
            if kind == 'program':
                tables.append(zero)
                programs.append(t)
                plain = False
                continue
            plain &= all(a == 1.0 and b == 0.0 and g == 1.0 and br == 0.0 and gr == 0.0 for a, b, g, br, gr in t)
            tables.append(t)
            programs.append(None)
        if plain:
            return None, None
        tables[0] = tuple((1.0, 0.0, 1.0, 0.0, 0.0) for _ in range(st.Q))
        return tuple(tables), (tuple(programs) if any(p is not None for p in programs) else None)
