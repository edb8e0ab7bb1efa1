"""Lattice Boltzmann update rules for ``AutoDiffLatticeBoltzmannStep`` (``lbm/_autodiff_lbstep.py``).

The reference builds its update rule with lbmpy [ext] (``lbmpy.creationfunctions.create_lb_update_rule``,
absent here: an un-vendored dependency of ``/root/reference/src/pystencils_autodiff/lbm/_autodiff_lbstep.py:8-10``).
This module restates the part of lbmpy the step consumes, as ``AssignmentCollection``s of this package's
``ps`` front-end: lbmpy's D2Q9 / D3Q19 / D3Q27 velocity sets (same direction order and weights), the
single-relaxation-time (SRT/BGK) method with the second-order equilibrium (compressible, or lbmpy's
incompressible form with reference density 1), and the ``stream_pull_collide`` kernel type:

    f_i(x) = src_i(x − c_i)                                  (pull streaming)
    ρ = Σ_i f_i,   u = Σ_i c_i f_i / ρ   (incompressible: / 1)
    feq_i = w_i ρ (1 + 3 c_i·u + 9/2 (c_i·u)² − 3/2 u²)     (incompressible: w_i (ρ + 3 c_i·u + …))
    dst_i(x) = f_i + ω (feq_i − f_i)

plus the macroscopic getter (ρ, u from the pdfs) and setter (pdfs = feq(ρ, u)) the step's
``create_macroscopic_*_op`` wrap. A constant body force F (``force_model``, lbmpy's ``forcemodels`` [ext]):

    'simple':  dst_i += 3 w_i (c_i·F)
    'guo':     u = (Σ_i c_i f_i + F/2) (/ρ),   dst_i += w_i (1 − ω/2) (3 (c_i − u)·F + 9 (c_i·u)(c_i·F))

(the getter reports Guo's shifted velocity). Parity with lbmpy is unpinned (lbmpy is absent); the oracle
(``oracle/lbm.py``) restates the same equations independently with array rolls.
"""
import sympy as sp

from .. import ps

__all__ = ['LBStencil', 'create_lb_update_rule', 'create_lb_adjoint_rule', 'macroscopic_getter',
           'equilibrium_setter', 'relaxation_rate_from_magic_number', 'mrt_moments', 'mrt_relaxation_matrices']


class LBStencil:
    """A DdQq velocity set in lbmpy's direction order (``lbmpy.stencils.LBStencil`` [ext]): ``directions``
    (tuples over the spatial axes, axis 0 first) and the lattice weights."""

    _SETS = {
        'D2Q9': ([(0, 0), (0, 1), (0, -1), (-1, 0), (1, 0), (-1, 1), (1, 1), (-1, -1), (1, -1)],
                 [sp.Rational(4, 9)] + [sp.Rational(1, 9)] * 4 + [sp.Rational(1, 36)] * 4),
        'D3Q19': ([(0, 0, 0), (0, 1, 0), (0, -1, 0), (-1, 0, 0), (1, 0, 0), (0, 0, 1), (0, 0, -1),
                   (-1, 1, 0), (1, 1, 0), (-1, -1, 0), (1, -1, 0), (0, 1, 1), (0, -1, 1), (-1, 0, 1),
                   (1, 0, 1), (0, 1, -1), (0, -1, -1), (-1, 0, -1), (1, 0, -1)],
                  [sp.Rational(1, 3)] + [sp.Rational(1, 18)] * 6 + [sp.Rational(1, 36)] * 12),
    }

    def __init__(self, name):
        name = str(name).upper().replace('STENCIL.', '')
        if name == 'D3Q27':
            dirs = [(0, 0, 0), (0, 1, 0), (0, -1, 0), (-1, 0, 0), (1, 0, 0), (0, 0, 1), (0, 0, -1),
                    (-1, 1, 0), (1, 1, 0), (-1, -1, 0), (1, -1, 0), (0, 1, 1), (0, -1, 1), (-1, 0, 1),
                    (1, 0, 1), (0, 1, -1), (0, -1, -1), (-1, 0, -1), (1, 0, -1),
                    (1, 1, 1), (-1, 1, 1), (1, -1, 1), (-1, -1, 1), (1, 1, -1), (-1, 1, -1), (1, -1, -1),
                    (-1, -1, -1)]
            w = {0: sp.Rational(8, 27), 1: sp.Rational(2, 27), 2: sp.Rational(1, 54), 3: sp.Rational(1, 216)}
            weights = [w[sum(abs(c) for c in d)] for d in dirs]
        elif name in self._SETS:
            dirs, weights = self._SETS[name]
        else:
            raise ValueError(f"unknown stencil '{name}' (D2Q9, D3Q19, D3Q27)")
        self.name = name
        self.directions = [tuple(d) for d in dirs]
        self.weights = list(weights)
        self.D = len(self.directions[0])
        self.Q = len(self.directions)
        assert sum(self.weights) == 1

    def __len__(self):
        return self.Q

    def inverse_direction_index(self, i):
        return self.directions.index(tuple(-c for c in self.directions[i]))


def _moments(stencil, f, compressible, shift=None):
    """ρ and u of the pdfs ``f``; ``shift``: a velocity shift per axis added to the momentum (Guo's F/2)."""
    rho = sp.Symbol('rho')
    us = sp.symbols(f'u_:{stencil.D}')
    subs = [ps.Assignment(rho, sum(f))]
    for a in range(stencil.D):
        mom = sum(c[a] * fi for c, fi in zip(stencil.directions, f) if c[a])
        if shift is not None:
            mom = mom + shift[a]
        subs.append(ps.Assignment(us[a], mom / rho if compressible else mom))
    return rho, us, subs


FORCE_MODELS = ('simple', 'guo')


def force_components(force, D):
    """The body force per axis as sympy expressions: numbers / symbols, or a force FIELD (a vector field of ``D``
    components, or a sequence of accesses) — a per-cell force, an additional input of the update rule."""
    if isinstance(force, ps.Field):
        if force.index_dimensions != 1 or int(force.index_shape[0]) != D:
            raise ValueError(f"force field '{force.name}' needs {D} components (one index dimension)")
        return [force.center(a) for a in range(D)]
    return [sp.sympify(v) for v in force]


def force_is_field(force):
    """Whether the (stored) force reads a field: a per-cell force."""
    return force is not None and any(sp.sympify(v).atoms(ps.Field.Access) for v in force)


def _force(force_model, force, stencil):
    """(velocity shift or None, per-direction force term builder) of a constant body force."""
    if force_model is None:
        if force is not None:
            raise ValueError('force given without force_model')
        return None, None
    fm = str(force_model).lower()
    if fm not in FORCE_MODELS:
        raise NotImplementedError(f"force_model '{force_model}': one of {FORCE_MODELS}")
    F = force_components(force, stencil.D)
    if len(F) != stencil.D:
        raise ValueError(f'force needs {stencil.D} components')

    def term(i, us, omega):
        c = stencil.directions[i]
        w = stencil.weights[i]
        cF = sum(ca * Fa for ca, Fa in zip(c, F) if ca)
        if fm == 'simple':
            return 3 * w * cF
        cu = sum(ca * ua for ca, ua in zip(c, us) if ca)
        cmu_F = sum((ca - ua) * Fa for ca, ua, Fa in zip(c, us, F))
        return w * (1 - omega / 2) * (3 * cmu_F + 9 * cu * cF)
    shift = [Fa / 2 for Fa in F] if fm == 'guo' else None
    return shift, term


def _feq(stencil, i, rho, us, compressible):
    c = stencil.directions[i]
    cu = sum(ca * ua for ca, ua in zip(c, us) if ca)
    usq = sum(ua ** 2 for ua in us)
    poly = 3 * cu + sp.Rational(9, 2) * cu ** 2 - sp.Rational(3, 2) * usq
    w = stencil.weights[i]
    return w * rho * (1 + poly) if compressible else w * (rho + poly)


def relaxation_rate_from_magic_number(relaxation_rate, magic_number=sp.Rational(3, 16)):
    """The odd-moment rate of a TRT method from the even one and the magic number
    Λ = (1/ω₊ − 1/2)(1/ω₋ − 1/2) (lbmpy ``relaxation_rate_from_magic_number`` [ext], default Λ = 3/16)."""
    w = sp.sympify(relaxation_rate)
    lam = sp.sympify(magic_number)
    return (4 - 2 * w) / (4 * lam * w + 2 - w)


METHODS = ('srt', 'trt', 'mrt')

# MRT moment polynomials (exponents per axis), grouped by relaxation rate: lbmpy's weighted-orthogonal MRT groups
# (shear, bulk, third order, fourth order) [ext]; conserved moments (density, momentum) first
_MRT_POLYS = {
    (2, 9): [('conserved', [(0, 0)]), ('conserved', [(1, 0)]), ('conserved', [(0, 1)]),
        ('bulk', [(2, 0), (0, 2)]), ('shear', [(2, 0), (0, 2, -1)]), ('shear', [(1, 1)]),
        ('third', [(2, 1)]), ('third', [(1, 2)]), ('fourth', [(2, 2)])],
    (3, 19): [('conserved', [(0, 0, 0)]), ('conserved', [(1, 0, 0)]), ('conserved', [(0, 1, 0)]), ('conserved', [(0, 0, 1)]),
        ('bulk', [(2, 0, 0), (0, 2, 0), (0, 0, 2)]),
        ('shear', [(2, 0, 0, 2), (0, 2, 0, -1), (0, 0, 2, -1)]), ('shear', [(0, 2, 0), (0, 0, 2, -1)]),
        ('shear', [(1, 1, 0)]), ('shear', [(1, 0, 1)]), ('shear', [(0, 1, 1)]),
        ('third', [(2, 1, 0)]), ('third', [(2, 0, 1)]), ('third', [(1, 2, 0)]), ('third', [(0, 2, 1)]),
        ('third', [(1, 0, 2)]), ('third', [(0, 1, 2)]),
        ('fourth', [(2, 2, 0)]), ('fourth', [(2, 0, 2)]), ('fourth', [(0, 2, 2)])],
}
# D3Q27: the D3Q19 moments plus xyz (third order) and the fourth- to sixth-order ones (all relaxing with the last rate)
_MRT_POLYS[(3, 27)] = _MRT_POLYS[(3, 19)][:16] + [('third', [(1, 1, 1)])] + _MRT_POLYS[(3, 19)][16:] + \
    [('fourth', [(2, 1, 1)]), ('fourth', [(1, 2, 1)]), ('fourth', [(1, 1, 2)]), ('fourth', [(2, 2, 1)]),
     ('fourth', [(2, 1, 2)]), ('fourth', [(1, 2, 2)]), ('fourth', [(2, 2, 2)])]
MRT_GROUPS = ('shear', 'bulk', 'third', 'fourth')


def mrt_moments(stencil):
    """The MRT moment basis of a D2Q9 / D3Q19 / D3Q27 stencil: ``[(group, row)]`` — each row the moment's values per
    direction (exact rationals), made orthogonal under the lattice weights (Σ_i w_i m_i n_i = 0) by Gram–Schmidt in
    the listed order (conserved → second order (bulk = |c|², shear = the traceless and off-diagonal parts) → third →
    fourth order; D3Q27's fifth- and sixth-order moments relax with the fourth-order rate). A polynomial is a list of
    monomial exponent tuples, an optional last entry the coefficient."""
    st = stencil if isinstance(stencil, LBStencil) else LBStencil(stencil)
    if (st.D, st.Q) not in _MRT_POLYS:
        raise NotImplementedError(f'MRT moments for {st.name}: D2Q9, D3Q19 and D3Q27 are restated')
    w = st.weights
    rows = []
    for group, terms in _MRT_POLYS[(st.D, st.Q)]:
        vec = [sp.Integer(0)] * st.Q
        for t in terms:
            e, coef = t[:st.D], (sp.Integer(t[st.D]) if len(t) > st.D else sp.Integer(1))
            for i, c in enumerate(st.directions):
                m = sp.Integer(1)
                for a in range(st.D):
                    m *= sp.Integer(c[a]) ** e[a]
                vec[i] += coef * m
        for _, r in rows:
            proj = sum(wi * a * b for wi, a, b in zip(w, vec, r)) / sum(wi * b * b for wi, b in zip(w, r))
            vec = [a - proj * b for a, b in zip(vec, r)]
        if all(v == 0 for v in vec):
            raise AssertionError(f'MRT moment basis of {st.name} is degenerate')
        rows.append((group, vec))
    return rows


def mrt_relaxation_matrices(stencil):
    """Per group: the projector ``P_g = M⁻¹ E_g M`` (E_g selects the group's moments) as exact rationals, ``P_g[i][k]``
    — the collision's relaxation matrix is ``Σ_g s_g P_g`` (the conserved group relaxes with 0). With the weighted-
    orthogonal rows m_k: ``P_g = Σ_{k∈g} W m_k m_kᵀ / (m_kᵀ W m_k)``."""
    st = stencil if isinstance(stencil, LBStencil) else LBStencil(stencil)
    w = st.weights
    out = {}
    for group, m in mrt_moments(st):
        nrm = sum(wi * a * a for wi, a in zip(w, m))
        P = out.setdefault(group, [[sp.Integer(0)] * st.Q for _ in range(st.Q)])
        for i in range(st.Q):
            for k in range(st.Q):
                P[i][k] += w[i] * m[i] * m[k] / nrm
    return out


def create_lb_update_rule(stencil='D2Q9', relaxation_rate=None, compressible=False, src_field=None, dst_field=None,
                          data_type='float64', layout='fzyx', kernel_type='stream_pull_collide', force_model=None,
                          force=None, method='srt', relaxation_rates=None, magic_number=sp.Rational(3, 16)):
    """SRT (BGK) or TRT ``stream_pull_collide`` update rule (lbmpy ``create_lb_update_rule(stencil=…,
    method='srt' | 'trt', relaxation_rate=…, compressible=…, kernel_type='stream_pull_collide')`` [ext]).
    ``relaxation_rate`` = ω: a number, or a sympy symbol left as a kernel parameter (default: the symbol ``omega``).
    TRT relaxes the symmetric part of each population pair (f_i + f_ī)/2 with ω (= ω₊, the shear rate) and the
    antisymmetric part with ω₋ — ``relaxation_rates=[ω₊, ω₋]``, or ω₋ from the magic number Λ
    (``relaxation_rate_from_magic_number``, lbmpy's default 3/16):

        dst_i = f_i − ω₊ (f_i⁺ − feq_i⁺) − ω₋ (f_i⁻ − feq_i⁻),   x_i^± = (x_i ± x_ī) / 2.

    MRT (D2Q9, D3Q19, D3Q27) relaxes the weighted-orthogonal moments (``mrt_moments``) group by group —
    ``relaxation_rates=[shear, bulk, third, fourth]`` (lbmpy's order; missing entries default to ω, the first to ω):

        dst = f − Σ_g s_g P_g (f − feq),   P_g = M⁻¹ E_g M   (``mrt_relaxation_matrices``)

    — all rates ω is SRT. On D2Q9 and D3Q19 ``[ω, ω, ω₋, ω]`` is TRT (there the odd non-conserved moments are exactly
    the third-order ones); on D3Q27 it is not: its odd fifth-order moments x²y²z, x²yz², xy²z² relax with the
    fourth-order rate (``tests/test_lbm.py::test_lbm_mrt_trt_equivalence_per_stencil``). The rule keeps
    ``ac.mrt_rates`` (per group) for the lattice kernels.

    Fields: ``src(q)``/``dst(q)`` vector fields in ``layout`` (``'fzyx'``: components slowest, lbmpy's default)
    unless given. ``force_model`` ('simple' or 'guo', with every method: Guo's force term is scaled by 1 − ω/2 with
    the shear rate ω) with ``force``: a body force — constant (numbers or symbols per axis) or per cell (a vector
    field of D components: an additional input of the rule, its adjoint accumulated over the steps)."""
    if kernel_type != 'stream_pull_collide':
        raise NotImplementedError("only kernel_type='stream_pull_collide' is restated")
    method = str(method).lower()
    if method not in METHODS:
        raise NotImplementedError(f"method '{method}': one of {METHODS} is restated (lbmpy's MRT / cumulant methods "
                                  'are not)')
    st = stencil if isinstance(stencil, LBStencil) else LBStencil(stencil)
    if src_field is None or dst_field is None:
        src_field, dst_field = ps.fields(f"src({st.Q}), dst({st.Q}): {data_type}[{st.D}D]", layout=layout)
    if relaxation_rates is not None:
        if method == 'trt' and len(relaxation_rates) != 2:
            raise ValueError('relaxation_rates: [even, odd] for the TRT method')
        if method == 'mrt' and not 1 <= len(relaxation_rates) <= 4:
            raise ValueError('relaxation_rates: [shear, bulk, third, fourth] for the MRT method')
        if method == 'srt':
            raise ValueError('relaxation_rates: for the TRT / MRT methods (SRT: relaxation_rate)')
        relaxation_rate = relaxation_rates[0]
    omega = sp.Symbol('omega') if relaxation_rate is None else sp.sympify(relaxation_rate)
    f = [src_field[tuple(-c for c in st.directions[i])](i) for i in range(st.Q)]
    # Guo with TRT / MRT: lbmpy's Guo model scales the force term by 1 − ω/2 with the shear rate ω [ext] (not by
    # moment group); the velocity shift F/2 as for SRT
    shift, term = _force(force_model, force, st)
    rho, us, subs = _moments(st, f, compressible, shift)
    feq = [_feq(st, i, rho, us, compressible) for i in range(st.Q)]
    mrt_rates = None
    if method == 'srt':
        omega_odd = None
        coll = [f[i] + omega * (feq[i] - f[i]) for i in range(st.Q)]
    elif method == 'mrt':
        omega_odd = None
        given = list(relaxation_rates or [])
        mrt_rates = {g: (sp.sympify(given[n]) if n < len(given) else omega) for n, g in enumerate(MRT_GROUPS)}
        P = mrt_relaxation_matrices(st)
        neq = [f[k] - feq[k] for k in range(st.Q)]
        coll = [f[i] - sum(mrt_rates[g] * sum(P[g][i][k] * neq[k] for k in range(st.Q) if P[g][i][k] != 0)
                           for g in MRT_GROUPS) for i in range(st.Q)]
    else:
        omega_odd = sp.sympify(relaxation_rates[1]) if relaxation_rates is not None else \
            relaxation_rate_from_magic_number(omega, magic_number)
        inv = [st.inverse_direction_index(i) for i in range(st.Q)]
        coll = [f[i] - omega * ((f[i] + f[inv[i]]) / 2 - (feq[i] + feq[inv[i]]) / 2)
                - omega_odd * ((f[i] - f[inv[i]]) / 2 - (feq[i] - feq[inv[i]]) / 2) for i in range(st.Q)]
    main = [ps.Assignment(dst_field.center(i), coll[i] + (term(i, us, omega) if term else 0)) for i in range(st.Q)]
    ac = ps.AssignmentCollection(main, subs)
    ac.stencil = st
    ac.compressible = compressible
    ac.relaxation_rate = omega
    ac.method = method
    ac.relaxation_rate_odd = omega_odd
    ac.magic_number = sp.sympify(magic_number) if method == 'trt' and relaxation_rates is None else None
    ac.mrt_rates = mrt_rates
    ac.force_model = None if force_model is None else str(force_model).lower()
    ac.force = None if force is None else tuple(force_components(force, st.D))
    return ac


def create_lb_adjoint_rule(update_rule, diff_fields_prefix='diff'):
    """The exact adjoint of a ``create_lb_update_rule`` rule in scatter form (what ``DiffModes.TRANSPOSED``
    derives, ``_autodiff.py:354-437``, written through the collision's structure instead of Q² expanded
    partial derivatives). With g_i = diffdst_i(y) and the pulled f_j = src_j(y − c_j) of cell y:

        diffsrc_j(y − c_j) = (1 − ω) g_j + ω (A + Σ_a B_a ∂u_a/∂f_j),
        A = Σ_i g_i ∂feq_i/∂ρ,   B_a = Σ_i g_i ∂feq_i/∂u_a,
        ∂u_a/∂f_j = (c_ja − u_a)/ρ  (compressible)   or   c_ja  (incompressible)

    — O(q·d) arithmetic per cell instead of O(q²). For a fixed component j the map y ↦ y − c_j is a
    bijection of the (periodic) lattice, so every (j, cell) of diffsrc is written exactly once. TRT
    (dst_i = (1 − a) f_i − b f_ī + a feq_i + b feq_ī, a = (ω₊ + ω₋)/2, b = (ω₊ − ω₋)/2): the same sums over
    h_i = a g_i + b g_ī, and diffsrc_j(y − c_j) = (1 − a) g_j − b g_ĵ + A_h + Σ_a B_h,a ∂u_a/∂f_j."""
    st = update_rule.stencil
    comp = update_rule.compressible
    omega = update_rule.relaxation_rate
    trt = getattr(update_rule, 'method', 'srt') == 'trt'
    mrt = getattr(update_rule, 'method', 'srt') == 'mrt'
    src = update_rule.free_fields
    dst = update_rule.bound_fields
    (src,), (dst,) = tuple(src), tuple(dst)
    from .._adjoint_field import AdjointField
    dsrc, ddst = AdjointField(src, diff_fields_prefix), AdjointField(dst, diff_fields_prefix)
    f = [src[tuple(-c for c in st.directions[i])](i) for i in range(st.Q)]
    g = [ddst.center(i) for i in range(st.Q)]
    rho, us, subs = _moments(st, f, comp)
    feq = [_feq(st, i, rho, us, comp) for i in range(st.Q)]
    A = sp.Symbol('adj_rho')
    B = sp.symbols(f'adj_u_:{st.D}')
    if trt:
        opp = [st.inverse_direction_index(i) for i in range(st.Q)]
        ka, kb = sp.Symbol('trt_a'), sp.Symbol('trt_b')
        subs += [ps.Assignment(ka, (omega + update_rule.relaxation_rate_odd) / 2),
                 ps.Assignment(kb, (omega - update_rule.relaxation_rate_odd) / 2)]
        h = [ka * g[i] + kb * g[opp[i]] for i in range(st.Q)]
    elif mrt:
        # h = Aᵀ g, A = Σ_g s_g P_g: dst = f − A (f − feq)  ⇒  v_j = g_j − h_j + (Jfeqᵀ h)_j
        P = mrt_relaxation_matrices(st)
        hs = sp.symbols(f'mrt_h_:{st.Q}')
        for i in range(st.Q):
            subs.append(ps.Assignment(hs[i], sum(update_rule.mrt_rates[gr] * sum(P[gr][k][i] * g[k] for k in range(st.Q)
                                                                                if P[gr][k][i] != 0)
                                                 for gr in MRT_GROUPS)))
        h = list(hs)
    else:
        h = g
    subs.append(ps.Assignment(A, sum(gi * sp.diff(fe, rho) for gi, fe in zip(h, feq))))
    for a in range(st.D):
        subs.append(ps.Assignment(B[a], sum(gi * sp.diff(fe, us[a]) for gi, fe in zip(h, feq))))
    if comp:
        inv = sp.Symbol('inv_rho')
        subs.append(ps.Assignment(inv, 1 / rho))
    main = []
    for j, c in enumerate(st.directions):
        du = [(c[a] - us[a]) * inv if comp else c[a] for a in range(st.D)]
        eq = A + sum(B[a] * du[a] for a in range(st.D) if du[a] != 0)
        if trt:
            rhs = (1 - ka) * g[j] - kb * g[opp[j]] + eq
        elif mrt:
            rhs = g[j] - h[j] + eq
        else:
            rhs = (1 - omega) * g[j] + omega * eq
        main.append(ps.Assignment(dsrc[tuple(-ci for ci in c)](j), rhs))
    return ps.AssignmentCollection(main, subs)


def macroscopic_getter(stencil, pdf_field, density_field, velocity_field, compressible=False, force_model=None,
                       force=None):
    """ρ = Σ f_i, u = Σ c_i f_i (/ρ): lbmpy's ``macroscopic_values_getter`` [ext] for the SRT method (Guo's
    forcing: the velocity shifted by F/2)."""
    st = stencil if isinstance(stencil, LBStencil) else LBStencil(stencil)
    f = [pdf_field.center(i) for i in range(st.Q)]
    shift, _ = _force(force_model, force, st)
    rho, us, subs = _moments(st, f, compressible, shift)
    main = [ps.Assignment(density_field.center, rho)] + \
        [ps.Assignment(velocity_field.center(a), us[a]) for a in range(st.D)]
    return ps.AssignmentCollection(main, subs)


def equilibrium_setter(stencil, pdf_field, density_field, velocity_field, compressible=False):
    """pdfs = feq(ρ, u): lbmpy's ``macroscopic_values_setter`` [ext] (equilibrium initialisation)."""
    st = stencil if isinstance(stencil, LBStencil) else LBStencil(stencil)
    rho = density_field.center
    us = [velocity_field.center(a) for a in range(st.D)]
    return ps.AssignmentCollection([ps.Assignment(pdf_field.center(i), _feq(st, i, rho, us, compressible))
                                    for i in range(st.Q)], [])


def _check_directions():
    for name in ('D2Q9', 'D3Q19', 'D3Q27'):
        st = LBStencil(name)
        assert len(set(st.directions)) == st.Q
        for a in range(st.D):                      # isotropy: Σ w c_a c_b = δ_ab / 3
            for b in range(st.D):
                m = sum(w * c[a] * c[b] for w, c in zip(st.weights, st.directions))
                assert m == (sp.Rational(1, 3) if a == b else 0), (name, a, b, m)
    return True
