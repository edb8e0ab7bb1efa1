"""TEST INFRASTRUCTURE ONLY (never imported by the package): an independent restatement of the lattice
Boltzmann time step the ``AutoDiffLatticeBoltzmannStep`` kernels compute, written with array rolls
instead of the symbolic pipeline.

Reference path: ``/root/reference/src/pystencils_autodiff/lbm/_autodiff_lbstep.py:189-247,372-398`` runs
lbmpy's [ext, absent] stream-pull-collide SRT kernel with periodic ghost-layer sync and buffer swaps;
the equations (lbmpy's published SRT method, second-order equilibrium) are restated here:

    f_i(x) = src_i(x − c_i)   (periodic)        ρ = Σ f_i,   u = Σ c_i f_i (/ρ if compressible)
    feq_i = w_i ρ (1 + 3 c·u + 4.5 (c·u)² − 1.5 u²)   or, incompressible, w_i (ρ + 3 c·u + 4.5 (c·u)² − 1.5 u²)
    dst_i = f_i + ω (feq_i − f_i)

``xp`` is numpy or torch (torch: an autograd-able restatement whose gradient, by torch's reverse mode, is
the adjoint oracle for the step's hand-derived transposed kernels). Pdf arrays are ``[*spatial, q]``.
Parity with lbmpy itself is unpinned (lbmpy is not importable here)."""
from fractions import Fraction

D2Q9 = ([(0, 0), (0, 1), (0, -1), (-1, 0), (1, 0), (-1, 1), (1, 1), (-1, -1), (1, -1)],
        [Fraction(4, 9)] + [Fraction(1, 9)] * 4 + [Fraction(1, 36)] * 4)
D3Q19 = ([(0, 0, 0), (0, 1, 0), (0, -1, 0), (-1, 0, 0), (1, 0, 0), (0, 0, 1), (0, 0, -1), (-1, 1, 0), (1, 1, 0),
          (-1, -1, 0), (1, -1, 0), (0, 1, 1), (0, -1, 1), (-1, 0, 1), (1, 0, 1), (0, 1, -1), (0, -1, -1),
          (-1, 0, -1), (1, 0, -1)],
         [Fraction(1, 3)] + [Fraction(1, 18)] * 6 + [Fraction(1, 36)] * 12)
D3Q27 = (D3Q19[0] + [(1, 1, 1), (-1, 1, 1), (1, -1, 1), (-1, -1, 1), (1, 1, -1), (-1, 1, -1), (1, -1, -1),
                     (-1, -1, -1)],
         [Fraction(8, 27)] + [Fraction(2, 27)] * 6 + [Fraction(1, 54)] * 12 + [Fraction(1, 216)] * 8)
SETS = {'D2Q9': D2Q9, 'D3Q19': D3Q19, 'D3Q27': D3Q27}


def _roll(xp, a, shift, axis):
    if xp.__name__ == 'torch':
        return xp.roll(a, shifts=shift, dims=axis)
    return xp.roll(a, shift, axis=axis)


def stream(f, stencil, xp):
    """Pull streaming with periodic wrap: out_i(x) = f_i(x − c_i)."""
    dirs, _ = SETS[stencil]
    comps = []
    for i, c in enumerate(dirs):
        g = f[..., i]
        for ax, s in enumerate(c):
            if s:
                g = _roll(xp, g, s, ax)
        comps.append(g)
    return xp.stack(comps, -1) if xp.__name__ != 'torch' else xp.stack(comps, dim=-1)


def trt_odd_rate(omega, magic=3.0 / 16.0):
    """ω₋ of a TRT method from ω₊ and the magic number Λ = (1/ω₊ − 1/2)(1/ω₋ − 1/2) (lbmpy's published
    relation, default Λ = 3/16)."""
    return 1.0 / (magic / (1.0 / omega - 0.5) + 0.5)


# MRT moments (lbmpy's weighted-orthogonal MRT groups, restated): monomials c_x^a c_y^b (c_z^c) with integer
# coefficients, Gram–Schmidt-orthogonalised under the lattice weights in this order
MRT_BASIS = {
    9: [('cons', {(0, 0): 1}), ('cons', {(1, 0): 1}), ('cons', {(0, 1): 1}), ('bulk', {(2, 0): 1, (0, 2): 1}),
        ('shear', {(2, 0): 1, (0, 2): -1}), ('shear', {(1, 1): 1}), ('third', {(2, 1): 1}), ('third', {(1, 2): 1}),
        ('fourth', {(2, 2): 1})],
    19: [('cons', {(0, 0, 0): 1}), ('cons', {(1, 0, 0): 1}), ('cons', {(0, 1, 0): 1}), ('cons', {(0, 0, 1): 1}),
        ('bulk', {(2, 0, 0): 1, (0, 2, 0): 1, (0, 0, 2): 1}),
        ('shear', {(2, 0, 0): 2, (0, 2, 0): -1, (0, 0, 2): -1}), ('shear', {(0, 2, 0): 1, (0, 0, 2): -1}),
        ('shear', {(1, 1, 0): 1}), ('shear', {(1, 0, 1): 1}), ('shear', {(0, 1, 1): 1}),
        ('third', {(2, 1, 0): 1}), ('third', {(2, 0, 1): 1}), ('third', {(1, 2, 0): 1}), ('third', {(0, 2, 1): 1}),
        ('third', {(1, 0, 2): 1}), ('third', {(0, 1, 2): 1}),
        ('fourth', {(2, 2, 0): 1}), ('fourth', {(2, 0, 2): 1}), ('fourth', {(0, 2, 2): 1})],
}
# D3Q27: + c_x c_y c_z (third order) and the fourth- to sixth-order monomials (relaxed with the fourth-order rate)
MRT_BASIS[27] = MRT_BASIS[19][:16] + [('third', {(1, 1, 1): 1})] + MRT_BASIS[19][16:] + \
    [('fourth', {e: 1}) for e in ((2, 1, 1), (1, 2, 1), (1, 1, 2), (2, 2, 1), (2, 1, 2), (1, 2, 2), (2, 2, 2))]


def mrt_matrix(stencil, rates):
    """The MRT collision matrix ``M⁻¹ S M`` (numpy float64, Q×Q) for group rates ``rates`` = {'shear', 'bulk',
    'third', 'fourth'} (the conserved moments relax with 0): ``dst = f − (M⁻¹ S M)(f − feq)``."""
    import numpy as np
    dirs, w = SETS[stencil]
    D = len(dirs[0])
    W = np.array([float(x) for x in w])
    rows, groups = [], []
    for grp, poly in MRT_BASIS[len(dirs)]:
        v = np.array([sum(cf * np.prod([c[a] ** e[a] for a in range(D)]) for e, cf in poly.items()) for c in dirs],
                     dtype=np.float64)
        for r in rows:
            v = v - (W * v * r).sum() / (W * r * r).sum() * r
        rows.append(v)
        groups.append(grp)
    M = np.array(rows)
    S = np.diag([0.0 if g == 'cons' else float(rates[g]) for g in groups])
    return np.linalg.inv(M) @ S @ M


def collide(f, omega, stencil, compressible, xp, force_model=None, force=None, omega_odd=None, mrt=None):
    """SRT collision, or TRT with ``omega_odd`` (the antisymmetric part of each population pair (f_i − f_ī)/2
    relaxes with ω₋, the symmetric part with ω), or MRT with ``mrt`` (a Q×Q collision matrix, ``mrt_matrix``:
    dst = f − A (f − feq)); ``force_model`` 'simple' (+3 w_i c_i·F) or 'guo' (velocity shifted by F/2,
    + w_i (1 − ω/2) (3 (c_i − u)·F + 9 (c_i·u)(c_i·F))) with a body force ``force`` (lbmpy's published force
    models)."""
    dirs, w = SETS[stencil]
    D = len(dirs[0])
    rho = f.sum(-1)
    u = []
    for a in range(D):
        m = sum(c[a] * f[..., i] for i, c in enumerate(dirs) if c[a])
        if force_model == 'guo':
            m = m + force[a] / 2
        u.append(m / rho if compressible else m)
    usq = sum(ua * ua for ua in u)
    feqs = []
    for i, c in enumerate(dirs):
        cu = sum(ca * ua for ca, ua in zip(c, u) if ca)
        poly = 3 * cu + 4.5 * cu * cu - 1.5 * usq
        feqs.append(float(w[i]) * rho * (1 + poly) if compressible else float(w[i]) * (rho + poly))
    opp = [dirs.index(tuple(-x for x in c)) for c in dirs]
    out = []
    for i, c in enumerate(dirs):
        cu = sum(ca * ua for ca, ua in zip(c, u) if ca)
        feq = feqs[i]
        if mrt is not None:
            g = f[..., i] - sum(float(mrt[i][k]) * (f[..., k] - feqs[k]) for k in range(len(dirs)) if mrt[i][k] != 0)
        elif omega_odd is None:
            g = f[..., i] + omega * (feq - f[..., i])
        else:
            j = opp[i]
            fs, fa = (f[..., i] + f[..., j]) / 2, (f[..., i] - f[..., j]) / 2
            es, ea = (feq + feqs[j]) / 2, (feq - feqs[j]) / 2
            g = f[..., i] - omega * (fs - es) - omega_odd * (fa - ea)
        if force_model is not None:
            cF = sum(ca * Fa for ca, Fa in zip(c, force) if ca)
            if force_model == 'simple':
                g = g + 3 * float(w[i]) * cF
            else:
                cmuF = sum((ca - ua) * Fa for ca, ua, Fa in zip(c, u, force))
                g = g + float(w[i]) * (1 - omega / 2) * (3 * cmuF + 9 * cu * cF)
        out.append(g)
    return xp.stack(out, -1) if xp.__name__ != 'torch' else xp.stack(out, dim=-1)


def step(f, omega, stencil='D2Q9', compressible=False, xp=None, force_model=None, force=None, omega_odd=None,
         mrt=None):
    """One stream-pull-collide time step on a periodic domain (``f``: ``[*spatial, q]``)."""
    if xp is None:
        import numpy as xp
    return collide(stream(f, stencil, xp), omega, stencil, compressible, xp, force_model, force, omega_odd, mrt)


def run(f, omega, steps, stencil='D2Q9', compressible=False, xp=None, force_model=None, force=None, omega_odd=None,
        mrt=None):
    for _ in range(steps):
        f = step(f, omega, stencil, compressible, xp, force_model, force, omega_odd, mrt)
    return f


def equilibrium(rho, u, stencil='D2Q9', compressible=False, xp=None):
    """feq(ρ, u) as ``[*spatial, q]`` (``u``: ``[*spatial, d]``)."""
    if xp is None:
        import numpy as xp
    dirs, w = SETS[stencil]
    usq = sum(u[..., a] * u[..., a] for a in range(len(dirs[0])))
    out = []
    for i, c in enumerate(dirs):
        cu = sum(ca * u[..., a] for a, ca in enumerate(c) if ca)
        poly = 3 * cu + 4.5 * cu * cu - 1.5 * usq
        out.append(float(w[i]) * rho * (1 + poly) if compressible else float(w[i]) * (rho + poly))
    return xp.stack(out, -1) if xp.__name__ != 'torch' else xp.stack(out, dim=-1)


def inverse(stencil):
    dirs, _ = SETS[stencil]
    return [dirs.index(tuple(-c for c in d)) for d in dirs]


def _roll_all(xp, a, c):
    for ax, s in enumerate(c):
        if s:
            a = _roll(xp, a, s, ax)
    return a


def stream_walls(f, stencil, wall, xp):
    """Pull streaming with half-way bounce-back at no-slip obstacle cells (``wall``: bool array over the domain):
    ``f_i(x) = f_ī(x)`` where ``x − c_i`` is an obstacle, else ``f_i(x − c_i)`` (periodic) — lbmpy's ``NoSlip``
    (``src_ī(x + c_i) := src_i(x)`` written into the obstacle cell, then the pull; ``adjoint_boundaryconditions.py``
    restates its adjoint)."""
    dirs, _ = SETS[stencil]
    inv = inverse(stencil)
    comps = []
    for i, c in enumerate(dirs):
        pulled = _roll_all(xp, f[..., i], c)
        nb_wall = _roll_all(xp, wall, c)
        comps.append(xp.where(nb_wall, f[..., inv[i]], pulled))
    return xp.stack(comps, -1) if xp.__name__ != 'torch' else xp.stack(comps, dim=-1)


def step_walls(f, omega, wall, stencil='D2Q9', compressible=False, xp=None, force_model=None, force=None,
               omega_odd=None, mrt=None):
    """One stream-pull-collide step with no-slip obstacles (and optionally a body force on the fluid cells, as
    ``collide``); obstacle cells keep their state."""
    if xp is None:
        import numpy as xp
    new = collide(stream_walls(f, stencil, wall, xp), omega, stencil, compressible, xp, force_model, force, omega_odd,
                  mrt)
    keep = wall[..., None] if xp.__name__ != 'torch' else wall.unsqueeze(-1)
    return xp.where(keep, f, new)


def run_walls(f, omega, wall, steps, stencil='D2Q9', compressible=False, xp=None, force_model=None, force=None,
              omega_odd=None, mrt=None):
    for _ in range(steps):
        f = step_walls(f, omega, wall, stencil, compressible, xp, force_model, force, omega_odd, mrt)
    return f


def stream_moving_walls(f, stencil, wall, wall_velocity, xp, density_weighted=False):
    """Pull streaming with bounce-back at wall cells that may move (lbmpy's ``UBB`` [ext], ``NoSlip`` where the
    velocity is 0): where ``x − c_i`` is a wall cell with velocity ``u_w``, ``f_i(x) = f_ī(x) + 6 w_i (c_i · u_w)``
    (the population that left ``x`` towards the wall, reflected with the wall's momentum: 2/c_s² = 6), else
    ``f_i(x − c_i)`` (periodic). ``wall_velocity``: ``[*spatial, d]`` (axis-0 component first; only read at wall
    cells). ``density_weighted``: the wall term times the fluid cell's density Σ_k f_k(x) (lbmpy's compressible UBB)."""
    dirs, w = SETS[stencil]
    inv = inverse(stencil)
    rho = f.sum(-1)
    comps = []
    for i, c in enumerate(dirs):
        pulled = _roll_all(xp, f[..., i], c)
        nb_wall = _roll_all(xp, wall, c)
        cu = sum(ca * _roll_all(xp, wall_velocity[..., a], c) for a, ca in enumerate(c) if ca)
        if density_weighted and any(c):
            cu = cu * rho
        bounced = f[..., inv[i]] + 6 * float(w[i]) * cu if any(c) else f[..., inv[i]]
        comps.append(xp.where(nb_wall, bounced, pulled))
    return xp.stack(comps, -1) if xp.__name__ != 'torch' else xp.stack(comps, dim=-1)


def run_moving_walls(f, omega, wall, wall_velocity, steps, stencil='D2Q9', compressible=False, xp=None,
                     density_weighted=False, omega_odd=None):
    """``steps`` stream-pull-collide steps with (moving) bounce-back walls; wall cells keep their state."""
    if xp is None:
        import numpy as xp
    keep = wall[..., None] if xp.__name__ != 'torch' else wall.unsqueeze(-1)
    for _ in range(steps):
        new = collide(stream_moving_walls(f, stencil, wall, wall_velocity, xp, density_weighted), omega, stencil,
                      compressible, xp, omega_odd=omega_odd)
        f = xp.where(keep, f, new)
    return f


def stream_pressure_walls(f, stencil, wall, pressure, rho_wall, compressible, xp, wall_velocity=None,
                          density_weighted=False):
    """Pull streaming with bounce-back walls and pressure cells (lbmpy's ``FixedDensity`` [ext], anti-bounce-back):
    where ``x − c_i`` is a pressure cell of density ``ρ_w`` (``pressure``: bool over the domain, a subset of
    ``wall``; ``rho_wall``: per cell, read at pressure cells), with ``d = ī`` the direction that left ``x`` towards
    it, ``f_i(x) = 2 w_d ρ_w (1 + 4.5 (c_d·u)² − 1.5 u²) − f_d(x)`` (incompressible: ``2 w_d (ρ_w + 4.5 (c_d·u)² −
    1.5 u²) − f_d(x)``) with ``u = Σ_k c_k f_k(x) / ρ_w`` (incompressible: without the division) of the fluid cell's
    own pdfs — lbmpy prints the equilibrium's velocity subexpression with its density symbol replaced by ρ_w. Other
    wall cells bounce back (moving with ``wall_velocity`` where given, as ``stream_moving_walls``, its wall term
    times the fluid cell's density with ``density_weighted``)."""
    dirs, w = SETS[stencil]
    inv = inverse(stencil)
    D = len(dirs[0])
    m = [sum(c[a] * f[..., k] for k, c in enumerate(dirs) if c[a]) for a in range(D)]
    comps = []
    for i, c in enumerate(dirs):
        pulled = _roll_all(xp, f[..., i], c)
        if not any(c):
            comps.append(pulled)
            continue
        d = inv[i]
        nb_wall = _roll_all(xp, wall, c)
        nb_p = _roll_all(xp, pressure, c)
        rw = _roll_all(xp, rho_wall, c)
        bounced = f[..., d]
        if wall_velocity is not None:
            cuw = sum(ca * _roll_all(xp, wall_velocity[..., a], c) for a, ca in enumerate(c) if ca)
            bounced = bounced + 6 * float(w[i]) * (cuw * f.sum(-1) if density_weighted else cuw)
        u = [ma / rw if compressible else ma for ma in m]
        cu = sum(dirs[d][a] * u[a] for a in range(D) if dirs[d][a])
        usq = sum(ua * ua for ua in u)
        sym = rw * (1 + 4.5 * cu * cu - 1.5 * usq) if compressible else rw + 4.5 * cu * cu - 1.5 * usq
        anti = 2 * float(w[d]) * sym - f[..., d]
        comps.append(xp.where(nb_wall, xp.where(nb_p, anti, bounced), pulled))
    return xp.stack(comps, -1) if xp.__name__ != 'torch' else xp.stack(comps, dim=-1)


def run_pressure_walls(f, omega, wall, pressure, rho_wall, steps, stencil='D2Q9', compressible=False, xp=None,
                       omega_odd=None, wall_velocity=None, density_weighted=False, mrt=None):
    """``steps`` stream-pull-collide steps with (moving) bounce-back walls and pressure cells; wall cells keep their
    state."""
    if xp is None:
        import numpy as xp
    keep = wall[..., None] if xp.__name__ != 'torch' else wall.unsqueeze(-1)
    for _ in range(steps):
        new = collide(stream_pressure_walls(f, stencil, wall, pressure, rho_wall, compressible, xp, wall_velocity,
                                            density_weighted), omega, stencil, compressible, xp, omega_odd=omega_odd,
                      mrt=mrt)
        f = xp.where(keep, f, new)
    return f
