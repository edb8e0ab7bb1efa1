"""Generate the golden fixtures in tests/golden/ (run: python tests/golden/make_golden.py).

The reference ships no numeric golden data and cannot be
run here (pystencils is absent), so these vectors come from the hand-written
float64 formulas in ``oracle/stencils.py`` — forward stencils and their TF-MAD
adjoints derived on paper (``_autodiff.py:104-109``; README op
``docs/index.rst:77-78``; the two-output op incl. the reference's
unshifted-partial quirk, ``tests/test_tfmad.py:244-248``). Seeds and
distributions follow SURVEY.md §8c / BASELINE.md §3.

Each ``<case>.npz`` holds the inputs (at their storage dtype), the upstream
gradients and the float64 expected forward outputs / input gradients.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, '..', '..')))

from oracle import stencils as S  # noqa: E402


def _u01(seed, shape, dtype):
    return np.random.default_rng(seed).uniform(0.0, 1.0, shape).astype(dtype)


def _um11(seed, shape, dtype):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, shape).astype(dtype)


def _interior(a, g):
    out = np.zeros_like(a)
    sl = tuple(slice(g, n - g) for n in a.shape)
    out[sl] = a[sl]
    return out


def cases():
    out = {}
    # README op, [20,30] fp32, x,y ~ U(0.5,1.5) seed 0, diffz ~ U(-1,1) seed 1
    rng = np.random.default_rng(0)
    x = rng.uniform(0.5, 1.5, (20, 30)).astype(np.float32)
    y = rng.uniform(0.5, 1.5, (20, 30)).astype(np.float32)
    dz = _um11(1, (20, 30), np.float32)
    dx, dy = S.readme_backward(x, y, dz)
    out['readme_f32_20x30'] = dict(x=x, y=y, diffz=dz, z=S.readme_forward(x, y), diffx=dx, diffy=dy)

    # 2-D 5-point Laplacian 64x64 fp32, zeros and interior-only (None)
    u = _u01(0, (64, 64), np.float32)
    do = _um11(1, (64, 64), np.float32)
    t = S.taps_laplace_5pt()
    out['laplace5_f32_64x64_zeros'] = dict(u=u, diffout=do, out=S.linear_stencil(u, t),
                                           diffu=S.linear_stencil(do, S.flip(t)))
    # None mode: iterate the interior [1, N-1) only, reads stay in-domain, border stays 0
    out['laplace5_f32_64x64_none'] = dict(u=u, diffout=do, out=_interior(S.linear_stencil(u, t), 1),
                                          diffu=_interior(S.linear_stencil(do, S.flip(t)), 1))

    # 3-D 7-point diffusion 32^3 fp32
    u = _u01(0, (32, 32, 32), np.float32)
    do = _um11(1, (32, 32, 32), np.float32)
    t = S.taps_diffusion_7pt()
    out['diffusion7_f32_32cube'] = dict(u=u, diffout=do, out=S.linear_stencil(u, t),
                                        diffu=S.linear_stencil(do, S.flip(t)))

    # asymmetric 3-D 7-point 16^3 fp32 (flip errors cannot hide)
    u = _u01(0, (16, 16, 16), np.float32)
    do = _um11(1, (16, 16, 16), np.float32)
    t = S.taps_asym_7pt()
    out['asym7_f32_16cube'] = dict(u=u, diffout=do, out=S.linear_stencil(u, t),
                                   diffu=S.linear_stencil(do, S.flip(t)))

    # 27-point fp16 16^3 (fp32 accumulate; expected from the fp16-rounded inputs in float64)
    u = _u01(0, (16, 16, 16), np.float16)
    do = _um11(1, (16, 16, 16), np.float16)
    t = S.taps_27pt()
    out['stencil27_f16_16cube'] = dict(u=u, diffout=do, out=S.linear_stencil(u, t),
                                       diffu=S.linear_stencil(do, S.flip(t)))

    # test_tfmad.py:195-200 stencil on float64[5,7], random inputs
    a = _u01(2, (5, 7), np.float64)
    b = _u01(3, (5, 7), np.float64)
    do = _um11(4, (5, 7), np.float64)
    ta = {(1, 0): 1.0, (-1, 0): -1.0, (0, 1): -0.75, (0, -1): 0.75, (0, 0): 1.2}
    tb = {(1, 0): -0.5, (-1, 0): 0.5, (0, 1): 1.5, (0, -1): -1.5}
    out['tfmad2d_f64_5x7'] = dict(a=a, b=b, diffout=do, out=S.linear_stencil(a, ta) + S.linear_stencil(b, tb),
                                  diffa=S.linear_stencil(do, S.flip(ta)), diffb=S.linear_stencil(do, S.flip(tb)))

    # test_tfmad.py:244-248 three outputs incl. exp(b[-1,0]) on float64[21,13]
    a = _um11(5, (21, 13), np.float64)
    b = _um11(6, (21, 13), np.float64)
    d1, d2, d3 = (_um11(s, (21, 13), np.float64) for s in (7, 8, 9))
    bp = np.pad(b, 1)
    b_w = bp[0:21, 1:14]                       # b[-1,0] zero-padded
    d3p = np.pad(d3, 1)
    d3_e = d3p[2:23, 1:14]                     # diffout3[1,0] zero-padded
    out['three_outputs_f64_21x13'] = dict(
        a=a, b=b, diffout1=d1, diffout2=d2, diffout3=d3, out1=a + b, out2=a - b, out3=np.exp(b_w),
        diffa=d1 + d2,
        # TF-MAD evaluates d exp(b[-1,0]) / d b[-1,0] at the forward cell: exp(b[-1,0]) * diffout3[1,0]
        diffb=d1 - d2 + d3_e * np.exp(b_w))
    return out


def main():
    for name, data in cases().items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **data)
        print('wrote', name, sorted(data))


if __name__ == '__main__':
    main()
