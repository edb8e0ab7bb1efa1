"""ctypes access to ``oracle/stencil_ref.c`` (ORACLE — test infrastructure only).

``load(build_dir=None, march=None)`` builds ``liboracle.so`` with ``make`` if needed and
returns a small wrapper. ``bench.py`` rebuilds it with ``-march=native`` on the GPU box so
the CPU baseline runs with the host's own ISA.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

__all__ = ['load', 'OracleLib']


class OracleLib:
    def __init__(self, path):
        L = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_longlong
        L.oracle_diffusion7_f32.argtypes = [vp, vp, i64, i64, i64, ctypes.c_float]
        L.oracle_linear3d_f64.argtypes = [vp, vp, i64, i64, i64, ctypes.c_int, vp, vp]
        L.oracle_stencil27_f16.argtypes = [vp, vp, i64, i64, i64, vp]
        L.oracle_readme_fwd_f32.argtypes = [vp, vp, vp, i64]
        L.oracle_readme_bwd_f32.argtypes = [vp, vp, vp, vp, vp, i64]
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_set_threads.restype = ctypes.c_int
        for name in ('oracle_diffusion7_f32', 'oracle_linear3d_f64', 'oracle_stencil27_f16',
                     'oracle_readme_fwd_f32', 'oracle_readme_bwd_f32'):
            getattr(L, name).restype = None
        self.lib = L
        self.path = path

    def set_threads(self, n):
        """OpenMP threads of the loops (1 = the reference's default, no cpu_openmp); returns the count."""
        return self.lib.oracle_set_threads(int(n))

    def diffusion7_f32(self, u, alpha, out=None):
        u = np.ascontiguousarray(u, dtype=np.float32)
        out = np.empty_like(u) if out is None else out
        Z, Y, X = u.shape
        self.lib.oracle_diffusion7_f32(u.ctypes.data, out.ctypes.data, Z, Y, X, alpha)
        return out

    def linear_f64(self, u, taps):
        u = np.ascontiguousarray(u, dtype=np.float64)
        shape3 = (1,) * (3 - u.ndim) + u.shape
        offs, w = [], []
        for off, wt in taps.items():
            off3 = (0,) * (3 - len(off)) + tuple(off)
            offs += list(off3)
            w.append(wt)
        offs = np.asarray(offs, np.int32)
        w = np.asarray(w, np.float64)
        out = np.empty_like(u)
        self.lib.oracle_linear3d_f64(u.ctypes.data, out.ctypes.data, *shape3, len(w), offs.ctypes.data, w.ctypes.data)
        return out

    def stencil27_f16(self, u, weights27):
        u = np.ascontiguousarray(u, dtype=np.float16)
        w = np.ascontiguousarray(weights27, dtype=np.float32)
        out = np.empty(u.shape, np.float32)
        Z, Y, X = u.shape
        self.lib.oracle_stencil27_f16(u.ctypes.data, out.ctypes.data, Z, Y, X, w.ctypes.data)
        return out

    def readme_fwd_f32(self, x, y):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.float32)
        z = np.empty_like(x)
        self.lib.oracle_readme_fwd_f32(x.ctypes.data, y.ctypes.data, z.ctypes.data, x.size)
        return z

    def readme_bwd_f32(self, x, y, dz):
        x, y, dz = (np.ascontiguousarray(a, np.float32) for a in (x, y, dz))
        dx, dy = np.empty_like(x), np.empty_like(x)
        self.lib.oracle_readme_bwd_f32(x.ctypes.data, y.ctypes.data, dz.ctypes.data, dx.ctypes.data,
                                       dy.ctypes.data, x.size)
        return dx, dy


def load(build_dir=None, march=None):
    build_dir = build_dir or os.path.join(HERE, 'build')
    path = os.path.join(build_dir, 'liboracle.so')
    if not os.path.exists(path) or march is not None:
        cmd = ['make', '-s', '-C', HERE, f'BUILD={os.path.abspath(build_dir)}']
        if march:
            cmd.append(f'MARCH={march}')
        if march is not None and os.path.exists(path):
            os.remove(path)
        subprocess.run(cmd, check=True, capture_output=True)
    return OracleLib(path)
