"""sha256 of the emitted HIP source of every default launch plan over a matrix of workloads, shapes, boundary modes
and pointer-alignment classes (no GPU: the plan selection of ``HipStencilKernel._plan_march`` runs on stand-in
tensors, the compile step is skipped). Used to show that a refactor of the emitters leaves every default kernel
byte-identical:

python scripts/probes/emit_snapshot.py > before.txt; (edit); python scripts/probes/emit_snapshot.py | diff before.txt -
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from pystencils_autodiff_amd import AutoDiffOp, workloads as W  # noqa: E402
from pystencils_autodiff_amd.backends import hip_kernel as HK  # noqa: E402
from pystencils_autodiff_amd.backends.kernel_ir import StencilKernel  # noqa: E402


class FakeTensor:
    """What ``_plan_march`` reads of a tensor: pointer, shape, dtype, contiguity."""
    is_cuda = True

    def __init__(self, shape, dtype, ptr):
        self.shape, self.dtype, self._ptr = tuple(shape), dtype, ptr

    def data_ptr(self):
        return self._ptr

    def is_contiguous(self):
        return True

    def stride(self):
        st, acc = [], 1
        for s in reversed(self.shape):
            st.append(acc)
            acc *= s
        return tuple(reversed(st))

    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


CASES = [
    ('diffusion7', W.diffusion_7pt, [(1024,) * 3, (512,) * 3, (768,) * 3, (128, 1024, 1024), (255,) * 3, (64, 300, 261)]),
    ('diffusion7_f16', lambda: W.diffusion_7pt(dtype='float16'), [(768,) * 3, (511,) * 3, (510,) * 3, (512, 512, 520)]),
    ('stencil27', W.stencil_27pt, [(768,) * 3, (1024,) * 3, (512,) * 3, (96, 768, 768), (511,) * 3, (510,) * 3,
                                   (255,) * 3, (512, 512, 1000), (512, 512, 320)]),
    ('laplace5', W.laplace_5pt, [(4096, 4096), (4097, 4097)]),
    ('asym7', W.asym_7pt, [(256,) * 3]),
    ('varcoef', W.varcoef_diffusion_7pt, [(768,) * 3, (512,) * 3]),
    ('varcoef_f16', lambda: W.varcoef_diffusion_7pt(dtype='float16'), [(768,) * 3]),
    ('veclap', W.vector_laplace_7pt, [(384,) * 3]),
]


def snapshot():
    HK.HipStencilKernel.function = lambda self, variant, device: None
    HK.HipStencilKernel._resident_slots = lambda self, fn, block, device: None
    out = []
    for name, builder, shapes in CASES:
        for bh in ('zeros', None):
            op = AutoDiffOp(builder(), boundary_handling=bh)
            for which, asg in (('fwd', op.forward_assignments), ('bwd', op.backward_assignments)):
                hk = HK.HipStencilKernel(StencilKernel(asg, boundary_handling=bh, function_name=f'{name}_{which}',
                                                       target='gpu'))
                if hk.schedule() != 'march':
                    out.append(f'{name} {bh} {which} {hk.schedule()}')
                    continue
                for shape in shapes:
                    for align in (256, 4):
                        ts = []
                        for f in hk.ir.fields:
                            dt = getattr(torch, f.dtype.numpy_dtype.name)
                            ts.append(FakeTensor(shape + tuple(f.index_shape), dt, (1 << 32) + align))
                        try:
                            plan = hk._plan_march(ts, [], shape, 0, None)
                        except Exception as exc:  # noqa: BLE001
                            out.append(f'{name} {bh} {which} {shape} a{align} ERROR {type(exc).__name__}: {exc}')
                            continue
                        src, kname = hk.source(plan.variant)
                        out.append(f'{name} {bh} {which} {shape} a{align} {kname} '
                                   f'{hashlib.sha256(src.encode()).hexdigest()[:16]}')
    return out


if __name__ == '__main__':
    print('\n'.join(snapshot()))
