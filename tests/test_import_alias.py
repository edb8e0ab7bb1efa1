"""The reference's import names (``pystencils_autodiff``, ``pystencils.autodiff``) resolve to this layer.

Runs the README example (reference ``README.rst:52-100``) with the reference's own imports; pystencils is not
installed here, so ``import pystencils`` binds this layer's symbolic front-end (``pystencils_autodiff_amd.ps``) after
``import pystencils_autodiff`` (see ``pystencils_autodiff/__init__.py``). Each test runs in a fresh interpreter so
the module aliases are observed from a clean ``sys.modules``."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))

README = '''
import pystencils_autodiff          # the reference's package name
import sympy
import pystencils

z, y, x = pystencils.fields("z, y, x: [20,30]")
forward_assignments = pystencils.AssignmentCollection({
    z[0, 0]: x[0, 0] * sympy.log(x[0, 0] * y[0, 0])
})
print(forward_assignments)

from pystencils.autodiff import AutoDiffOp, create_backward_assignments
backward_assignments = create_backward_assignments(forward_assignments)
print(backward_assignments)
rhs = {str(a.lhs): str(a.rhs) for a in backward_assignments.main_assignments}
assert rhs == {r'\\hat{x}[0,0]': 'diffz_C*(log(x_C*y_C) + 1)', r'\\hat{y}[0,0]': 'diffz_C*x_C/y_C'}, rhs

op = AutoDiffOp(forward_assignments)
backward_assignments = op.backward_assignments
torch_op = op.create_tensorflow_op(backend='torch_native', use_cuda=False)

import numpy as np
import torch
xv = torch.rand(20, 30, dtype=torch.float64) + 0.5
yv = torch.rand(20, 30, dtype=torch.float64) + 0.5
xt, yt = xv.clone().requires_grad_(True), yv.clone().requires_grad_(True)
(zt,) = torch_op.apply(xt, yt)
assert torch.allclose(zt, xv * torch.log(xv * yv))
zt.backward(torch.ones_like(zt))
assert torch.allclose(xt.grad, torch.log(xv * yv) + 1) and torch.allclose(yt.grad, xv / yv)
print('README OK')
'''


def _run(src):
    proc = subprocess.run([sys.executable, '-c', textwrap.dedent(src)], cwd=ROOT, capture_output=True, text=True,
                          timeout=300, env=dict(os.environ, PYTHONPATH=ROOT))
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-3000:]
    return proc.stdout


def test_readme_example_with_reference_imports():
    out = _run(README)
    assert 'README OK' in out and 'diffz_C' in out


def test_reference_module_paths():
    out = _run('''
        import pystencils_autodiff
        import pystencils_autodiff_amd as amd
        import pystencils.autodiff
        import pystencils.autodiff.backends
        assert pystencils.autodiff is pystencils_autodiff and pystencils.autodiff.backends is amd.backends
        from pystencils_autodiff._autodiff import AutoDiffOp, DiffModes, create_backward_assignments
        assert AutoDiffOp is amd.AutoDiffOp and DiffModes is amd.DiffModes
        from pystencils_autodiff.backends._torch_native import create_autograd_function
        from pystencils_autodiff._adjoint_field import AdjointField
        from pystencils_autodiff.transformations import add_fixed_constant_boundary_handling
        from pystencils_autodiff.framework_integration.printer import show_code, get_code_str
        from pystencils_autodiff.lbm import AutoDiffLatticeBoltzmannStep
        from pystencils_autodiff.lbm.adjoint_boundaryconditions import AdjointBoundaryCondition, AdjointNoSlip
        from pystencils_autodiff.lbm._autodiff_lbstep import AutoDiffLatticeBoltzmannStep as S2
        assert S2 is AutoDiffLatticeBoltzmannStep
        import pystencils_autodiff.backends as b
        assert b is amd.backends and pystencils_autodiff.backends is amd.backends
        print('paths OK')
    ''')
    assert 'paths OK' in out
