"""The reference's import name, bound to the MI355X layer: ``import pystencils_autodiff`` and
``import pystencils.autodiff`` resolve to ``pystencils_autodiff_amd``.

The reference registers itself as ``pystencils.autodiff`` / ``pystencils.autodiff.backends``
(``src/pystencils_autodiff/__init__.py:26-27``); this package does the same for the module objects of
``pystencils_autodiff_amd`` and maps the reference's submodule paths that have a counterpart here onto it, so user
code written against the reference keeps its imports:

* ``pystencils_autodiff._autodiff`` → ``autodiff`` (``AutoDiffOp``, ``create_backward_assignments``, …),
  ``._adjoint_field``, ``.transformations``, ``.backends`` (+ ``._torch_native``),
  ``.framework_integration.printer`` → ``printing`` (``show_code``, ``get_code_str``),
  ``.lbm`` (+ ``._autodiff_lbstep``, ``.adjoint_boundaryconditions`` → ``lbm.boundaries``).

pystencils itself is an un-vendored dependency of the reference (``setup.cfg:35``). When it is not installed, the
name ``pystencils`` is bound to this layer's restatement of the symbolic front-end the path consumes
(``pystencils_autodiff_amd.ps``: ``fields``, ``Field``, ``Assignment``, ``AssignmentCollection``, ``fd``), so that
``import pystencils.autodiff`` works as in the reference. An installed pystencils is left alone (only its
``autodiff`` attribute is set, as the reference does).
"""
import importlib
import importlib.util
import sys

import pystencils_autodiff_amd as _impl
from pystencils_autodiff_amd import (  # noqa: F401
    AdjointField, AutoDiffAstPair, AutoDiffBoundaryHandling, AutoDiffOp, DiffModes, backends,
    create_backward_assignments, get_jacobian_of_assignments, ps, show_code)

__version__ = _impl.__version__
__all__ = ['backends', 'AdjointField', 'get_jacobian_of_assignments', 'create_backward_assignments', 'AutoDiffOp',
           'AutoDiffAstPair', 'DiffModes', 'AutoDiffBoundaryHandling', 'show_code']

_this = sys.modules[__name__]

# reference submodule path → module of this layer
_ALIASES = {
    '_autodiff': 'pystencils_autodiff_amd.autodiff',
    '_adjoint_field': 'pystencils_autodiff_amd._adjoint_field',
    'transformations': 'pystencils_autodiff_amd.transformations',
    'backends': 'pystencils_autodiff_amd.backends',
    'backends._torch_native': 'pystencils_autodiff_amd.backends._torch_native',
    'framework_integration.printer': 'pystencils_autodiff_amd.printing',
    'lbm': 'pystencils_autodiff_amd.lbm',
    'lbm._autodiff_lbstep': 'pystencils_autodiff_amd.lbm._autodiff_lbstep',
    'lbm.adjoint_boundaryconditions': 'pystencils_autodiff_amd.lbm.boundaries',
}


def _register():
    import types
    for sub, target in _ALIASES.items():
        mod = importlib.import_module(target)
        sys.modules[f'{__name__}.{sub}'] = mod
        parent, _, leaf = sub.rpartition('.')
        if parent:
            pname = f'{__name__}.{parent}'
            if pname not in sys.modules:           # a package path with no module of its own here
                pkg = types.ModuleType(pname)
                pkg.__path__ = []
                sys.modules[pname] = pkg
            setattr(sys.modules[pname], leaf, mod)
        else:
            setattr(_this, sub, mod)
    _this.framework_integration = sys.modules[f'{__name__}.framework_integration']

    # pystencils.autodiff (reference __init__.py:26-27)
    if 'pystencils' in sys.modules:
        pystencils = sys.modules['pystencils']
    elif importlib.util.find_spec('pystencils') is not None:
        pystencils = importlib.import_module('pystencils')
    else:
        pystencils = ps
        sys.modules['pystencils'] = ps
    pystencils.autodiff = _this
    sys.modules['pystencils.autodiff'] = _this
    sys.modules['pystencils.autodiff.backends'] = backends


_register()
