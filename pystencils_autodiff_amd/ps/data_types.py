"""Scalar element types of fields.

Restates the small part of pystencils' type system the autodiff path touches
([ext] pystencils ``data_types.create_type`` / ``BasicType``): a field dtype
has a ``numpy_dtype`` (used by the torch op to allocate outputs,
reference ``backends/_pytorch.py:95-97``) and a C spelling (used by the
kernel emitters).
"""
import numpy as np

_ALIASES = {
    'double': 'float64', 'float64': 'float64', 'f8': 'float64',
    'float': 'float32', 'float32': 'float32', 'f4': 'float32',
    'half': 'float16', 'float16': 'float16', 'f2': 'float16',
    'int': 'int32', 'int32': 'int32', 'int64': 'int64',
}

_C_NAMES = {
    'float64': 'double', 'float32': 'float', 'float16': '_Float16',
    'int32': 'int', 'int64': 'long long',
}


class BasicType:
    """An element type, e.g. ``BasicType('float32')``."""

    def __init__(self, name):
        if isinstance(name, BasicType):
            name = name.numpy_dtype.name
        if isinstance(name, np.dtype) or (isinstance(name, type) and issubclass(name, np.generic)):
            name = np.dtype(name).name
        name = str(name).strip()
        if name.startswith('torch.'):
            name = name[len('torch.'):]
        if name not in _ALIASES:
            raise ValueError(f"unsupported field data type '{name}'")
        self._name = _ALIASES[name]
        self.numpy_dtype = np.dtype(self._name)

    @property
    def base_type(self):
        return self

    @property
    def c_name(self):
        return _C_NAMES[self._name]

    @property
    def is_float(self):
        return self.numpy_dtype.kind == 'f'

    @property
    def itemsize(self):
        return self.numpy_dtype.itemsize

    def __eq__(self, other):
        return isinstance(other, BasicType) and other._name == self._name

    def __hash__(self):
        return hash(('BasicType', self._name))

    def __str__(self):
        return self.c_name

    def __repr__(self):
        return self._name


def create_type(spec):
    return spec if isinstance(spec, BasicType) else BasicType(spec)
