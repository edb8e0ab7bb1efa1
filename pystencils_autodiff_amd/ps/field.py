"""Fields and field accesses — the symbolic objects stencils are written in.

The reference builds on pystencils' ``Field`` / ``Field.Access`` ([ext]
pystencils ``field.py``; used throughout ``_autodiff.py:47-152`` and
``_adjoint_field.py:9-30``). pystencils is not vendored and not installable
here, so this module restates the parts of its contract the autodiff hot path
depends on:

* a ``Field.Access`` is a SymPy ``Symbol`` named ``<field>_<direction>``
  (``x_C``, ``a_E``, ``u_TN`` ...) so that ``sympy.diff(rhs, access)`` works and
  printed expressions match the reference's known-answer strings
  (``tests/test_autodiff.py:21``, ``docs/index.rst:77-78``);
* ``str(access)`` is the bracket form ``x[0,0]`` (with the field's LaTeX name,
  e.g. ``\\hat{x}[0,0]`` for adjoint fields);
* spatial coordinate 0 is the first (slowest, C-layout) array axis;
* vector fields come in pystencils' two memory layouts: ``'numpy'``/``'zyxf'``
  (AoS, components fastest) and ``'fzyx'``/``'soa'`` (SoA, one C-ordered
  spatial array per component, components slowest); for scalar fields both
  are the same memory (pystencils ``layout_string_to_tuple`` [ext]);
* fields are compared by value (name, dtype, shape, strides, memory layout).
"""
import re
from enum import Enum
from typing import Sequence

import numpy as np
import sympy as sp

from .data_types import BasicType, create_type

__all__ = ['Field', 'FieldType', 'fields', 'offset_to_direction_string',
           'direction_string_to_offset', 'FieldShapeSymbol', 'FieldStrideSymbol']


class FieldType(Enum):
    GENERIC = 0
    INDEXED = 1
    BUFFER = 2
    CUSTOM = 3


_DIR_NAMES = (('E', 'W'), ('N', 'S'), ('T', 'B'))


def offset_to_direction_string(offsets: Sequence[int]) -> str:
    """``(1, -1, 0)`` -> ``'SE'``, ``(0, 0, -3)`` -> ``'3B'``, zeros -> ``'C'``.

    Highest coordinate first, coordinate 0 labelled E/W, 1 N/S, 2 T/B
    (pystencils ``stencil.offset_to_direction_string`` [ext]).
    """
    if len(offsets) > 3:
        return str(tuple(offsets))
    res = ''
    for d in reversed(range(len(offsets))):
        o = offsets[d]
        if not isinstance(o, (int, np.integer)) and not (isinstance(o, sp.Integer)):
            return str(tuple(offsets))
        o = int(o)
        if o == 0:
            continue
        if abs(o) > 1:
            res += str(abs(o))
        res += _DIR_NAMES[d][0 if o > 0 else 1]
    return res or 'C'


def direction_string_to_offset(direction: str, dim: int = 3):
    offset = [0] * 3
    num = ''
    for ch in direction.upper():
        if ch.isdigit():
            num += ch
            continue
        if ch == 'C':
            continue
        for d, (pos, neg) in enumerate(_DIR_NAMES):
            if ch in (pos, neg):
                step = int(num) if num else 1
                offset[d] += step if ch == pos else -step
                break
        else:
            raise ValueError(f"invalid direction string '{direction}'")
        num = ''
    return tuple(offset[:dim])


class FieldShapeSymbol(sp.Symbol):
    """Symbolic extent of a variable-size field (printed ``_size_<name>_<d>``)."""

    def __new__(cls, field_names, coordinate):
        names = tuple(field_names) if not isinstance(field_names, str) else (field_names,)
        obj = sp.Symbol.__xnew__(cls, f"_size_{'_'.join(names)}_{coordinate}", integer=True, positive=True)
        obj.field_names = names
        obj.coordinate = coordinate
        return obj

    def __getnewargs__(self):
        return self.field_names, self.coordinate

    def __getnewargs_ex__(self):
        return (self.field_names, self.coordinate), {}

    def _hashable_content(self):
        return super()._hashable_content() + (self.field_names, self.coordinate)


class FieldStrideSymbol(sp.Symbol):
    """Symbolic element stride of a variable-size field."""

    def __new__(cls, field_name, coordinate):
        obj = sp.Symbol.__xnew__(cls, f"_stride_{field_name}_{coordinate}", integer=True)
        obj.field_name = field_name
        obj.coordinate = coordinate
        return obj

    def __getnewargs__(self):
        return self.field_name, self.coordinate

    def __getnewargs_ex__(self):
        return (self.field_name, self.coordinate), {}

    def _hashable_content(self):
        return super()._hashable_content() + (self.field_name, self.coordinate)


def _soa_strides(shape, index_dimensions):
    """Element strides of an ``fzyx`` (SoA) field: C order over the spatial axes, the component axes
    slowest (each component a whole spatial array)."""
    spatial = len(shape) - index_dimensions
    sp_strides = _c_strides(shape[:spatial])
    vol = 1
    for n in shape[:spatial]:
        vol = vol * n
    idx_strides = tuple(s * vol for s in _c_strides(shape[spatial:]))
    return tuple(sp_strides) + idx_strides


def _c_strides(shape):
    strides = []
    acc = 1
    for s in reversed(shape):
        strides.append(acc)
        acc = acc * s
    return tuple(reversed(strides))


class Field:
    """A named n-dimensional array with ``spatial_dimensions`` stencil axes
    followed by ``index_dimensions`` component axes (C / "numpy" layout)."""

    def __init__(self, field_name, field_type, dtype, layout, shape, strides, latex_name=None):
        self._field_name = field_name
        self.field_type = field_type if isinstance(field_type, FieldType) else FieldType(field_type)
        self._dtype = create_type(dtype)
        self._layout = tuple(layout)
        self.shape = tuple(shape)
        self.strides = tuple(strides)
        self.latex_name = latex_name
        self._index_dimensions = None
        self._soa = False

    # -- construction ---------------------------------------------------------------------------
    @staticmethod
    def create_fixed_size(field_name, shape, index_dimensions=0, dtype=np.float64, layout='numpy',
                          strides=None, field_type=FieldType.GENERIC):
        shape = tuple(int(s) for s in shape)
        spatial = len(shape) - index_dimensions
        soa = _check_layout(layout) == 'fzyx' and index_dimensions > 0
        if strides is None:
            strides = _soa_strides(shape, index_dimensions) if soa else _c_strides(shape)
        f = Field(field_name, field_type, dtype, tuple(range(spatial)), shape, strides)
        f._index_dimensions = index_dimensions
        f._soa = soa
        return f

    @staticmethod
    def create_generic(field_name, spatial_dimensions, dtype=np.float64, index_dimensions=0,
                       layout='numpy', index_shape=None, field_type=FieldType.GENERIC):
        soa = _check_layout(layout) == 'fzyx'
        if index_shape is not None:
            index_dimensions = len(index_shape)
        total = spatial_dimensions + index_dimensions
        shape = [FieldShapeSymbol([field_name], i) for i in range(spatial_dimensions)]
        if index_shape is not None:
            shape += list(index_shape)
        else:
            shape += [FieldShapeSymbol([field_name], i) for i in range(spatial_dimensions, total)]
        strides = [FieldStrideSymbol(field_name, i) for i in range(total)]
        f = Field(field_name, field_type, dtype, tuple(range(spatial_dimensions)), shape, strides)
        f._index_dimensions = index_dimensions
        f._soa = soa and index_dimensions > 0
        return f

    @staticmethod
    def create_from_numpy_array(field_name, array, index_dimensions=0, field_type=FieldType.GENERIC):
        shape = tuple(int(s) for s in array.shape)
        if hasattr(array, 'stride') and callable(array.stride):       # torch tensor: element strides
            strides = tuple(int(s) for s in array.stride())
            dtype = str(array.dtype)
        else:                                                         # numpy: byte strides
            strides = tuple(int(s) // array.itemsize for s in array.strides)
            dtype = array.dtype
        f = Field(field_name, field_type, dtype, tuple(range(len(shape) - index_dimensions)), shape, strides)
        f._index_dimensions = index_dimensions
        # components slowest in memory: an fzyx (SoA) array
        f._soa = index_dimensions > 0 and tuple(strides) == _soa_strides(shape, index_dimensions) and \
            tuple(strides) != _c_strides(shape)
        return f

    def new_field_with_different_name(self, new_name):
        """The same field (type, dtype, layout, shape, strides) under another name (pystencils' method of the same
        name [ext]; symbolic shape / stride symbols are renamed with it)."""
        shape = tuple(FieldShapeSymbol([new_name], s.coordinate) if isinstance(s, FieldShapeSymbol) else s
                      for s in self.shape)
        strides = tuple(FieldStrideSymbol(new_name, s.coordinate) if isinstance(s, FieldStrideSymbol) else s
                        for s in self.strides)
        f = Field(new_name, self.field_type, self.dtype, self._layout, shape, strides)
        f._index_dimensions = self._index_dimensions
        f._soa = self._soa
        return f

    # -- properties -----------------------------------------------------------------------------
    @property
    def name(self):
        return self._field_name

    @property
    def dtype(self):
        return self._dtype

    @property
    def layout(self):
        return self._layout

    @property
    def is_soa(self):
        """A vector field in ``fzyx`` layout (components slowest in memory)."""
        return bool(self._soa) and self.index_dimensions > 0

    @property
    def memory_layout(self):
        """``'fzyx'`` for SoA vector fields, ``'numpy'`` otherwise."""
        return 'fzyx' if self.is_soa else 'numpy'

    def component_field(self, idx):
        """The scalar field holding component ``idx`` of an fzyx (SoA) field: the same spatial shape, C
        strides, named ``<name>__c<i>[_<j>...]`` (the kernels bind it to the component's sub-array)."""
        if not self.is_soa:
            raise ValueError(f"'{self.name}' is not an fzyx vector field")
        idx = tuple(int(i) for i in idx)
        name = f"{self.name}__c{'_'.join(str(i) for i in idx)}"
        sshape = tuple(self.spatial_shape)
        if self.has_fixed_shape:
            strides = _c_strides(tuple(int(n) for n in sshape))
        else:
            strides = tuple(FieldStrideSymbol(name, d) for d in range(len(sshape)))
        f = Field(name, self.field_type, self.dtype, tuple(range(len(sshape))), sshape, strides)
        f._index_dimensions = 0
        f.soa_parent = (self, idx)
        return f

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def index_dimensions(self):
        return self._index_dimensions or 0

    @property
    def spatial_dimensions(self):
        return len(self.shape) - self.index_dimensions

    @property
    def spatial_shape(self):
        return self.shape[:self.spatial_dimensions]

    @property
    def index_shape(self):
        return self.shape[self.spatial_dimensions:]

    @property
    def spatial_strides(self):
        return self.strides[:self.spatial_dimensions]

    @property
    def index_strides(self):
        return self.strides[self.spatial_dimensions:]

    @property
    def has_fixed_shape(self):
        return all(isinstance(s, (int, np.integer)) or (isinstance(s, sp.Integer)) for s in self.shape)

    @property
    def has_fixed_index_shape(self):
        return all(isinstance(s, (int, np.integer)) for s in self.index_shape)

    @property
    def center(self):
        return Field.Access(self, (0,) * self.spatial_dimensions)

    @property
    def center_vector(self):
        if self.index_dimensions == 0:
            return sp.Matrix([self.center])
        if self.index_dimensions == 1:
            return sp.Matrix([self.center(i) for i in range(self.index_shape[0])])
        raise NotImplementedError('center_vector for more than one index dimension')

    def neighbor(self, coord_id, offset):
        offsets = [0] * self.spatial_dimensions
        offsets[coord_id] = offset
        return Field.Access(self, tuple(offsets))

    def absolute_access(self, offset, index):
        return Field.Access(self, tuple(offset), tuple(index), is_absolute_access=True)

    def __getitem__(self, offset):
        if isinstance(offset, np.ndarray):
            offset = tuple(offset)
        if isinstance(offset, str):
            offset = direction_string_to_offset(offset, self.spatial_dimensions)
        if not isinstance(offset, (tuple, list)):
            offset = (offset,)
        if len(offset) != self.spatial_dimensions:
            raise ValueError(f"Wrong number of spatial indices: got {len(offset)}, "
                             f"expected {self.spatial_dimensions}")
        return Field.Access(self, tuple(offset))

    def __call__(self, *args, **kwargs):
        return self.center(*args, **kwargs)

    # -- identity -------------------------------------------------------------------------------
    def _hashable_contents(self):
        return (self._field_name, self._dtype, self.shape, self.strides, self.index_dimensions, self.is_soa)

    def __hash__(self):
        return hash(self._hashable_contents())

    def __eq__(self, other):
        if not isinstance(other, Field):
            return False
        return self._hashable_contents() == other._hashable_contents()

    def __str__(self):
        return self._field_name

    def __repr__(self):
        return self._field_name

    # ------------------------------------------------------------------------------------------
    class Access(sp.Symbol):
        """A read or write of ``field`` at a constant offset from the current cell."""

        _iterable = False   # has __getitem__ (component index) but is an atom for sympy

        def __new__(cls, field, offsets=(0, 0, 0), idx=None, is_absolute_access=False, dtype=None):
            offsets = tuple(int(o) if isinstance(o, (int, np.integer, sp.Integer)) else o for o in offsets)
            if idx is None:
                idx = (0,) * field.index_dimensions
            idx = tuple(int(i) if isinstance(i, (int, np.integer, sp.Integer)) else i for i in idx)
            offset_name = offset_to_direction_string(offsets)
            if field.index_dimensions == 0:
                name = f"{field.name}_{offset_name}"
            else:
                name = f"{field.name}_{offset_name}^" + ','.join(str(i) for i in idx)
            obj = sp.Symbol.__xnew__(cls, name)
            obj._field = field
            obj._offsets = offsets
            obj._offset_name = offset_name
            obj._index = idx
            obj._is_absolute_access = is_absolute_access
            return obj

        def __getnewargs__(self):
            return self._field, self._offsets, self._index, self._is_absolute_access

        def __getnewargs_ex__(self):
            return self.__getnewargs__(), {}

        def _hashable_content(self):
            return super()._hashable_content() + (self._field._hashable_contents(), self._offsets,
                                                  self._index, self._is_absolute_access)

        # pystencils-compatible accessors
        @property
        def field(self):
            return self._field

        @property
        def offsets(self):
            return self._offsets

        @property
        def index(self):
            return self._index

        @property
        def offset_name(self):
            return self._offset_name

        @property
        def dtype(self):
            return self._field.dtype

        @property
        def is_absolute_access(self):
            return self._is_absolute_access

        @property
        def required_ghost_layers(self):
            return int(np.max(np.abs(self._offsets))) if self._offsets else 0

        @property
        def nr_of_coordinates(self):
            return len(self._offsets)

        def neighbor(self, coord_id, offset):
            offsets = list(self._offsets)
            offsets[coord_id] += offset
            return Field.Access(self._field, tuple(offsets), self._index)

        def get_shifted(self, *shift):
            return Field.Access(self._field, tuple(a + b for a, b in zip(self._offsets, shift)), self._index)

        def at_index(self, *idx):
            return Field.Access(self._field, self._offsets, tuple(idx))

        def __call__(self, *idx):
            if self._index != (0,) * self._field.index_dimensions:
                raise ValueError('Indexing an already indexed Field.Access')
            idx = tuple(idx)
            if self._field.index_dimensions == 0 and idx == (0,):
                idx = ()
            if len(idx) != self._field.index_dimensions:
                raise ValueError(f"Wrong number of indices: got {len(idx)}, "
                                 f"expected {self._field.index_dimensions}")
            return Field.Access(self._field, self._offsets, idx)

        def __getitem__(self, *idx):
            if len(idx) == 1 and isinstance(idx[0], tuple):
                idx = idx[0]
            return self.__call__(*idx)

        def __str__(self):
            n = self._field.latex_name if self._field.latex_name else self._field.name
            offset_str = ','.join(str(o) for o in self._offsets)
            if self._field.index_dimensions and self._index:
                offset_str += ',' + ','.join(str(i) for i in self._index)
            return f"{n}[{offset_str}]"

        def _latex(self, _printer):
            n = self._field.latex_name if self._field.latex_name else self._field.name
            return f"{{{n}}}_{{{self._offset_name}}}"


def _check_layout(layout):
    """Normalised memory layout: ``'numpy'`` (C order, components fastest: also ``'c'``, ``'zyxf'``,
    ``'aos'``) or ``'fzyx'`` (components slowest: also ``'soa'``). Fortran-ordered spatial axes
    (``'f'``, ``'reverse_numpy'``) are not handled."""
    if layout is None:
        return 'numpy'
    lay = str(layout).lower()
    if lay in ('numpy', 'c', 'zyxf', 'aos'):
        return 'numpy'
    if lay in ('fzyx', 'soa'):
        return 'fzyx'
    raise NotImplementedError(f"layout '{layout}' is not supported; C-ordered spatial axes with the "
                              "components fastest ('numpy'/'zyxf') or slowest ('fzyx') are")


_NAME_RE = re.compile(r'\s*([A-Za-z_]\w*)\s*(\(([^)]*)\))?\s*$')
_TYPE_RE = re.compile(r'\s*([A-Za-z_]\w*)?\s*(\[(.*)\])?\s*$')


def _split_names(names):
    out, depth, cur = [], 0, ''
    for ch in names:
        if ch == '(':
            depth += 1
        elif ch == ')':
            depth -= 1
        if ch == ',' and depth == 0:
            out.append(cur)
            cur = ''
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _parse_description(description):
    if ':' in description:
        names_part, type_part = description.split(':', 1)
    else:
        names_part, type_part = description, ''
    field_descs = []
    for part in _split_names(names_part):
        m = _NAME_RE.match(part)
        if not m:
            raise ValueError(f"could not parse field name '{part}'")
        idx_shape = tuple(int(i) for i in m.group(3).split(',') if i.strip()) if m.group(3) else ()
        field_descs.append((m.group(1), idx_shape))
    m = _TYPE_RE.match(type_part)
    if not m:
        raise ValueError(f"could not parse field type '{type_part}'")
    dtype = m.group(1) or 'double'
    shape = None
    if m.group(2) is not None:
        content = m.group(3).strip()
        dm = re.fullmatch(r'(\d+)\s*[dD]', content)
        if dm:
            shape = int(dm.group(1))
        else:
            shape = tuple(int(s) for s in content.split(',') if s.strip())
    return field_descs, dtype, shape


def fields(description=None, index_dimensions=0, layout=None, field_type=FieldType.GENERIC, **kwargs):
    """``fields("a, b, out: float64[5,7]")`` / ``fields("x, y: float32[3d]")`` / ``fields(x=array)``."""
    result = []
    if description:
        field_descs, dtype, shape = _parse_description(description)
        for field_name, idx_shape in field_descs:
            if field_name in kwargs:
                f = Field.create_from_numpy_array(field_name, kwargs[field_name],
                                                  index_dimensions=len(idx_shape), field_type=field_type)
            elif isinstance(shape, tuple):
                f = Field.create_fixed_size(field_name, shape + idx_shape, dtype=dtype,
                                            index_dimensions=len(idx_shape), layout=layout or 'numpy',
                                            field_type=field_type)
            elif isinstance(shape, int):
                f = Field.create_generic(field_name, spatial_dimensions=shape, dtype=dtype,
                                         index_shape=idx_shape if idx_shape else None,
                                         layout=layout or 'numpy', field_type=field_type)
            else:
                f = Field.create_generic(field_name, spatial_dimensions=2, dtype=dtype,
                                         index_shape=idx_shape if idx_shape else None,
                                         layout=layout or 'numpy', field_type=field_type)
            result.append(f)
    else:
        for field_name, arr in kwargs.items():
            result.append(Field.create_from_numpy_array(field_name, arr, index_dimensions=index_dimensions,
                                                        field_type=field_type))
    if not result:
        return None
    if len(result) == 1:
        return result[0]
    return result


# ``BasicType`` is re-exported for convenience (``Field.dtype.numpy_dtype``).
__all__.append('BasicType')
