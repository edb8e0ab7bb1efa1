"""Adjoint fields: the gradient storage that mirrors a forward field.

Follows ``_adjoint_field.py:9-30`` of the reference: an adjoint field is named
``<prefix><name>`` (``diffx`` for ``x``), has the forward field's dtype,
shape and strides, is a BUFFER field iff the forward field is, rebinds
symbolic shape/stride symbols to its own name (so a backward kernel does not
need the forward tensor just for its extents), and prints as ``\\hat{x}``.
"""
from .ps.field import Field, FieldShapeSymbol, FieldStrideSymbol, FieldType

ADJOINT_FIELD_LATEX_HIGHLIGHT = r"\hat{%s}"

__all__ = ['AdjointField', 'ADJOINT_FIELD_LATEX_HIGHLIGHT']


class AdjointField(Field):
    """Field holding the adjoint (gradient) of ``forward_field``."""

    def __init__(self, forward_field, name_prefix='diff'):
        name = name_prefix + forward_field.name
        ftype = FieldType.BUFFER if forward_field.field_type == FieldType.BUFFER else FieldType.GENERIC
        shape = tuple(FieldShapeSymbol([name], s.coordinate) if isinstance(s, FieldShapeSymbol) else s
                      for s in forward_field.shape)
        strides = tuple(FieldStrideSymbol(name, s.coordinate) if isinstance(s, FieldStrideSymbol) else s
                        for s in forward_field.strides)
        super().__init__(name, ftype, forward_field.dtype, forward_field.layout, shape, strides)
        self._index_dimensions = forward_field.index_dimensions
        self._soa = forward_field.is_soa
        self.corresponding_forward_field = forward_field
        self.name_prefix = name_prefix
        self.latex_name = ADJOINT_FIELD_LATEX_HIGHLIGHT % (forward_field.latex_name or forward_field.name)
