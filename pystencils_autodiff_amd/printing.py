"""``show_code`` / ``get_code_str`` (reference ``framework_integration/printer.py:200-201``)."""

__all__ = ['show_code', 'get_code_str']


def get_code_str(obj):
    """Source of a kernel, a kernel pair module or an autograd op class."""
    if hasattr(obj, 'code'):
        return obj.code
    return str(obj)


def show_code(obj, custom_backend=None):
    code = get_code_str(obj)
    try:
        from IPython.display import Code, display  # noqa: F401
        display(Code(code, language='c++'))
    except Exception:  # noqa: BLE001 - not in a notebook
        print(code)
