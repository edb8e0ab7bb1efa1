"""ctypes binding of ``libpsad_hip.so`` (``include/psad.h``) and the code-object cache.

Replaces the reference's JIT build layer (``backends/astnodes.py:148-182``:
write ``<md5>.cu`` into pystencils' object cache and
``torch.utils.cpp_extension.load`` it, 10-60 s cold). Here an emitted HIP
translation unit is compiled by hiprtc for gfx950 (about a second), the code
object is cached on disk keyed by ``sha256(source, options, hiprtc version)``
and in memory per device, and kernels are launched with a packed argument
buffer on the caller's HIP stream.

The library is built in-tree (``python -m pystencils_autodiff_amd.build``);
if it is missing every GPU entry point raises — there is no CPU fallback on
the GPU path.
"""
import ctypes
import hashlib
import os
import struct
import tempfile
import threading

__all__ = ['lib', 'library_path', 'compile_hip', 'load_function', 'launch', 'HipError', 'ARCH',
           'DEFAULT_OPTIONS', 'pack_args', 'cache_dir']

ARCH = os.environ.get('PSAD_ARCH', 'gfx950')
DEFAULT_OPTIONS = (f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-Wno-unused-variable')

_HERE = os.path.dirname(os.path.abspath(__file__))
library_path = os.path.join(os.path.dirname(_HERE), 'libpsad_hip.so')

_lib = None
_lock = threading.Lock()


class HipError(RuntimeError):
    pass


def lib():
    """The loaded C-ABI library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(library_path):
            raise HipError(f"{library_path} is missing: build the MI355X extension with "
                           "`python -m pystencils_autodiff_amd.build` (no CPU fallback exists for the GPU path)")
        # Calls keep the GIL (PyDLL): launches and stream-ordered enqueues return in microseconds, and
        # dropping the GIL around each one (ctypes.CDLL) hands it to torch's autograd device thread and
        # back — 2-D 4096² apply+backward 115 -> 52 us per step with the default multithreaded engine
        # (scripts/probes/autograd_handoff.py, profiles/r02_autograd_handoff.log). The calls that can
        # run for milliseconds (hiprtc compile, code-object load) go through a CDLL handle and release it.
        L = ctypes.PyDLL(library_path)
        C = ctypes.CDLL(library_path)
        L.psad_rtc_compile = C.psad_rtc_compile
        L.psad_module_load = C.psad_module_load
        L.psad_rccl_open = C.psad_rccl_open               # and the collective RCCL setup calls
        L.psad_rccl_unique_id = C.psad_rccl_unique_id
        L.psad_rccl_comm_init = C.psad_rccl_comm_init
        L.psad_rccl_comm_destroy = C.psad_rccl_comm_destroy
        c_int, c_size, vp, cp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
        L.psad_abi_version.restype = c_int
        L.psad_rtc_version.restype = c_int
        L.psad_rtc_compile.argtypes = [cp, cp, ctypes.POINTER(cp), c_int, ctypes.POINTER(vp),
                                       ctypes.POINTER(c_size), cp, c_size]
        L.psad_rtc_compile.restype = c_int
        L.psad_free.argtypes = [vp]
        L.psad_free.restype = None
        L.psad_module_load.argtypes = [vp, c_size, ctypes.POINTER(vp)]
        L.psad_module_load.restype = c_int
        L.psad_module_unload.argtypes = [vp]
        L.psad_module_unload.restype = c_int
        L.psad_module_get_function.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.psad_module_get_function.restype = c_int
        L.psad_launch.argtypes = [vp, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                  ctypes.c_uint, ctypes.c_uint, vp, vp, c_size]
        L.psad_launch.restype = c_int
        L.psad_function_attributes.argtypes = [vp, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                               ctypes.POINTER(c_int)]
        L.psad_function_attributes.restype = c_int
        L.psad_get_device.argtypes = [ctypes.POINTER(c_int)]
        L.psad_get_device.restype = c_int
        L.psad_device_count.argtypes = [ctypes.POINTER(c_int)]
        L.psad_device_count.restype = c_int
        L.psad_last_error.restype = c_int
        L.psad_memcpy_d2d_async.argtypes = [vp, vp, c_size, vp]
        L.psad_memcpy_d2d_async.restype = c_int
        L.psad_error_string.argtypes = [c_int]
        L.psad_error_string.restype = cp
        L.psad_rccl_open.argtypes = [cp]
        L.psad_rccl_open.restype = c_int
        L.psad_rccl_unique_id.argtypes = [vp]
        L.psad_rccl_unique_id.restype = c_int
        L.psad_rccl_comm_init.argtypes = [vp, c_int, c_int, ctypes.POINTER(vp)]
        L.psad_rccl_comm_init.restype = c_int
        L.psad_rccl_comm_destroy.argtypes = [vp]
        L.psad_rccl_comm_destroy.restype = c_int
        L.psad_halo_exchange.argtypes = [vp, c_int, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                         ctypes.POINTER(vp), ctypes.POINTER(c_size), c_int, c_int, vp]
        L.psad_halo_exchange.restype = c_int
        L.psad_rccl_error_string.argtypes = [c_int]
        L.psad_rccl_error_string.restype = cp
        if L.psad_abi_version() != 3:
            raise HipError(f'{library_path}: ABI version {L.psad_abi_version()}, this tree needs 3 (a stale build): '
                           'rebuild with `python -m pystencils_autodiff_amd.build`')
        L.psad_source_hash.restype = cp
        _check_stamp(L.psad_source_hash().decode(), 'lib', library_path)
        _lib = L
        return _lib


def _check_stamp(stamp, which, path):
    """Refuse a native library not built from the sources of this tree (``build.source_hash``): a stale ``.so``
    shipped next to changed sources would otherwise run silently. Skipped when the sources are not present."""
    from .. import build
    srcs = build.lib_sources() if which == 'lib' else build.torch_sources()
    if not all(os.path.exists(p) for p in srcs) or os.environ.get('PSAD_SKIP_STAMP') == '1':
        return
    want = build.source_hash(srcs)
    if stamp != want:
        raise HipError(f'{path} was built from other sources (stamp {stamp}, sources {want}): rebuild with '
                       '`python -m pystencils_autodiff_amd.build`')


def _check(code, what):
    if code != 0:
        msg = lib().psad_error_string(code)
        raise HipError(f"{what} failed: {msg.decode() if msg else code} (code {code})")


def cache_dir():
    d = os.environ.get('PSAD_CACHE_DIR')
    if not d:
        base = os.environ.get('XDG_CACHE_HOME') or os.path.join(os.path.expanduser('~'), '.cache')
        d = os.path.join(base, 'pystencils_autodiff_amd')
    try:
        os.makedirs(d, exist_ok=True)
        probe = os.path.join(d, '.w')
        with open(probe, 'w'):
            pass
        os.remove(probe)
    except OSError:
        d = os.path.join(tempfile.gettempdir(), f'pystencils_autodiff_amd_{os.getuid()}')
        os.makedirs(d, exist_ok=True)
    return d


_code_cache = {}


def compile_hip(source, options=DEFAULT_OPTIONS, name='psad.hip'):
    """hiprtc-compile ``source``; returns the code object bytes (disk + memory cached)."""
    L = lib()
    options = tuple(options)
    key = hashlib.sha256((source + '\0' + '\0'.join(options) + f"\0rtc{L.psad_rtc_version()}").encode()).hexdigest()
    if key in _code_cache:
        return _code_cache[key]
    path = os.path.join(cache_dir(), f"{key}.co")
    if os.path.exists(path):
        with open(path, 'rb') as fh:
            code = fh.read()
        if code:
            _code_cache[key] = code
            return code
    opts = (ctypes.c_char_p * len(options))(*[o.encode() for o in options])
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    log = ctypes.create_string_buffer(1 << 16)
    rc = L.psad_rtc_compile(source.encode(), name.encode(), opts, len(options), ctypes.byref(out),
                            ctypes.byref(size), log, len(log))
    if rc != 0:
        msg = L.psad_error_string(rc)
        raise HipError(f"hiprtc compilation failed ({msg.decode() if msg else rc}):\n{log.value.decode(errors='replace')}"
                       f"\n--- source ---\n{source}")
    try:
        code = ctypes.string_at(out, size.value)
    finally:
        L.psad_free(out)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, 'wb') as fh:
        fh.write(code)
    os.replace(tmp, path)
    _code_cache[key] = code
    return code


_modules = {}


def load_function(code, kernel_name, device):
    """hipFunction_t (as int) of ``kernel_name`` in ``code`` loaded on ``device`` (cached)."""
    key = (hashlib.sha256(code).hexdigest(), device)
    mod = _modules.get(key)
    L = lib()
    if mod is None:
        handle = ctypes.c_void_p()
        _check(L.psad_module_load(code, len(code), ctypes.byref(handle)), 'hipModuleLoadData')
        mod = {'module': handle.value, 'functions': {}}
        _modules[key] = mod
    fn = mod['functions'].get(kernel_name)
    if fn is None:
        h = ctypes.c_void_p()
        _check(L.psad_module_get_function(mod['module'], kernel_name.encode(), ctypes.byref(h)),
               f"hipModuleGetFunction({kernel_name})")
        fn = h.value
        mod['functions'][kernel_name] = fn
    return fn


def function_attributes(fn):
    regs, lds, thr = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().psad_function_attributes(fn, ctypes.byref(regs), ctypes.byref(lds), ctypes.byref(thr)),
           'hipFuncGetAttribute')
    return {'num_regs': regs.value, 'shared_bytes': lds.value, 'max_threads': thr.value}


_FMT = {'ptr': ('Q', 8), 'i32': ('i', 4), 'i64': ('q', 8), 'f32': ('f', 4), 'f64': ('d', 8)}


def pack_args(args):
    """Pack ``[(kind, value), ...]`` at natural alignment (HIP_LAUNCH_PARAM_BUFFER layout)."""
    buf = bytearray()
    for kind, value in args:
        fmt, size = _FMT[kind]
        pad = (-len(buf)) % size
        buf += b'\0' * pad
        buf += struct.pack('<' + fmt, value if kind != 'ptr' else (value or 0))
    buf += b'\0' * ((-len(buf)) % 8)
    return bytes(buf)


def launch(fn, grid, block, args_packed, stream, shared_bytes=0):
    gx, gy, gz = (tuple(grid) + (1, 1))[:3]
    bx, by, bz = (tuple(block) + (1, 1))[:3]
    _check(lib().psad_launch(fn, gx, gy, gz, bx, by, bz, shared_bytes, stream, args_packed, len(args_packed)),
           'hipModuleLaunchKernel')
