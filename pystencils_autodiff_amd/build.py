"""Build the in-tree native libraries (``python -m pystencils_autodiff_amd.build``).

* ``libpsad_hip.so`` — the C ABI (``include/psad.h``). ``hipcc --offload-arch=gfx950`` is not needed for
  the shim itself (it holds no device code — kernels are emitted at run time and compiled by hiprtc); it
  is compiled with hipcc so the HIP runtime / hiprtc headers and libraries resolve.
* ``_psad_torch.so`` — the op's native autograd node (``csrc/psad_torch.cpp``), a torch extension module
  compiled with g++ against torch's headers and linked to ``libpsad_hip.so`` (host code only).
"""
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, 'csrc', f) for f in ('psad_hip.cpp', 'psad_halo.cpp')]
OUT = os.path.join(HERE, 'libpsad_hip.so')
TORCH_SRC = os.path.join(HERE, 'csrc', 'psad_torch.cpp')
TORCH_OUT = os.path.join(HERE, '_psad_torch.so')
HEADER = os.path.join(ROOT, 'include', 'psad.h')


def source_hash(paths):
    """First 16 hex digits of sha256 over the files' contents (sorted by name): the stamp each library embeds
    (``PSAD_SOURCE_HASH``) so a loaded library can be checked against the sources of the tree it runs from."""
    h = hashlib.sha256()
    for p in sorted(paths, key=os.path.basename):
        with open(p, 'rb') as fh:
            h.update(os.path.basename(p).encode() + b'\0' + fh.read() + b'\0')
    return h.hexdigest()[:16]


def lib_sources():
    return SRCS + [HEADER]


def torch_sources():
    return [TORCH_SRC, HEADER]


def embedded_hash(path):
    """The ``PSAD_SOURCE_HASH=`` stamp inside a built library (read from its bytes, nothing loaded), or None."""
    try:
        with open(path, 'rb') as fh:
            m = re.search(rb'PSAD_SOURCE_HASH=([0-9a-f]{16})', fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def stale(path, sources):
    """True if ``path`` is missing or was not built from exactly these sources."""
    return embedded_hash(path) != source_hash(sources)


def build(force=False, verbose=False):
    if not force and not stale(OUT, lib_sources()):
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc, '-O2', '-fPIC', '-shared', '-std=c++17', f"-I{os.path.join(ROOT, 'include')}",
           f'-DPSAD_SOURCE_HASH="{source_hash(lib_sources())}"', '-o', OUT + '.tmp', *SRCS, '-lhiprtc', '-ldl']
    if verbose:
        print(' '.join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"building libpsad_hip.so failed:\n{proc.stdout}\n{proc.stderr}")
    os.replace(OUT + '.tmp', OUT)
    return OUT


def build_torch_ext(force=False, verbose=False):
    """``_psad_torch.so``: g++ (no device code) with torch's include / library paths."""
    if not force and not stale(TORCH_OUT, torch_sources()) and os.path.getmtime(TORCH_OUT) >= os.path.getmtime(OUT):
        return TORCH_OUT
    import sysconfig

    import torch
    from torch.utils import cpp_extension
    cxx = os.environ.get('CXX', 'g++')
    tlib = cpp_extension.library_paths()[0]
    cmd = [cxx, '-O2', '-fPIC', '-shared', '-std=c++17', '-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1',
           '-DTORCH_EXTENSION_NAME=_psad_torch', f'-DPSAD_SOURCE_HASH="{source_hash(torch_sources())}"',
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           *[f'-I{p}' for p in cpp_extension.include_paths()], f"-I{sysconfig.get_paths()['include']}",
           '-I/opt/rocm/include', f"-I{os.path.join(ROOT, 'include')}", TORCH_SRC, '-o', TORCH_OUT + '.tmp',
           f'-L{tlib}', '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_python', '-l:libamdhip64.so', f'-L{HERE}', '-lpsad_hip',
           f'-Wl,-rpath,$ORIGIN:{tlib}']
    if verbose:
        print(' '.join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"building _psad_torch.so failed:\n{proc.stdout}\n{proc.stderr}")
    os.replace(TORCH_OUT + '.tmp', TORCH_OUT)
    return TORCH_OUT


def build_all(force=False, verbose=False):
    return build(force, verbose), build_torch_ext(force, verbose)


if __name__ == '__main__':
    print(build_all(force='--force' in sys.argv, verbose=True))
