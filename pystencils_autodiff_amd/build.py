"""Build the in-tree native library ``libpsad_hip.so`` (``python -m pystencils_autodiff_amd.build``).

``hipcc --offload-arch=gfx950`` is not needed for the shim itself (it holds no
device code — kernels are emitted at run time and compiled by hiprtc); it is
compiled with hipcc so the HIP runtime / hiprtc headers and libraries resolve.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, 'csrc', f) for f in ('psad_hip.cpp', 'psad_halo.cpp')]
OUT = os.path.join(HERE, 'libpsad_hip.so')


def build(force=False, verbose=False):
    deps = SRCS + [os.path.join(ROOT, 'include', 'psad.h')]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc, '-O2', '-fPIC', '-shared', '-std=c++17', f"-I{os.path.join(ROOT, 'include')}",
           '-o', OUT + '.tmp', *SRCS, '-lhiprtc', '-ldl']
    if verbose:
        print(' '.join(cmd))
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"building libpsad_hip.so failed:\n{proc.stdout}\n{proc.stderr}")
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
