"""Forced LBM rules through the timestep op: the lattice kernels (constant force terms compiled in, or a per-cell force
field read per cell with its adjoint accumulated) vs the rule's own AutoDiffOp kernels (PSAD_LBM_LATTICE=0), same
process. python scripts/probes/lbm_force_ab.py [field]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from bench_configs import run_lbm  # noqa: E402

field = 'field' in sys.argv[1:]
for stencil, shape, comp, model in (('D2Q9', (2048, 2048), False, 'simple'), ('D2Q9', (2048, 2048), True, 'guo'),
                                     ('D3Q19', (192, 192, 192), False, 'guo')):
    for sched in ('lattice', 'autodiffop'):
        os.environ['PSAD_LBM_LATTICE'] = '1' if sched == 'lattice' else '0'
        run_lbm(f'lbm_{stencil}_{model}{"_field" if field else ""}_{sched}', stencil, shape, torch.float32,
                compressible=comp, force_model=model, force_field=field)
