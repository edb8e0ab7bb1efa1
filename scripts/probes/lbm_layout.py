"""LBM timestep op in the two pdf layouts lbmpy offers: 'fzyx' (SoA, one plane per component, the default)
and 'numpy' / zyxf (AoS, a cell's q values contiguous), D3Q19 192^3 and D2Q9 2048^2 fp32, 10 steps, same
process (scripts/bench_configs.run_lbm with the layout swapped in)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts'))
import torch  # noqa: E402

import bench_configs as B  # noqa: E402
from pystencils_autodiff_amd import lbm  # noqa: E402

orig = lbm.create_lb_update_rule


def main():
    for layout in ('fzyx', 'numpy', 'fzyx', 'numpy'):
        lbm.create_lb_update_rule = lambda *a, **k: orig(*a, **{**k, 'layout': layout})
        print(f'# layout {layout}', flush=True)
        B.run_lbm(f'lbm_d3q19_f32_192^3_{layout}', 'D3Q19', (192, 192, 192), torch.float32)
        B.run_lbm(f'lbm_d2q9_f32_2048^2_{layout}', 'D2Q9', (2048, 2048), torch.float32)


if __name__ == '__main__':
    main()
