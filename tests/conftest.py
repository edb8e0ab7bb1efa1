import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu on the GPU box)')
    config.addinivalue_line('markers', 'slow: long-running')


def golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture
def load_golden():
    return golden


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


def assert_close_rel(actual, expected, rtol, what=''):
    """|actual - expected| <= rtol * max|expected| (SURVEY.md §7 tolerance form)."""
    actual = np.asarray(actual, dtype=np.float64)
    expected = np.asarray(expected, dtype=np.float64)
    assert actual.shape == expected.shape, f"{what}: shape {actual.shape} != {expected.shape}"
    scale = max(float(np.max(np.abs(expected))) if expected.size else 0.0, 1e-30)
    err = float(np.max(np.abs(actual - expected))) if expected.size else 0.0
    assert err <= rtol * scale, f"{what}: max abs err {err:.3e} > {rtol:.1e} * {scale:.3e}"
