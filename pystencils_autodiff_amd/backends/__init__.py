"""Framework backends for ``AutoDiffOp`` (reference ``backends/__init__.py:9``).

The names are kept so ``create_tensorflow_op(backend=...)`` validates the same
way; only ``'torch_native'`` is implemented by the MI355X execution layer
(HIP kernels via hiprtc on ``use_cuda=True``, C kernels on ``use_cuda=False``).
"""

AVAILABLE_BACKENDS = ['tensorflow', 'torch', 'tensorflow_native', 'torch_native']
