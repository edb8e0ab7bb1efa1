#!/bin/bash
# fp16 half-precision-ring A/B: parity subset on the GPU, then interleaved timing vs the current default.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "ws_loader or zsum_schedule or interior_tiles or golden or 27" > gpurun_out/half_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/half_pytest.log; [ $rc -eq 0 ] || exit $rc
C="${C:-default}" TAG="${TAG:-half}" bash scripts/ab27_once.sh
