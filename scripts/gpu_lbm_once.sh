#!/bin/bash
# LBM GPU tests + LBM bench lines, then the rest of the GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 400 python -u -m pytest tests/test_lbm.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    > gpurun_out/lbm_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/lbm_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_configs.py lbm_d2q9_f32_2048^2 lbm_d3q19_f32_192^3 > gpurun_out/lbm_configs.jsonl 2> gpurun_out/lbm_configs.err
rc=$?; cat gpurun_out/lbm_configs.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/lbm_configs.err; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu_lbm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_lbm.log; exit $rc
