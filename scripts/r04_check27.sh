set -u
# round 4: constant-force LBM on the lattice kernels — GPU tests, then lattice vs AutoDiffOp kernels
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 400 python -u -m pytest tests/test_lbm.py -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r04_lbm_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04_lbm_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04_lbm_gpu_tests.log
timeout -k 10 300 python -u scripts/probes/lbm_force_ab.py > gpurun_out/r04_lbm_force_ab.jsonl 2> gpurun_out/r04_lbm_force_ab.err || { tail -20 gpurun_out/r04_lbm_force_ab.err; exit 1; }
cut -c1-260 gpurun_out/r04_lbm_force_ab.jsonl
