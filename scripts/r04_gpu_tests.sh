set -u
# round 4: the whole GPU test suite, then one default bench.py line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r04_pytest_gpu.log
if [ $rc -ne 0 ]; then grep -B2 -A15 "^E " gpurun_out/r04_pytest_gpu.log | head -80; exit $rc; fi
timeout -k 10 150 python bench.py > gpurun_out/r04_bench_a.json 2> gpurun_out/r04_bench_a.err || { tail -20 gpurun_out/r04_bench_a.err; exit 1; }
cat gpurun_out/r04_bench_a.json
