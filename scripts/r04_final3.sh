set -u
# round 4, final tree (round end: + lattice force terms, per-cell forces, BMBR tests): the whole GPU suite, every config, the bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04h_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r04h_pytest_gpu.log
if [ $rc -ne 0 ]; then grep -B2 -A15 "^E " gpurun_out/r04h_pytest_gpu.log | head -60; exit $rc; fi
timeout -k 10 300 python -u scripts/bench_configs.py > gpurun_out/r04h_configs.jsonl 2> gpurun_out/r04h_configs.err || { tail -20 gpurun_out/r04h_configs.err; exit 1; }
timeout -k 10 200 python bench.py > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err || { tail -20 gpurun_out/r04h_bench.err; exit 1; }
cut -c1-220 gpurun_out/r04h_configs.jsonl
cut -c1-400 gpurun_out/r04h_bench.json
