set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 500 python scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err; rc=$?
cat gpurun_out/configs.jsonl; tail -3 gpurun_out/configs.err; exit $rc
