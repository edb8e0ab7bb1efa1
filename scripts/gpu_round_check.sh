#!/bin/bash
# Full GPU check of the tree: smoke, GPU suite, all-config op measurements, bench line + kernel stats.
# Every GPU step has its own time limit; the script stops at the first fault / abort / timeout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r02}"
fatal() { echo "[$2] rc=$1" | tee -a "$OUT/status_$TAG.log"; if [ "$1" -ge 2 ] && [ "$1" -ne 5 ]; then exit "$1"; fi; }
python -m pystencils_autodiff_amd.build > "$OUT/build_$TAG.log" 2>&1 || exit 3
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke_$TAG.log" 2>&1; fatal $? smoke
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu_$TAG.log"; fatal $rc pytest_gpu
timeout -k 10 500 python scripts/bench_configs.py > "$OUT/configs_$TAG.jsonl" 2> "$OUT/configs_$TAG.err"; fatal $? configs
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; fatal $? bench
cat "$OUT/configs_$TAG.jsonl" "$OUT/bench_$TAG.json"
