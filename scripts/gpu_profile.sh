#!/bin/bash
# Profiles for a round: all-config measurements, rocprofv3 kernel trace + stats of bench.py, and the
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, no tracing domains mixed in), then bench.py itself.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r01}"
fatal() { echo "[$2] rc=$1" | tee -a "$OUT/status_$TAG.log"; if [ "$1" -ge 2 ]; then exit "$1"; fi; }
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 500 python scripts/bench_configs.py > "$OUT/configs_$TAG.jsonl" 2> "$OUT/configs_$TAG.err"; fatal $? configs
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace -- \
    python "$ROOT/bench.py" --steps 30 --warmup 2 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1; fatal $? trace
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1; fatal $? pmc_fetch
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1; fatal $? pmc_write
cd "$ROOT"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; fatal $? bench
cat "$OUT/configs_$TAG.jsonl" "$OUT/bench_$TAG.json"
