#!/bin/bash
# Round-3 evidence: rocprofv3 kernel trace + stats of bench.py (headline + config 5, kernels named per workload),
# the FETCH_SIZE / WRITE_SIZE passes (separate runs, no trace domains mixed in), bench_configs, bench.py itself.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r03}"
fatal() { echo "[$2] rc=$1" | tee -a "$OUT/status_$TAG.log"; if [ "$1" -ne 0 ]; then exit "$1"; fi; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace -- \
    python "$ROOT/bench.py" --steps 30 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1; fatal $? trace
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1; fatal $? pmc_fetch
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1; fatal $? pmc_write
cd "$ROOT"
timeout -k 10 500 python scripts/bench_configs.py > "$OUT/configs_$TAG.jsonl" 2> "$OUT/configs_$TAG.err"; fatal $? configs
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; fatal $? bench
cat "$OUT/prof_$TAG/trace_kernel_stats.csv" | cut -c1-160 | head -8
cat "$OUT/bench_$TAG.json"
