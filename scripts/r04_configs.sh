#!/bin/bash
# Round-4 evidence, part 2: every BASELINE config (scripts/bench_configs.py), then bench.py as the driver runs it.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r04}"
timeout -k 10 700 python -u scripts/bench_configs.py > "$OUT/configs_$TAG.jsonl" 2> "$OUT/configs_$TAG.err" || { tail -20 "$OUT/configs_$TAG.err"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -20 "$OUT/bench_$TAG.err"; exit 1; }
cut -c1-200 "$OUT/configs_$TAG.jsonl"
cat "$OUT/bench_$TAG.json"
