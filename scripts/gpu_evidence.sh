#!/bin/bash
# Profile evidence for a round's final tree: rocprofv3 kernel trace + stats of bench.py, FETCH_SIZE /
# WRITE_SIZE PMC passes of the same command (separate runs), the host CPU baselines, and the SQ / HBM
# counter passes of the 27-point fp16 768^3 sweep (scripts/pmc27h_once.sh). Each GPU step has its own
# time limit; the script stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r02}"
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace -- \
    python "$ROOT/bench.py" --steps 30 --warmup 2 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1 || exit $?
cd "$ROOT"
timeout -k 10 400 python scripts/cpu_baselines.py > "$OUT/cpu_baselines_$TAG.jsonl" 2> "$OUT/cpu_baselines_$TAG.err" || exit $?
TAG="pmc27h_$TAG" timeout -k 10 400 bash scripts/pmc27h_once.sh || exit $?
echo evidence done
