#!/bin/bash
# One GPU-box session: build, smoke, GPU parity tests, bench, rocprofv3 kernel trace + HBM counters.
# Every GPU step has its own time limit; the script stops at the first fault / abort / timeout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
export PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r01}"
STEPS="${STEPS:-all}"

stop_if_fatal() {  # $1 = rc, $2 = step name ; test failures (rc 1) are not fatal
  echo "[$2] rc=$1" | tee -a "$OUT/status.log"
  if [ "$1" -ge 2 ] && [ "$1" -ne 5 ]; then echo "fatal rc in $2, stopping" | tee -a "$OUT/status.log"; exit "$1"; fi
}

python -m pystencils_autodiff_amd.build > "$OUT/build.log" 2>&1 || { echo build failed; cat "$OUT/build.log"; exit 3; }

if [[ "$STEPS" == *smoke* || "$STEPS" == all ]]; then
  timeout -k 10 400 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; rc=$?
  tail -3 "$OUT/smoke.log"; stop_if_fatal $rc smoke
fi
if [[ "$STEPS" == *tests* || "$STEPS" == all ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -15 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest_gpu
fi
if [[ "$STEPS" == *bench* || "$STEPS" == all ]]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 --kernel-only > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; rc=$?
  cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"; stop_if_fatal $rc bench
fi
if [[ "$STEPS" == *prof* || "$STEPS" == all ]]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace -- \
      python "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1; rc=$?
  tail -3 "$OUT/prof_$TAG.log"; stop_if_fatal $rc rocprof_trace
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o pmc -- \
      python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1; rc=$?
  tail -3 "$OUT/pmc_fetch_$TAG.log"; stop_if_fatal $rc rocprof_pmc_fetch
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o pmc -- \
      python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1; rc=$?
  tail -3 "$OUT/pmc_write_$TAG.log"; stop_if_fatal $rc rocprof_pmc_write
  cd "$ROOT"
fi
echo done | tee -a "$OUT/status.log"
