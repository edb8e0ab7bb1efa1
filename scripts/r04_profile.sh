#!/bin/bash
# Round-4 evidence, part 1: rocprofv3 kernel trace + stats of bench.py (headline + config 5), the FETCH_SIZE /
# WRITE_SIZE passes (separate runs, no trace domains), two SQ counter passes over config 5's band kernels.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r04}"
fatal() { echo "[$2] rc=$1" | tee -a "$OUT/status_$TAG.log"; if [ "$1" -ne 0 ]; then exit "$1"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_bench_rehearsal.py -m gpu -q --timeout 250 --timeout-method thread > "$OUT/pytest_rehearsal_$TAG.log" 2>&1; fatal $? rehearsal
tail -2 "$OUT/pytest_rehearsal_$TAG.log"
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/warm_$TAG.log" 2>&1; fatal $? warm
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace -- \
    python "$ROOT/bench.py" --steps 30 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1; fatal $? trace
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch_$TAG.log" 2>&1; fatal $? pmc_fetch
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$TAG" -o pmc -- \
    python "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write_$TAG.log" 2>&1; fatal $? pmc_write
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmcband_${TAG}_$i" -o pmc -- python "$ROOT/bench.py" \
      --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmcband_${TAG}_$i.log" 2>&1
  fatal $? "pmc_sq_$i"
done
cd "$ROOT"
cut -c1-160 "$OUT/prof_$TAG/trace_kernel_stats.csv" | head -8
echo done-profile
