#!/bin/bash
# SQ counters of config 5's band kernels (27-point fp16 768^3) under each plane-synchronisation variant: the plane
# barrier (default) and the LDS handshake (BFREE), two separate --pmc passes per variant (no trace domains), summarised
# by scripts/sq_summary.py.   usage: gpurun -- "bash scripts/probes/band_sync_pmc.sh r06 '' BFREE=2 ..."
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="$1"; shift
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
for V in "$@"; do
  N="${V:-default}"; N="${N//[=,]/_}"
  export PSAD_MARCH="$V"
  [ -z "$V" ] && unset PSAD_MARCH
  timeout -k 10 200 python bench.py --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline \
      > "$OUT/bsync_${TAG}_${N}_warm.log" 2>&1 || { echo "warm $N failed"; exit 1; }
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$OUT/bsync_${TAG}_${N}_$i" -o pmc -- \
        python "$ROOT/bench.py" --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline \
        > "$OUT/bsync_${TAG}_${N}_$i.log" 2>&1) || { echo "pmc $N $i failed"; exit 1; }
  done
  echo "== $N (PSAD_MARCH='$V')" >> "$OUT/bsync_${TAG}.txt"
  python scripts/sq_summary.py "$OUT/bsync_${TAG}_${N}_1/pmc_counter_collection.csv" \
      "$OUT/bsync_${TAG}_${N}_2/pmc_counter_collection.csv" --select stencil27_f16 >> "$OUT/bsync_${TAG}.txt" || exit 1
done
cat "$OUT/bsync_${TAG}.txt"
