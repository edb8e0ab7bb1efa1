#!/bin/bash
# Perf evidence of the tree being benched, stamped with its commit:
#   1. rocprofv3 --kernel-trace --stats of bench.py (headline + config 5 as `secondary`)
#   2. rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs (no trace domains) -> traffic_<TAG>.json
#      (scripts/pmc_summary.py: FETCH_SIZE doubled, the gfx950 wide-read correction), each entry carrying the commit
#      and bench.py's kernel_sha16 of the launches it measured (bench.py reports whether they match the running tree)
#   3. two SQ counter passes over config 5's band kernels (pmcband_<TAG>_1/2)
# usage (the commit is expanded on the CPU side: the box has no .git):
#   gpurun -- "bash scripts/profile_evidence.sh r05 $(git rev-parse --short HEAD)"
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r05}"
HEAD="${2:-unknown}"
fatal() { echo "[$2] rc=$1" | tee -a "$OUT/status_$TAG.log"; if [ "$1" -ne 0 ]; then exit "$1"; fi; }
echo "$HEAD" > "$OUT/head_$TAG.txt"
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
# traffic_<TAG>.json: the committed summary updated with this run's passes (copied into profiles/traffic.json)
cp profiles/traffic.json "$OUT/traffic_$TAG.json"
F="$OUT/pmc_fetch_$TAG/pmc_counter_collection.csv"; W="$OUT/pmc_write_$TAG/pmc_counter_collection.csv"
SRC="profiles/${TAG}_pmc_fetch_size.csv + profiles/${TAG}_pmc_write_size.csv (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of bench.py --steps 3; scripts/profile_evidence.sh)"
python - "$OUT/pmc_fetch_$TAG.log" > "$OUT/ksha_$TAG.txt" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
r = json.loads(line)
print(r['roofline']['kernel_sha16'], r['secondary']['roofline']['kernel_sha16'])
EOF
fatal $? ksha
read KS1 KS2 < "$OUT/ksha_$TAG.txt"
python scripts/pmc_summary.py "$F" "$W" --workload "diffusion7_f32_1024^3" --bytes 8589934592 --select diffusion7_f32 \
    --json "$OUT/traffic_$TAG.json" --source "$SRC" --git-head "$HEAD" --kernel-sha "$KS1" > "$OUT/traffic_$TAG.txt"; fatal $? sum1
python scripts/pmc_summary.py "$F" "$W" --workload "stencil27_f16_768^3" --bytes 1811939328 --select stencil27_f16 \
    --json "$OUT/traffic_$TAG.json" --source "$SRC" --git-head "$HEAD" --kernel-sha "$KS2" >> "$OUT/traffic_$TAG.txt"; fatal $? sum2
python scripts/sq_summary.py "$OUT/pmcband_${TAG}_1/pmc_counter_collection.csv" "$OUT/pmcband_${TAG}_2/pmc_counter_collection.csv" \
    --select stencil27_f16 > "$OUT/pmc_band_sq_$TAG.txt"; fatal $? sq
cut -c1-160 "$OUT/prof_$TAG/trace_kernel_stats.csv" | head -8
echo done-profile
