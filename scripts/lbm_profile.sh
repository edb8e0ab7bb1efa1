#!/bin/bash
# rocprofv3 evidence for the LBM lattice kernels (D3Q19 192^3 fp32, periodic / MRT / pressure channel, 10-step ops):
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate passes (no trace domains).
#   gpurun -- 'bash scripts/lbm_profile.sh r05'
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r05}"
CFGS="lbm_d3q19_f32_192^3 lbm_d3q19_f32_192^3_mrt lbm_d3q19_f32_192^3_pressure"
cd "$ROOT"
timeout -k 10 300 python scripts/bench_configs.py $CFGS > "$OUT/lbmprof_warm_$TAG.jsonl" 2>/dev/null || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lbmprof_$TAG" -o trace -- \
    python "$ROOT/scripts/bench_configs.py" $CFGS > "$OUT/lbmprof_trace_$TAG.log" 2>&1 || exit 2
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/lbmpmc_fetch_$TAG" -o pmc -- \
    python "$ROOT/scripts/bench_configs.py" $CFGS > "$OUT/lbmpmc_fetch_$TAG.log" 2>&1 || exit 3
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/lbmpmc_write_$TAG" -o pmc -- \
    python "$ROOT/scripts/bench_configs.py" $CFGS > "$OUT/lbmpmc_write_$TAG.log" 2>&1 || exit 4
echo done-lbm-profile
