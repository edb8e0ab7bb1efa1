#!/bin/bash
# HBM traffic of configs 2 and 3 (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, one config per process):
#   gpurun -- 'bash scripts/config_traffic.sh r05'
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r05}"
cd "$ROOT"
timeout -k 10 200 python scripts/bench_configs.py laplace5_f32_4096^2 diffusion7_f32_512^3 > /dev/null 2>&1 || exit 1
cd /tmp
for C in laplace5_f32_4096^2 diffusion7_f32_512^3; do
  N="${C//^/}"
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/cfgpmc_${TAG}_${N}_$P" -o pmc -- \
        python "$ROOT/scripts/bench_configs.py" "$C" > "$OUT/cfgpmc_${TAG}_${N}_$P.log" 2>&1 || exit 2
  done
done
echo done-config-traffic
