#!/bin/bash
# L2 (TCC) stall / queue counters of the band kernels on rows of different pitch (the row-pitch cliff: 27-point fp16
# 511^3 against 512^3), one rocprofv3 --pmc pass per counter group (<= 4 TCC counters each, no trace domains), over
# scripts/probes/pitch_pmc.py (4 fwd+bwd steps per size).  usage: gpurun -- bash scripts/probes/pitch_stall_pmc.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
TAG="${1:-r06}"
SIZES="${2:-s27:511 s27:512}"
timeout -k 10 200 python scripts/probes/pitch_pmc.py $SIZES > "$OUT/pstall_${TAG}_warm.log" 2>&1 || { echo warm failed; exit 1; }
i=0
for P in "TCC_WRREQ_STALL_max TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
         "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum TCC_CYCLE_sum" \
         "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUSY_avr"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$OUT/pstall_${TAG}_$i" -o pmc -- \
      python "$ROOT/scripts/probes/pitch_pmc.py" $SIZES > "$OUT/pstall_${TAG}_$i.log" 2>&1) || { echo "pass $i failed"; exit 1; }
done
python - "$OUT" "$TAG" $SIZES <<'PY'
import csv, sys, glob, collections
out, tag, sizes = sys.argv[1], sys.argv[2], sys.argv[3:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(f'{out}/pstall_{tag}_*/pmc_counter_collection.csv')):
    rows = [r for r in csv.DictReader(open(p, newline='')) if 'band' in r['Kernel_Name']]
    ids = sorted({int(r['Dispatch_Id']) for r in rows})
    per = len(ids) // len(sizes)          # the probe runs the sizes one after another, the same launches each
    size_of = {d: sizes[min(i // per, len(sizes) - 1)] for i, d in enumerate(ids)}
    for r in rows:
        kind = 'fwd' if 'forward' in r['Kernel_Name'] else 'bwd'
        acc[(size_of[int(r['Dispatch_Id'])], kind)][r['Counter_Name']].append(float(r['Counter_Value']))
for key, cs in sorted(acc.items()):
    print(key[0], key[1], ' '.join(f'{c}={sum(v) / len(v):.4g}' for c, v in sorted(cs.items())))
PY
