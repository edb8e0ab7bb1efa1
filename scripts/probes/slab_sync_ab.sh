#!/bin/bash
# Loopback proxy of the N=8 slab step (scripts/probes/slab_step.py) under each cross-stream ordering of the sweep:
# PSAD_SLAB_SYNC=value (stream memory operations both ways, the round-4 default), mixed (compute -> halo by event,
# halo -> compute by stream memory operation), event (both by events); a mode cp-<m> runs <m> with the HIP runtime's
# GPU_STREAMOPS_CP_WAIT=1 (stream-op waits by the command processor instead of a blit kernel); ns-<m> runs <m> with
# PSAD_SLAB_START_SIG=0 (the compute -> halo signal by hipStreamWriteValue32 instead of the interior launch's store);
# fw-<m> with PSAD_SLAB_FACE_WAIT=1 (the face launches on the compute stream, their loaders waiting for the halos).
# usage: gpurun -- bash scripts/probes/slab_sync_ab.sh TAG ["value mixed cp-value ..."]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG="${1:-r06}"
LOG="gpurun_out/slab_sync_${TAG}.log"
MODES="${2:-value mixed event}"
for R in 1 2; do
  for V in $MODES; do
    for W in "96 stencil27" "128 diffusion7"; do
      echo "== round $R PSAD_SLAB_SYNC=$V $W" >> "$LOG"
      if [ "${V#cp-}" != "$V" ]; then CPW=1; M="${V#cp-}"; else CPW=0; M="$V"; fi
      if [ "${M#ns-}" != "$M" ]; then SS=0; M="${M#ns-}"; else SS=1; fi
      if [ "${M#fw-}" != "$M" ]; then FW=1; M="${M#fw-}"; else FW=0; fi
      PSAD_SLAB_FACE_WAIT=$FW PSAD_SLAB_START_SIG=$SS GPU_STREAMOPS_CP_WAIT=$CPW PSAD_SLAB_SYNC=$M timeout -k 10 150 python scripts/probes/slab_step.py $W 2>&1 | \
          grep -E "zslab native|plain" >> "$LOG" || exit 1
    done
  done
done
cat "$LOG"
