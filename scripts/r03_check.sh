#!/bin/bash
# round-3 GPU check: selected test files, then probes / benches; every GPU step under its own time limit,
# stops at the first fatal status (fault, abort, timeout)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
mkdir -p gpurun_out
TAG="$1"; shift
TESTS="$1"; shift
fatal() { [ "$1" -ge 2 ] && [ "$1" -ne 5 ]; }
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread $TESTS -m gpu > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -4 gpurun_out/${TAG}_pytest.log; echo "pytest rc=$rc"
  if fatal $rc; then exit $rc; fi
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 300 bash -c "$cmd" > gpurun_out/${TAG}_step$i.log 2>&1; r=$?
  echo "== step $i rc=$r: $cmd"; tail -40 gpurun_out/${TAG}_step$i.log
  if [ $r -ne 0 ]; then exit $r; fi
done
