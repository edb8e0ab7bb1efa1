#!/bin/bash
# round 5: new band / WS parity tests, then the band-kernel edge-read / store-interleave / loader-priority A/B through
# the op (same process per line). A test failure (exit 1) still runs the A/B; a timeout / crash ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py::test_ws_tilings_bitwise_same_process tests/test_band.py::test_band_chunk_length_and_band_height_bitwise \
  tests/test_band.py::test_band_padded_rows_vs_oracle > gpurun_out/r05_tests1.log 2>&1
rc=$?; tail -3 gpurun_out/r05_tests1.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/probes/op_band_ab.py s27:768::BPE=3:BSI=1:BPE=3,BSI=1:BPRIO=3 2>&1 | tee gpurun_out/r05_band_ab1.log && \
timeout -k 10 300 python -u scripts/probes/op_band_ab.py s27:1024::BPE=3:BSI=1:BPE=3,BSI=1 s27:512::BPE=3:BSI=1 h7:768::BSI=1 2>&1 | tee gpurun_out/r05_band_ab2.log
