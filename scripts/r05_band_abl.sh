#!/bin/bash
# round 5: where the 27-point fp16 768^3 band sweep's time goes (ablation probes, timing only) + occupancy variants
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u scripts/probes/op_band_ab.py s27:768::BABL=1:BABL=2:BABL=3:BABL=1,BABL=1 h7:768::BABL=1:BABL=2:BABL=3 2>&1 | tee gpurun_out/r05_band_abl1.log && \
timeout -k 10 400 python -u scripts/probes/op_band_ab.py s27:768::D=1,BWPE=4:BTY=16,D=1:D=1:BTY=16,BAND=2,D=2 2>&1 | tee gpurun_out/r05_band_abl2.log && \
timeout -k 10 120 python -u scripts/probes/torch_stream.py 768 2>&1 | tee gpurun_out/r05_torch_stream.log
