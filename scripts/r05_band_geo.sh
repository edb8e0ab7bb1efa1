#!/bin/bash
# round 5: band geometry sweep for the 27-point fp16 sweep (rows per band, rows per lane, planes in flight, chunks)
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u scripts/probes/op_band_ab.py s27:768::BTY=16,BAND=2,D=2:BTY=16,BAND=2,D=1:BTY=16,BAND=2,D=3:BTY=32,BAND=2,D=1:BTY=16,BAND=2,D=2,ZMIN=32,ZMAX=32:BTY=16,BAND=2,D=2,BABL=1 2>&1 | tee gpurun_out/r05_band_geo1.log && \
timeout -k 10 500 python -u scripts/probes/op_band_ab.py s27:1024::BTY=8,BAND=2,D=2:BTY=8,BAND=2,D=3:BTY=8,BAND=4,D=2 s27:512::BTY=16,BAND=2,D=2:BTY=8,BAND=2,D=2 h7:768::BTY=16,BAND=2,D=2:BTY=16,BAND=2,D=1 2>&1 | tee gpurun_out/r05_band_geo2.log
