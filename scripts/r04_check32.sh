set -u
# round 4: fp16 16-row bands of 2 rows per lane ahead of (8,2,3), the 16-row zc rule only for the 1024-wide box rule —
# parity, then defaults vs zsum
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 500 python -u -m pytest tests/test_band.py -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r04_band_gpu4.log 2>&1 || { tail -30 gpurun_out/r04_band_gpu4.log; exit 1; }
tail -2 gpurun_out/r04_band_gpu4.log
L=gpurun_out/r04_op_band_1622.log
run() { timeout -k 10 250 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:512x512x320 s27:512x512x384 s27:512x512x576 s27:512x512x640 s27:512x512x448
run h7:512x512x384 h7:512x512x640
grep -v amdgpu.ids $L
