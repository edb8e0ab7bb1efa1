set -u
# round 4: branch-free masked band stores (range-check drops) — parity, then A/B vs the branched form (BMBR=1)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 400 python -u -m pytest tests/test_band.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04_band_mask_tests.log 2>&1 || { tail -30 gpurun_out/r04_band_mask_tests.log; exit 1; }
tail -2 gpurun_out/r04_band_mask_tests.log
L=gpurun_out/r04_op_band_mask.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:512 s27:512x510x512:BMBR=1 s27:510:BMBR=1 s27:511:BMBR=1 s27:255:BMBR=1 s27:256
run h7:512 h7:510:BMBR=1 h7:511:BMBR=1 h7:512x510x512:BMBR=1 f7:512x510x512:BMBR=1 s27:512x512x520:BMBR=1
grep -v amdgpu.ids $L
