set -u
# round 4: idle-lane band defaults — parity (test_band.py) then op-level A/B vs the zsum schedule they replace
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 400 python -u -m pytest tests/test_band.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04_band_idle_tests.log 2>&1 || { tail -30 gpurun_out/r04_band_idle_tests.log; exit 1; }
tail -2 gpurun_out/r04_band_idle_tests.log
L=gpurun_out/r04_op_band_idle2.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:512x512x520:ZMIN=32,ZMAX=32 s27:512x512x504 s27:512x512x760 s27:512x512x1000:ZMIN=32,ZMAX=32
run h7:512x512x520 h7:512x512x504 h7:512x512x760 h7:512x512x1000
run f7:512x512x520 f7:512x512x504:BAND=4,BTY=8 f7:512x512x760 f7:512x512x1000 f7:256x256x1000
grep -v amdgpu.ids $L
