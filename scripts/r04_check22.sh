set -u
# round 4: band schedule with idle lanes in the last compute wave, rows whose chunk count has no whole-wave band
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_band_idle.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:512x512x520:BAND=4,BTY=8:BAND=2,BTY=16:BAND=4,BTY=16,D=1:BAND=4,BTY=32,D=1
run s27:512x512x504:BAND=4,BTY=8:BAND=2,BTY=16
run s27:512x512x760:BAND=4,BTY=8:BAND=2,BTY=16
run s27:512x512x1000:BAND=4,BTY=8:BAND=4,BTY=16,D=1
run h7:512x512x520:BAND=4,BTY=8:BAND=2,BTY=16:BAND=4,BTY=32,D=1
run h7:512x512x504:BAND=4,BTY=8
run h7:512x512x1000:BAND=4,BTY=8
run f7:512x512x520:BAND=4,BTY=8:BAND=2,BTY=8:BAND=4,BTY=4
run f7:512x512x504:BAND=4,BTY=8:BAND=4,BTY=4
grep -v amdgpu.ids $L
