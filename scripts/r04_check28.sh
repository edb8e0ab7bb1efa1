set -u
# round 4: band output stores' cache policy (BNT: 2 = non-temporal default, 0 = default policy, 1 / 3)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_band_nt.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:768:BNT=0:BNT=1:BNT=3:BNT=2
run h7:768:BNT=0:BNT=1:BNT=3
run f7:512:BNT=0:BNT=1:BNT=3
run s27:96x768:BNT=0:BNT=1
grep -v amdgpu.ids $L
