set -u
# round 4: 27-point partial rows — band height / rows per lane / chunk variants
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_pitch27b.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run s27:510:BAND=2,BTY=16:BAND=2,BTY=16,ZMIN=16,ZMAX=16:ZMIN=16,ZMAX=16:ZMIN=64,ZMAX=64:BREG=1:BAND=4,BTY=16,D=1
run s27:511:BAND=2,BTY=16:ZMIN=16,ZMAX=16:BREG=1
run s27:255:BAND=2,BTY=16:ZMIN=16,ZMAX=16:ZMIN=4,ZMAX=4:BREG=1
run s27:512:BAND=2,BTY=16:ZMIN=16,ZMAX=16
grep -v amdgpu.ids $L
