set -u
# round 4: fp32 7-point band geometries at 768 / 1024 (4-row bands; zsum is the default there)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_f7_ab6.log
run() { timeout -k 10 250 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run f7:768:BAND=4,BTY=4:BAND=2,BTY=4:BAND=4,BTY=8,D=1:BAND=2,BTY=4,D=3:BAND=4,BTY=4,ZMIN=32,ZMAX=32
run f7:1024:BAND=4,BTY=4:BAND=2,BTY=4:BAND=4,BTY=8,D=1:BAND=4,BTY=4,ZMIN=32,ZMAX=32
grep -v amdgpu.ids $L
