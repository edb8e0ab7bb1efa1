set -u
# round 4: 512^3 fp32 7-point band geometries (rows per lane, band height) — BASELINE config 3
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_f7_ab5.log
run() { timeout -k 10 200 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
run f7:512:BAND=2,BTY=8:BAND=4,BTY=16,D=1:BAND=2,BTY=8,ZMIN=8,ZMAX=8:BAND=2,BTY=8,ZMIN=32,ZMAX=32:BAND=4,BTY=8
run f7:512:BAND=2,BTY=8:BAND=4,BTY=8
grep -v amdgpu.ids $L
