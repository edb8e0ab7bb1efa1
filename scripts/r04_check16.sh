set -u
# round 4: 27-point 768^3 on padded rows -- band height / depth / chunk length variants (shared inputs)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 700 python -u scripts/probes/op_band_ab.py "s27:768:BTY=16,D=1:BTY=16,D=1,ZMIN=32,ZMAX=32:ZMIN=32,ZMAX=32:ZMIN=24,ZMAX=24:BLDR=1:BTY=12:BAND=2,BTY=8" > gpurun_out/r04_op_band_ab10.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab10.log
