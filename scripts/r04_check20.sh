set -u
# round 4: 27-point 768^3 occupancy variants (one plane in flight: smaller LDS ring, more workgroups per CU)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_band_ab12.log
timeout -k 10 400 python -u scripts/probes/op_band_ab.py \
  s27:768:D=1:D=1,ZMIN=32,ZMAX=32:D=1,ZMIN=96,ZMAX=96:BAND=2,BTY=16:BAND=2,BTY=16,D=1:BAND=2,BTY=16,ZMIN=32,ZMAX=32:BAND=4,BTY=8 >> $L 2>&1 || { tail -5 $L; exit 1; }
timeout -k 10 400 python -u scripts/probes/op_band_ab.py \
  s27:1024:D=1,BTY=8:BAND=2,BTY=16:BAND=2,BTY=32,D=1 >> $L 2>&1 || { tail -5 $L; exit 1; }
grep -v amdgpu.ids $L
