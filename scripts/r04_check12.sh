set -u
# round 4: fp32 7-point 512^3 / 768^3 schedules on shared inputs (op A/B)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 700 python -u scripts/probes/op_band_ab.py "f7:512:ZMIN=64,ZMAX=64:ZMIN=16,ZMAX=16:BAND=4:BAND=4,BTY=8:BAND=4,ZMIN=64,ZMAX=64:BAND=4,BPAD=1:NR=4:MAP=1" "f7:768:BAND=4:BAND=4,ZMIN=64,ZMAX=64:ZMIN=64,ZMAX=64" > gpurun_out/r04_op_f7_ab2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_f7_ab2.log
