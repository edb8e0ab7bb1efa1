set -u
# round 4: the headline fp32 7-point 1024^3 -- zsum chunk lengths, fp32 bands with one plane in flight (shared inputs)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 900 python -u scripts/probes/op_band_ab.py "f7:1024:ZMIN=64,ZMAX=64:ZMIN=48,ZMAX=48:ZMIN=128,ZMAX=128:BAND=4,BTY=8,D=1:BAND=4,BTY=4:BAND=4,BTY=8,D=1,ZMIN=32,ZMAX=32" > gpurun_out/r04_op_f7_1024.log 2>&1 || { tail -5 gpurun_out/r04_op_f7_1024.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_op_f7_1024.log
