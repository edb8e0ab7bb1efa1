set -u
# round 4: fp32 7-point -- band with 8-row bands at 512^3, zsum chunk lengths at 768^3 / 1024^3 (shared inputs)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 900 python -u scripts/probes/op_band_ab.py "f7:512:BAND=4,BTY=8:BAND=4,BTY=8,ZMIN=64,ZMAX=64:BAND=4,BTY=8,ZMIN=16,ZMAX=16:BAND=4,BTY=8,BPAD=1:ZMIN=64,ZMAX=64" "f7:768:ZMIN=48,ZMAX=48:ZMIN=64,ZMAX=64:ZMIN=96,ZMAX=96:BAND=4,BTY=8" "f7:1024:ZMIN=64,ZMAX=64:ZMIN=48,ZMAX=48:BAND=4,BTY=8" > gpurun_out/r04_op_f7_ab3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_f7_ab3.log
