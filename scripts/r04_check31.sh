set -u
# round 4: rows whose whole-wave band choice is (8,2,3) (384 / 640 / 896 chunks-of-8 multiples of 16 but not 32):
# 16-row bands of 2 rows per lane instead
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_band_823.log
run() { timeout -k 10 250 python -u scripts/probes/op_band_ab.py "$@" >> $L 2>&1 || { tail -5 $L; exit 1; }; }
# (27-point 640 / 384 above)
run h7:512x512x640:BAND=2,BTY=16,D=2:BAND=4,BTY=8 h7:512x512x384:BAND=2,BTY=16,D=2
grep -v amdgpu.ids $L
