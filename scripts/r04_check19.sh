set -u
# round 4: band variants for 512^3 fp32 7-point (VERDICT: >= 74 % per sweep) and 768^3 fp16 27-point
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_band_ab11.log
timeout -k 10 300 python -u scripts/probes/op_band_ab.py \
  f7:512:ZMIN=12,ZMAX=12:ZMIN=8,ZMAX=8:ZMIN=24,ZMAX=24:BTRIM=1:MAP=1:BLAUX=2:BWPE=3:D=3:BEDGE=0 >> $L 2>&1 || { tail -5 $L; exit 1; }
timeout -k 10 400 python -u scripts/probes/op_band_ab.py \
  s27:768:BTY=16,D=1:BTY=16,D=1,ZMIN=32,ZMAX=32:D=3:BTY=12:BAND=2:BAND=2,BTY=16:MAP=1 >> $L 2>&1 || { tail -5 $L; exit 1; }
grep -v amdgpu.ids $L
