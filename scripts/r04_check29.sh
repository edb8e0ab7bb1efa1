set -u
# round 4: 27-point 96x768^2 slab proxy — band chunk length on the slab (interior z range + two-face launch)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_slab27_zc.log
for m in "" "BAND=4,ZMIN=8,ZMAX=8" "BAND=4,ZMIN=16,ZMAX=16" "BAND=4,ZMIN=24,ZMAX=24" "BAND=4,ZMIN=47,ZMAX=47" ""; do
  echo "== PSAD_MARCH=$m" >> $L
  PSAD_MARCH="$m" timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
grep -v amdgpu.ids $L | grep -E "==|native faces on halo|plain op"
