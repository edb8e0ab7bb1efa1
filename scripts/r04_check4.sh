set -u
# round 4: slab sync A/B (event vs stream memory ops), allocation-order probe, band chunk-length sweeps
# (wave quantisation at 256..768), 7-point edge mapping under BTRIM=3
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/r04_slab27_event.log 2>&1 || exit 1
PSAD_SLAB_SYNC=value timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/r04_slab27_value.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/r04_slab7_event.log 2>&1 || exit 1
PSAD_SLAB_SYNC=value timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/r04_slab7_value.log 2>&1 || exit 1
for f in gpurun_out/r04_slab*_*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -6; done
echo done-slab
timeout -k 10 300 python -u scripts/probes/alloc_ab.py > gpurun_out/r04_alloc_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_alloc_ab.log
timeout -k 10 500 python -u scripts/probes/op_band_ab.py "s27:768:BTRIM=3:BTRIM=3,ZMIN=96,ZMAX=96:BTRIM=3,ZMIN=32,ZMAX=32:BTRIM=3,BEDGE=0:BTRIM=3,BLAUX=2:BTRIM=3,BWPE=3" "h7:768:BTRIM=3:BTRIM=3,BEDGE=0:BTRIM=1,BEDGE=0:BTRIM=3,BEDGE=0,ZMIN=96,ZMAX=96:BTRIM=3,BEDGE=0,ZMIN=32,ZMAX=32" "h7:1024:BTRIM=3:BTRIM=3,BEDGE=0" > gpurun_out/r04_op_band_ab5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab5.log
Z="BAND=4,BTRIM=3"
timeout -k 10 600 python -u scripts/probes/op_band_ab.py "s27:512:$Z,ZMIN=8,ZMAX=8:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=12,ZMAX=12:$Z,ZMIN=16,ZMAX=16:$Z,ZMIN=22,ZMAX=22:$Z,ZMIN=32,ZMAX=32:$Z,ZMIN=64,ZMAX=64" "s27:510:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=12,ZMAX=12:$Z,ZMIN=16,ZMAX=16:$Z,ZMIN=32,ZMAX=32:$Z,ZMIN=64,ZMAX=64" "s27:511:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=12,ZMAX=12:$Z,ZMIN=16,ZMAX=16:$Z,ZMIN=32,ZMAX=32" "h7:512:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=16,ZMAX=16:$Z,ZMIN=32,ZMAX=32:$Z,ZMIN=64,ZMAX=64:$Z,BEDGE=0,ZMIN=32,ZMAX=32" "h7:510:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=16,ZMAX=16:$Z,ZMIN=32,ZMAX=32:$Z,ZMIN=64,ZMAX=64:$Z,BEDGE=0,ZMIN=32,ZMAX=32" "s27:256:$Z,ZMIN=4,ZMAX=4:$Z,ZMIN=6,ZMAX=6:$Z,ZMIN=8,ZMAX=8:$Z,ZMIN=11,ZMAX=11:$Z,ZMIN=16,ZMAX=16" "s27:255:$Z,ZMIN=4,ZMAX=4:$Z,ZMIN=6,ZMAX=6:$Z,ZMIN=8,ZMAX=8:$Z,ZMIN=11,ZMAX=11" > gpurun_out/r04_op_zc_sweep.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_zc_sweep.log
echo done-all
