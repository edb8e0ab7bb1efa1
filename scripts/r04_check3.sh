set -u
# round 4: GPU tests of this round's changes, then op-level A/B (band variants, fp32 7-point tiles, unaligned rows)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 900 python -u -m pytest tests/test_band.py tests/test_gpu_parity.py tests/test_lbm.py tests/test_cpu_backend.py -m gpu -x -q --timeout 300 --timeout-method thread -k "band or golden_linear or full_size_properties or 512_vs_c_oracle or lbm or iteration_slice" > gpurun_out/r04_pytest3.log 2>&1 || { tail -40 gpurun_out/r04_pytest3.log; exit 1; }
tail -3 gpurun_out/r04_pytest3.log
timeout -k 10 60 python -u scripts/probes/simd_place.py > gpurun_out/r04_simd_place.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_simd_place.log
timeout -k 10 400 python -u scripts/probes/op_band_ab.py "s27:768:BTRIM=3,BLDR=1:BTRIM=1,BLAUX=2:BTRIM=3,BLDR=1,BLAUX=2:BEDGE=0:BTRIM=1:BTRIM=3:BTRIM=3,ZMIN=24,ZMAX=24:BTRIM=3,ZMIN=16,ZMAX=16:BTRIM=1,BEDGE=0:BTRIM=1,BSTAG=40:BTRIM=1,BSTAG=100:BTRIM=1,MAP=1:BTRIM=1,ZMIN=64,ZMAX=64" > gpurun_out/r04_op_band_ab3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab3.log
timeout -k 10 400 python -u scripts/probes/op_band_ab.py "h7:510:BTRIM=1" "s27:766:BTRIM=1" "s27:510:BAND=4,ZMIN=24,ZMAX=24,BTRIM=1:BAND=4,ZMIN=16,ZMAX=16,BTRIM=1" "s27:512:BAND=4,ZMIN=24,ZMAX=24,BTRIM=1:BAND=4,ZMIN=16,ZMAX=16,BTRIM=1" "h7:512:BTRIM=1" "s27:511:BAND=4,ZMIN=24,ZMAX=24,BTRIM=1:BAND=4,ZMIN=16,ZMAX=16,BTRIM=1" "s27:255:BAND=4,ZMIN=8,ZMAX=8,BTRIM=1:BAND=4,ZMIN=16,ZMAX=16,BTRIM=1" "s27:256:BAND=4,ZMIN=8,ZMAX=8,BTRIM=1" "s27:96x768:BAND=4,ZMIN=12,ZMAX=12,BTRIM=3:BAND=4,ZMIN=8,ZMAX=8,BTRIM=3:BAND=4,ZMIN=24,ZMAX=24,BTRIM=3" "h7:511" "h7:255" "h7:256" > gpurun_out/r04_op_unaligned.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_unaligned.log
timeout -k 10 400 python -u scripts/probes/op_band_ab.py "s27:1024:BTRIM=1,ZMIN=32,ZMAX=32:BTRIM=3,ZMIN=32,ZMAX=32:BTRIM=3:BTRIM=3,ZMIN=16,ZMAX=16:BTRIM=1,ZMIN=32,ZMAX=32,BEDGE=0" "h7:768:BTRIM=1,BEDGE=0:BTRIM=1:BTRIM=3:BTRIM=3,ZMIN=16,ZMAX=16" > gpurun_out/r04_op_band_ab4.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab4.log
timeout -k 10 400 python -u scripts/probes/op_band_ab.py "f7:512:CX=2:NR=2:ZMIN=64,ZMAX=64:MAP=1:D=3:CX=2,ZMIN=64,ZMAX=64:CX=2,MAP=1:BAND=4,BTRIM=1:BAND=4,BTRIM=1,ZMIN=16,ZMAX=16" "f7:768:CX=2:MAP=0:D=3:ZMIN=64,ZMAX=64:BAND=4,BTRIM=1" > gpurun_out/r04_op_f7_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_f7_ab.log
echo done-ab
timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/r04_slab27_event.log 2>&1 || exit 1
PSAD_SLAB_SYNC=value timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/r04_slab27_value.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/r04_slab7_event.log 2>&1 || exit 1
PSAD_SLAB_SYNC=value timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/r04_slab7_value.log 2>&1 || exit 1
for f in gpurun_out/r04_slab*_*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -6; done
echo done-slab
timeout -k 10 300 python -u scripts/probes/alloc_ab.py > gpurun_out/r04_alloc_ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_alloc_ab.log
echo done-all
