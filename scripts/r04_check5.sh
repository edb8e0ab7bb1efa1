set -u
# round 4: zero-padded band image rows (BPAD) parity + A/B, star-stencil chunk lengths, slab defaults (value sync,
# faces on the halo stream)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 900 python -u -m pytest tests/test_band.py tests/test_distributed.py tests/test_native_abi.py tests/test_native_autograd.py -m gpu -q --deselect tests/test_band.py::test_band_chunk_length_and_band_height_bitwise --timeout 300 --timeout-method thread > gpurun_out/r04_pytest5.log 2>&1 || { tail -40 gpurun_out/r04_pytest5.log; exit 1; }
tail -3 gpurun_out/r04_pytest5.log
timeout -k 10 500 python -u scripts/probes/op_band_ab.py "s27:768:BPAD=1:BPAD=1,BEDGE=0:BAND=4,ZMIN=96,ZMAX=96:BPAD=1,BAND=4,ZMIN=96,ZMAX=96" "s27:1024:BPAD=1" "s27:512:BPAD=1" "h7:768:BPAD=1:BAND=4,ZMIN=64,ZMAX=64:BAND=4,ZMIN=96,ZMAX=96:BAND=4,ZMIN=128,ZMAX=128" "h7:1024:BPAD=1:BAND=4,ZMIN=64,ZMAX=64:BAND=4,ZMIN=128,ZMAX=128:BAND=4,ZMIN=171,ZMAX=171" "h7:256:BAND=4,ZMIN=16,ZMAX=16:BAND=4,ZMIN=32,ZMAX=32:BAND=4,ZMIN=64,ZMAX=64" > gpurun_out/r04_op_band_ab6.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab6.log
timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/r04_slab27_defaults.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/r04_slab7_defaults.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_slab27_defaults.log gpurun_out/r04_slab7_defaults.log | grep -v "^.*RCCL\|HIP ver\|ROCm\|Hostname\|Librccl"
echo done-all
