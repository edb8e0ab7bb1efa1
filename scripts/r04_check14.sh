set -u
# round 4: fp32 star stencils on 8-row bands by default (rows <= 768): parity (band + parity suites), then A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 900 python -u -m pytest tests/test_band.py tests/test_gpu_parity.py tests/test_native_autograd.py -m gpu -q --timeout 250 --timeout-method thread > gpurun_out/r04_pytest14.log 2>&1 || { grep -B2 -A12 "^E " gpurun_out/r04_pytest14.log | head -50; tail -3 gpurun_out/r04_pytest14.log; exit 1; }
tail -2 gpurun_out/r04_pytest14.log
timeout -k 10 600 python -u scripts/probes/op_band_ab.py "f7:512:BAND=4,BTY=8,ZMIN=8,ZMAX=8:BAND=4,BTY=8,ZMIN=32,ZMAX=32" "f7:768:BAND=4,BTY=8,ZMIN=8,ZMAX=8" "f7:510" "f7:256" > gpurun_out/r04_op_f7_ab4.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_f7_ab4.log
