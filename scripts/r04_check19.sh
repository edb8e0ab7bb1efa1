set -u
# round 4: staged aligned-DMA loader for partial rows (BREG=2): parity, then A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 600 python -u -m pytest tests/test_band.py -m gpu -q --timeout 200 --timeout-method thread -k "unaligned_variants and BREG2" > gpurun_out/r04_pytest19.log 2>&1 || { grep -B2 -A12 "^E " gpurun_out/r04_pytest19.log | head -50; tail -3 gpurun_out/r04_pytest19.log; exit 1; }
tail -2 gpurun_out/r04_pytest19.log
timeout -k 10 600 python -u scripts/probes/op_band_ab.py "s27:510:BREG=2:BREG=2,D=1" "s27:511:BREG=2:BREG=2,D=1" "s27:255:BREG=2:BREG=2,D=1" "s27:766:BREG=2,D=1" "h7:510:BREG=2:BREG=2,D=1" "s27:512" > gpurun_out/r04_op_band_ab11.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab11.log
