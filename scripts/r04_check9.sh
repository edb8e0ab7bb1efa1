set -u
# round 4: band compute barrier as asm with a memory clobber -- determinism, bitwise variants, parity, then BPAD A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 300 python -u scripts/probes/band_determinism.py > gpurun_out/r04_band_det2.log 2>&1 || { tail -20 gpurun_out/r04_band_det2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_band_det2.log
timeout -k 10 900 python -u -m pytest tests/test_band.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r04_pytest9.log 2>&1 || { grep -B2 -A12 "^E " gpurun_out/r04_pytest9.log | head -60; tail -3 gpurun_out/r04_pytest9.log; exit 1; }
tail -2 gpurun_out/r04_pytest9.log
timeout -k 10 600 python -u scripts/probes/op_band_ab.py "s27:768:BPAD=0" "s27:1024:BPAD=0" "s27:512:BPAD=0" "s27:96x768:BPAD=0" "h7:768" "h7:512" > gpurun_out/r04_op_band_ab8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab8.log
echo done-all
