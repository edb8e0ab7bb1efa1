set -u
# round 4: compute-side zero past row ends (BZF=0) parity + A/B, new defaults (box: padded rows; star: 64-plane
# chunks at <= 512), where the padded-row variant differs bitwise
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 600 python -u -m pytest tests/test_band.py -m gpu -q --timeout 200 --timeout-method thread -k "chunk_length_and_band_height or register_zero or unaligned_vs_oracle" > gpurun_out/r04_pytest7.log 2>&1 || { grep -B2 -A12 "^E " gpurun_out/r04_pytest7.log | head -60; tail -3 gpurun_out/r04_pytest7.log; }
tail -2 gpurun_out/r04_pytest7.log
timeout -k 10 600 python -u scripts/probes/op_band_ab.py "s27:510:BZF=0" "s27:511:BZF=0" "s27:255:BZF=0" "s27:766:BZF=0" "h7:510:BZF=0" "h7:511:BZF=0" "s27:512" "h7:512" "s27:256" "s27:768:BPAD=0" > gpurun_out/r04_op_band_ab7.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab7.log
echo done-all
