set -u
# round 4: which band variants differ bitwise (test_band_chunk_length_and_band_height_bitwise), then check 5's A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 300 python -u -m pytest tests/test_band.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chunk_length_and_band_height or padded_rows" > gpurun_out/r04_pytest6.log 2>&1 || { grep -A12 "^E " gpurun_out/r04_pytest6.log | head -30; tail -3 gpurun_out/r04_pytest6.log; }
tail -2 gpurun_out/r04_pytest6.log
bash scripts/r04_check5.sh
