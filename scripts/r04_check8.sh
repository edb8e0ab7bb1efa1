set -u
# round 4: run-to-run determinism of the band variants (padded image rows)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 300 python -u scripts/probes/band_determinism.py > gpurun_out/r04_band_det.log 2>&1 || { tail -20 gpurun_out/r04_band_det.log; exit 1; }
timeout -k 10 300 python -u scripts/probes/band_determinism.py 37,48,256 >> gpurun_out/r04_band_det.log 2>&1 || { tail -20 gpurun_out/r04_band_det.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_band_det.log
