set -u
# round 4: CU-masked slab sweeps (PSAD_SLAB_CUMASK=K: exchange + faces on K CUs, the interior on the others)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -q --timeout 250 --timeout-method thread -k "native or loopback" > gpurun_out/r04_pytest15.log 2>&1 || { tail -30 gpurun_out/r04_pytest15.log; exit 1; }
PSAD_SLAB_CUMASK=16 timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -q --timeout 250 --timeout-method thread -k "native or loopback" >> gpurun_out/r04_pytest15.log 2>&1 || { tail -30 gpurun_out/r04_pytest15.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04_pytest15.log
for K in 0 8 16 32; do
  for W in "96 stencil27" "128 diffusion7"; do
    PSAD_SLAB_CUMASK=$K timeout -k 10 200 python -u scripts/probes/slab_step.py $W > gpurun_out/r04_slab_cumask.tmp 2>&1 || { tail -20 gpurun_out/r04_slab_cumask.tmp; exit 1; }
    echo "== PSAD_SLAB_CUMASK=$K slab_step.py $W" >> gpurun_out/r04_slab_cumask.log
    grep -E "plain op|native faces on halo" gpurun_out/r04_slab_cumask.tmp >> gpurun_out/r04_slab_cumask.log
  done
done
cat gpurun_out/r04_slab_cumask.log
