set -u
# z-chunk length sweep on the per-rank slabs of the multi-GPU configs (wave quantisation of the grid)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-zcslab}"
C27="${C27:-default;ZC=12;ZC=14;ZMIN=12;ZMIN=8;BLK=4096;BLK=3072}"
timeout -k 10 200 python scripts/tune_march.py --workload stencil27 --shape 96,768,768 --rounds 5 \
  --configs "$C27" > gpurun_out/${TAG}_27slab8.log 2>&1 && \
timeout -k 10 200 python scripts/tune_march.py --workload stencil27 --shape 192,768,768 --rounds 5 \
  --configs "$C27" > gpurun_out/${TAG}_27slab4.log 2>&1 && \
timeout -k 10 300 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 5 \
  --configs "$C27" > gpurun_out/${TAG}_27full.log 2>&1
cat gpurun_out/${TAG}_*.log | grep -v amdgpu.ids | grep -E "^tune|mul"
