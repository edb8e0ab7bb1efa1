set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
C="${C:-default}"
TAG="${TAG:-ab27}"
timeout -k 10 300 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 5 --configs "$C" > gpurun_out/${TAG}_768.log 2>&1 && \
timeout -k 10 200 python scripts/tune_march.py --workload stencil27 --shape 96,768,768 --rounds 5 --configs "$C" > gpurun_out/${TAG}_slab8.log 2>&1
cat gpurun_out/${TAG}_768.log gpurun_out/${TAG}_slab8.log | grep -v amdgpu.ids
