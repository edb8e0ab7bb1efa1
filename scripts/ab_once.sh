set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
C="${C:-default}"
TAG="${TAG:-ab}"
timeout -k 10 300 python scripts/tune_march.py --n 1024 --rounds 5 --configs "$C" > gpurun_out/${TAG}_1024.log 2>&1 && \
timeout -k 10 200 python scripts/tune_march.py --n 512 --rounds 5 --configs "$C" > gpurun_out/${TAG}_512.log 2>&1 && \
timeout -k 10 200 python scripts/tune_march.py --shape 128,1024,1024 --rounds 5 --configs "$C" > gpurun_out/${TAG}_slab8.log 2>&1
cat gpurun_out/${TAG}_1024.log gpurun_out/${TAG}_512.log gpurun_out/${TAG}_slab8.log | grep -v amdgpu.ids
