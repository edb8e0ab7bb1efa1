set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 300 python scripts/tune_march.py --workload veclap3 --n 384 --rounds 5 --configs "$C" > gpurun_out/${TAG}_384.log 2>&1
cat gpurun_out/${TAG}_384.log | grep -v amdgpu.ids
