set -u
# broad tile sweep of the 27-point fp16 forward (768^3 and the 8-GPU slab)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 500 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 3 --configs-file scripts/tune_cfgs_27d.txt > gpurun_out/sweep27_768.log 2>&1 && \
timeout -k 10 400 python scripts/tune_march.py --workload stencil27 --shape 96,768,768 --rounds 3 --configs-file scripts/tune_cfgs_27d.txt > gpurun_out/sweep27_slab8.log 2>&1
grep -E "^tune" gpurun_out/sweep27_768.log | sort -k4 -n | head -8
grep -E "^tune" gpurun_out/sweep27_slab8.log | sort -k4 -n | head -8
