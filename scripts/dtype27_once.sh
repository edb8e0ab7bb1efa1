set -u
# Is the 27-point fp16 sweep's ~5 TB/s a property of fp16 storage or of the 27-point box? Same 768^3 grid:
# 7-point fp32 / fp16, 27-point fp32 / fp16, default schedules (each tune_march run prints its own copy refs).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-dt27}"
for w in diffusion7 diffusion7_f16 stencil27_f32 stencil27; do
  timeout -k 10 200 python scripts/tune_march.py --workload $w --n 768 --rounds 5 --configs "default;default" > gpurun_out/${TAG}_$w.log 2>&1 || exit $?
  echo "== $w"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$w.log
done
