set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
for S in 512,512,512 768,768,768 1024,512,512 512,1024,512 512,512,1024 256,1024,1024 384,384,384; do
  echo "== $S" >> gpurun_out/aux_shapes.log
  timeout -k 10 120 python scripts/tune_march.py --shape $S --rounds 5 --configs "default;DMA_AUX=2;default;DMA_AUX=2" 2>&1 | grep -E "^tune|torch.mul" >> gpurun_out/aux_shapes.log || exit 1
done
