set -u
# new fp32 WS default (CX=2,NR=8,D=2 + one-workgroup-per-CU rounds) vs the previous default tile across shapes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
rm -f gpurun_out/tile_b2.log
for S in 1024,1024,1024 768,768,768 640,640,640 512,512,512 384,384,384 128,1024,1024 256,1024,1024 96,768,768; do
  echo "== $S" >> gpurun_out/tile_b2.log
  timeout -k 10 150 python scripts/tune_march.py --shape $S --rounds 5 --configs "default;CX=4,NR=4,D=4;default" 2>&1 | grep -E "^tune|torch.mul" >> gpurun_out/tile_b2.log || exit 1
done
cat gpurun_out/tile_b2.log
