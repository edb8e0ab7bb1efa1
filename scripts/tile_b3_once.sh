set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
rm -f gpurun_out/tile_b3.log
O="CX=4,NR=4,D=4"
for S in 256,1024,1024 768,768,768; do
  echo "== $S" >> gpurun_out/tile_b3.log
  timeout -k 10 150 python scripts/tune_march.py --shape $S --rounds 7 --configs "default;$O;ZC=64;ZC=48;$O,ZC=110;default;$O" 2>&1 | grep -E "^tune|torch.mul" >> gpurun_out/tile_b3.log || exit 1
done
cat gpurun_out/tile_b3.log
