set -u
# 7-point fp32 forward at power-of-two and other cube edges / slabs: defaults vs fixed chunk lengths
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
rm -f gpurun_out/odd.log
for S in 1024,1024,1024 512,512,512 128,1024,1024 768,768,768 640,640,640 384,384,384 256,1024,1024 96,768,768; do
  echo "== $S" >> gpurun_out/odd.log
  timeout -k 10 150 python scripts/tune_march.py --shape $S --rounds 5 --configs "${C:-default;ZC=128}" 2>&1 | grep -E "^tune|torch.mul" >> gpurun_out/odd.log || exit 1
done
cat gpurun_out/odd.log
