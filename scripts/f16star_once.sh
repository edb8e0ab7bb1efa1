set -u
# fp16 star stencils (7-point, half-precision ring): 256x32 tiles (NR=8) vs the fp32-tuned 256x16 default
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-f16s}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 ${2} --rounds 4 --configs "$3" > gpurun_out/${TAG}_$4.log 2>&1 || exit $?; echo "== $4"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$4.log; }
run diffusion7_f16 "--n 512" "default;NR=8;NR=6;default" 512
run diffusion7_f16 "--n 768" "default;NR=8;NR=6;NR=8,ZC=64;default" 768
run diffusion7_f16 "--n 1024" "default;NR=8;NR=8,D=3;default" 1024
run diffusion7_f16 "--shape 128,1024,1024" "default;NR=8;default" slab8
run diffusion7_f16 "--shape 200,300,260" "default;NR=8;default" odd
