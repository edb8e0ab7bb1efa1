set -u
# Which of {fp16 storage, 27-point box, the 768 extent} holds the sweeps below the copy rate?
# 1024^3: 7-point fp32 / fp16, 27-point fp32 / fp16 (default + larger tiles); 768^3 7-point fp32 tile variants.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-sd}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --n $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$1_$2.log; }
run diffusion7 1024 "default"
run diffusion7_f16 1024 "default;NR=8;default"
run stencil27_f32 1024 "default"
run stencil27 1024 "default;NR=4,D=4,ZC=128;NR=4,ZC=64;default"
run diffusion7 768 "default;CX=2;NR=2;ZC=64;CX=2,ZC=64;CX=2,NR=8;default"
