set -u
# 27-point fp16 half ring at 1024^3: tiles 256 wide (default) vs 512 / 1024 wide made of waves side by side
# (WX), i.e. 512-B vs 1-2 KB contiguous row segments per load / store, same lane work (CX=4).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-wx27}"
C="default;CX=4,WX=2,NR=2,ZC=24;CX=4,WX=2,NR=4,ZC=24;CX=4,WX=4,NR=4,ZC=24;CX=4,WX=4,NR=2,ZC=24;CX=4,WX=1,NR=4,ZC=24;default"
timeout -k 10 400 python scripts/tune_march.py --workload stencil27 --n 1024 --rounds 5 --configs "$C" > gpurun_out/${TAG}_1024.log 2>&1
grep -v amdgpu.ids gpurun_out/${TAG}_1024.log
