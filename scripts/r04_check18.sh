set -u
# round 4: bench.py's adjoint-slower-than-forward gap vs the allocation sequence; headline A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
for v in bench inplace d_first bench inplace; do
  timeout -k 10 120 python -u scripts/probes/bench_alloc.py $v >> gpurun_out/r04_bench_alloc.log 2>&1 || { tail -5 gpurun_out/r04_bench_alloc.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r04_bench_alloc.log
bash scripts/r04_check17.sh
