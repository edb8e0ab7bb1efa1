set -u
# SQ counter passes (separate runs, --pmc only) over bench.py's 27-point fp16 768^3 step on the row-band schedule,
# then the one-GPU loopback proxy of the N=8 slab step (scripts/probes/slab_step.py) for both configs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 200 python bench.py --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcband_0.log 2>&1 || exit $?
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmcband_$i" -o pmc -- python "$GRAFT_REPO_ROOT/bench.py" --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/pmcband_$i.log" 2>&1 || exit $?
done
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u scripts/probes/slab_step.py 96 stencil27 > gpurun_out/slab27_r03f.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/probes/slab_step.py 128 diffusion7 > gpurun_out/slab7_r03f.log 2>&1 || exit $?
cat gpurun_out/slab27_r03f.log gpurun_out/slab7_r03f.log | grep -v amdgpu.ids
echo done
