set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_avail.txt 2>&1 || true
python scripts/tune_march.py --workload stencil27 --n 768 --rounds 1 --reps 1 --configs "default" > /dev/null 2>&1   # warm the code cache
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc27" -o pmc -- python "$GRAFT_REPO_ROOT/scripts/tune_march.py" --workload stencil27 --n 768 --rounds 1 --reps 1 --configs "${C:-default}" > "$GRAFT_REPO_ROOT/gpurun_out/pmc27.log" 2>&1
echo rc=$?
