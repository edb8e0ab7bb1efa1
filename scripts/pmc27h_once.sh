set -u
# SQ + HBM counter passes over the 27-point fp16 768^3 forward kernel variants (tune_march, one launch per config)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 120 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 1 --reps 1 --configs "${C:-default}" > /dev/null 2>&1 || exit $?
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc27h}_$i" -o pmc -- python "$GRAFT_REPO_ROOT/scripts/tune_march.py" --workload stencil27 --n 768 --rounds 1 --reps 1 --configs "${C:-default}" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc27h}_$i.log" 2>&1 || exit $?
done
echo done
