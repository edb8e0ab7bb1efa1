set -u
# SQ counter passes over the row-band 27-point probe (one config per argument, scripts/probes/rowblock27r.py)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 120 python scripts/probes/rowblock27r.py 768 "$@" > gpurun_out/${TAG:-pmcrb}_0.log 2>&1 || exit $?
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcrb}_$i" -o pmc -- python "$GRAFT_REPO_ROOT/scripts/probes/rowblock27r.py" 768 "$@" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcrb}_$i.log" 2>&1 || exit $?
done
cat "$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcrb}_0.log"
echo done
