set -u
# round 4: band schedule A/B through the op (peeled chunk-edge planes, chunk lengths) + parity + LDS bank-conflict pass
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 400 python -u -m pytest tests/test_band.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_band_pytest.log 2>&1 || { tail -30 gpurun_out/r04_band_pytest.log; exit 1; }
tail -2 gpurun_out/r04_band_pytest.log
timeout -k 10 300 python -u scripts/probes/op_band_ab.py "s27:768:BTRIM=1:BTRIM=1,ZMIN=32,ZMAX=32:BTRIM=1,ZMIN=24,ZMAX=24:BTRIM=1,ZMIN=16,ZMAX=16:BTRIM=2,ZMIN=16,ZMAX=16:ZMIN=24,ZMAX=24:BTRIM=2,ZMIN=24,ZMAX=24" > gpurun_out/r04_op_band_ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab1.log
timeout -k 10 300 python -u scripts/probes/op_band_ab.py "s27:1024:BTRIM=1:BTRIM=1,ZMIN=32,ZMAX=32:BTRIM=1,ZMIN=24,ZMAX=24" "h7:768:BTRIM=1:BTRIM=1,ZMIN=16,ZMAX=16" > gpurun_out/r04_op_band_ab2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04_op_band_ab2.log
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04_pmc_lds" -o pmc -- python "$GRAFT_REPO_ROOT/bench.py" --workload stencil27_f16 --secondary none --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r04_pmc_lds.log" 2>&1 || exit 1
echo done
