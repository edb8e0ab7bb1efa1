set -u
# per-rank slab step (scripts/probes/slab_step.py) under halo-exchange scheduling variants
cd "$GRAFT_REPO_ROOT"
for V in "X=1" "PSAD_HALO_PRIORITY=-1" "PSAD_HALO_FACES=halo" "PSAD_HALO_FACES=halo PSAD_HALO_PRIORITY=-1"; do
  echo "== $V" >> gpurun_out/slab_env.log
  env $V timeout -k 10 120 python scripts/probes/slab_step.py 128 2>&1 | grep -E "zslab" >> gpurun_out/slab_env.log || exit 1
done
