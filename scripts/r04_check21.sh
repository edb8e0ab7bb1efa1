set -u
# round 4: 27-point row-pitch cliff — masked stores (ragged Y) vs partial rows (X % 8) vs aligned non-power-of-two X
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
L=gpurun_out/r04_op_pitch27.log
for s in s27:512 s27:512x510x512 s27:512x512x510 s27:512x512x520 s27:512x512x504 s27:510 s27:512x512x511 s27:256 s27:256x256x255 s27:256x255x256; do
  timeout -k 10 200 python -u scripts/probes/op_band_ab.py $s >> $L 2>&1 || { tail -5 $L; exit 1; }
done
grep -v amdgpu.ids $L
