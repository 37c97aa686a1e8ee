# Same-box A/B of variant libraries (pc-nerf_amd/lib/variants/*.so) on the full train_step and config3 bench lines
# (the default sizes): ROUNDS interleaved runs per variant; prints ms per step and the backward kernel averages
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUNDS=${ROUNDS:-2}
mkdir -p gpurun_out/libab_full
for r in $(seq 1 $ROUNDS); do
  for so in pc-nerf_amd/lib/variants/*.so; do
    v=$(basename $so .so); v=${v#libpcnerf_}
    PCNERF_HIP_LIB=$PWD/$so timeout -k 10 200 python3 bench.py --mode train_step --steps 3 --warmup 1 \
      --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline > gpurun_out/libab_full/$v.ts.$r.json 2> gpurun_out/libab_full/$v.ts.$r.err
    rc=$?; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json; d=json.loads(open('gpurun_out/libab_full/$v.ts.$r.json').read().strip().splitlines()[-1]); print('$v train_step', $r, d['value'], d['ms_per_step'])"
  done
done
