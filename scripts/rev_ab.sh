# bench train_fwd under several tile-reversal masks (PCNERF_TILE_REV), one line each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rev
for m in ${MASKS:-0xAA 0x00 0x52 0x54 0xA2 0x2A}; do
  PCNERF_TILE_REV=$m timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-line \
    > gpurun_out/rev/$m.json 2> gpurun_out/rev/$m.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/rev/$m.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$m', d['ms_per_step'], {n: k[n]['avg_us'] for n in ('train_hidden','train_skip','train_first','train_out')})"
done
