# Generic variant-library A/B (pc-nerf_amd/lib/variants/*.so): the backward / config GPU tests on the default
# library, then ROUNDS interleaved short training-step benches per variant; prints ms per step and the bench's
# per-tag kernel averages named in KEYS (comma-separated, bench.py 'kernels' keys)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
KEYS=${KEYS:-bwd_fused,bwd_other}
ROUNDS=${ROUNDS:-3}
mkdir -p gpurun_out/libab
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_backward_gpu.py \
  tests/test_configs_gpu.py -k "fused or config3 or trajectory" > gpurun_out/libab/pytest.log 2>&1 || { tail -30 gpurun_out/libab/pytest.log; exit 1; }
tail -1 gpurun_out/libab/pytest.log
for r in $(seq 1 $ROUNDS); do
  for so in pc-nerf_amd/lib/variants/*.so; do
    v=$(basename $so .so); v=${v#libpcnerf_}
    PCNERF_HIP_LIB=$PWD/$so timeout -k 10 120 python3 bench.py --mode train_step --rays 16384 --steps 3 --warmup 1 \
      --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline > gpurun_out/libab/$v.$r.json 2> gpurun_out/libab/$v.$r.err
    rc=$?; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json; d=json.loads(open('gpurun_out/libab/$v.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', $r, d['ms_per_step'], {n: k[n]['avg_us'] for n in '$KEYS'.split(',') if n in k})"
  done
done
