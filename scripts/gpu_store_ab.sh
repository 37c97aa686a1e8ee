# Store-writing train query A/B across variant libraries (pc-nerf_amd/lib/variants/*.so): the backward / config
# GPU tests on the default library first, then fused_ab.py with the store written (FA_STORE=1) and one short
# training-step bench per variant, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/stab
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_backward_gpu.py \
  tests/test_configs_gpu.py -k "fused or config3 or trajectory" > gpurun_out/stab/pytest.log 2>&1 || { tail -30 gpurun_out/stab/pytest.log; exit 1; }
tail -3 gpurun_out/stab/pytest.log
FA_STORE=1 FA_ROUNDS=6 timeout -k 10 240 python3 scripts/fused_ab.py > gpurun_out/stab/fused_ab.json || exit 1
cat gpurun_out/stab/fused_ab.json
for r in 1 2; do
  for so in pc-nerf_amd/lib/variants/*.so; do
    v=$(basename $so .so); v=${v#libpcnerf_}
    PCNERF_HIP_LIB=$PWD/$so timeout -k 10 120 python3 bench.py --mode train_step --rays 16384 --steps 3 --warmup 1 \
      --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline > gpurun_out/stab/$v.$r.json 2> gpurun_out/stab/$v.$r.err
    rc=$?; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json; d=json.loads(open('gpurun_out/stab/$v.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', $r, d['ms_per_step'], {n: k[n]['avg_us'] for n in k if 'query' in n})"
  done
done
