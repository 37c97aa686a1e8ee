# k_bwd_fused A/B across variant libraries (pc-nerf_amd/lib/variants/*.so): one short training-step bench per variant,
# interleaved rounds; prints the fused kernel's average launch time per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fbab
for r in 1 2 3; do
  for so in pc-nerf_amd/lib/variants/*.so; do
    v=$(basename $so .so); v=${v#libpcnerf_}
    PCNERF_HIP_LIB=$PWD/$so timeout -k 10 120 python3 bench.py --mode train_step --rays 16384 --steps 3 --warmup 1 \
      --no-extra --no-ceiling --no-fp32-line --no-cpu-baseline > gpurun_out/fbab/$v.$r.json 2> gpurun_out/fbab/$v.$r.err
    rc=$?; [ $rc -ne 0 ] && exit $rc
    python3 -c "import json; d=json.loads(open('gpurun_out/fbab/$v.$r.json').read().strip().splitlines()[-1]); k=d['kernels']['bwd_fused']; print('$v', $r, k['avg_us'], d['ms_per_step'])"
  done
done
