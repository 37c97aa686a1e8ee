export TMPDIR=/tmp
mkdir -p gpurun_out/prof/r02h_train_step_pmc
VB_BWD=0 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_h1i.json 2> gpurun_out/vb_h1i.err
echo vb rc=$?
rm -rf pc-nerf_amd/lib/variants
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/r02h_train_step_pmc/pmc_$C -o run -- \
    python3 bench.py --no-cpu-baseline --no-fp32-line --mode train_step --rays 16384 --steps 1 --warmup 0 > gpurun_out/prof/r02h_train_step_pmc/pmc_$C.json 2> gpurun_out/prof/r02h_train_step_pmc/pmc_$C.err
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/compact_pmc.py gpurun_out/prof/r02h_train_step_pmc/pmc_$C
done
echo rc=$?
