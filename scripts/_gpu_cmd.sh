export TMPDIR=/tmp
mkdir -p gpurun_out
VB_BWD=0 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_h64.json 2> gpurun_out/vb_h64.err
echo vb rc=$?
