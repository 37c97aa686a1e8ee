export TMPDIR=/tmp
mkdir -p gpurun_out
VB_BWD=1 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_wred.json 2> gpurun_out/vb_wred.err
echo vb rc=$?
