export TMPDIR=/tmp
mkdir -p gpurun_out
VB_BWD=0 VB_RAYS=32768 timeout -k 10 300 python scripts/variant_bench.py > gpurun_out/vb_ts.json 2> gpurun_out/vb_ts.err
echo vb rc=$?
