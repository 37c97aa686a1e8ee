# variant_bench.py (train query + backward per tag) over the variant libraries in VB_ONLY
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/vb
timeout -k 10 400 python -u scripts/variant_bench.py > gpurun_out/vb/vb.json 2> gpurun_out/vb/vb.err
rc=$?; cat gpurun_out/vb/vb.json; tail -3 gpurun_out/vb/vb.err; echo "vb rc=$rc"; exit $rc
