# One GPU call: fb_diag.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/fb_diag.py pcnerf original > gpurun_out/fb_diag.log 2>&1
rc=$?
cat gpurun_out/fb_diag.log | grep -v amdgpu.ids
exit $rc
