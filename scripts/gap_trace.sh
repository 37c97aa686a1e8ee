# rocprofv3 kernel trace of one bench line, kept whole (for idle-gap analysis: scripts/gaps.py)
# usage: bash scripts/gap_trace.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-gaps}; shift
OUT=gpurun_out/trace/$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 bench.py --no-cpu-baseline --no-fp32-line --no-ceiling --no-extra "$@" > $OUT/bench.json 2> $OUT/bench.err
