# rocprofv3 passes for one bench workload: a --kernel-trace --stats pass, then one PMC pass per counter group
# (FETCH_SIZE and WRITE_SIZE in passes of their own: MI355X_MICROARCH.md rocprofv3 slot limits; each PMC pass
# runs one step, no warmup, whatever steps the stats pass was given); outputs under
# gpurun_out/prof/<tag>.   usage: bash scripts/profile.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}; shift
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
# heartbeat: PMC passes of a long workload print nothing for minutes
( while sleep 50; do date +%s >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
echo "python3 bench.py --no-cpu-baseline --no-fp32-line $*" > $OUT/command.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-fp32-line --detail $OUT/stats_detail.json "$@" > $OUT/stats_bench.json 2> $OUT/stats.err
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -f $OUT/stats/*kernel_trace.csv   # per-dispatch trace: the stats file carries the averages
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$N -o run -- \
    python3 bench.py --no-cpu-baseline --no-fp32-line --detail "" "$@" --steps 1 --warmup 0 > $OUT/pmc_$N.json 2> $OUT/pmc_$N.err
  rc=$?; echo "pmc $N rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 scripts/compact_pmc.py $OUT/pmc_$N
done
exit 0
