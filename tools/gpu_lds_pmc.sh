# GPU-box script (r3): SQ / LDS counters of the cfg3 decode kernel (Neural, B=16384), one rocprofv3
# --pmc pass per group (groups separated by ';' in $GROUPS_, each within the hardware's per-block
# limits), plus the list of available counters.  Usage: TAG=name GROUPS_="A B;C D" bash tools/gpu_lds_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
T=${TAG:-r3lds}
cd /tmp && export TMPDIR=/tmp
[ -f $O/r3_counters_avail.txt ] || timeout -k 10 120 rocprofv3 -L > $O/r3_counters_avail.txt 2>&1 || true
ARGS="--steps 2 --warmup 1 --batch 16384 --no-cpu-baseline --no-profile --no-sweep --no-count-only ${BENCH_ARGS}"
IFS=';' read -ra GS <<< "${GROUPS_}"
i=0
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $O/${T}_g$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/${T}_g$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -3 $O/${T}_g$i.log; exit 1; }
done
python3 $R/tools/sq_summary.py $O/${T}_g* > $O/${T}_summary.txt 2>&1
grep -A16 "fused_bg2_z384::kernel<3, 0>" $O/${T}_summary.txt
