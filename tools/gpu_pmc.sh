# GPU-box script: PMC counters of one bench workload, one rocprofv3 --pmc pass per counter group (groups separated
# by ';' in GROUPS_, each within the hardware's per-block limits; --kernel-trace only beside --pmc), summarised by
# tools/pmc_summary.py (FETCH_SIZE / WRITE_SIZE -> bytes per launch) and tools/sq_summary.py (everything else).
# Usage (gpurun): TAG=name BENCH_ARGS="--workload cfg5 --steps 2 --warmup 1" GROUPS_="FETCH_SIZE;WRITE_SIZE" \
#   [NLDPC_LIB_PATH=...] bash tools/gpu_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-pmc}; mkdir -p $O
GROUPS_=${GROUPS_:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"}
ARGS="--no-cpu-baseline --no-profile --no-sweep --no-count-only ${BENCH_ARGS:---steps 2 --warmup 1}"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra GS <<< "${GROUPS_}"
i=0
for grp in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $grp --kernel-trace -d $O/g$i -o run --output-format csv -- \
      python3 $R/bench.py $ARGS > $O/g$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -3 $O/g$i.log; exit 1; }
done
python3 $R/tools/sq_summary.py $O/g* > $O/summary.txt 2>&1
cat $O/summary.txt | cut -c1-220
