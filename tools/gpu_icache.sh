# GPU-box script: instruction-cache and issue-stall counters of the cfg3 fused kernel (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
ARGS="--steps 1 --warmup 1 --batch 16384 --no-cpu-baseline --no-profile --no-sweep"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-trace -d $R/gpurun_out/ic_g1 -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/ic_g1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/ic_g2 -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/ic_g2.log 2>&1
rc=$?
python3 $R/tools/sq_summary.py $R/gpurun_out/ic_g1 $R/gpurun_out/ic_g2 2>&1 | grep -A14 "fused"
exit $rc
