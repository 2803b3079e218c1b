# GPU-box script: rocprofv3 kernel-trace summary (--kernel-trace --stats) of one bench run.
# Usage (gpurun): TAG=name BENCH_ARGS="--workload cfg5 --steps 3 --warmup 1" bash tools/gpu_trace.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; grep '^{' $O/bench.log | tail -1 | cut -c1-300; echo "exit $rc"; exit $rc
