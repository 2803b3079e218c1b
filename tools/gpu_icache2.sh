# GPU-box script: instruction-cache counters of the cfg5 kernels (saving forward, backward) and of the
# Boosted MS UCN decode kernel (run via gpurun; library built on the CPU side).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r3}
cd /tmp && export TMPDIR=/tmp
P="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace -d $O/${TAG}_ic5 -o run --output-format csv -- \
    python3 $R/bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $O/${TAG}_ic5.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace -d $O/${TAG}_icu -o run --output-format csv -- \
    python3 $R/bench.py --workload cfg3ucn --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-count-only > $O/${TAG}_icu.log 2>&1
rc=$?
python3 $R/tools/sq_summary.py $O/${TAG}_ic5 $O/${TAG}_icu > $O/${TAG}_icache2.txt 2>&1
grep -A5 "fused" $O/${TAG}_icache2.txt
exit $rc
