# GPU-box script (run via gpurun; library built on the CPU side): GPU parity tests, smoke, the cfg3
# bench line, then the Boosted inference side lines (cfg3ucn: MS NW(1,1,2) with UCN, MS NW(1,0,0),
# QMS NW(1,1,2)).  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r2b}
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail 40 -p no:cacheprovider ${PYTEST_ARGS} > $O/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" $O/${TAG}_gpu_tests.log | tail -25
case $rc in 0|1) ;; *) exit $rc ;; esac
[ -n "$NO_SMOKE" ] || { timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?; }
[ -n "$NO_CFG3" ] || { timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/${TAG}_bench_cfg3.log 2>&1 || exit $?; tail -c 600 $O/${TAG}_bench_cfg3.log; }
for spec in "MS 1,1,2" "MS 1,0,0" "QMS 1,1,2"; do
    set -- $spec
    timeout -k 10 300 python -u bench.py --workload cfg3ucn --kind $1 --nw $2 --steps 5 --warmup 2 --no-count-only \
        > $O/${TAG}_bench_ucn_$1_${2//,/}.log 2>&1 || exit $?
    python3 - $O/${TAG}_bench_ucn_$1_${2//,/}.log "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"cfg3ucn {sys.argv[2]:10s} {d['value']:>12.0f} cw/s  kernel {d['roofline']['avg_launch_ms']:.3f} ms")
PY
done
[ -n "$NO_CFG5" ] || { timeout -k 10 600 python -u bench.py --workload cfg5 --steps 10 --warmup 3 > $O/${TAG}_bench_cfg5.log 2>&1 || exit $?;
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cfg5', d['value'], 'cw/s', d['ms_per_step'], 'ms/step')" $O/${TAG}_bench_cfg5.log; }
exit $rc
