# GPU-box script (run via gpurun; the library is built on the CPU side and travels with the tree):
# GPU parity tests, smoke, then the default bench line.  Every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r2}
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail 40 -p no:cacheprovider > $O/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/${TAG}_gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/${TAG}_bench.log 2>&1
rc=$?; tail -c 3000 $O/${TAG}_bench.log; exit $rc
