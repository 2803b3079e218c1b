# GPU-box script: the GPU parity tests only (library built on the CPU side).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r2}
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail 40 -p no:cacheprovider ${PYTEST_ARGS} > $O/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" $O/${TAG}_gpu_tests.log | tail -25; exit $rc
