# GPU-box script (r5l): the training forward with the degree-1 bypass (savepipe = + the two-buffer schedule) -- z=384 oracle
# tests on it, then cfg5 A/B base | savecn | saved1b, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5m; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
NLDPC_LIB_PATH=$A/saved1b/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/savepipe_tests.log 2>&1 || { echo "savepipe tests failed"; tail -15 $O/savepipe_tests.log; exit 1; }
echo "savepipe z384 tests: $(tail -1 $O/savepipe_tests.log)"
TAG=r5m NOTESTS=1 VARIANTS="lib_ab/saved1b lib_ab/savepipe" bash tools/gpu_ab_cfg5.sh
