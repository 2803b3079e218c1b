# GPU-box script (r5l): the training forward with the degree-1 bypass (saved1b = SAVECN + SAVED1B) -- z=384 oracle
# tests on it, then cfg5 A/B base | savecn | saved1b, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5l; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
NLDPC_LIB_PATH=$A/saved1b/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/saved1b_tests.log 2>&1 || { echo "saved1b tests failed"; tail -15 $O/saved1b_tests.log; exit 1; }
echo "saved1b z384 tests: $(tail -1 $O/saved1b_tests.log)"
TAG=r5l NOTESTS=1 VARIANTS="lib_ab/base lib_ab/savecn lib_ab/saved1b" bash tools/gpu_ab_cfg5.sh
