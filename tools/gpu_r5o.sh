# GPU-box script (r5o): tied-weight backward with per-row epilogue masks (samew) -- z=384 oracle tests on it, then
# cfg5 A/B against the in-tree library, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5o; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
NLDPC_LIB_PATH=$A/samew2/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/samew_tests.log 2>&1 || { echo "samew tests failed"; tail -15 $O/samew_tests.log; exit 1; }
echo "samew2 z384 tests: $(tail -1 $O/samew_tests.log)"
TAG=r5o NOTESTS=1 VARIANTS="lib lib_ab/samew lib_ab/samew2" bash tools/gpu_ab_cfg5.sh
