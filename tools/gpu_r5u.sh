# GPU-box script (r5u): backward staging through a buffer descriptor (stageb) -- z=384 oracle tests, gradient digests
# (lib, stageb), cfg5 A/B lib | stageb interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5u; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
NLDPC_LIB_PATH=$A/stageb/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/stageb_tests.log 2>&1 || { echo "stageb tests failed"; tail -15 $O/stageb_tests.log; exit 1; }
echo "stageb z384 tests: $(tail -1 $O/stageb_tests.log)"
TAG=r5u VARIANTS="lib lib_ab/stageb" bash tools/gpu_digest.sh || exit 1
TAG=r5u NOTESTS=1 VARIANTS="lib lib_ab/stageb" bash tools/gpu_ab_cfg5.sh
