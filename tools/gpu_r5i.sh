# GPU-box script (r5i): UREMAT (lane offsets re-derived per phase in the SAVE kernels, buffer-descriptor saves):
# z=384 oracle + stateful tests on it, then cfg5 A/B against lib_ab/base (interleaved, 2 rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5i; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
NLDPC_LIB_PATH=$A/urm/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/urm_tests.log 2>&1 || { echo "urm tests failed"; tail -15 $O/urm_tests.log; exit 1; }
echo "urm tests: $(tail -1 $O/urm_tests.log)"
TAG=r5i NOTESTS=1 VARIANTS="lib_ab/base lib_ab/urm" bash tools/gpu_ab_cfg5.sh
