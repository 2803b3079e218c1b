# GPU-box script (r5k): the in-tree library (UREMAT) -- GPU suite, smoke; cfg5 A/B base | lib | savecn (check-node
# threads store the saved v2c); z=384 oracle tests on savecn; cfg5 PMC passes on lib; phase stamps of the training
# forward (lib_ab/st_save, a stamp build).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5k; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
NLDPC_LIB_PATH=$A/savecn/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/savecn_tests.log 2>&1 || { echo "savecn tests failed"; tail -15 $O/savecn_tests.log; exit 1; }
echo "savecn z384 tests: $(tail -1 $O/savecn_tests.log)"
TAG=r5k NOTESTS=1 VARIANTS="lib_ab/base lib lib_ab/savecn" bash tools/gpu_ab_cfg5.sh || exit 1
NLDPC_LIB_PATH=$A/st_save/libnldpc.so NLDPC_STAMPS=$O/stamps_save.bin timeout -k 10 300 python -u bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $O/stamps_bench.log 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_bench.log; exit 1; }
python tools/stamps2.py $O/stamps_save.bin > $O/stamps_save.txt && head -20 $O/stamps_save.txt
TAG=r5k NOTESTS=1 ROUNDS=0 PMC=1 bash tools/gpu_ab_cfg5.sh
