# GPU-box script: GPU tests, cfg3 bench line, then the phase stamps of the diagnostic build (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 STAMPS=1 > $R/gpurun_out/build_st.log 2>&1 &&
timeout -k 10 600 python -u -m pytest $R/tests -x -q -m gpu --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python $R/bench.py --no-cpu-baseline --no-sweep > $R/gpurun_out/bench_cfg3.log 2>&1 &&
NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_stamps/libnldpc.so NLDPC_STAMPS=$R/gpurun_out/stamps.bin timeout -k 10 300 python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-sweep --batch 16384 --no-profile > $R/gpurun_out/stamps_bench.log 2>&1 &&
python $R/tools/stamps.py $R/gpurun_out/stamps.bin
rc=$?; tail -2 $R/gpurun_out/gpu_tests.log; grep -o '"value": [0-9.]*' $R/gpurun_out/bench_cfg3.log; echo "exit $rc"; exit $rc
