# GPU-box script: build, GPU parity tests, then one full-size bench line (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -m pytest $R/tests -x -q -m gpu > $R/gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python $R/bench.py --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/bench_quick.log 2>&1
rc=$?; tail -3 $R/gpurun_out/gpu_tests.log; echo "exit $rc"; exit $rc
