# GPU-box script: build, GPU parity tests, then the cfg5 training bench line (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -u -m pytest $R/tests -x -q -m gpu --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python $R/bench.py --workload cfg5 --steps 3 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bench_cfg5.log 2>&1
rc=$?; tail -3 $R/gpurun_out/gpu_tests.log; tail -1 $R/gpurun_out/bench_cfg5.log | cut -c1-300; echo "exit $rc"; exit $rc
