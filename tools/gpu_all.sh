# GPU-box script: build, GPU parity tests, then the bench lines of every GPU workload (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -m pytest $R/tests -x -q -m gpu > $R/gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python $R/bench.py > $R/gpurun_out/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/bench_cfg2.log 2>&1 &&
timeout -k 10 600 python $R/bench.py --workload cfg5 --steps 3 --warmup 1 > $R/gpurun_out/bench_cfg5.log 2>&1
rc=$?; tail -3 $R/gpurun_out/gpu_tests.log; echo "exit $rc"; exit $rc
