# GPU-box script: build and one full-size bench line with the CPU baseline (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python $R/bench.py ${BENCH_ARGS} > $R/gpurun_out/bench.log 2>&1
rc=$?; tail -2 $R/gpurun_out/bench.log; echo "exit $rc"; exit $rc
