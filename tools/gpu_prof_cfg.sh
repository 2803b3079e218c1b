# GPU-box script: rocprofv3 kernel-trace summary of one bench workload (run via gpurun).
# Usage: TAG=name BENCH_ARGS="--workload cfg5 --steps 3 --warmup 1" bash tools/gpu_prof_cfg.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
TAG=${TAG:-prof}
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG} -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/${TAG}.log 2>&1
rc=$?; tail -1 $R/gpurun_out/${TAG}.log | cut -c1-300; echo "exit $rc"; exit $rc
