# GPU-box script: build, small + full bench, rocprofv3 kernel-trace summary (run via gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python $R/bench.py --batch 4096 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_small.log 2>&1 &&
timeout -k 10 600 python $R/bench.py > $R/gpurun_out/bench_full.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1
echo "exit $?"
