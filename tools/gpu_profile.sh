# GPU-box script: rocprofv3 kernel-trace summary + HBM traffic counters of the bench (run via gpurun).
# Counters are collected in their own passes (FETCH_SIZE and WRITE_SIZE cannot share one pass),
# with --kernel-trace/--stats only, as MI355X_MICROARCH.md §rocprofv3 prescribes.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
TAG=${TAG:-r1}
ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_${TAG}_trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/prof_${TAG}_fetch -o run --output-format csv -- python3 $R/bench.py $ARGS --no-profile > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/prof_${TAG}_write -o run --output-format csv -- python3 $R/bench.py $ARGS --no-profile > $R/gpurun_out/prof_${TAG}_write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU --kernel-trace -d $R/gpurun_out/prof_${TAG}_sq -o run --output-format csv -- python3 $R/bench.py $ARGS --no-profile > $R/gpurun_out/prof_${TAG}_sq.log 2>&1
rc=$?; echo "exit $rc"; exit $rc
