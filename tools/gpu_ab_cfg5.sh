# GPU-box A/B of cfg5 (training step) between libraries: VARIANTS="lib_ab/base lib" (directories under
# neural-ldpc-decoder-torch_amd/ holding a libnldpc.so), interleaved ROUNDS times; prints the saving
# forward, the backward and the median step per run.  Then (unless NOTESTS) the GPU suite on the in-tree
# library and (PMC=1) FETCH_SIZE / WRITE_SIZE passes of cfg5 on it.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-ab5}; mkdir -p $O
cd $R
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in ${VARIANTS}; do
    n=${v//\//_}
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so timeout -k 10 300 python -u bench.py --workload cfg5 \
        --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/ab_${n}_$rnd.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/ab_${n}_$rnd.log; exit 1; }
    python3 - $v $O/ab_${n}_$rnd.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
pk = d["roofline"]["per_kernel"]
print(f"{sys.argv[1]:14s} forward {pk['fused']['avg_ms']:.3f} ms  backward {pk['fusedb']['avg_ms']:.3f} ms  "
      f"median step {d['ms_per_step_median']:.3f} ms  loss {d['loss']}")
PY
done
done
if [ -z "$NOTESTS" ]; then
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -15 $O/gpu_tests.log; exit 1; }
    tail -1 $O/gpu_tests.log
fi
if [ -n "$PMC" ]; then
    cd /tmp && export TMPDIR=/tmp
    B="python3 $R/bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline --no-profile"
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/cfg5_fetch -o run --output-format csv -- $B > $O/cfg5_fetch.log 2>&1 &&
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/cfg5_write -o run --output-format csv -- $B > $O/cfg5_write.log 2>&1 &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg5_trace -o run --output-format csv -- $B > $O/cfg5_trace.log 2>&1 || { echo "pmc failed"; exit 1; }
    echo "pmc done"
fi
