# GPU-box script (r3): parity tests of the in-tree library, then an A/B of experiment builds
# (VARIANTS, lib_exp/<name>) on the cfg3 bench, then the stamps of STAMPS_LIB if given.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
T=${TAG:-r3}
if [ -z "$NO_TESTS" ]; then
  rm -f $O/${T}_sp_log.txt
  NLDPC_SP_LOG=$O/${T}_sp_log.txt timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1
  rc=$?; tail -3 $O/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${VARIANTS}; do
  NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_exp/$v/libnldpc.so timeout -k 10 240 python -u bench.py --steps ${STEPS:-6} --warmup 2 \
      --no-cpu-baseline --no-sweep --no-count-only ${BENCH_ARGS} > $O/${T}_ab_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/${T}_ab_$v.log; exit 1; }
  python3 - $v $O/${T}_ab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:14s} {d['value']:>12.0f} cw/s  kernel {d['roofline']['avg_launch_ms']:.3f} ms  median step {d['ms_per_step_median']:.3f} ms")
PY
done
if [ -n "$STAMPS_LIB" ]; then
  NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_exp/$STAMPS_LIB/libnldpc.so NLDPC_STAMPS=$O/${T}_stamps.bin timeout -k 10 300 python bench.py --steps 1 --warmup 1 \
      --no-cpu-baseline --no-sweep --no-count-only --batch 16384 --no-profile > $O/${T}_stamps_bench.log 2>&1 || exit 1
  python tools/stamps2.py $O/${T}_stamps.bin VN "VN+W0" "CN0+W1" "R0+CN1" "W2+R1" "CN2+W3" "R2+CN3" "R3"
fi
