# GPU-box A/B of experiment builds (tools/exp_build.sh): the cfg3 decode kernel time of each variant,
# measured by bench.py with the variant's library.  VARIANTS="base cn4 ..." (lib_exp/<name>).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for v in ${VARIANTS}; do
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_exp/$v/libnldpc.so timeout -k 10 240 python -u bench.py --steps ${STEPS:-6} --warmup 2 \
        --no-cpu-baseline --no-sweep --no-count-only ${BENCH_ARGS} > $O/ab_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/ab_$v.log; exit 1; }
    python3 - $v $O/ab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:12s} {d['value']:>12.0f} cw/s  kernel {d['roofline']['avg_launch_ms']:.3f} ms  median step {d['ms_per_step_median']:.3f} ms")
PY
done
