# GPU-box A/B of experiment builds (tools/exp_build.sh): for each variant, the fused kernels checked bit for
# bit against the streaming kernels of the same library (tools/ab_check.py), then the cfg3 decode kernel
# time measured by bench.py with the variant's library.  VARIANTS="lib_ab/base lib_ab/cn4 ..." (directories under
# neural-ldpc-decoder-torch_amd/ holding a libnldpc.so: copy lib_exp/<name>/libnldpc.so there -- lib_exp/ does not travel);
# ROUNDS=2 runs the whole list twice (interleaved, to see box drift).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-ab}; mkdir -p $O
cd $R
for rnd in $(seq 1 ${ROUNDS:-1}); do
for v in ${VARIANTS}; do
    L=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so
    n=${v//\//_}
    if [ -z "${NOCHECK}" ]; then
        NLDPC_LIB_PATH=$L timeout -k 10 180 python -u tools/ab_check.py ${CHECK_KINDS} > $O/abchk_$n.log 2>&1 || { echo "$v check failed rc=$?"; tail -5 $O/abchk_$n.log; exit 1; }
    fi
    NLDPC_LIB_PATH=$L timeout -k 10 240 python -u bench.py --steps ${STEPS:-6} --warmup 2 \
        --no-cpu-baseline --no-sweep --no-count-only --no-side-lines ${BENCH_ARGS} > $O/ab_$n.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/ab_$n.log; exit 1; }
    python3 - $v $O/ab_$n.log $O/abchk_$n.log <<'PY'
import json, os, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
chk = open(sys.argv[3]).read().strip().splitlines()[-1] if os.path.exists(sys.argv[3]) else ""
print(f"{sys.argv[1]:12s} {d['value']:>12.0f} cw/s  kernel {d['roofline']['avg_launch_ms']:.3f} ms  median step {d['ms_per_step_median']:.3f} ms  | {chk}")
PY
done
done
