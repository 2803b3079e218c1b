# GPU-box script (r5h): spill-reload experiments.  (1) UCN bit addresses per iteration (ucn_a) and
# + branch-free OR (ucn_b) vs ucn_base: fused vs streaming bit-exact (MS, QMS, with and without UCN), then
# cfg3ucn MS / QMS kernel times interleaved; (2) UREMAT (lane offsets re-derived per phase in the SAVE
# kernels, buffer-descriptor saves): z=384 oracle tests on it, cfg5 A/B against lib_ab/base.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
for v in ucn_base ucn_a ucn_b; do
    NLDPC_LIB_PATH=$A/$v/libnldpc.so timeout -k 10 180 python -u tools/ab_check.py 1 2 > $O/abchk_$v.log 2>&1 || { echo "$v check failed"; tail -5 $O/abchk_$v.log; exit 1; }
    echo "$v: $(tail -2 $O/abchk_$v.log | tr '\n' ' ')"
done
for rnd in 1 2; do for k in MS QMS; do for v in ucn_base ucn_a ucn_b; do
    NLDPC_LIB_PATH=$A/$v/libnldpc.so timeout -k 10 240 python -u bench.py --workload cfg3ucn --kind $k \
        --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-count-only > $O/ucn_${k}_${v}_$rnd.log 2>&1 || { echo "$v $k failed"; tail -5 $O/ucn_${k}_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$O/ucn_${k}_${v}_$rnd.log') if l.startswith('{')][-1])
print('$k $v', 'kernel', d['roofline']['avg_launch_ms'], 'median step', d['ms_per_step_median'], 'ber', d['ber']['bit_errors_last_iter'])"
done; done; done
NLDPC_LIB_PATH=$A/urm/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py tests/test_gpu_stateful.py -x -q --timeout 300 --timeout-method thread > $O/urm_tests.log 2>&1 || { echo "urm tests failed"; tail -15 $O/urm_tests.log; exit 1; }
echo "urm tests: $(tail -1 $O/urm_tests.log)"
TAG=r5h NOTESTS=1 VARIANTS="lib_ab/base lib_ab/urm" bash tools/gpu_ab_cfg5.sh
