# GPU-box script (r5g): packed Q(xa) bytes.  (1) cfg5 A/B: lib_ab/base (the previous library) vs lib
# (XQ in the training forward), interleaved; (2) the QMS decode kernels with XQ (lib_ab/xqdec) checked bit
# for bit against the streaming kernels, and cfg3ucn QMS A/B base vs xqdec; (3) the GPU suite on lib;
# (4) cfg5 FETCH/WRITE PMC passes and a kernel trace on lib.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5g; mkdir -p $O
cd $R
TAG=r5g NOTESTS=1 VARIANTS="lib_ab/base lib" bash tools/gpu_ab_cfg5.sh || exit 1
NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_ab/xqdec/libnldpc.so timeout -k 10 180 python -u tools/ab_check.py 2 > $O/abchk_xqdec.log 2>&1 || { echo "xqdec check failed"; tail -5 $O/abchk_xqdec.log; exit 1; }
tail -1 $O/abchk_xqdec.log
for rnd in 1 2; do for v in lib_ab/base lib_ab/xqdec; do
    n=${v//\//_}
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so timeout -k 10 240 python -u bench.py --workload cfg3ucn --kind QMS \
        --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-count-only > $O/ucn_qms_${n}_$rnd.log 2>&1 || { echo "$v failed"; tail -5 $O/ucn_qms_${n}_$rnd.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('$O/ucn_qms_${n}_$rnd.log') if l.startswith('{')][-1])
print('$v', 'ucn QMS kernel', d['roofline']['avg_launch_ms'], 'median step', d['ms_per_step_median'])"
done; done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
TAG=r5g NOTESTS=1 ROUNDS=0 PMC=1 bash tools/gpu_ab_cfg5.sh
