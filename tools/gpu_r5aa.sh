# GPU-box script (r5aa): degree-1 channel values requested before the row's stores (d1x) -- gradient digests, z=384
# oracle tests, cfg5 A/B lib | d1x and cfg3ucn QMS A/B lib | d1x, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5aa; mkdir -p $O
cd $R
A=$R/neural-ldpc-decoder-torch_amd/lib_ab
TAG=r5aa VARIANTS="lib lib_ab/d1x" bash tools/gpu_digest.sh || exit 1
NLDPC_LIB_PATH=$A/d1x/libnldpc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_z384_oracle.py -x -q --timeout 300 --timeout-method thread > $O/d1x_tests.log 2>&1 || { echo "d1x tests failed"; tail -15 $O/d1x_tests.log; exit 1; }
echo "d1x z384 tests: $(tail -1 $O/d1x_tests.log)"
NLDPC_LIB_PATH=$A/d1x/libnldpc.so timeout -k 10 180 python -u tools/ab_check.py 2 > $O/abchk_d1x.log 2>&1 || { echo "d1x check failed"; tail -5 $O/abchk_d1x.log; exit 1; }
tail -1 $O/abchk_d1x.log
TAG=r5aa NOTESTS=1 VARIANTS="lib lib_ab/d1x" bash tools/gpu_ab_cfg5.sh || exit 1
for rnd in 1 2; do for v in lib lib_ab/d1x; do
    n=${v//\//_}
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so timeout -k 10 240 python -u bench.py --workload cfg3ucn --kind QMS \
        --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-count-only > $O/ucn_qms_${n}_$rnd.log 2>&1 || { echo "$v failed"; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/ucn_qms_${n}_$rnd.log') if l.startswith('{')][-1])
print('$v', 'ucn QMS kernel', d['roofline']['avg_launch_ms'])"
done; done
