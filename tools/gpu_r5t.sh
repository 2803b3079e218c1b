# GPU-box script (r5t): cfg3 decode kernel, the r5f library (lib_ab/base) vs the in-tree library, same box, interleaved
# (the cfg3 kernel's generated code changed only by dead-branch removal in r5; this checks it did not move).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5t; mkdir -p $O
cd $R
for rnd in 1 2; do for v in lib_ab/base lib; do
    n=${v//\//_}
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 \
        --no-cpu-baseline --no-sweep --no-count-only > $O/cfg3_${n}_$rnd.log 2>&1 || { echo "$v failed"; tail -5 $O/cfg3_${n}_$rnd.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/cfg3_${n}_$rnd.log') if l.startswith('{')][-1])
print('$v', 'cfg3 kernel', d['roofline']['avg_launch_ms'], 'median step', d['ms_per_step_median'])"
done; done
