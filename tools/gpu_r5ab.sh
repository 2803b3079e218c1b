# GPU-box script (r5ab): final validation of the in-tree library (early degree-1 loads in the Boosted kernels) -- GPU
# suite, smoke, gradient digest against the r5f library (r4 kernels), cfg5 / cfg3 / cfg3ucn MS+QMS bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ab; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r5ab VARIANTS="lib_ab/base lib" bash tools/gpu_digest.sh || exit 1
timeout -k 10 600 python bench.py --workload cfg5 --steps 5 --warmup 2 > $O/bench_cfg5.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3ucn --kind MS --no-cpu-baseline > $O/bench_ucn_ms.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3ucn --kind QMS --no-cpu-baseline > $O/bench_ucn_qms.log 2>&1 || { echo "bench failed"; exit 1; }
python3 -c "
import json
for f in ('cfg5', 'cfg3', 'ucn_ms', 'ucn_qms'):
    d=json.loads([l for l in open('$O/bench_'+f+'.log') if l.startswith('{')][-1]); r=d['roofline']; pk=r.get('per_kernel', {})
    print(f, d['value'], 'median step', d['ms_per_step_median'], 'kernel', r['avg_launch_ms'], r['bound'], {k: v['avg_ms'] for k, v in pk.items()})"
