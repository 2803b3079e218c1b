# GPU-box script (r5v): final validation of the in-tree library (buffer-descriptor staging in the backward) -- GPU suite,
# smoke, gradient digests (the r5f library with r4 kernels, lib), the cfg5 and cfg3 bench lines, kernel traces of both.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5v; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r5v VARIANTS="lib_ab/base lib" bash tools/gpu_digest.sh || exit 1
timeout -k 10 600 python bench.py --workload cfg5 --steps 5 --warmup 2 > $O/bench_cfg5.log 2>&1 || { echo "bench cfg5 failed"; tail -5 $O/bench_cfg5.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_cfg3.log 2>&1 || { echo "bench cfg3 failed"; tail -5 $O/bench_cfg3.log; exit 1; }
python3 -c "
import json
for f in ('cfg5', 'cfg3'):
    d=json.loads([l for l in open('$O/bench_'+f+'.log') if l.startswith('{')][-1]); r=d['roofline']
    print(f, d['value'], 'median step', d['ms_per_step_median'], 'kernel', r['avg_launch_ms'], r['bound'], r.get('issue_frac'), r['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg5_trace -o run --output-format csv -- python3 $R/bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $O/cfg5_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg3_trace -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --no-count-only > $O/cfg3_trace.log 2>&1 && echo "traces ok"
