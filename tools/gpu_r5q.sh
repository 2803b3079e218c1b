# GPU-box script (r5q): the in-tree library after the r5 training-path changes -- GPU suite, smoke, gradient digest
# against the r5f library (lib_ab/base: r4's kernels), cfg5 bench line, cfg5 kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5q; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r5q VARIANTS="lib_ab/base lib" bash tools/gpu_digest.sh || exit 1
timeout -k 10 600 python bench.py --workload cfg5 --steps 5 --warmup 2 > $O/bench_cfg5.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_cfg5.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_cfg5.log') if l.startswith('{')][-1]); pk=d['roofline']['per_kernel']
print('cfg5', d['value'], 'median step', d['ms_per_step_median'], 'fwd', pk['fused']['avg_ms'], 'bwd', pk['fusedb']['avg_ms'], d['roofline']['bound'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cfg5_trace -o run --output-format csv -- python3 $R/bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $O/cfg5_trace.log 2>&1 && echo "trace ok"
