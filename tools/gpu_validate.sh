# GPU-box script (run via gpurun): the prebuilt in-tree library's GPU suite, smoke, the default bench line (cfg3 with
# the cfg5 / cfg2 side lines), the Boosted cfg3ucn side lines and a rocprofv3 kernel-trace summary of the default
# bench.  Every GPU step has its own time limit; steps are chained with && so the first failure ends the call.
# Usage: TAG=r6x [NOTESTS=1] [NOUCN=1] [NOTRACE=1] bash tools/gpu_validate.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-validate}; mkdir -p $O
cd $R || exit 1
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -15 $O/gpu_tests.log; exit 1; }
  echo "gpu tests: $(tail -1 $O/gpu_tests.log)"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
if [ -z "$NOUCN" ]; then
  timeout -k 10 300 python bench.py --workload cfg3ucn --kind MS --no-cpu-baseline --no-sweep > $O/bench_ucn_ms.log 2>&1 &&
  timeout -k 10 300 python bench.py --workload cfg3ucn --kind QMS --no-cpu-baseline --no-sweep > $O/bench_ucn_qms.log 2>&1 || { echo "ucn bench failed"; exit 1; }
fi
python3 - $O <<'PY'
import json, os, sys
for f in ("bench", "bench_ucn_ms", "bench_ucn_qms"):
    p = os.path.join(sys.argv[1], f + ".log")
    if not os.path.exists(p):
        continue
    d = json.loads([l for l in open(p) if l.startswith("{")][-1]); r = d.get("roofline", {})
    print(f, d["value"], "median step", d.get("ms_per_step_median"), "kernel", r.get("avg_launch_ms"), r.get("bound"))
    for k, v in d.get("side_lines", {}).items():
        print("  side", k, v.get("value"), "median step", v.get("ms_per_step_median"), "kernels",
              {kk: vv["avg_ms"] for kk, vv in v.get("roofline", {}).get("per_kernel", {}).items()})
PY
if [ -z "$NOTRACE" ]; then
  cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_prof.log 2>&1 || { echo "trace failed"; exit 1; }
fi
echo "validate done"
