# GPU-box script (run via gpurun): the prebuilt in-tree library's GPU suite, smoke, bench lines and a
# rocprofv3 kernel-trace summary of the headline bench.  Every GPU step has its own time limit; steps
# are chained with && so the first failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r5}; mkdir -p $O
cd $R &&
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 &&
timeout -k 10 600 python bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cfg5.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3ucn --kind MS --no-cpu-baseline > $O/bench_ucn_ms.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3ucn --kind QMS --no-cpu-baseline > $O/bench_ucn_qms.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_prof.log 2>&1
echo "exit $?"
