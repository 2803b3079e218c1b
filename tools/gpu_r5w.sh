# GPU-box script (r5w): the side lines on the final library -- cfg3ucn MS / QMS NW(1,1,2)+UCN and cfg2 (graph replay).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5w; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --workload cfg3ucn --kind MS --no-cpu-baseline > $O/bench_ucn_ms.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg3ucn --kind QMS --no-cpu-baseline > $O/bench_ucn_qms.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg2 --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_cfg2.log 2>&1 || { echo "bench failed"; exit 1; }
python3 -c "
import json
for f in ('ucn_ms', 'ucn_qms', 'cfg2'):
    d=json.loads([l for l in open('$O/bench_'+f+'.log') if l.startswith('{')][-1]); r=d['roofline']
    print(f, d['value'], 'median step', d['ms_per_step_median'], 'kernel', r['avg_launch_ms'], r['bound'])"
