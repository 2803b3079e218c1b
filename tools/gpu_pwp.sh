# GPU-box: partial-line byte stores vs L2 fetch (tools/dev/partial_write_probe.hip, prebuilt as lib_ab/pwp)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pwp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv -- $R/neural-ldpc-decoder-torch_amd/lib_ab/pwp > $O/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv -- $R/neural-ldpc-decoder-torch_amd/lib_ab/pwp > $O/write.log 2>&1 &&
python3 - $O <<'PY'
import csv, sys
for c in ("fetch", "write"):
    rows = list(csv.DictReader(open(f"{sys.argv[1]}/{c}/run_counter_collection.csv")))
    for i, r in enumerate(rows):
        print(c, "kind", i, r["Counter_Name"], float(r["Counter_Value"]) * 1024 / 2**30, "GiB (KiB units)")
PY
cd $R && timeout -k 10 300 python bench.py --workload cfg2 --steps 200 --warmup 10 --no-cpu-baseline > $O/bench_cfg2_graph.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg2 --steps 200 --warmup 10 --no-cpu-baseline --graph off > $O/bench_cfg2_eager.log 2>&1 &&
for f in bench_cfg2_graph bench_cfg2_eager; do python3 -c "
import json; d=json.loads([l for l in open('$O/'+'$f'+'.log') if l.startswith('{')][-1])
print('$f', d['value'], 'ms', d['ms_per_step'], 'median', d['ms_per_step_median'], 'kernel', d['roofline']['avg_launch_ms'], d['config'].get('graph'))"; done
