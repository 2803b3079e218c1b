# GPU-box script: rocprofv3 kernel-trace summaries and PMC passes (one counter group per run, with
# --kernel-trace only, as MI355X_MICROARCH.md prescribes) for cfg3 and cfg5, plus the probe kernels
# that calibrate FETCH_SIZE / WRITE_SIZE.  Library built on the CPU side.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r2}
cd /tmp && export TMPDIR=/tmp
run() {  # name, timeout, rocprof args..., -- command
    local name=$1 t=$2; shift 2
    timeout -k 10 $t rocprofv3 "$@" > $O/${TAG}_${name}.log 2>&1 || { echo "$name failed rc=$?"; tail -5 $O/${TAG}_${name}.log; exit 1; }
    echo "$name ok"
}
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sweep --no-count-only"
[ -n "$NO_PROBE" ] || run probe_fetch 120 --pmc FETCH_SIZE --kernel-trace -d $O/${TAG}_probe_fetch -o run --output-format csv -- python3 $R/tools/probe_pmc.py
[ -n "$NO_PROBE" ] || run probe_write 120 --pmc WRITE_SIZE --kernel-trace -d $O/${TAG}_probe_write -o run --output-format csv -- python3 $R/tools/probe_pmc.py
# WORKLOADS entries: cfg3 | cfg5 | cfg2 | cfg3ucn@KIND@CN,UCN,VN (a Boosted side line, e.g. cfg3ucn@QMS@1,1,2)
for WS in ${WORKLOADS:-cfg3 cfg5}; do
    IFS=@ read -r W K NW <<< "$WS"
    A="--workload $W"; N=$W
    if [ -n "$K" ]; then A="$A --kind $K --nw $NW"; N=${W}_${K}_NW${NW//,/}; fi
    run ${N}_trace 300 --kernel-trace --stats -d $O/${TAG}_${N}_trace -o run --output-format csv -- $B $A
    run ${N}_fetch 300 --pmc FETCH_SIZE --kernel-trace -d $O/${TAG}_${N}_fetch -o run --output-format csv -- $B $A --no-profile
    run ${N}_write 300 --pmc WRITE_SIZE --kernel-trace -d $O/${TAG}_${N}_write -o run --output-format csv -- $B $A --no-profile
    run ${N}_sq 300 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/${TAG}_${N}_sq -o run --output-format csv -- $B $A --no-profile
done
echo "all passes done"
