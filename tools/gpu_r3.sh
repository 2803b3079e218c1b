# GPU-box script (run via gpurun; the library is built on the CPU side and travels with the tree):
# GPU parity tests, smoke, the bench lines of every workload and a rocprofv3 kernel-trace summary of the
# headline (cfg3) bench.  Every GPU step has its own time limit; the first failing step ends the script.
# TAG=r3a PHASES="tests smoke cfg3 prof cfg5 cfg2 ucn" bash tools/gpu_r3.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r3}
PHASES=${PHASES:-"tests smoke cfg3 prof cfg5 cfg2 ucn"}
cd $R
export TMPDIR=/tmp
for s in $PHASES; do
    echo "== $s $(date +%T)"
    case $s in
    tests) NLDPC_JIT_LOG=$O/${TAG}_jit_compiles.txt timeout -k 10 ${TESTS_TIMEOUT:-600} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x \
               -p no:cacheprovider > $O/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 $O/${TAG}_gpu_tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1; rc=$? ;;
    cfg3)  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/${TAG}_bench_cfg3.log 2>&1; rc=$?; tail -c 1500 $O/${TAG}_bench_cfg3.log ;;
    prof)  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_cfg3 -o run --output-format csv \
               -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sweep > $O/${TAG}_bench_cfg3_under_rocprof.log 2>&1); rc=$? ;;
    cfg5)  timeout -k 10 600 python -u bench.py --workload cfg5 --steps 5 --warmup 2 > $O/${TAG}_bench_cfg5.log 2>&1; rc=$?; tail -c 800 $O/${TAG}_bench_cfg5.log ;;
    prof5) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_cfg5 -o run --output-format csv \
               -- python3 $R/bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_bench_cfg5_under_rocprof.log 2>&1); rc=$? ;;
    cfg2)  timeout -k 10 300 python -u bench.py --workload cfg2 --steps 50 --warmup 5 --no-cpu-baseline > $O/${TAG}_bench_cfg2.log 2>&1; rc=$?; tail -c 800 $O/${TAG}_bench_cfg2.log ;;
    ucn)   timeout -k 10 600 python -u bench.py --workload cfg3ucn --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench_ucn_MS_112.log 2>&1 &&
           timeout -k 10 600 python -u bench.py --workload cfg3ucn --kind QMS --steps 3 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench_ucn_QMS_112.log 2>&1; rc=$?
           tail -c 600 $O/${TAG}_bench_ucn_MS_112.log; tail -c 600 $O/${TAG}_bench_ucn_QMS_112.log ;;
    ab)    VARIANTS="${VARIANTS}" STEPS=6 bash tools/gpu_ab.sh > $O/${TAG}_ab.txt 2>&1; rc=$?; cat $O/${TAG}_ab.txt ;;
    icache) bash tools/gpu_icache.sh > $O/${TAG}_icache.txt 2>&1; rc=$?; cat $O/${TAG}_icache.txt ;;
    host)  timeout -k 10 300 python -u tools/dev/host_overhead.py > $O/${TAG}_host_overhead.txt 2>&1; rc=$?; head -30 $O/${TAG}_host_overhead.txt ;;
    cfg2np) timeout -k 10 300 python -u bench.py --workload cfg2 --steps 500 --warmup 20 --no-cpu-baseline --no-profile --no-count-only > $O/${TAG}_bench_cfg2_noprof.log 2>&1 &&
           (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_cfg2 -o run --output-format csv \
               -- python3 $R/bench.py --workload cfg2 --steps 500 --warmup 20 --no-cpu-baseline --no-profile --no-count-only > $O/${TAG}_bench_cfg2_under_rocprof.log 2>&1); rc=$?
           tail -c 400 $O/${TAG}_bench_cfg2_noprof.log ;;
    valumix) (cd /tmp && timeout -s KILL 120 rocprofv3 -L > $O/${TAG}_counters_list.txt 2>&1; \
             timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_LDS \
               --kernel-trace -d $O/${TAG}_valumix -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --batch 16384 --no-cpu-baseline --no-profile --no-sweep --no-count-only > $O/${TAG}_valumix.log 2>&1); rc=$?
           python3 tools/sq_summary.py $O/${TAG}_valumix | grep -A9 "kernel<3" ;;
    stampsucn) NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_stamps/libnldpc.so NLDPC_STAMPS=$O/${TAG}_stamps_ucn.bin \
             timeout -k 10 300 python -u bench.py --workload cfg3ucn --steps 1 --warmup 1 --batch 16384 --no-profile --no-cpu-baseline > $O/${TAG}_stamps_ucn_bench.log 2>&1 &&
           python3 tools/stamps2.py $O/${TAG}_stamps_ucn.bin > $O/${TAG}_stamps_ucn.txt 2>&1; rc=$?; head -30 $O/${TAG}_stamps_ucn.txt ;;
    stamps3|stamps2) W=cfg3; BA="--batch 16384"; [ $s = stamps2 ] && { W=cfg2; BA=""; }
           NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_stamps/libnldpc.so NLDPC_STAMPS=$O/${TAG}_$s.bin \
             timeout -k 10 300 python -u bench.py --workload $W --steps 1 --warmup 1 $BA --no-profile --no-cpu-baseline --no-sweep --no-count-only > $O/${TAG}_${s}_bench.log 2>&1 &&
           python3 tools/stamps2.py $O/${TAG}_$s.bin > $O/${TAG}_$s.txt 2>&1; rc=$?; head -30 $O/${TAG}_$s.txt ;;
    abq)   for v in ${VARIANTS}; do
               NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_exp/$v/libnldpc.so timeout -k 10 300 python -u bench.py --workload ${WL:-cfg3ucn} ${BENCH_ARGS} \
                   --steps ${NSTEPS:-4} --warmup 2 --no-cpu-baseline > $O/${TAG}_abq_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/${TAG}_abq_$v.log; exit 1; }
               python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d.get('ms_per_step_median'), d.get('roofline',{}).get('per_kernel'))" $O/${TAG}_abq_$v.log $v | cut -c1-400
           done; rc=0 ;;
    stamps5) NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_stamps/libnldpc.so NLDPC_STAMPS=$O/${TAG}_stamps5_fwd.bin NLDPC_STAMPS_BWD=$O/${TAG}_stamps5_bwd.bin \
             timeout -k 10 300 python -u bench.py --workload cfg5 --steps 1 --warmup 0 --batch 512 --no-profile --no-cpu-baseline > $O/${TAG}_stamps5_bench.log 2>&1 &&
           python3 tools/stamps2.py $O/${TAG}_stamps5_fwd.bin > $O/${TAG}_stamps5_fwd.txt 2>&1 && python3 tools/stamps_bwd.py $O/${TAG}_stamps5_bwd.bin ${KB:-3} > $O/${TAG}_stamps5_bwd.txt 2>&1; rc=$?
           head -14 $O/${TAG}_stamps5_fwd.txt; head -20 $O/${TAG}_stamps5_bwd.txt ;;
    *) echo "unknown step $s"; rc=2 ;;
    esac
    echo "== $s rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
