# GPU-box script: phase stamps of experiment stamp builds (tools/exp_build.sh NAME NLDPC_GEN_STAMPS=1 ...), one
# cfg3 launch of 16 384 codewords each, parsed by tools/stamps2.py into gpurun_out/stamps_<NAME>.txt.
# Usage (gpurun): STAMP_VARIANTS="r5st_a r5st_b" bash tools/gpu_stamps.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for v in ${STAMP_VARIANTS}; do
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_exp/$v/libnldpc.so NLDPC_STAMPS=$O/stamps_$v.bin \
        timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-sweep --no-count-only \
        --batch 16384 --no-profile > $O/stamps_bench_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/stamps_bench_$v.log; exit 1; }
    python tools/stamps2.py $O/stamps_$v.bin > $O/stamps_$v.txt || exit 1
    echo "== $v"; cat $O/stamps_$v.txt
done
