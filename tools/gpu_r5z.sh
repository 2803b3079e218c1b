# GPU-box script (r5z): phase stamps of the final training kernels (cfg5 at B=512, one step: the training forward and the
# tied backward), from a stamp build of the final generator copied to lib_ab/st (make STAMPS=1 NLDPC_GEN_KINDS=2).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5z; mkdir -p $O
cd $R
NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_ab/st/libnldpc.so NLDPC_STAMPS=$O/stamps_fwd.bin NLDPC_STAMPS_BWD=$O/stamps_bwd.bin \
    timeout -k 10 300 python -u bench.py --workload cfg5 --steps 1 --warmup 0 --batch 512 --no-profile --no-cpu-baseline > $O/stamps_bench.log 2>&1 &&
python3 tools/stamps2.py $O/stamps_fwd.bin VN "W0" "CN0" "R0" "W1" "CN1" "R1" > $O/stamps_fwd.txt 2>&1 && python3 tools/stamps_bwd.py $O/stamps_bwd.bin 3 > $O/stamps_bwd.txt 2>&1 || { echo "stamps failed"; tail -5 $O/stamps_bench.log; exit 1; }
head -12 $O/stamps_fwd.txt; head -14 $O/stamps_bwd.txt
