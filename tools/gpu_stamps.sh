# GPU-box script: phase stamps of stamp builds (tools/exp_build.sh NAME NLDPC_GEN_STAMPS=1 ..., or make STAMPS=1).
#   default: one cfg3 launch of 16 384 codewords per variant, parsed by tools/stamps2.py
#   CFG5=1: one cfg5 step at B=512 (the training forward and the backward), parsed by stamps2.py / stamps_bwd.py
# Usage (gpurun): STAMP_VARIANTS="lib_exp/r5st_a lib_stamps" [CFG5=1] bash tools/gpu_stamps.sh
#   (directories under neural-ldpc-decoder-torch_amd/ holding a libnldpc.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-stamps}; mkdir -p $O
cd $R
for v in ${STAMP_VARIANTS}; do
  n=${v//\//_}
  L=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so
  if [ -n "$CFG5" ]; then
    NLDPC_LIB_PATH=$L NLDPC_STAMPS=$O/fwd_$n.bin NLDPC_STAMPS_BWD=$O/bwd_$n.bin \
      timeout -k 10 300 python -u bench.py --workload cfg5 --steps 1 --warmup 0 --batch 512 --no-profile \
      --no-cpu-baseline > $O/bench_$n.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/bench_$n.log; exit 1; }
    python3 tools/stamps2.py $O/fwd_$n.bin VN W0 CN0 R0 W1 CN1 R1 W2 CN2 R2 > $O/fwd_$n.txt 2>&1 &&
    python3 tools/stamps_bwd.py $O/bwd_$n.bin ${NCHUNK:-3} > $O/bwd_$n.txt 2>&1 || { echo "stamp parse failed"; exit 1; }
    echo "== $v forward"; head -14 $O/fwd_$n.txt; echo "== $v backward"; head -16 $O/bwd_$n.txt
  else
    NLDPC_LIB_PATH=$L NLDPC_STAMPS=$O/$n.bin \
      timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-sweep --no-count-only \
      --batch 16384 --no-profile > $O/bench_$n.log 2>&1 || { echo "$v failed rc=$?"; tail -5 $O/bench_$n.log; exit 1; }
    python3 tools/stamps2.py $O/$n.bin > $O/$n.txt || exit 1
    echo "== $v"; cat $O/$n.txt
  fi
done
