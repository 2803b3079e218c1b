# GPU-box script: SQ instruction / stall counters of the bench's kernels, one rocprofv3 pass per
# counter group (--pmc with --kernel-trace only).  Usage: TAG=name bash tools/gpu_sq.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
TAG=${TAG:-sq}
ARGS="--steps 2 --warmup 1 --batch ${SQ_BATCH:-16384} --no-cpu-baseline --no-profile ${BENCH_ARGS}"
make -C $R/neural-ldpc-decoder-torch_amd/csrc -j16 > $R/gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $R/gpurun_out/${TAG}_g$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/${TAG}_g$i.log 2>&1 || { echo "group $i failed"; exit 1; }
done
python3 $R/tools/sq_summary.py $R/gpurun_out/${TAG}_g* > $R/gpurun_out/${TAG}_summary.txt 2>&1
cat $R/gpurun_out/${TAG}_summary.txt
