set -o pipefail; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6e; mkdir -p $O; cd $R || exit 1
TAG=r6e/ab5 VARIANTS="lib_ab/b_sp1b lib_ab/b_sp1c lib_ab/b_sp2" NOTESTS=1 ROUNDS=2 bash tools/gpu_ab_cfg5.sh || exit 1
TAG=r6e/dig VARIANTS="lib_ab/f_base lib_ab/b_sp1c lib_ab/b_sp2" bash tools/gpu_digest.sh || exit 1
TAG=r6e/stamps CFG5=1 STAMP_VARIANTS="lib_ab/b_sp1bst" bash tools/gpu_stamps.sh || exit 1
TAG=r6e/ab3 VARIANTS="lib_ab/c_base lib_ab/c_ms6 lib_ab/c_ms4 lib_ab/c_ms10" CHECK_KINDS=3 ROUNDS=2 bash tools/gpu_ab.sh || exit 1
for v in b_sp1c b_sp2; do
  NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/lib_ab/$v/libnldpc.so TAG=r6e/pmc_$v GROUPS_="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" BENCH_ARGS="--workload cfg5 --steps 2 --warmup 1" bash tools/gpu_pmc.sh > $O/pmc_$v.txt 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo r6e done
