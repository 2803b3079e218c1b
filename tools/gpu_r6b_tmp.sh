set -o pipefail; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6c; mkdir -p $O; cd $R || exit 1
TAG=r6c/ab3 VARIANTS="lib_ab/c_base lib_ab/c_ms lib_ab/c_ms6 lib_ab/c_s6" CHECK_KINDS=3 ROUNDS=2 bash tools/gpu_ab.sh || exit 1
TAG=r6c/ab5 VARIANTS="lib_ab/f_base lib_ab/b_bp1 lib_ab/b_p1s lib_ab/b_p2 lib_ab/b_p2s" NOTESTS=1 ROUNDS=2 bash tools/gpu_ab_cfg5.sh || exit 1
TAG=r6c/dig VARIANTS="lib_ab/f_base lib_ab/b_p1s lib_ab/b_p2 lib_ab/b_p2s" bash tools/gpu_digest.sh || exit 1
TAG=r6c/stamps CFG5=1 STAMP_VARIANTS="lib_ab/b_st2" bash tools/gpu_stamps.sh || exit 1
echo r6c done
