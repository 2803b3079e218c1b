# Experiment build: a libnldpc.so whose generated fused kernels cover only BG2 z=384 / Neural, built
# with the generator knobs given in the environment (NLDPC_GEN_*), into lib_exp/<name>/.  The
# hand-written units are reused from lib/obj (built by the main Makefile).  Used by the GPU A/B runs
# (NLDPC_LIB_PATH=lib_exp/<name>/libnldpc.so python bench.py ...).
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/neural-ldpc-decoder-torch_amd
OUT=$P/lib_exp/$NAME
mkdir -p $OUT/obj $OUT/gen
for f in nldpc_graph.cpp nldpc_profile.cpp nldpc_forward.hip nldpc_backward.hip nldpc_aux.hip; do
    cp -p $P/lib/obj/$f.o $OUT/obj/
done
cd $P/csrc
env NLDPC_GEN_ONLY=bg2_z384 NLDPC_GEN_KINDS=${KINDS:-3} "$@" python3 gen_fused.py $OUT/gen $R/resources
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -fno-slp-vectorize -I$R/include -I$P/csrc ${EXTRA_FLAGS}"
pids=""
for g in $OUT/gen/*.hip; do
    b=$(basename $g)
    /opt/rocm/bin/hipcc $FLAGS -x hip -c $g -o $OUT/obj/gen_$b.o &
    pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnldpc.so $OUT/obj/*.o
echo "built $OUT/libnldpc.so"
