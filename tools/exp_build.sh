# Experiment build: a libnldpc.so whose generated fused kernels cover only BG2 z=384 / Neural, built
# with the generator knobs given in the environment (NLDPC_GEN_*), into lib_exp/<name>/, with its own
# build of the hand-written units (same headers, EXTRA_FLAGS).  Used by the GPU A/B runs
# (NLDPC_LIB_PATH=lib_exp/<name>/libnldpc.so python bench.py ...).
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/neural-ldpc-decoder-torch_amd
OUT=$P/lib_exp/$NAME
mkdir -p $OUT/obj $OUT/gen
cd $P/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -fno-slp-vectorize -I$R/include -I$P/csrc ${EXTRA_FLAGS}"
# the hand-written units (launchers, streaming kernels) are compiled here against the same headers as the
# variant's generated kernels: r3 copied them from lib/obj, and a variant whose FusedArgs layout had
# changed ran its kernels on a launcher that filled the old layout (the qms3 hang)
# (cached by the hash of the sources, headers and flags: lib_exp/.hw/<hash>/; a variant that changes none of them
# reuses them, one whose headers differ gets its own)
HW="nldpc_graph.cpp nldpc_profile.cpp nldpc_forward.hip nldpc_backward.hip nldpc_aux.hip"
KEY=$( (cat $HW *.h $R/include/nldpc.h; echo "$FLAGS") | sha1sum | cut -c1-16)
# HWKEY=<key>: reuse an existing hand-written build (lib_exp/.hw/<key>) -- only when the header edits since it change no
# struct layout or code those units compile (e.g. code behind a generator macro); the layout signature still guards
KEY=${HWKEY:-$KEY}
HWD=$P/lib_exp/.hw/$KEY
hpids=""
if [ -f $HWD/done ]; then
    for f in $HW; do cp -p $HWD/$f.o $OUT/obj/; done
else
    mkdir -p $HWD
    for f in $HW; do
        ( /opt/rocm/bin/hipcc ${FLAGS/-fno-slp-vectorize/} -x hip -c $f -o $HWD/$f.o && cp -p $HWD/$f.o $OUT/obj/ ) &
        hpids="$hpids $!"
    done
fi
env NLDPC_GEN_ONLY=${GEN_ONLY:-bg2_z384} NLDPC_GEN_KINDS=${KINDS:-3} "$@" python3 gen_fused.py $OUT/gen $R/resources
pids="$hpids"
for g in $OUT/gen/*.hip; do
    b=$(basename $g)
    /opt/rocm/bin/hipcc $FLAGS -x hip -c $g -o $OUT/obj/gen_$b.o &
    pids="$pids $!"
done
for p in $pids; do wait $p; done
touch $HWD/done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnldpc.so $OUT/obj/*.o
echo "built $OUT/libnldpc.so"
