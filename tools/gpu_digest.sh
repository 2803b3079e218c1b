# GPU-box: gradient digests (tools/grad_digest.py) of one cfg5 step on each library in VARIANTS -- equal lines mean
# bit-identical loss and gradients.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-digest}; mkdir -p $O
cd $R
for v in ${VARIANTS}; do
    n=${v//\//_}
    NLDPC_LIB_PATH=$R/neural-ldpc-decoder-torch_amd/$v/libnldpc.so timeout -k 10 300 python -u tools/grad_digest.py ${B:-256} > $O/digest_$n.log 2>&1 || { echo "$v failed"; tail -5 $O/digest_$n.log; exit 1; }
    echo "$v: $(tail -1 $O/digest_$n.log)"
done
