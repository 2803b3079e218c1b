# ISA metadata (VGPRs, SGPRs, scratch, spills) of an experiment variant's z=384 Neural decode kernel.
R=$(cd "$(dirname "$0")/.." && pwd); P=$R/neural-ldpc-decoder-torch_amd
G=$P/lib_exp/$1/gen/fused_bg2_z384_s${2:-0}.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function -fno-slp-vectorize -I$R/include -I$P/csrc ${EXTRA_FLAGS} -x hip --cuda-device-only -S $G -o /tmp/exp_$1.s 2>/dev/null
grep -E "^\s+\.(vgpr_count|sgpr_count|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|agpr_count):" /tmp/exp_$1.s | tr -s ' ' | tr '\n' ' '; echo
