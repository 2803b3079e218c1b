#!/bin/bash
# The ISA of the cfg3 decode kernel (fused_bg2_z384::kernel<3,0>), one single-part build per part, and the
# instruction budget tools/isa_budget.py reads from it.  CPU only (hipcc -S); about a minute per part.
# Usage: bash tools/isa_budget.sh [OUTDIR]   (default /tmp/isa)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/neural-ldpc-decoder-torch_amd/csrc
OUT=${1:-/tmp/isa}
mkdir -p "$OUT/parts"
for p in 0 1 2 3 4 5 6 7; do
  NLDPC_GEN_PARTS=$p NLDPC_GEN_KINDS=${KIND:-3} NLDPC_GEN_ONLY=bg2_z384 NLDPC_GEN_NOBWD=1 \
    python3 "$CS/gen_fused.py" "$OUT/parts/g$p" "$ROOT/resources" > /dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -I"$ROOT/include" -I"$CS" -x hip --cuda-device-only -S "$OUT/parts/g$p/fused_bg2_z384_s0.hip" \
    -o "$OUT/parts/p$p.s" &
done
wait
python3 "$ROOT/tools/isa_budget.py" ${ISA_JSON:+--json=$ISA_JSON} "$OUT"/parts/p{0,1,2,3,4,5,6,7}.s
