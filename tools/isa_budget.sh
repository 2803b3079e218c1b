#!/bin/bash
# The ISA instruction budget of a generated fused kernel (tools/isa_budget.py): one single-part build per part (gfx950
# asm, hipcc -S, CPU only, about a minute per part, parts in parallel), the kernel's hot loop per part, VALU issue cycles.
# LINES=1: asm with line tables, and the hot loop's VALU cycles by source line (isa_budget.py --lines) instead of the budget
# Usage: [TAG=bg2_z384] [UNIT=s0|s1|s2|s3|bwd] [MODE=<kernel MODE, default the unit's>] [KIND=3] [TIED=0|1] [ISA_JSON=profiles/isa_budget.json] bash tools/isa_budget.sh [OUTDIR]
#   UNIT s<MODE>: the forward kernel<KIND, MODE> (MODE=5 with UNIT=s1: the tied saving forward); bwd: the backward bwd_kernel<KIND, TIED>.  Default: the cfg3 decode kernel.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/neural-ldpc-decoder-torch_amd/csrc
TAG=${TAG:-bg2_z384}; UNIT=${UNIT:-s0}; KIND=${KIND:-3}; TIED=${TIED:-0}
OUT=${1:-/tmp/isa_${TAG}_${UNIT}_${KIND}}
GEO=$(cd "$CS" && python3 -c "
import gen_fused as g, numpy as np, os
t = [s for s in g.SPECS if s[0] == '$TAG'][0]
hb = np.loadtxt(os.path.join('$ROOT/resources', t[1]), int, delimiter='\t')
G, P, Q = t[3:] if t[3] else g.auto_geometry(hb, t[2])
S = g.Spec('$TAG', hb, t[2], G, P, Q)
print(G, P, S.lanes_pad // 64, S.threads)")
read G P WPP THREADS <<< "$GEO"
mkdir -p "$OUT/parts"
NOBWD=1; [ "$UNIT" = bwd ] && NOBWD=0
for p in $(seq 0 $((P - 1))); do
  NLDPC_GEN_PARTS=$p NLDPC_GEN_KINDS=$KIND NLDPC_GEN_ONLY=$TAG NLDPC_GEN_NOBWD=$NOBWD \
    python3 "$CS/gen_fused.py" "$OUT/parts/g$p" "$ROOT/resources" > /dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -Wno-unused-function ${LINES:+-gline-tables-only} -I"$ROOT/include" -I"$CS" -x hip --cuda-device-only -S "$OUT/parts/g$p/fused_${TAG}_${UNIT}.hip" \
    -o "$OUT/parts/p$p.s" 2> /dev/null &
done
wait
if [ "$UNIT" = bwd ]; then FUNC="bwd_kernelILi${KIND}ELi${TIED}E"; NAME="_bg2_z384::bwd_kernel<${KIND}, ${TIED}>"; NAME="${TAG}::bwd_kernel<${KIND}, ${TIED}>";
else M=${MODE:-${UNIT#s}}; FUNC="kernelILi${KIND}ELi${M}E"; NAME="fused_${TAG}::kernel<${KIND}, ${M}>"; fi
if [ -n "$LINES" ]; then
  python3 "$ROOT/tools/isa_budget.py" --func="$FUNC" --lines=${LINES_TOP:-30} $(for p in $(seq 0 $((P - 1))); do echo "$OUT/parts/p$p.s"; done); exit $?
fi
python3 "$ROOT/tools/isa_budget.py" --func="$FUNC" --name="$NAME" --geom="$G,$P,$WPP,$THREADS" ${ISA_JSON:+--json=$ISA_JSON} \
  $(for p in $(seq 0 $((P - 1))); do echo "$OUT/parts/p$p.s"; done)
