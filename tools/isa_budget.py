"""Per-edge instruction budget and issue-cycle floor of the cfg3 decode kernel, read from its ISA
(VERDICT r3 item 1).

Input: the gfx950 asm of single-part builds of fused_bg2_z384::kernel<3,0> (NLDPC_GEN_PARTS=p, one file per
part p = 0..7; tools/isa_budget.sh makes them).  For each part the hot loop (from the loop header to its back
edge, the cold zero-message blocks after the loop excluded) is split at its s_barrier instructions into the
six barrier phases of an iteration, and every instruction is classed:

  VALU full   v_add/sub/mul/fma_f32, v_add/sub_u32, v_and/or/xor_b32, v_mov_b32 ...   2.08-2.37 SIMD cycles
  VALU half   v_min/max/med3/min3_f32, v_cndmask_b32, shifts, 3-input integer ops      ~4.2
  VOPC        v_cmp_* (into VCC or an SGPR pair)                                       ~5.2
  (measured issue costs at 4 waves per SIMD, profiles/r3_valu_rate2*.txt)
  SALU, LDS (ds_*), VMEM (buffer_*), WAIT (s_waitcnt), NOP (s_nop: stalls only its wave)

A part is two waves (128 lanes x 3 lane copies = the 384 copies of its columns); a SIMD hosts one wave of
four parts (even parts on two SIMDs, odd parts on the other two: gen_fused.py Spec, SIMDBAL), so a SIMD's
VALU issue cycles per codeword-iteration are the sum over its four parts' loops.  That sum is the floor the
SIMD cannot beat whatever the latency hiding, barrier balance or memory system do.

Usage: python tools/isa_budget.py /tmp/isa/parts/p{0..7}.s   (prints the tables committed in
profiles/r4_isa_budget.txt)
"""
import collections

import sys

FULL = ("v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_add_u32",
        "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32", "v_add_co_u32",
        "v_readfirstlane_b32", "v_not_b32")
COST = {"full": 2.2, "half": 4.2, "vopc": 5.2}
CLK_GHZ = 2.45     # the clock the cfg3 launches run at (r3 PMC: GRBM_GUI_ACTIVE over the profiled duration)
ITERS_PER_CU = 20 * 65536 / 256   # T x codeword-workgroups per CU at cfg3


def vclass(op):
    if op.startswith("v_cmp"):
        return "vopc"
    if any(op.startswith(f) for f in FULL):
        return "full"
    return "half"


def parse(path):
    raw = open(path).read().split("\n")
    # the iteration loop: of the labels the asm comments as "Loop Header", the one whose body (header to the
    # last branch back to it) holds the most s_barrier instructions (the Boosted kernels have other loops)
    best = None
    for i, ln in enumerate(raw):
        if "Loop Header" in ln and ln.startswith(".LBB"):
            label = ln.split(":")[0]
            ends = [k for k in range(len(raw) - 1, i, -1)
                    if raw[k].strip().startswith("s_") and raw[k].strip().split()[-1] == label
                    and "branch" in raw[k]]
            if ends:
                nb = sum(1 for k in range(i, ends[0]) if raw[k].strip() == "s_barrier")
                if best is None or nb > best[0]:
                    best = (nb, i, ends[0])
    _, hi, back = best
    phases, cur = [], collections.Counter()
    for ln in raw[hi + 1:back + 1]:
        t = ln.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_barrier":
            phases.append(cur)
            cur = collections.Counter()
            continue
        if op.startswith("v_"):
            cur[vclass(op)] += 1
            cur["valu"] += 1
            if op.startswith("v_add_f32"):
                cur["add_f32"] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
        elif op.startswith(("buffer_", "global_")):
            cur["vmem"] += 1
        elif op == "s_waitcnt":
            cur["wait"] += 1
        elif op == "s_nop":
            cur["nop"] += 1
        elif op.startswith("s_"):
            cur["salu"] += 1
    phases.append(cur)
    # the part before the first barrier and the tail after the last one belong to one phase: the tail's
    # [R_{K-1}] read-back runs into the next iteration's VN (gen_fused.py pipelined schedule)
    return [phases[0] + phases[-1]] + phases[1:-1]


def cycles(c):
    return sum(c[k] * COST[k] for k in COST)


def main(paths):
    parts = [parse(p) for p in paths]
    names = ["VN+W0 (+R3)", "CN0+W1", "R0+CN1", "W2+R1", "CN2+W3", "R2+CN3"]
    print("VALU instructions per wave and iteration, by barrier phase (hot loop, one wave of each part)")
    print("part " + "".join(f"{n:>13s}" for n in names) + "     total  add_f32   full   half   vopc    LDS  VMEM  SALU")
    tot = []
    for p, ph in enumerate(parts):
        s = sum(ph, collections.Counter())
        tot.append(s)
        print(f"{p:4d} " + "".join(f"{c['valu']:13d}" for c in ph) +
              f"{s['valu']:10d}{s['add_f32']:9d}{s['full']:7d}{s['half']:7d}{s['vopc']:7d}{s['lds']:7d}{s['vmem']:6d}{s['salu']:6d}")
    print()
    print("VALU issue cycles per wave and iteration at the measured class costs (full 2.2, half 4.2, VOPC 5.2)")
    for p, s in enumerate(tot):
        print(f"part {p}: {cycles(s):8.0f}")
    simd = {0: [0, 2, 4, 6], 1: [1, 3, 5, 7]}
    print()
    worst = 0
    for k, ps in simd.items():
        c = sum(cycles(tot[p]) for p in ps)
        worst = max(worst, c)
        print(f"SIMD set {k} (parts {ps}): {c:8.0f} VALU issue cycles per codeword-iteration")
    E, Z = 197, 384
    edges = E * Z / 64 / 4   # wave-edge-copies per SIMD and iteration
    allv = sum(s["valu"] for s in tot) / 2   # per SIMD (four of the eight parts' waves)
    print()
    print(f"per SIMD and iteration: {allv:.0f} VALU instructions for {edges:.0f} wave-edge copies "
          f"= {allv / edges:.2f} per edge copy; of them add_f32 {sum(s['add_f32'] for s in tot) / 2 / edges:.2f}, "
          f"half-rate {sum(s['half'] for s in tot) / 2 / edges:.2f}, VOPC {sum(s['vopc'] for s in tot) / 2 / edges:.2f}")
    floor_ms = worst * ITERS_PER_CU / (CLK_GHZ * 1e9) * 1e3
    print(f"issue-cycle floor: {worst:.0f} cycles per codeword-iteration on the busier SIMD set = {floor_ms:.1f} ms "
          f"per cfg3 launch at {CLK_GHZ} GHz ({ITERS_PER_CU:.0f} codeword-iterations per CU)")
    print(f"the north-star 22.9 ms (0.60 of HBM) allows {22.9e-3 * CLK_GHZ * 1e9 / ITERS_PER_CU:.0f} cycles per "
          f"codeword-iteration")
    return worst


def write_json(path, worst, source):
    """The budget bench.py reads (roofline.issue_floor_ms): busier-set SIMD issue cycles per workgroup-iteration."""
    import json
    import os
    d = json.load(open(path)) if os.path.exists(path) else {}
    d["fused_bg2_z384::kernel<3, 0>"] = {"simd_issue_cycles_per_wg_iter": int(round(worst)), "G": 1,
                                          "clock_ghz": CLK_GHZ, "source": source}
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    args = sys.argv[1:]
    js = None
    if args and args[0].startswith("--json="):
        js, args = args[0][7:], args[1:]
    worst = main(args)
    if js:
        write_json(js, worst, "tools/isa_budget.sh (gfx950 asm of single-part builds of the library's generator)")
