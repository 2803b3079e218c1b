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

Usage: python tools/isa_budget.py [--func=MANGLED_SUBSTRING --name=KEY --geom=G,P,WPP,THREADS --json=FILE] p0.s p1.s ...
       python tools/isa_budget.py --func=... --lines=30 p0.s   (r6: the loop's VALU cycles by source line; LINES=1 builds)
(tools/isa_budget.sh runs it for any generated kernel; the defaults are the cfg3 decode kernel of
profiles/r4_isa_budget.txt).  r6: any geometry -- the SIMD issue cycles of one workgroup-iteration are the busiest
SIMD's under round-robin wave placement when one workgroup fills the CU (1024 threads), else the workgroup's total
over the 4 SIMDs (a lower bound whatever the residency); per-part register metadata (VGPRs, spills) printed too.
The counts are static: exact for kernels without run-time branches in the loop (the Neural decode kernels; PMC
SQ_INSTS_VALU agrees within 1 %), an over-count for kernels whose loop carries unexecuted branches (UCN, fallbacks).
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


def func_lines(path, func):
    """The asm lines of the kernel whose mangled name contains `func` (all lines when func is None) and its
    register metadata."""
    raw = open(path).read().split("\n")
    meta = {}
    if func:
        start = next(i for i, ln in enumerate(raw)
                     if ln.split(";")[0].strip().endswith(":") and func in ln and not ln.startswith((".", " ", "\t")))
        end = next(i for i in range(start, len(raw)) if raw[i].startswith(".Lfunc_end"))
        name = raw[start].split(";")[0].strip()[:-1]
        text = "\n".join(raw)
        import re
        for blk in re.split(r"\n  - \.", text):
            if f".name:           {name}" in blk or f"name:           {name}" in blk:
                for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
                    m = re.search(rf"\.{key}:\s+(\d+)", blk)
                    if m:
                        meta[key] = int(m.group(1))
        raw = raw[start:end]
    return raw, meta


def parse(path, func=None):
    raw, meta = func_lines(path, func)
    parse.meta = meta
    # the iteration loop: of the labels the asm comments as "Loop Header", the one whose body (header to the
    # last branch back to it) holds the most s_barrier instructions (the Boosted kernels have other loops)
    best = None
    for i, ln in enumerate(raw):
        # (any label with a later branch back to it: the asm does not always comment the loop header)
        if ln.startswith(".LBB") and ln.split(";")[0].strip().endswith(":"):
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


def line_costs(path, func, top=30):
    """(r6, --lines=N) VALU issue cycles of the hot loop by source line, from asm compiled with -gline-tables-only
    (tools/isa_budget.sh LINES=1): the .loc before each instruction names the innermost inlined source line."""
    import re
    text = open(path).read().split("\n")
    files = {}
    for ln in text:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', ln)
        if m:
            files[int(m.group(1))] = m.group(3).split("/")[-1]
    raw, _ = func_lines(path, func)
    best = None
    for i, ln in enumerate(raw):
        if ln.startswith(".LBB") and ln.split(";")[0].strip().endswith(":"):
            label = ln.split(":")[0]
            ends = [k for k in range(len(raw) - 1, i, -1) if raw[k].strip().startswith("s_")
                    and raw[k].strip().split()[-1] == label and "branch" in raw[k]]
            if ends:
                nb = sum(1 for k in range(i, ends[0]) if raw[k].strip() == "s_barrier")
                if best is None or nb > best[0]:
                    best = (nb, i, ends[0])
    _, hi, back = best
    cur, cyc, ops = "?", collections.Counter(), collections.defaultdict(collections.Counter)
    for ln in raw[hi + 1:back + 1]:
        t = ln.split(";")[0].strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = f"{files.get(int(m.group(1)), m.group(1))}:{m.group(2)}"
            continue
        if t and not t.startswith(".") and not t.endswith(":") and t.split()[0].startswith("v_"):
            op = t.split()[0]
            cyc[cur] += COST[vclass(op)]
            ops[cur][op] += 1
    tot = sum(cyc.values())
    print(f"{path}: {tot:.0f} VALU issue cycles per wave and iteration, by source line")
    for k, v in cyc.most_common(top):
        print(f"{v:8.0f} {100 * v / tot:5.1f}%  {k:30s} " + " ".join(f"{o}:{n}" for o, n in ops[k].most_common(4)))


def cycles(c):
    return sum(c[k] * COST[k] for k in COST)


def main(paths, func=None, geom=(1, 8, 2, 1024)):
    parts, metas = [], []
    for p in paths:
        parts.append(parse(p, func))
        metas.append(parse.meta)
    G, P, WPP, THREADS = geom
    nph = max(len(ph) for ph in parts)
    names = (["VN+W0 (+R3)", "CN0+W1", "R0+CN1", "W2+R1", "CN2+W3", "R2+CN3"] if nph == 6 and func is None
             else [f"phase {k}" for k in range(nph)])
    if any(metas):
        print("registers per part (single-part builds): " + "; ".join(
            f"p{p}: {m.get('vgpr_count')} VGPR / {m.get('vgpr_spill_count')} spilled, {m.get('sgpr_spill_count')} SGPR spills"
            for p, m in enumerate(metas)))
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
    print()
    if THREADS == 1024:  # one workgroup per CU: waves placed round-robin, wave w = p * WPP + k on SIMD w % 4
        load = [0.0] * 4
        for p, s_ in enumerate(tot):
            for k in range(WPP):
                load[(p * WPP + k) % 4] += cycles(s_)
        worst = max(load)
        print("SIMD issue cycles per workgroup-iteration (one workgroup per CU, round-robin waves): " +
              ", ".join(f"SIMD {k} {c:.0f}" for k, c in enumerate(load)))
    else:  # several workgroups per CU: the workgroup's total over the 4 SIMDs (a lower bound)
        worst = sum(cycles(s_) * WPP for s_ in tot) / 4
        print(f"SIMD issue cycles per workgroup-iteration (workgroup total / 4 SIMDs): {worst:.0f}")
    if func is not None:
        return worst
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


def write_json(path, worst, source, name="fused_bg2_z384::kernel<3, 0>", G=1, threads=1024):
    """The budget bench.py reads (roofline.issue_floor_ms): busiest-SIMD issue cycles per workgroup-iteration."""
    import json
    import os
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[name] = {"simd_issue_cycles_per_wg_iter": int(round(worst)), "G": G, "threads": threads,
               "model": "busiest SIMD, one workgroup per CU" if threads == 1024 else "workgroup total / 4 SIMDs",
               "clock_ghz": CLK_GHZ, "source": source}
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    opts = {a.split("=", 1)[0][2:]: a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--")}
    files = [a for a in sys.argv[1:] if not a.startswith("--")]
    geom = tuple(int(v) for v in opts["geom"].split(",")) if "geom" in opts else (1, 8, 2, 1024)
    if "lines" in opts:
        for f_ in files:
            line_costs(f_, opts.get("func"), int(opts["lines"]))
        sys.exit(0)
    worst = main(files, opts.get("func"), geom)
    if "json" in opts:
        write_json(opts["json"], worst, "tools/isa_budget.sh (gfx950 asm of single-part builds of the library's generator)",
                   opts.get("name", "fused_bg2_z384::kernel<3, 0>"), geom[0], geom[3])
