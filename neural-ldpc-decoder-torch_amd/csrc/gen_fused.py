"""Generate the register-resident fused decoder kernels (lib/gen/fused_*.hip) for known base graphs.

Design (DESIGN.md §Fused kernel): one workgroup decodes G codewords for all T iterations without
touching HBM for message state.  The c2v messages of a codeword (E*Z floats, 302 KB for BG2 z=384)
live in the REGISTERS of the threads that own their variable copies: the columns are split into P
parts; thread (part p, codeword g, lane copy u) owns every edge of the columns of part p at the Q
copies v = u + q*Z/Q, so the variable-node update (sum of the others, sequential fp32 in ascending
check row: the reference's sgemm order) is register-only code.  The check-node update needs each
row's messages at cyclically shifted copies, so per iteration the v2c messages go through LDS in row
chunks: owners write a chunk, every thread runs the check nodes of its rows of that chunk in LDS
(gather at (h + s) mod Z, update, scatter back to the same addresses), owners read the new c2v
back.  Degree-1 columns keep no state at all (their v2c is the channel value; their c2v only feeds
their own posterior, written as soon as it comes back).  HBM traffic per codeword: the channel LLRs
(re-read from L2 every iteration) and the T posteriors the API returns.

Everything that indexes registers is emitted as straight-line code with literal indices, so the
generator needs the graph structure at build time; the per-edge arithmetic is the shared
nldpc_node.h / nldpc_fused.h code, identical to the streaming kernels (tests compare both paths).

Usage: python3 gen_fused.py OUTDIR RESOURCE_DIR   (or --list: the generated file names)
"""
import os
import sys

import numpy as np

PARTS = [int(x) for x in filter(None, os.environ.get("NLDPC_GEN_PARTS", "").split(","))]  # debug
# graphs whose decode unit also carries the MODE-6 kernels (UCN with CN / UCN / cumulative VN weights: the Boosted
# NW(1,1,2) decode of the bench's cfg3ucn side lines); the others decode such configurations on MODE 0
UCNW_TAGS = set(filter(None, os.environ.get("NLDPC_GEN_UCNW", "bg2_z384").split(",")))
SKIP = set(filter(None, os.environ.get("NLDPC_GEN_SKIP", "").split(",")))  # debug: drop phases
# diagnostic build only (make STAMPS=1 -> lib_stamps/): s_memtime at every phase boundary of the forward
# kernels, lane 0 of each wave, first 256 workgroups (FusedArgs::stamps, tools/stamps.py)
STAMPS = os.environ.get("NLDPC_GEN_STAMPS") == "1"
LDS_BYTES = 160 * 1024 - 2048  # leave room for the compiler / alignment


def app_words(N, Z):
    """32-bit words of one codeword's UCN hard-decision bit array (bit (j, v) = APP[j][v] >= 0): per column
    the Z bits and one more word (word 0 again, so a 32-bit window at any start reads two words)."""
    return N * ((Z + 31) // 32 + 1)
# Generator knobs left after the r5 prune (every measured loser is gone; its A/B stays in profiles/):
#   NLDPC_GEN_PARTS / _SKIP / _STAMPS / _ONLY / _KINDS / _NOBWD   debug and diagnostic builds (above / main)
#   NLDPC_GEN_GEOM    experiment: override a spec's (G, P, Q)
#   NLDPC_GEN_WLATE   when a chunk's check-node weights are loaded (below)
#   NLDPC_FUSED_EXTRA more built-in (graph, Z) pairs
# Settled choices, no longer knobs (cfg3 kernel ms in the same-box A/B records):
# * VN lane copies as scalar v_add_f32 chains, two chains (k, k+1) interleaved: packed v_pk_add_f32 pairs issue
#   at the same adds per cycle on gfx950 (tools/dev/valu_rate2.hip) and spilled (profiles/r2_ab_schedule.txt)
# * pipelined chunk schedule for the decode / count-only kernels (two LDS buffers, each phase mixes one chunk's
#   check nodes with another chunk's owner traffic; cfg3 55.2 vs 58.7 ms, r2); the SAVE kernels keep one buffer
# * check-node row copies software-pipelined one ahead (the next row copy's LDS reads issued before the current
#   one computes); deeper prefetch 48.5 / 48.8 (profiles/r4_ab.txt)
# * check-node work balanced by (row, lane copy) units (LPT by degree)
# * check-row LDS addresses from one 32-bit base per thread (Neural / MS; cfg3 51.7 -> 50.9 ms)
# * SAVE kernels copy the chunk image to the saved v2c buffer in 16-byte pieces (profiles/r3f_stamps.txt)
# * backward weight-gradient sums per lane copy (QMS z=384 3135 -> 16 spilled VGPRs), one fence per lane copy
#   (profiles/r4_ab.txt: 27.97 -> 27.32 ms without the per-row fence)
# * VN chains keep the reference's explicit "0 +" starts (without them 48.49 -> 48.94 ms, profiles/r3b_ab.txt)
# * QMS VN as total minus own message (QEXACT, r4: exact on the quantiser's 0.5 grid)
# * degree-1 bypass for Neural, MS and QMS decode (D1B, r4)
# * Boosted posterior channel values (cumulative VN weights) requested before a VN call's first store (XPRE=2,
#   cfg3 MS NW(1,0,2) 99.9 -> 92.5 ms)
# * UCN flag of a check copy: the row's bit words all read before the shifts and XORs (UCNB, r4p)
# Removed as measured losers: wave-ballot UCN bits (UCNWAVE, UCNBW), lane-mask wrapped copies (WRAPMASK),
# paired check rows (CNPAIR, CNPAIR2), owner / check-node ds_write_addtid (OWNTID, CNTID), s_setprio by phase
# (PRIO), early VN sums in the LDS-only phase (EARLYVN), owner-traffic-aware CN balance (CNBAL_ALPHA), phase
# weight loads (WPHASE), tied backward by units (TIEDUNITS), QMS wave UCN (UCNW_QMS), no row-base barrier (NORO).

# When a chunk's check-node weights are loaded: a phase ahead (with the chunk's owner writes; Neural) or at
# the start of its check-node phase (one chunk's weights in SGPRs at a time instead of two; Boosted, whose
# kernels spilled SGPRs: cfg3ucn MS NW(1,1,2) 97.3 -> 92.6 ms, QMS 100.1 -> 99.8, profiles/r4_ab.txt).
# NLDPC_GEN_WLATE: "boosted" (default), "0" every kind early, "1" every kind late
WLATE = os.environ.get("NLDPC_GEN_WLATE", "boosted")
WLATE_COND = {"boosted": "KIND != NLDPC_NEURAL", "0": "false", "1": "true"}[WLATE]
NOBWD = os.environ.get("NLDPC_GEN_NOBWD") == "1"  # experiment builds without backward kernels (faster)
# SAVE kernels of one-codeword geometries: lane offsets re-derived per phase, buffer-descriptor saves (r5: the
# cfg5 training forward 11.57 -> 11.38 ms, profiles/r5i_ab_uremat.txt); NLDPC_GEN_UREMAT=0 turns it off
UREMAT = os.environ.get("NLDPC_GEN_UREMAT", "1") == "1"
# r6 backward (cfg5, profiles/r6_ab_cfg5_bwd.txt; every variant's gradients bit-identical, tools/grad_digest.py):
#   NLDPC_GEN_BWDPIPE (default 1): the read-backs' degree-1 VN-weight chains software-pipelined one deep (25.0 -> 24.0 ms)
#   NLDPC_GEN_CNBSPARSE (default 1): the tied kernel's check node with a third fewer VALU (nldpc_node.h NLDPC_CNB_SPARSE:
#   QMS ordering keys, branch-free minima, sparse pass 3) and its wave sum in a register (24.0 -> 20.7 ms)
BWDPIPE = os.environ.get("NLDPC_GEN_BWDPIPE", "1") == "1"
CNBSPARSE = os.environ.get("NLDPC_GEN_CNBSPARSE", "1") == "1"
TACC = CNBSPARSE
# r6 cache policies (profiles/r6_ab_cfg5_cache.txt): NLDPC_GEN_BWDCACHE (default 2) -- the backward's VN-weight carry
# stored temporal (1) and its per-iteration streams (xin, dL/dy, masks, staged messages) loaded non-temporal (2), so the
# carry's read-back one iteration later hits L2 (nldpc_fused.h bload_nt / gy_masked_nt / bstore_keep): backward 20.8 ->
# 20.3 ms, fetch 36.5 -> 27.9 GB; NLDPC_GEN_FWDNT8 (default 1) -- the training forward's byte stores (clamp masks, QMS
# saved codes) non-temporal like its fp32 stores: they were evicting the channel values its posteriors re-read (fetch
# 9.8 -> 1.8 GB, 10.3 -> 9.7 ms)
BWDCACHE = int(os.environ.get("NLDPC_GEN_BWDCACHE", "2"))
_CY_ST = "bstore_keep" if BWDCACHE >= 1 else "bstore"
_LD_NT = "bload_nt" if BWDCACHE >= 2 else "bload"
_GY = "gy_masked_nt" if BWDCACHE >= 2 else "gy_masked"
FWDNT8 = os.environ.get("NLDPC_GEN_FWDNT8", "1") == "1"  # (see nldpc_fused.h bstore8_nt)
_S8 = "bstore8_nt" if FWDNT8 else "bstore8"
_SI8 = "bstore_i8_nt" if FWDNT8 else "bstore_i8"

# (tag, base graph file, Z, codewords per workgroup G, parts P, copies per thread Q); G/P/Q None =
# chosen by auto_geometry
SPECS = [
    ("bg2_z384", "basegraph2_set0.txt", 384, 1, 8, 3),
    ("bg2_z16", "basegraph2_set0.txt", 16, 16, 2, 1),
    ("wimax_z24", "wman_N0576_R34_z24.txt", 24, 8, 4, 1),  # r4: 0.160 -> 0.114 ms at cfg2 (profiles/r4_ab.txt)
    ("bg2_z96", "basegraph2_set0.txt", 96, None, None, None),
]
# More (graph, Z) pairs at build time: NLDPC_FUSED_EXTRA="bg2:192,wimax:48,<file.txt>:Z" (base graph
# files from resources/; bg2 / wimax name the two shipped ones).  Every other lifted graph decodes on
# the streaming kernels.
_GRAPH_FILES = {"bg2": "basegraph2_set0.txt", "wimax": "wman_N0576_R34_z24.txt"}
for _item in filter(None, os.environ.get("NLDPC_FUSED_EXTRA", "").split(",")):
    _g, _z = _item.rsplit(":", 1)
    _f = _GRAPH_FILES.get(_g, _g)
    _tag = f"{_g if _g in _GRAPH_FILES else os.path.splitext(os.path.basename(_g))[0]}_z{int(_z)}"
    if all(t[0] != _tag for t in SPECS):
        SPECS.append((_tag, _f, int(_z), None, None, None))

# experiment knob: NLDPC_GEN_GEOM="bg2_z384:1,4,3" overrides a spec's (G, P, Q)
for _item in filter(None, os.environ.get("NLDPC_GEN_GEOM", "").split(";")):
    _t, _g = _item.split(":")
    SPECS = [(t, f, z, *[int(v) for v in _g.split(",")]) if t == _t else (t, f, z, g, p, q) for t, f, z, g, p, q in SPECS]


MAX_STATE_REGS = 72  # register-resident c2v floats per thread (the z=384 kernel holds 69 at 124 VGPRs)
REG_ROOM = 81  # state + degree-1 channel values per thread (r4's z=384 part 0: 69 + 12, no VGPR spills)


def auto_geometry(hb, Z):
    """(G, P, Q) for a lifted graph: G codewords x P parts x Z/Q lanes per workgroup, at most 1024
    threads, at most MAX_STATE_REGS state floats per thread, check rows that fit LDS.  A part's lanes are
    padded to whole waves (the extra lanes repeat live ones, Spec.lanes_pad), at most a third of them
    idle.  Prefers >= 512 threads, then fewer LDS chunks (fewer barriers), then fewer idle lanes, then
    more threads, then fewer copies per thread."""
    rows, cols = np.nonzero(hb != -1)
    deg = np.bincount(cols, minlength=hb.shape[1])
    multi = [int(d) for d in deg if d > 1]
    row_deg = np.bincount(rows, minlength=hb.shape[0])
    best = None
    for Q in [q for q in range(1, Z + 1) if Z % q == 0]:
        ZT = Z // Q
        for G in (1, 2, 4, 8, 16, 32):
            lanes = G * ZT
            pad = -(-lanes // 64) * 64
            if pad * 3 > lanes * 4:  # more than a quarter of the part idle
                continue
            for P in (8, 7, 6, 5, 4, 3, 2, 1):
                threads = P * pad
                if threads > 1024:
                    continue
                load = [0] * P
                for d in sorted(multi, reverse=True):
                    load[int(np.argmin(load))] += d
                if Q * max(load) > MAX_STATE_REGS:
                    continue
                GL = G + (1 if pad != lanes else 0)  # (+1: the repeating lanes' LDS region, Spec.G_lds)
                cap = ((LDS_BYTES - 4 * GL * app_words(hb.shape[1], Z)) // (4 * GL) - 32) // Z  # edges per LDS chunk
                if cap < int(row_deg.max()):
                    continue
                nchunks, acc = 1, 0
                for d in row_deg:
                    if acc + d > cap:
                        nchunks, acc = nchunks + 1, 0
                    acc += int(d)
                key = (threads >= 512, -nchunks, -(pad - lanes) / pad, threads, -Q)
                if best is None or key > best[0]:
                    best = (key, (G, P, Q))
    if best is None:
        raise SystemExit(f"gen_fused: no register-resident geometry for Z={Z}")
    return best[1]


def balance(items, weight, P):
    """Greedy partition of items (heaviest first) into P bins of similar total weight."""
    load = [0] * P
    bins = [[] for _ in range(P)]
    for it in sorted(items, key=lambda x: -weight(x)):
        k = int(np.argmin(load))
        bins[k].append(it)
        load[k] += weight(it)
    return [sorted(b) for b in bins]


class Spec:
    def __init__(self, tag, hb, Z, G, P, Q, sched="one", stage=0):
        """sched: the per-iteration chunk schedule -- "one" (one LDS image: write | check nodes | read-back
        per chunk; the SAVE kernels) or "pipe2" (two buffers, pipelined: the decode and count-only kernels);
        see emit().
        stage (backward kernels): bytes per message of the saved v2c staged in LDS beside the chunk
        image (4 fp32, 1 QMS int8 codes; 0 = none, the check nodes gather from global memory)."""
        assert Z % Q == 0
        self.tag, self.hb, self.Z, self.G, self.P, self.Q = tag, hb, Z, G, P, Q
        assert sched in ("one", "pipe2"), sched
        self.sched = sched
        self.pipe = sched != "one"  # two LDS buffers (not the SAVE kernels' schedule)
        self.ZT = Z // Q
        self.M, self.N = hb.shape
        rows, cols = np.nonzero(hb != -1)
        self.E = len(rows)
        self.shift = hb[rows, cols] % Z
        self.row_edges = [[int(e) for e in np.nonzero(rows == i)[0]] for i in range(self.M)]
        self.col_edges = [[int(e) for e in np.nonzero(cols == j)[0]] for j in range(self.N)]
        deg = lambda j: len(self.col_edges[j])  # noqa: E731
        multi = [j for j in range(self.N) if deg(j) > 1]
        single = [j for j in range(self.N) if deg(j) == 1]
        self.reg_cols = balance(multi, deg, P)  # columns whose messages live in registers
        # waves of a workgroup go round the 4 SIMDs, so with 2-wave parts the even parts share SIMDs
        # {0,1} and the odd parts SIMDs {2,3}; the VN phase saturates the SIMDs, so order the parts
        # for equal VN work (sequential adds per lane copy) on the two sets
        if P == 8 and G * self.ZT == 128:
            import itertools
            cost = [sum(deg(j) * (deg(j) - 1) // 2 + 2 * deg(j) + 1 for j in c) for c in self.reg_cols]
            best = min(itertools.combinations(range(P), P // 2),
                       key=lambda e: abs(sum(cost[k] for k in e) * 2 - sum(cost)))
            odd = [k for k in range(P) if k not in best]
            self.reg_cols = [self.reg_cols[k] for pair in zip(best, odd) for k in pair]
        self.d1_cols = balance(single, lambda j: 1, P)  # stateless degree-1 columns
        self.slots = [[e for j in cols_ for e in self.col_edges[j]] for cols_ in self.reg_cols]
        self.smax = max(1, max(len(s) for s in self.slots)) * Q
        # row chunks: contiguous row ranges whose messages (edges x Z x G) fit in LDS beside the UCN bits
        self.WZ = (Z + 31) // 32
        self.WZX = self.WZ + 1  # words per column in the bit array
        self.lanes = G * self.ZT  # live threads per part
        # A part occupies whole waves.  The lanes past the live ones (padded parts) run the code of the
        # first live lanes (same copies) on an LDS region of their own and with global offsets out of
        # every descriptor's range: nothing they compute reaches the live codewords' messages, outputs,
        # counters or gradient sums.  (Sharing the live lanes' LDS would race: a check node updates its
        # slots in place, and a repeating lane in a later wave could read the updated value.)
        self.lanes_pad = -(-self.lanes // 64) * 64
        self.padded = self.lanes_pad != self.lanes
        self.G_lds = G + (1 if self.padded else 0)  # codeword LDS regions (+1: the repeating lanes')
        self.threads = P * self.lanes_pad
        assert self.threads <= 1024, (tag, self.threads)
        GL = self.G_lds
        cap = ((LDS_BYTES - 4 * GL * app_words(self.N, Z)) // (4 * GL) - 32) // Z
        row_max = max(len(r) for r in self.row_edges)
        if self.pipe:  # two buffers; only the count-only counters (G*128 B) share the remaining KiB
            cap = ((160 * 1024 - 1024 - 4 * GL * app_words(self.N, Z)) // (8 * GL) - (32 if GL > 1 else 0)) // Z

        def chunking(cap, stage):
            chunks, r0 = [], 0  # (row_begin, row_end, edge_begin, edge_end)
            while r0 < self.M:
                e0 = self.row_edges[r0][0]
                r1 = r0
                while r1 < self.M and self.row_edges[r1][-1] - e0 + 1 <= cap:
                    r1 += 1
                if r1 == r0:
                    return None
                chunks.append((r0, r1, e0, self.row_edges[r1 - 1][-1] + 1))
                r0 = r1
            cf = max(e1 - e0 for _, _, e0, e1 in chunks) * Z
            if GL > 1:  # codeword stride = 1 (mod 32 banks) so lanes of different codewords do not collide
                cf += (1 - cf) % 32
            # staged saved messages: one region per codeword, 16-byte aligned
            sf = -(-(max(e1 - e0 for _, _, e0, e1 in chunks) * Z * stage) // 16) * 4 if stage else 0
            return chunks, cf, sf

        if stage:  # the largest chunks whose image and staged messages fit beside each other
            c = cap
            while c >= row_max:
                got = chunking(c, stage)
                if got and (got[1] + got[2]) * 4 * GL <= LDS_BYTES - 4 * GL * app_words(self.N, Z):
                    break
                c -= 1
            else:
                stage = 0  # a row and its staged messages do not fit: gather from global memory
            if stage:
                cap = c
        got = chunking(cap, stage)
        if got is None:
            raise SystemExit(f"{tag}: a single check row does not fit in LDS")
        self.chunks, self.chunk_floats, self.stage_floats = got
        self.nbuf = 2 if self.pipe and len(self.chunks) > 1 else 1  # (one chunk: the second buffer would stay unused)
        # LDS float offset of chunk c's image in a codeword's block, and the block's size
        self.region_off = [(c % self.nbuf) * self.chunk_floats for c in range(len(self.chunks))]
        self.cw_floats = self.chunk_floats * self.nbuf
        self.stage = stage
        # LDS-DMA width of the staging: 16 B when every chunk's block (and the per-codeword stride of
        # the saved buffer) is a multiple of 16 B, else 4 B
        blocks = [(e0 * Z * stage, (e1 - e0) * Z * stage) for _, _, e0, e1 in self.chunks] + [(0, self.E * Z * stage)]
        self.stage_width = 16 if stage and all(o % 16 == 0 and n % 16 == 0 for o, n in blocks) else \
            4 if stage and all(o % 4 == 0 and n % 4 == 0 for o, n in blocks) else 0
        if stage and not self.stage_width:
            self.stage, self.stage_floats = 0, 0
        self.cn_rows = [balance(list(range(r0, r1)), lambda i: len(self.row_edges[i]), P)
                        for (r0, r1, _, _) in self.chunks]
        # forward check-node work units (row i, lane copy q) of each chunk, balanced over the parts by
        # degree (LPT): a row's Q copies may go to different parts.  A check-node phase is bound by
        # its busiest wave (a chain of LDS round trips, one per row copy), and whole rows balanced
        # badly: BG2 z=384 chunk 0 has 7 rows for 8 parts (edge copies per lane 30, 30, 24, 24, 18,
        # 18, 12, 0; by units at most 21)
        # Register room: a unit's degree-1 edges stay in its part's registers for the whole decode (the bypass,
        # `cd`), on top of the part's state; a part is offered a unit only while state + cd fits REG_ROOM (the
        # z=384 parts 0/1 hold 69/66 state floats), else the least-loaded part takes it anyway.
        d1e = {self.col_edges[j][0] for j in single}
        nd1 = [sum(1 for e in self.row_edges[i] if e in d1e) for i in range(self.M)]
        regs = [Q * len(sl) for sl in self.slots]
        self.cn_units = []
        for ci, (r0, r1, _, _) in enumerate(self.chunks):
            units = sorted(((i, q) for i in range(r0, r1) for q in range(Q)),
                           key=lambda iq: (-len(self.row_edges[iq[0]]), iq[0], iq[1]))
            load = [0] * P
            bins = [[] for _ in range(P)]
            for i, q in units:
                fit = [k for k in range(P) if regs[k] + nd1[i] <= REG_ROOM]
                k = min(fit or range(P), key=lambda k_: (load[k_], k_))
                bins[k].append((i, q))
                load[k] += len(self.row_edges[i]) + 1  # + the row's fixed work
                regs[k] += nd1[i]
            self.cn_units.append([sorted(b, key=lambda iq: (-len(self.row_edges[iq[0]]), iq[0], iq[1])) for b in bins])
        self.max_dc = max(len(r) for r in self.row_edges)
        # UREMAT applies where a wave's lanes are consecutive copies of one codeword: u = (wave base) + lane
        self.uremat = UREMAT and not self.pipe and G == 1 and not self.padded and self.ZT % 64 == 0  # (the SAVE kernels)
        self.hb_cols = cols  # column of each C-order edge


def emit(S: Spec) -> str:
    Z, G, Q, ZT, NZ = S.Z, S.G, S.Q, S.ZT, S.N * S.Z
    L = []
    w = L.append
    CF = S.chunk_floats
    # wrapped lane copies by scalar lane masks (own_lv): needs waves of 64 consecutive copies of one codeword
    w(f"// ---- {S.tag}: M={S.M} N={S.N} E={S.E} Z={Z}; workgroup = {G} codeword(s) x {S.P} part(s) x {ZT} lanes "
      f"= {S.threads} threads{' (padded parts)' if S.padded else ''}, {Q} cop{'y' if Q == 1 else 'ies'} per lane; register slots/part "
      f"{[len(s) * Q for s in S.slots]}; {len(S.chunks)} LDS chunk(s) of <= {CF * G * 4} B")
    w(f"namespace fused_{S.tag} {{")
    w(f"constexpr int Z = {Z}, ZT = {ZT}, N = {S.N}, E = {S.E};")
    w("// degree-1 edges bypass LDS (Neural inference; see the check-node section)")
    # MODE 0: decode, MODE 1: decode and save what the backward needs, MODE 2 / 3: count-only decode
    # (the posteriors are compared with the codeword and counted instead of stored):
    # 2 = all-zero codeword, decoder convention; 3 = either convention, against y when given
    # MODE 5 (r6): MODE 1 specialised for one CN weight per iteration (sharing code 3) and no UCN -- the tied saving
    # forward fused_forward picks for NLDPC_FLAG_CN_TIED (FusedSpec::save_tied)
    w("#define SAVE (MODE == 1 || MODE == 5)")
    w("#define CNT (MODE == 2 || MODE == 3)")
    w("#define CM (CNT ? MODE - 1 : 0)  // put_post: store / count / count against y")
    w("#define TIEDW (MODE == 5)")
    # MODE 6 (r6): MODE 0 specialised for UCN on with CN weights, UCN weights and cumulative VN weights all given -- the
    # Boosted NW(1,1,2)-like decode: its runtime flags become constants, so their uniform branches and the SGPRs holding
    # the conditions leave the loop (a part of the MS kernel spilled 110 SGPRs, 48 specialised)
    w("#define UCNW (MODE == 6)")
    w("#define UCN_ON (!TIEDW && (UCNW || a.ucn))  // (the tied saving forward has no UCN code)")
    w("#define WVN_ON (UCNW || a.w_vn != nullptr)")
    w("// check-row LDS addresses from one 32-bit base (ROADDR); in the QMS / SP kernels it measured slower")
    w("#define ROA (KIND == NLDPC_NEURAL || KIND == NLDPC_MS)")
    assert NZ < 65536  # per-codeword error counts are packed two to an LDS word

    # Register state of part p: one float array per lane copy q (cs{q}[slot]).  The channel values a thread
    # needs every iteration are loaded once into registers (xs{q} for its register columns; those of the
    # degree-1 columns are held by the check-node threads, cd).
    def ref(p, q, k):
        return f"cs{q}[{k}]"

    def xref(p, j, q):
        return f"xs{q}[{S.reg_cols[p].index(j)}]"

    def state_params(p, const=False):
        sp = len(S.slots[p])
        c = "const " if const else ""
        return ", ".join(f"{c}float (&cs{i})[{max(sp, 1)}]" for i in range(Q))

    def state_args(p):
        return ", ".join(f"cs{i}" for i in range(Q))

    def x_params(p):
        nr = max(len(S.reg_cols[p]), 1)
        return ", ".join(f"const float (&xs{i})[{nr}]" for i in range(Q))

    def x_args(p):
        return ", ".join(f"xs{i}" for i in range(Q))

    # UCN hard decisions of the posteriors of a thread's cd entries (cdm) -- a bit array of 32-bit words, as many
    # as the part needs (a run-time geometry with few parts can hold more than 32)
    def nwords(p):
        return max(1, -(-len(S.cd_index[p]) // 32))

    def bit_get(arr, b):
        return f"({arr}[{b >> 5}] >> {b & 31})"

    def bit_set(arr, b, cond):
        return f"{arr}[{b >> 5}] = ({arr}[{b >> 5}] & ~(1u << {b & 31})) | (({cond}) ? 1u : 0u) << {b & 31}"

    # ---------------------------------------------------------------- variable nodes
    # global accesses: bload/bstore(descriptor, lane byte offset vo, constant byte offset)
    def X(j, q):  # byte offset of variable copy (column j, lane copy q) in a [N][Z] codeword
        return 4 * (j * Z + q * ZT)

    def vn_col(p, n, j, s, d, final):
        """VN (or final posterior) of column j (n-th register column of part p) for every lane copy at
        once: the copies' chains are emitted interleaved, so consecutive adds never depend on each other.
        Each chain is the reference's sequential fp32 order: S_k = ((P_{k-1} + c_{k+1}) + ...) + c_{d-1},
        v2c_k = x0 + S_k, P_k = P_{k-1} + c_k (the chains start from the reference's explicit 0)."""
        grp = [(f"cs{i}", f"xs{i}[{n}]", f"s{i}") for i in range(Q)]
        w(f"        {{  // column {j}, degree {d}")
        for arr, xin, g in grp:
            w(f"            float P_{g} = 0.f;")
        if final:
            for k in range(d):
                for arr, xin, g in grp:
                    w(f"            P_{g} = fadd(P_{g}, {arr}[{s + k}]);")
            return
        for arr, xin, g in grp:
            w(f"            const float x0_{g} = fadd(0.f, chan<KIND>({xin}, a));")
        # QMS: every VN input lies on the quantiser's 0.5 grid with |x| <= 15.5, so every partial sum of a
        # column (<= 24 terms) is exact in fp32 and the reference's sequential S_k equals (x0 + C) - c_k bit
        # for bit (C = the posterior's own sum): d + 1 adds per column copy instead of d(d-1)/2 + d (QEXACT)
        w("            if constexpr (KIND == NLDPC_QMS) {")
        for k in range(d):
            for arr, xin, g in grp:
                w(f"                P_{g} = fadd(P_{g}, {arr}[{s + k}]);")
        for arr, xin, g in grp:
            w(f"                const float tq_{g} = fadd(x0_{g}, P_{g});")
        for k in range(d):
            for arr, xin, g in grp:
                w(f"                {arr}[{s + k}] = __fsub_rn(tq_{g}, {arr}[{s + k}]);")
        w("            } else {")
        # edges two at a time: the chains of k and k+1 (S_k from P_{k-1}, S_{k+1} from P_k) run interleaved --
        # twice the independent adds per wave for the VN's dependent-add tail.  Chain k reads c_{k+1} first,
        # before chain k+1 overwrites it with v2c_{k+1}.
        ind = "            "
        for k in range(0, d, 2):
            w(f"{ind}{{")
            if k + 1 < d:
                for arr, xin, g in grp:
                    w(f"{ind}    const float Pk_{g} = fadd(P_{g}, {arr}[{s + k}]);  // P_k")
                for arr, xin, g in grp:
                    w(f"{ind}    float S_{g} = fadd(P_{g}, {arr}[{s + k + 1}]);")
                    w(f"{ind}    float U_{g} = Pk_{g};")
                for m in range(k + 2, d):
                    for arr, xin, g in grp:
                        w(f"{ind}    S_{g} = fadd(S_{g}, {arr}[{s + m}]);")
                        w(f"{ind}    U_{g} = fadd(U_{g}, {arr}[{s + m}]);")
                for arr, xin, g in grp:
                    w(f"{ind}    const float o_{g} = {arr}[{s + k + 1}];")
                    w(f"{ind}    {arr}[{s + k}] = fadd(x0_{g}, S_{g}); {arr}[{s + k + 1}] = fadd(x0_{g}, U_{g});")
                # the fake dependence of the running prefix on the new messages keeps the compiler from
                # running the prefix chain ahead and holding every partial sum in a register
                for arr, xin, g in grp:
                    w(f"{ind}    asm volatile(\"\" : \"+v\"(P_{g}) : \"v\"({arr}[{s + k}]), \"v\"({arr}[{s + k + 1}]));")
                for arr, xin, g in grp:
                    w(f"{ind}    P_{g} = fadd(Pk_{g}, o_{g});")
            else:
                for arr, xin, g in grp:
                    w(f"{ind}    float S_{g} = P_{g};")
                for arr, xin, g in grp:
                    w(f"{ind}    const float o_{g} = {arr}[{s + k}]; {arr}[{s + k}] = fadd(x0_{g}, S_{g});")
                for arr, xin, g in grp:
                    w(f"{ind}    asm volatile(\"\" : \"+v\"(P_{g}) : \"v\"({arr}[{s + k}]));")
                for arr, xin, g in grp:
                    w(f"{ind}    P_{g} = fadd(P_{g}, o_{g});")
            w(f"{ind}}}")
        w("            }")

    for p in range(S.P):
        cols = S.reg_cols[p]
        for final in (False, True):
            fname = f"post_p{p}" if final else f"vn_p{p}"
            w("template <int KIND, int MODE>")
            w(f"__device__ __forceinline__ void {fname}({state_params(p)}, {x_params(p)}, const FusedArgs& a, "
              f"uint32_t vo, int it, rsrc_t pr, uint32_t vm, rsrc_t xr, rsrc_t pm, PostSink& ps, uint32_t* appw, int u, "
              f"rsrc_t apr) {{")
            if not final:
                w("    const bool ucn_ = KIND != NLDPC_NEURAL && UCN_ON;  // UCN: hard decisions of the previous posterior")
            # every posterior's xa (cumulative VN weights) requested before the first posterior store: a later
            # load would wait (vmcnt counts loads and stores in order) for every store issued before it (XPRE)
            # (r6: one branch for the whole group -- a select per load compiled to a branch per load, each reloading the
            # spilled descriptor's four SGPRs by v_readlane)
            xls = [(n, j, i) for n, j in enumerate(cols) for i in range(Q)]
            if "xlreg" in SKIP:  # (fetch bisect, wrong results: the posterior's xa re-read replaced by xin)
                for n, j, i in xls:
                    w(f"    const float xl_{n}_{i} = xs{i}[{n}];")
            elif xls:
                w("    float " + ", ".join(f"xl_{n}_{i}" for n, j, i in xls) + ";")
                w("    if (KIND != NLDPC_NEURAL && WVN_ON) {")
                for n, j, i in xls:
                    w(f"        xl_{n}_{i} = bload(xr, vo, {X(j, i)});")
                w("    } else {")
                for n, j, i in xls:
                    w(f"        xl_{n}_{i} = xs{i}[{n}];")
                w("    }")
            s = 0
            for n, j in enumerate(cols):
                d = len(S.col_edges[j])
                vn_col(p, n, j, s, d, final)
                for q in range(Q):
                    w("            {")
                    w(f"            const float xo_ = xl_{n}_{q};")
                    w("            float y_;")
                    w("            if constexpr (SAVE && KIND != NLDPC_NEURAL) {")
                    w("                bool m_;")
                    w(f"                y_ = posterior_m<KIND>(xo_, P_s{q}, a, m_);")
                    w(f"                bstore(pr, vo, {X(j, q)}, y_);")
                    w(f"                {_S8}(pm, vm, {X(j, q) // 4}, m_);")
                    w("            } else {")
                    w(f"                y_ = posterior<KIND>(xo_, P_s{q}, a);")
                    w(f"                put_post<CM>(pr, vo, {X(j, q)}, y_, ps);")
                    w("            }")
                    if not final:
                        app0 = f"(a.first_iter > 0 ? bload(apr, vo, {X(j, q)}) : chan<KIND>(xs{q}[{n}], a))"
                        w(f"            if (ucn_) app_or(appw, {j * S.WZX}, u + {q * ZT}, (it == 0 ? {app0} : y_) >= 0.f);")
                    w("            }")
                w("        }")
                w("        __builtin_amdgcn_sched_barrier(0);")
                s += d
            # (degree-1 columns: their UCN hard decisions are the check-node threads' own, cdm)
            w("}")

    # ---------------------------------------------------------------- LDS chunk write / read-back
    def own(e, q, e0):
        """LDS index (expression in u) where the owner of variable copy u + q*ZT puts edge e's message:
        check copy h = (v - s_e) mod Z of the chunk's check-ordered image.  Only one of the Q copies
        of a shifted edge can wrap inside the lane range; the others are a constant offset."""
        cq = (q * ZT - int(S.shift[e])) % Z
        base = (e - e0) * Z + cq
        if cq + ZT <= Z:
            return f"{base} + u"
        return f"{base} + u - (u >= {Z - cq} ? {Z} : 0)"

    def own_lv(e, q, e0):
        return f"lds[{own(e, q, e0)}]"

    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            mine = [(k, e) for k, e in enumerate(S.slots[p]) if e0 <= e < e1]
            # (degree-1 edges never enter the image: their check-node threads form their v2c, posteriors, clamp
            # masks, saved v2c and xin themselves -- cn_p)
            w("template <int KIND, int MODE>")
            w(f"__device__ __forceinline__ void wr_p{p}_c{ci}({state_params(p, True)}, {x_params(p)}, float* lds, "
              f"int u, const FusedArgs& a, int it, rsrc_t sv, uint32_t vc) {{")
            w("    asm volatile(\"\" : \"+v\"(u));  // LDS addresses are recomputed here, not hoisted out of the loop")
            for q in range(Q):
                for k, e in mine:
                    w(f"    {own_lv(e, q, e0)} = {ref(p, q, k)};")
            w("}")
            w("template <int KIND, int MODE>")
            w(f"__device__ __forceinline__ void rd_p{p}_c{ci}({state_params(p)}, {x_params(p)}, const float* lds, "
              f"int u, const FusedArgs& a, uint32_t vo, rsrc_t pr, rsrc_t cr, uint32_t vc, bool has_co, "
              f"uint32_t vm, rsrc_t xr, rsrc_t pm, PostSink& ps) {{")
            w("    asm volatile(\"\" : \"+v\"(u));")
            for q in range(Q):
                for k, e in mine:
                    w(f"    {ref(p, q, k)} = {own_lv(e, q, e0)};")
            w("}")

    # ---------------------------------------------------------------- check nodes
    # LDS holds each edge's Z messages in CHECK order (the owners rotate on write/read-back), so the
    # thread of check copy h reads every edge of its row at h: one address per row copy, the edges at
    # immediate offsets k*Z.  Rows are emitted inline per part and chunk (literal edges and degree).
    # Degree-1 bypass (every kernel; the training forward since r5): a degree-1 edge's v2c is its channel value
    # itself, so instead of a round trip owner -> LDS -> check node -> LDS -> owner, the check-node thread keeps
    # that edge's xa (at its rotated copies, advanced by the cumulative VN weights) in registers from the start
    # and writes the edge's posterior (and final c2v; training: its saved v2c, clamp mask and xin) itself:
    # ~19% of the LDS traffic of BG2 (38 of 197 edges) disappears.
    d1set = {S.col_edges[j][0] for j in range(S.N) if len(S.col_edges[j]) == 1}
    S.cd_index = {}  # part -> list of (edge, q) whose xa the check-node thread holds
    for p in range(S.P):
        lst = []
        for ci in range(len(S.chunks)):
            for i, q in S.cn_units[ci][p]:
                for e in S.row_edges[i]:
                    if e in d1set:
                        lst.append((e, q))
        S.cd_index[p] = lst

    S.cn_order, S.cn_nw = {}, {}
    for p in range(S.P):
        for ci in range(len(S.chunks)):
            S.cn_order[(p, ci)] = list(dict.fromkeys(i for i, _ in S.cn_units[ci][p]))  # distinct rows, unit order
            S.cn_nw[(p, ci)] = max(sum(len(S.row_edges[i]) for i in S.cn_order[(p, ci)]), 1)

    def rot(e, q):  # check copy h = u + q*ZT of edge e sits at variable copy (u + c) mod Z
        c = (q * ZT + int(S.shift[e])) % Z
        if c + ZT <= Z:
            return c, "0u"
        return c, f"(u >= {Z - c} ? {(-4 * Z) & 0xFFFFFFFF}u : 0u)"

    for p in range(S.P):
        ncd = max(len(S.cd_index[p]), 1)
        for ci, (r0, r1, e0c, e1c) in enumerate(S.chunks):
            w("template <int KIND, int MODE>")
            w(f"__device__ __forceinline__ void cn_p{p}_c{ci}(float* lds, int u, const FusedArgs& a, int it, "
              f"const float (&cd)[{ncd}], uint32_t vo, rsrc_t nr, rsrc_t cr, uint32_t vc, bool co_last, "
              f"const float (&W)[{S.cn_nw[(p, ci)]}], const float (&Bv)[{S.cn_nw[(p, ci)]}], PostSink& ps, "
              f"const uint32_t* appw, rsrc_t xr, rsrc_t apr, uint32_t (&cdm)[{nwords(p)}]"
              f", rsrc_t sv, rsrc_t nm, rsrc_t sxd) {{")
            w("    asm volatile(\"\" : \"+v\"(u));")
            w("    const uint32_t lu_ = (uint32_t)(uintptr_t)(lds_fp)lds + 4u * (uint32_t)u;")
            # row copies in order; weight offsets of each row in the preloaded W/Bv arrays
            rcs, woff, wo = list(S.cn_units[ci][p]), {}, 0
            for i in S.cn_order[(p, ci)]:
                woff[i] = wo
                wo += len(S.row_edges[i])

            def row_slots(i):
                """The row's first edge and each edge's float offset from it in the chunk image."""
                es = S.row_edges[i]
                return es[0], {e: k * Z for k, e in enumerate(es)}

            def rc_load(n):
                i, q = rcs[n]
                es = S.row_edges[i]
                DC = len(es)
                e0, off = row_slots(i)
                w(f"    float m{n}[{DC}];  // row {i} copy {q}")
                # the row copy's LDS byte address = lu_ + constant: one v_add_u32 (ROA kinds); the edges ride
                # in the 16-bit DS offset
                w(f"    std::conditional_t<ROA, lds_fp, float*> rq{n};")
                w("    if constexpr (ROA) {")
                w(f"        uint32_t rb = lu_ + {4 * ((e0 - e0c) * Z + q * ZT)}u;")
                w("        asm volatile(\"\" : \"+v\"(rb));")
                w(f"        rq{n} = (decltype(rq{n}))(uintptr_t)rb;")
                w("    } else {")
                w(f"        int ro = {(e0 - e0c) * Z + q * ZT} + u;")
                w("        asm volatile(\"\" : \"+v\"(ro));")
                w(f"        rq{n} = (decltype(rq{n}))(lds + ro);")
                w("    }")
                for k, e in enumerate(es):
                    if e in d1set:
                        w(f"    m{n}[{k}] = d1_v2c<KIND, 1>(cd[{S.cd_index[p].index((e, q))}], a);")
                    elif "cnread" in SKIP:  # (timing experiment: no check-node LDS reads, junk inputs)
                        w(f"    m{n}[{k}] = __uint_as_float(0x3f800000u + ((uint32_t)u << 8) + {k * 977 + n * 131}u);")
                    else:
                        w(f"    m{n}[{k}] = rq{n}[{off[e]}];")

            def rc_compute(n):
                i, q = rcs[n]
                es = S.row_edges[i]
                DC = len(es)
                _, off = row_slots(i)
                w("    {")
                # the degree-1 posteriors' channel values (Boosted with cumulative VN weights: from memory) requested
                # before the row's saved-message stores and check-node work -- a load after a store waits for it
                # (vmcnt counts both in order): r5, cfg5 training forward 10.8 -> 10.3 ms, cfg3ucn QMS 98.3 -> 95.3 ms
                d1k = []
                for k, e in enumerate(es):
                    if e in d1set:
                        j = int(S.hb_cols[e])
                        c, dv = rot(e, q)
                        ix = S.cd_index[p].index((e, q))
                        d1k.append((k, j, c, dv, ix))
                if "xld1" in SKIP:  # (fetch bisect, wrong results: the degree-1 posteriors' xa re-read replaced by xin)
                    for k, j, c, dv, ix in d1k:
                        w(f"        const float xo{k}_ = cd[{ix}];")
                elif d1k:  # (one branch for the row copy's loads, as in vn_p)
                    w("        float " + ", ".join(f"xo{k}_" for k, *_ in d1k) + ";")
                    w("        if (KIND != NLDPC_NEURAL && WVN_ON) {")
                    for k, j, c, dv, ix in d1k:
                        w(f"            xo{k}_ = bload(xr, vo + {dv}, {4 * (j * Z + c)});")
                    w("        } else {")
                    for k, j, c, dv, ix in d1k:
                        w(f"            xo{k}_ = cd[{ix}];")
                    w("        }")
                # SAVE: the row copy's v2c, as read, into the saved [E][Z] image by check copy h = u + q*ZT (r5: the
                # check-node threads store it from their registers; before, the whole workgroup copied each chunk
                # image between two extra barriers)
                w("        if constexpr (SAVE) {")
                # (one-codeword geometries: the codeword's element offset is u itself, no other value kept live)
                eo = "(uint32_t)u" if S.uremat else "(vc >> 2)"
                for k, e in enumerate(es):
                    w(f"            if constexpr (KIND == NLDPC_QMS) {_SI8}(sv, {eo} + {q * ZT}u, {e * Z}, qms_code_p(m{n}[{k}], a.qp));")
                    w(f"            else bstore(sv, 4u * {eo} + {4 * q * ZT}u, {4 * e * Z}, m{n}[{k}]);")
                w("        }")
                w(f"        float wv[{DC}], bv[{DC}];")
                w(f"        for (int k = 0; k < {DC}; ++k) {{ wv[k] = W[{woff[i]} + k]; bv[k] = Bv[{woff[i]} + k]; }}")
                w("        const bool wc = UCNW || a.w_cn != nullptr;")
                w("        float uf_ = 0.f;  // UCN: unsatisfied check (odd number of row variables with APP >= 0)")
                w("        bool ufb_ = false;  // (the same as a lane mask: MS / QMS select on it, SP multiplies by uf_)")
                w("        if (KIND != NLDPC_NEURAL && UCN_ON) {")
                w("            uint32_t par_ = 0;")
                # every word of the row requested first, then the shifts and XORs (one LDS wait, not DC; UCNB)
                ks = [(k, e) for k, e in enumerate(es) if e not in d1set]
                for k, e in ks:
                    c, dvu = rot(e, q)
                    j = int(S.hb_cols[e])
                    # (u + c) mod Z as min(v, v - Z) on unsigned: v - Z wraps above v unless v >= Z
                    vexpr = f"(uint32_t)u + {c}u" if c + ZT <= Z else f"min((uint32_t)u + {c}u, (uint32_t)u + {c - Z}u)"
                    w(f"            const uint32_t v{k}_ = {vexpr}; const uint32_t w{k}_ = appw[{j * S.WZX} + (v{k}_ >> 5)];")
                for k, e in ks:
                    w(f"            par_ ^= w{k}_ >> (v{k}_ & 31u);")
                for k, e in enumerate(es):
                    if e not in d1set:
                        continue
                    c, dvu = rot(e, q)
                    j = int(S.hb_cols[e])
                    # the hard decision of this thread's own previous posterior of that edge's column copy
                    ix = S.cd_index[p].index((e, q))
                    # (r6: iteration 0's bits -- APP = xa_input or the previous call's posterior -- are set into cdm at
                    # the top of iteration 0, run_p: no per-iteration select between the two sources)
                    w(f"            par_ ^= {bit_get('cdm', ix)};")
                w("            ufb_ = (par_ & 1u) != 0u;")
                w("            uf_ = ufb_ ? 1.f : 0.f;")
                w("        }")
                if "cnmath" not in SKIP:  # (timing experiment: SKIP=cnmath leaves the messages unchanged)
                    w(f"        cn_copy<KIND, {DC}, TIEDW>(m{n}, wv, bv, a, wc, {i}, uf_, UCN_ON, ufb_);")
                for k, e in enumerate(es):
                    if e in d1set:
                        j = int(S.hb_cols[e])
                        c, dv = rot(e, q)
                        ix = S.cd_index[p].index((e, q))
                        pm = f"fadd(0.f, m{n}[{k}])"
                        w("        {")
                        w(f"            const uint32_t dv_ = {dv};")
                        w("            float y_;")
                        w(f"            if constexpr (KIND == NLDPC_NEURAL) y_ = fadd(cd[{ix}], {pm});")
                        w("            else {  // Boosted: the unweighted channel value (cumulative VN weights: from memory)")
                        w(f"                const float xo_ = xo{k}_;")
                        # the training forward: the clamp mask (byte offset = the float offset / 4) and this
                        # iteration's xin too (the owners keep no degree-1 state)
                        w("                if constexpr (SAVE) { bool m_; "
                          f"y_ = posterior_m<KIND>(xo_, {pm}, a, m_); {_S8}(nm, (vo + dv_ + {4 * (j * Z + c)}u) >> 2, 0, m_); "
                          f"bstore(sxd, vo + dv_, {4 * (j * Z + c)}, cd[{ix}]); }}")
                        w(f"                else y_ = posterior<KIND>(xo_, {pm}, a);")
                        w(f"                if (UCN_ON) {bit_set('cdm', ix, 'y_ >= 0.f')};")
                        w("            }")
                        if "d1post" in SKIP:  # (timing experiment: no degree-1 posterior stores)
                            w("            asm volatile(\"\" :: \"v\"(y_));")
                        else:
                            w(f"            put_post<CM>(nr, vo + dv_, {4 * (j * Z + c)}, y_, ps);")
                        w(f"            if (co_last) bstore(cr, vc + dv_, {4 * (e * Z + c)}, m{n}[{k}]);")
                        w("        }")
                    elif "cnwrite" in SKIP:  # (timing experiment: keep the value live without the LDS write)
                        w(f"        asm volatile(\"\" :: \"v\"(m{n}[{k}]));")
                    else:
                        w(f"        rq{n}[{off[e]}] = m{n}[{k}];")
                w("    }")

            # the next row copy's reads go out before this one computes (its slots are disjoint from every
            # slot this one writes, so program order already allows it)
            if rcs:
                rc_load(0)
            for n in range(len(rcs)):
                if n + 1 < len(rcs):
                    rc_load(n + 1)
                w("    __builtin_amdgcn_sched_barrier(0);")
                rc_compute(n)
            w("}")

    # ---------------------------------------------------------------- the kernel
    def each_part(fmt, indent="        "):
        ps_ = list(PARTS or range(S.P))
        for p in ps_:
            w(f"{indent}{'if' if p == ps_[0] else 'else if'} (p == {p}) {fmt.format(p=p)};")

    # Each part runs its own copy of the whole iteration loop: its register state never meets another
    # part's at a control-flow join (per-phase part branches inside one loop made the register
    # allocator insert phi copies and spill).  The parts still meet at every s_barrier: a hardware
    # barrier counts waves, not program counters, and every part executes the same barrier sequence.
    def pipe_phases(K):
        # [W0] | [CN0, W1] | [R0, CN1] | [W2, R1] | [CN2, W3] | [R2, CN3] | ... (see the pipelined schedule below)
        phases = [[("w", 0)]]
        c = 0
        while c < K:
            phases.append([("cn", c)] + ([("w", c + 1)] if c + 1 < K else []))
            phases.append([("r", c)] + ([("cn", c + 1)] if c + 1 < K else []))
            if c + 1 < K:
                phases.append(([("w", c + 2)] if c + 2 < K else []) + [("r", c + 1)])
            c += 2
        return phases

    # this thread's codeword counters (recomputed at each flush: no register held across the iteration)
    cnt_slot = "cntl"  # the kernel passes this codeword's counters
    cnt_flush = "flush_wave" if G == 1 else "flush"  # one codeword per wave: reduce the wave first
    for p in range(S.P):
        if PARTS and p not in PARTS:
            continue
        sp = max(len(S.slots[p]), 1)
        nr = max(len(S.reg_cols[p]), 1)
        w("template <int KIND, int MODE>")
        w(f"__device__ __forceinline__ void run_p{p}(const FusedArgs& a, float* lds, int u, int64_t blk, int nlive, "
          f"rsrc_t xr, uint32_t vo, rsrc_t cr, uint32_t vc, uint32_t vm, int* cntl, uint32_t* app_all, uint32_t* appw, bool dup_, "
          f"const float* lds_all{', int ub' if S.uremat else ''}) {{")
        # UREMAT (the SAVE kernels of a one-codeword, unpadded geometry): the lane offsets u / vo / vc / vm are
        # re-derived from the wave-uniform base ub and the lane id before each phase, so none of them lives across
        # the iteration (the QMS training forward at the 128-VGPR cap spilled them and reloaded each phase with a
        # vmcnt(0) wait -- behind every posterior / saved-state store in flight)
        remat = ("        if constexpr (SAVE) { u = ub + lane_id(); vo = 4u * (uint32_t)u; vc = vo; vm = (uint32_t)u; }"
                 if S.uremat else None)
        if S.pipe:  # (r2: the pipelined schedule made the training forward slower; r5 with the check-node saves: still)
            w("    static_assert(!SAVE, \"the SAVE kernels use the one-buffer schedule\");")
        for i in range(Q):
            w(f"    float cs{i}[{sp}], xs{i}[{nr}];")
        w("#pragma unroll")
        w(f"    for (int k = 0; k < {sp}; ++k) {{")
        for i in range(Q):
            w(f"        cs{i}[k] = 0.f;")
        w("    }")
        w("    // this thread's channel values, loaded once for all T iterations")
        for n, j in enumerate(S.reg_cols[p]):
            for i in range(Q):
                w(f"    xs{i}[{n}] = bload(xr, vo, {X(j, i)});")
        w(f"    PostSink ps{{make_rsrc((const float*)(a.cnt_y ? a.cnt_y + blk * {NZ} : nullptr), "
          f"a.cnt_y ? nlive * {NZ} : 0), 0, a.cnt_conv}};")
        ncd = max(len(S.cd_index[p]), 1)
        w(f"    float cd[{ncd}];  // xa of the degree-1 edges of this part's check rows, rotated copies")
        w("    {")
        for idx, (e, q) in enumerate(S.cd_index[p]):
            c, dv = rot(e, q)
            # (0 + xa): the v2c of a degree-1 edge, canonical (never -0), as the check node sees it
            w(f"        {{ const float x_ = bload(xr, vo + {dv}, {4 * (int(S.hb_cols[e]) * Z + c)}); "
              f"cd[{idx}] = KIND == NLDPC_NEURAL ? fadd(0.f, x_) : x_; }}")
        if not S.cd_index[p]:
            w("        cd[0] = 0.f;")
        w("    }")
        # cumulative VN weighting: the channel registers hold xin and advance one step per iteration
        def chan_steps(step_expr, indent):
            w(f"{indent}{{ const cfloat_p wr_ = (cfloat_p)(a.w_vn + (int64_t)({step_expr}) * N);")
            for n, j in enumerate(S.reg_cols[p]):
                for i in range(Q):
                    w(f"{indent}  xs{i}[{n}] = chan_step<KIND>(xs{i}[{n}], a, wr_[{j}]);")
            if S.cd_index[p]:  # (the degree-1 channel values the check-node thread holds)
                w(f"{indent}  {{")
                for idx, (e, q) in enumerate(S.cd_index[p]):
                    w(f"{indent}    cd[{idx}] = chan_step<KIND>(cd[{idx}], a, wr_[{int(S.hb_cols[e])}]);")
                w(f"{indent}  }}")
            w(f"{indent}}}")

        def rs(ptr, size):  # descriptor over this block's part of a per-iteration buffer, or an empty one
            return f"make_rsrc({ptr} ? {ptr} + blk * {size} : a.xa, {ptr} ? nlive * {size} : 0)"

        w("    if (KIND != NLDPC_NEURAL && WVN_ON) {  // steps applied before this call's first iteration")
        w("        for (int s_ = 0; s_ < a.vn_prefix; ++s_)")
        chan_steps("s_", "            ")
        w("    }")
        def stamp(ph):
            if STAMPS:
                assert ph < 16
                w(f"        stamp_store(a.stamps, {S.threads // 64}, a.T, it, {ph});")
        # UCN: the hard-decision bit array of the codewords starts at zero (bits are OR-ed in); every later
        # iteration's array is cleared in the read-back phase of the iteration before
        w(f"    uint32_t cdm[{nwords(p)}] = {{}};  // UCN: hard decisions of the posteriors of its cd entries")
        w(f"    const rsrc_t apr = make_rsrc(a.app_prev ? a.app_prev + blk * {NZ} : a.xa, a.app_prev ? nlive * {4 * NZ} : 0);")
        w("    if (KIND != NLDPC_NEURAL && UCN_ON) {")
        w(f"        for (int i_ = threadIdx.x; i_ < {S.G_lds * S.N * S.WZX}; i_ += {S.threads}) app_all[i_] = 0u;")
        w("        __syncthreads();")
        w("    }")
        w("    for (int it = 0; it < a.T; ++it) {")
        stamp(0)
        w("        if (KIND != NLDPC_NEURAL && WVN_ON) {")
        chan_steps("a.vn_prefix + it", "            ")
        w("            if constexpr (SAVE) {")
        w("                float* sx_ = a.sxin ? a.sxin + it * a.sxin_stride : nullptr;")
        w(f"                const rsrc_t sx = make_rsrc(sx_ ? sx_ + blk * {NZ} : a.xa, sx_ ? nlive * {4 * NZ} : 0);")
        for n, j in enumerate(S.reg_cols[p]):
            for q in range(Q):
                w(f"                bstore(sx, vo, {X(j, q)}, {xref(p, j, q)});")
        w("            }")
        w("        }")
        # UCN, iteration 0: the degree-1 entries' hard decisions of APP = xa_input (after this iteration's VN-weight step)
        # or of the previous call's posterior, into cdm once (the check nodes read cdm in every iteration)
        if S.cd_index[p]:
            w("        if (KIND != NLDPC_NEURAL && UCN_ON && it == 0) {")
            for ix, (e, q) in enumerate(S.cd_index[p]):
                j = int(S.hb_cols[e])
                c, dvu = rot(e, q)
                app0 = f"(a.first_iter > 0 ? bload(apr, vo + {dvu}, {4 * (j * Z + c)}) : chan<KIND>(cd[{ix}], a))"
                w(f"            {bit_set('cdm', ix, app0 + ' >= 0.f')};")
            w("        }")
        # (the check-node threads store the degree-1 columns' xin: cn_p)
        w("        float* sxd_ = (SAVE && KIND != NLDPC_NEURAL && WVN_ON && a.sxin) ? a.sxin + it * a.sxin_stride : nullptr;")
        w(f"        const rsrc_t sxd = make_rsrc(sxd_ ? sxd_ + blk * {NZ} : a.xa, sxd_ ? nlive * {4 * NZ} : 0);")
        w("        const float* pp = it >= 1 ? a.outs.p[it - 1] : nullptr;  // previous iteration's posterior")
        w(f"        const rsrc_t pr = make_rsrc(pp ? pp + blk * {NZ} : a.xa, pp ? nlive * {4 * NZ} : 0);  // no output: stores dropped")
        w("        const uint8_t* pmp = (SAVE && a.symask && it >= 1) ? a.symask + (it - 1) * a.symask_stride : nullptr;")
        w(f"        const rsrc_t pm = make_rsrc((const float*)(pmp ? pmp + blk * {NZ} : nullptr), pmp ? nlive * {NZ} : 0);")
        if remat:
            w(remat)
        if "vn" not in SKIP:
            w(f"        vn_p{p}<KIND, MODE>({state_args(p)}, {x_args(p)}, a, vo, it, pr, vm, xr, pm, ps, appw, u, apr);")
        # iteration it-1 is complete (at it = 0 the VN step made no output: nothing to count)
        w(f"        if constexpr (CNT) {{ if (dup_) ps.ec = 0; if (it >= 1) ps.{cnt_flush}({cnt_slot}, it - 1); else ps.ec = 0; }}")
        w("        const float* pn = a.outs.p[it];  // this iteration's posterior (degree-1 columns)")
        w(f"        const rsrc_t nr = make_rsrc(pn ? pn + blk * {NZ} : a.xa, pn ? nlive * {4 * NZ} : 0);")
        w("        const uint8_t* nmp = (SAVE && a.symask) ? a.symask + it * a.symask_stride : nullptr;")
        w(f"        const rsrc_t nm = make_rsrc((const float*)(nmp ? nmp + blk * {NZ} : nullptr), nmp ? nlive * {NZ} : 0);")
        w("        constexpr int SB = saved_msg_bytes<KIND>();")
        w("        const char* svp = SAVE ? a.sv2c + it * a.sv2c_stride * SB : nullptr;")
        w(f"        const rsrc_t sv = make_rsrc((const float*)(svp ? svp + blk * {S.E * Z} * SB : nullptr), "
          f"svp ? nlive * {S.E * Z} * SB : 0);")
        w("        (void)sv;")
        w("        const bool co_last = a.c2v_out && it == a.T - 1;")
        stamp(1)
        def declare_w(ci):
            nw = S.cn_nw[(p, ci)]
            w(f"        float W{ci}[{nw}], B{ci}[{nw}];")

        def preload(ci):
            nw = S.cn_nw[(p, ci)]
            # this chunk's check-node weights, by whole-row scalar loads issued a phase ahead of its check
            # nodes (their latency overlaps LDS traffic and a barrier, not the check rows' LDS waits), or
            # at the start of the check-node phase (WLATE)
            w("        {")
            w("            const cfloat_p wc_ = a.w_cn ? (cfloat_p)(a.w_cn + (int64_t)it * E) : nullptr;")
            w("            const float* bsrc_ = KIND == NLDPC_NEURAL ? a.bias : (UCN_ON ? a.w_ucn : nullptr);  // bias / UCN weight")
            w("            const cfloat_p bs_ = bsrc_ ? (cfloat_p)(bsrc_ + (int64_t)it * E) : nullptr;")
            wo, wl, bl = 0, [], []
            for i in S.cn_order[(p, ci)]:
                for k, e in enumerate(S.row_edges[i]):
                    wl.append(f"W{ci}[{wo}] = wc_[{e}];")
                    bl.append(f"B{ci}[{wo}] = bs_[{e}];")
                    wo += 1
            w("            if constexpr (TIEDW) {  // one CN weight per iteration: the row's first entry, one scalar")
            w("                const float w0_ = wc_ ? wc_[0] : 1.f;")
            w(f"                for (int k = 0; k < {nw}; ++k) {{ W{ci}[k] = w0_; B{ci}[k] = 0.f; }}")
            w("            } else {")
            if "wload" in SKIP:  # timing experiment only: constant weights, no scalar loads
                w(f"            for (int k = 0; k < {nw}; ++k) {{ W{ci}[k] = 0.5f; B{ci}[k] = 0.f; }}")
            else:
                w(f"            if (KIND == NLDPC_NEURAL || UCNW || wc_) {{ {' '.join(wl)} }}")
                w(f"            else {{ for (int k = 0; k < {nw}; ++k) W{ci}[k] = 1.f; }}")
                w(f"            if (KIND == NLDPC_NEURAL || bs_) {{ {' '.join(bl)} }}")
                w(f"            else {{ for (int k = 0; k < {nw}; ++k) B{ci}[k] = 0.f; }}")
            w("            }")
            w("        }")

        def buf(ci):
            return f"lds + {S.region_off[ci]}" if S.region_off[ci] else "lds"

        def op_w(ci):
            declare_w(ci)
            w(f"        if constexpr (!({WLATE_COND}))")
            preload(ci)
            if remat:
                w(remat)
            w(f"        wr_p{p}_c{ci}<KIND, MODE>({state_args(p)}, {x_args(p)}, {buf(ci)}, u, a, it, sv, vc);")

        def op_cn(ci):
            w(f"        if constexpr ({WLATE_COND})")
            preload(ci)
            if remat:
                w(remat)
            if "cn" not in SKIP:
                w(f"        cn_p{p}_c{ci}<KIND, MODE>({buf(ci)}, u, a, it, cd, vo, nr, cr, vc, co_last, W{ci}, B{ci}, ps, appw, xr, apr, cdm, sv, nm, sxd);")

        def op_r(ci):
            if remat:
                w(remat)
            w(f"        rd_p{p}_c{ci}<KIND, MODE>({state_args(p)}, {x_args(p)}, {buf(ci)}, u, a, vo, nr, cr, vc, co_last, vm, xr, nm, "
              f"ps);")
            if ci == len(S.chunks) - 1:  # every check node of the iteration has read the bits
                w("        if (KIND != NLDPC_NEURAL && UCN_ON) {")
                w(f"            for (int i_ = threadIdx.x; i_ < {S.G_lds * S.N * S.WZX}; i_ += {S.threads}) app_all[i_] = 0u;")
                w("        }")

        K = len(S.chunks)
        if not S.pipe:
            for ci in range(K):
                op_w(ci)
                stamp(2 + 3 * ci)
                w("        __syncthreads();")
                op_cn(ci)
                stamp(3 + 3 * ci)
                w("        __syncthreads();")
                op_r(ci)
                stamp(4 + 3 * ci)
                w("        __syncthreads();")
        else:
            # phases: [W0] | [CN0, W1] | [R0, CN1] | [W2, R1] | [CN2, W3] | [R2, CN3] | ... | [R_{K-1}] (the last
            # read-back runs into the next iteration's VN and W0, whose buffer was last read two phases back).
            # W_c reuses the buffer of chunk c-2, read (R_{c-2}) a phase earlier.
            phases = pipe_phases(K)
            # phase dependencies hold: each W_c is after R_{c-2}'s phase, each CN_c after W_c's, each R_c after CN_c's
            for k, ph in enumerate(phases):
                for kind_, ci in ph:
                    {"w": op_w, "r": op_r, "cn": op_cn}[kind_](ci)
                stamp(2 + k)  # arrival at the barrier that ends phase k (stamp 1: after the VN)
                if k < len(phases) - 1:
                    # (timing experiment SKIP=sync: no barrier -- racy results, the cost of waiting at them)
                    w("        __builtin_amdgcn_sched_barrier(0);" if "sync" in SKIP else "        __syncthreads();")
            # a K-odd schedule ends with [R_{K-1}] alone after [R_{K-2}... ]: the next W0 (buffer 0) follows
            # R_{K-1} (buffer 0) in other waves -> keep a barrier; K even: R_{K-1} reads buffer 1
            if K % 2 == 1:
                w("        __syncthreads();")
            else:  # UCN: the bits cleared in R_{K-1} must be clear before any wave's next VN
                w("        if (KIND != NLDPC_NEURAL && UCN_ON) __syncthreads();")
        w("    }")
        w("    const float* pl = a.outs.p[a.T - 1];")
        w(f"    const rsrc_t lr = make_rsrc(pl ? pl + blk * {NZ} : a.xa, pl ? nlive * {4 * NZ} : 0);")
        w("    const uint8_t* lmp = (SAVE && a.symask) ? a.symask + (a.T - 1) * a.symask_stride : nullptr;")
        w(f"    const rsrc_t lm = make_rsrc((const float*)(lmp ? lmp + blk * {NZ} : nullptr), lmp ? nlive * {NZ} : 0);")
        if remat:
            w(remat)
        w(f"    post_p{p}<KIND, MODE>({state_args(p)}, {x_args(p)}, a, vo, a.T, lr, vm, xr, lm, ps, appw, u, apr);")
        w(f"    if constexpr (CNT) {{ if (dup_) ps.ec = 0; ps.{cnt_flush}({cnt_slot}, a.T - 1); }}")
        w("    if (a.c2v_out) {")
        for q in range(Q):
            for k, e in enumerate(S.slots[p]):
                w(f"        bstore(cr, vc, {4 * (e * Z + q * ZT)}, {ref(p, q, k)});")
        w("    }")
        w("}")
    w("template <int KIND, int MODE>")
    w("__device__ __forceinline__ void kernel_body(const FusedArgs& a) {")
    w("    if (a.sig != kFusedArgsSig) return;  // a launcher built against another FusedArgs layout")
    w(f"    __shared__ __attribute__((aligned(16))) float lds_all[{S.cw_floats * S.G_lds}];")
    w("    const int t = threadIdx.x;")
    w(f"    // every wave lies in one part ({S.lanes_pad} threads per part): the part is wave-uniform")
    w(f"    const int p = __builtin_amdgcn_readfirstlane(t / {S.lanes_pad});")
    if S.padded:  # lanes past the live ones repeat live lanes (Spec.lanes_pad)
        w(f"    const int r0_ = t - p * {S.lanes_pad};")
        w(f"    const bool dup_ = r0_ >= {S.lanes};")
        w(f"    const int r = dup_ ? r0_ - {S.lanes} : r0_;")
    else:
        w(f"    const int r = t - p * {S.lanes};")
        w("    const bool dup_ = false;")
    w(f"    const int g = r / {ZT};")
    w(f"    const int u = r - g * {ZT};")
    w(f"    const int64_t blk = (int64_t)blockIdx.x * {G};  // first codeword of the workgroup")
    w(f"    const int nlive = a.B - blk < {G} ? (int)(a.B - blk) : {G};")
    w("    // lane byte offsets into the block's codewords; a lane past the last codeword gets an offset")
    w("    // beyond every descriptor's range (its loads read 0, its stores are dropped)")
    w(f"    const uint32_t vo = g < nlive && !dup_ ? 4u * (g * {NZ} + u) : 0x80000000u;  // [N][Z] layouts")
    w(f"    const uint32_t vc = g < nlive && !dup_ ? 4u * (g * {S.E * Z} + u) : 0x80000000u;  // [E][Z] c2v state")
    w(f"    const rsrc_t xr = make_rsrc(a.xa + blk * {NZ}, nlive * {4 * NZ});")
    w(f"    const rsrc_t cr = make_rsrc(a.c2v_out ? a.c2v_out + blk * {S.E * Z} : a.xa, nlive * {4 * S.E * Z});")
    w(f"    float* lds = lds_all + (dup_ ? {G} : g) * {S.cw_floats};  // (repeating lanes: their own region)")
    w("    const uint32_t vm = vo >> 2;  // byte offsets of the uint8 clamp masks")
    w(f"    __shared__ int cnt_all[{G * 32}];  // count-only decode: per codeword, two iterations per word")
    w(f"    __shared__ uint32_t app_all[{S.G_lds * S.N * S.WZX}];  // UCN: bit (j, v) = APP[j][v] >= 0, per codeword")
    w(f"    uint32_t* appw = app_all + (dup_ ? {G} : g) * {S.N * S.WZX};")
    w(f"    if constexpr (CNT) {{ for (int i = t; i < {G * 32}; i += {S.threads}) cnt_all[i] = 0; }}  // first use after iteration 0's barriers")
    if S.uremat:
        w("    const int ub = __builtin_amdgcn_readfirstlane(u - lane_id());  // (UREMAT) u of the wave's lane 0")
    each_part("run_p{p}<KIND, MODE>(a, lds, u, blk, nlive, xr, vo, cr, vc, vm, cnt_all + g * 32, app_all, appw, dup_, lds_all"
              + (", ub)" if S.uremat else ")"), indent="    ")
    w("    if constexpr (CNT) {")
    w("        __syncthreads();")
    w("        if (t < a.T) count_iteration(a, cnt_all, nlive, t);")
    w("    }")
    w("}")
    w("template <int KIND, int MODE>")
    w(f"__global__ __launch_bounds__({S.threads}, {(S.threads + 255) // 256}) void kernel(FusedArgs a) {{")
    w("    kernel_body<KIND, MODE>(a);")
    w("}")
    w("#undef ROA")
    w("#undef SAVE")
    w("#undef CNT")
    w("#undef CM")
    w("#undef TIEDW")
    w("#undef UCN_ON")
    w("#undef UCNW")
    w("#undef WVN_ON")
    w("}  // namespace")
    return "\n".join(L)


def emit_bwd(S: Spec, ns: str = "fusedb") -> str:
    """Backward kernels (training): the forward's ownership and LDS exchange, run in reverse.

    State: dL/dc2v_{k+1} of every register edge copy (the forward's c2v slots), one float array per
    lane copy.  Per iteration k = T-1..0: owners write the state into the check-ordered LDS image
    (degree-1 edges: dL/dy_k * mask_k), the check-node threads read v2c_k (saved in check order; staged
    into LDS per chunk when S.stage) at their check copy, run cn_backward (nldpc_node.h, the streaming cnb_kernel's arithmetic) and put
    dL/dv2c_k back in place, owners read it back; then the variable-node step: dL/dc2v_k = dL/dy_{k-1}
    * mask_{k-1} + sum of the column's other dL/dv2c_k (prefix + suffix, as vnb_kernel), and the
    cumulative VN-weight chain (carry per channel value).  Weight gradients: per-wave partial sums."""
    Z, G, Q, ZT, NZ, E, N = S.Z, S.G, S.Q, S.ZT, S.N * S.Z, S.E, S.N
    WP = S.lanes_pad // 64  # waves per part
    L = []
    w = L.append
    CF = S.chunk_floats
    w(f"// ---- {S.tag} backward: {S.threads} threads, {WP} wave(s) per part")
    w(f"namespace {ns}_{S.tag} {{")
    w(f"constexpr int Z = {Z}, ZT = {ZT}, N = {N}, E = {E}, WP = {WP}, MDC = {S.max_dc};")

    def X(j, q):
        return 4 * (j * Z + q * ZT)

    def own(e, q, e0):
        cq = (q * ZT - int(S.shift[e])) % Z
        base = (e - e0) * Z + cq
        if cq + ZT <= Z:
            return f"{base} + u"
        return f"{base} + u - (u >= {Z - cq} ? {Z} : 0)"

    def sref(q, k):
        return f"g{q}[{k}]"

    def state_params(p):
        sp = max(len(S.slots[p]), 1)
        return ", ".join(f"float (&g{q})[{sp}]" for q in range(Q))

    def state_args():
        return ", ".join(f"g{q}" for q in range(Q))

    # the VN-weight chain of one channel value: carry (a workspace buffer, one float per variable copy:
    # registers are all taken by the state) and this column's weight-gradient contribution
    # (vnb_kernel's arithmetic: u = xprev * w, STE mask of Q on u, du = (gsum + carry) * mask)
    def chain(p, j, q, gsum, indent):
        w(f"{indent}{{ const float xp_ = it >= 1 ? {_LD_NT}(sxp, vo, {X(j, q)}) : {_LD_NT}(xr, vo, {X(j, q)});")
        w(f"{indent}  const float u_ = fmul(xp_, wvn[{j}]);")
        w(f"{indent}  const float mk_ = (KIND == NLDPC_QMS && qr.active) ? in_range(u_, qr.lo, qr.hi) : 1.f;")
        w(f"{indent}  const float cy_ = it == a.T - 1 ? 0.f : bload(cyr, vo, {X(j, q)});")
        w(f"{indent}  const float du_ = ({gsum} + cy_) * mk_;")
        w(f"{indent}  ctb_ += du_ * xp_;")
        w(f"{indent}  {_CY_ST}(cyr, vo, {X(j, q)}, du_ * wvn[{j}]); }}")

    # r6 (BWDPIPE): the degree-1 chains of a read-back software-pipelined one deep -- the next chain's loads are issued before
    # this chain computes and stores its carry, so no load waits behind a carry store (vmcnt counts loads and stores
    # in issue order: each chain used to wait a full memory round trip behind the previous chain's store)
    def chain_load(n, j, q, indent):
        w(f"{indent}const float xp{n}_ = it >= 1 ? {_LD_NT}(sxp, vo, {X(j, q)}) : {_LD_NT}(xr, vo, {X(j, q)});")
        w(f"{indent}const float cy{n}_ = it == a.T - 1 ? 0.f : bload(cyr, vo, {X(j, q)});")

    def chain_pre(n, j, q, gsum, indent):
        w(f"{indent}{{ const float xp_ = xp{n}_;")
        w(f"{indent}  const float u_ = fmul(xp_, wvn[{j}]);")
        w(f"{indent}  const float mk_ = (KIND == NLDPC_QMS && qr.active) ? in_range(u_, qr.lo, qr.hi) : 1.f;")
        w(f"{indent}  const float cy_ = cy{n}_;")
        w(f"{indent}  const float du_ = ({gsum} + cy_) * mk_;")
        w(f"{indent}  ctb_ += du_ * xp_;")
        w(f"{indent}  {_CY_ST}(cyr, vo, {X(j, q)}, du_ * wvn[{j}]); }}")

    def col_partial(j, indent):  # (lanes repeating a live one add nothing: Spec.lanes_pad)
        # (a tied VN weight keeps these: one wave reduction per column either way; a per-lane running sum over
        # the columns instead spilled 122 VGPRs)
        w(f"{indent}if (a.p_vn) {{ const float s_ = wave_sum(dup_ ? 0.f : ctb_); if (lane0) a.p_vn[pv + {j}] = s_; }}")

    # ---------------------------------------------------------------- LDS write / read-back
    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            mine = [(k, e) for k, e in enumerate(S.slots[p]) if e0 <= e < e1]
            d1 = [(j, S.col_edges[j][0]) for j in S.d1_cols[p] if e0 <= S.col_edges[j][0] < e1]
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void wrb_p{p}_c{ci}({state_params(p)}, float* lds, int u, rsrc_t gr, "
              f"rsrc_t mr, uint32_t vo, uint32_t vm) {{")
            w("    asm volatile(\"\" : \"+v\"(u));")
            for q in range(Q):
                for k, e in mine:
                    w(f"    lds[{own(e, q, e0)}] = {sref(q, k)};")
            for j, e in d1:  # dL/dc2v_{k+1} of a degree-1 edge: only its own posterior
                for q in range(Q):
                    w(f"    lds[{own(e, q, e0)}] = {_GY}<KIND>(gr, mr, vo, vm, {X(j, q)});")
            w("}")
            w("template <int KIND, int TIED>")
            w(f"__device__ __forceinline__ void rdb_p{p}_c{ci}({state_params(p)}, const float* lds, "
              f"int u, const FusedBwdArgs& a, int it, uint32_t vo, rsrc_t xr, rsrc_t sxp, rsrc_t cyr, cfloat_p wvn, "
              f"int64_t pv, bool lane0, bool dup_) {{")
            w("    asm volatile(\"\" : \"+v\"(u));")
            for q in range(Q):
                for k, e in mine:
                    w(f"    {sref(q, k)} = lds[{own(e, q, e0)}];")
            if d1 and BWDPIPE:
                w("    if (KIND != NLDPC_NEURAL && a.w_vn) {  // VN chain of the degree-1 columns (gsum = their one edge)")
                w("        const QRange qr = q_range(a.qbit);")
                items = [(j, e, q) for j, e in d1 for q in range(Q)]
                chain_load(0, items[0][0], items[0][2], "        ")
                w("        float ctb_;")
                for n, (j, e, q) in enumerate(items):
                    if q == 0:
                        w("        ctb_ = 0.f;")
                    if n + 1 < len(items):
                        chain_load(n + 1, items[n + 1][0], items[n + 1][2], "          ")
                    w(f"          {{ const float gs_ = 0.f + lds[{own(e, q, e0)}];")
                    chain_pre(n, j, q, "gs_", "            ")
                    w("          }")
                    w("          __builtin_amdgcn_sched_barrier(0);")
                    if q == Q - 1:
                        col_partial(j, "          ")
                w("    }")
            elif d1:
                w("    if (KIND != NLDPC_NEURAL && a.w_vn) {  // VN chain of the degree-1 columns (gsum = their one edge)")
                w("        const QRange qr = q_range(a.qbit);")
                for j, e in d1:
                    w("        { float ctb_ = 0.f;")
                    for q in range(Q):
                        w(f"          {{ const float gs_ = 0.f + lds[{own(e, q, e0)}];")
                        chain(p, j, q, "gs_", "            ")
                        w("          }")
                        w("          __builtin_amdgcn_sched_barrier(0);")
                    col_partial(j, "          ")
                    w("        }")
                w("    }")
            w("}")

    # ---------------------------------------------------------------- variable-node backward
    for p in range(S.P):
        w("template <int KIND, int TIED>")
        w(f"__device__ __forceinline__ void vnb_p{p}({state_params(p)}, const FusedBwdArgs& a, "
          f"int it, uint32_t vo, uint32_t vm, rsrc_t gr, rsrc_t mr, rsrc_t xr, rsrc_t sxp, rsrc_t cyr, cfloat_p wvn, "
          f"int64_t pv, bool lane0, bool dup_) {{")
        w("    const bool chain_on = KIND != NLDPC_NEURAL && a.w_vn;")
        w("    const QRange qr = q_range(a.qbit);")
        s0 = 0
        for j in S.reg_cols[p]:
            d = len(S.col_edges[j])
            w(f"    {{  // column {j}, degree {d}")
            w("        float ctb_ = 0.f;")
            for q in range(Q):
                c = lambda k: sref(q, s0 + k)  # noqa: E731
                w("        {")
                w("            float gs_ = 0.f;")
                for k in range(d):
                    w(f"            gs_ = gs_ + {c(k)};")
                w("            if (it >= 1) {")
                w(f"                const float gyv_ = {_GY}<KIND>(gr, mr, vo, vm, {X(j, q)});")
                w(f"                float suf_[{d + 1}];")
                w(f"                suf_[{d}] = 0.f;")
                for k in range(d - 1, -1, -1):
                    w(f"                suf_[{k}] = suf_[{k + 1}] + {c(k)};")
                w("                float pre_ = 0.f;")
                for k in range(d):
                    w(f"                {{ const float o_ = {c(k)}; {c(k)} = gyv_ + (pre_ + suf_[{k + 1}]); pre_ += o_; }}")
                w("            }")
                w("            if (chain_on) {")
                chain(p, j, q, "gs_", "                ")
                w("            }")
                w("        }")
                w("        __builtin_amdgcn_sched_barrier(0);  // one column copy at a time (register pressure)")
            w("        if (chain_on) {")
            col_partial(j, "            ")
            w("        }")
            w("    }")
            s0 += d
        w("}")

    # ---------------------------------------------------------------- check-node backward
    # The saved v2c of an iteration is check-ordered ([E][Z] by check copy h), so a chunk's messages are
    # one contiguous block: with S.stage the block is copied into LDS beside the chunk image by LDS-DMA
    # (global_load_lds, issued at the start of the chunk's write phase, landed by the barrier before the
    # check nodes), and each check copy reads its row's messages from LDS at h -- no global gathers in
    # the check-node phase.  Without staging they are read from global memory at h (coalesced).
    SBY = S.stage
    w("template <int KIND, int DC, int TIED, int Q0, int Q1>  // the row's copies Q0 .. Q1-1")
    w("__device__ __forceinline__ void cnb_row(float* rp, const char* sq, int u, const FusedBwdArgs& a, int it, "
      "int e0, int row, rsrc_t svr, uint32_t vcw, int64_t pc, bool lane0, bool dup_, float* gacc, float& tacc) {")
    # a scheduling fence after each lane copy, none per row: the row fence pushed the tied QMS kernel to 123
    # VGPR spills (21 without) and cfg5's backward measured 27.97 -> 27.32 ms without it (no fence at all:
    # 27.49; profiles/r4_ab.txt)
    w("    float wv[DC], bv[DC];")
    w("    const cfloat_p wc = a.w_cn ? (cfloat_p)(a.w_cn + (int64_t)it * E + e0) : nullptr;")
    w("    const cfloat_p bs = a.bias ? (cfloat_p)(a.bias + (int64_t)it * E + e0) : nullptr;")
    w("    if (KIND == NLDPC_NEURAL || wc) {")
    w("#pragma unroll")
    w("        for (int k = 0; k < DC; ++k) wv[k] = wc[k];")
    w("    } else {")
    w("#pragma unroll")
    w("        for (int k = 0; k < DC; ++k) wv[k] = 1.f;")
    w("    }")
    w("    if (KIND == NLDPC_NEURAL) {")
    w("#pragma unroll")
    w("        for (int k = 0; k < DC; ++k) bv[k] = bs[k];")
    w("    } else {")
    w("#pragma unroll")
    w("        for (int k = 0; k < DC; ++k) bv[k] = 0.f;")
    w("    }")
    w("#pragma unroll")
    w("    for (int q = Q0; q < Q1; ++q) {")
    # per-copy partial sums (slot q of the wave's Q): no accumulator lives across the copies (QMS z=384 with
    # 3 chunks 3135 -> 16 spilled VGPRs against per-lane accumulators over the copies)
    w("        float gwa[DC], gba[DC];")
    w("#pragma unroll")
    w("        for (int k = 0; k < DC; ++k) gwa[k] = gba[k] = 0.f;")
    w("        auto load_m = [&](int k) {  // saved v2c of edge k at check copy h = u + q*ZT")
    if SBY:
        w("            if constexpr (KIND == NLDPC_QMS)")
        w(f"                return qms_decode(((const int8_t*)sq)[k * {Z} + q * {ZT}]);")
        w("            else")
        w(f"                return ((const float*)sq)[k * {Z} + q * {ZT}];")
    else:
        w("            if constexpr (KIND == NLDPC_QMS)")
        w("                return qms_decode((int8_t)bload8(svr, (vcw >> 2) + (uint32_t)(u + q * ZT), (e0 + k) * Z));")
        w("            else")
        w("                return bload(svr, vcw + 4u * (uint32_t)(u + q * ZT), 4 * (e0 + k) * Z);")
    w("        };")
    w("        if constexpr (KIND == NLDPC_SP) {")
    w("            float m[DC], gc[DC], gm[DC], gw[DC], gu[DC], gb[DC];")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) {")
    w("                m[k] = load_m(k);")
    w("                gc[k] = rp[k * Z + q * ZT];")
    w("            }")
    w("            cn_backward<DC, KIND, false>(m, gc, DC, 0.f, wv, wv, bv, wc != nullptr, false, a.qbit, a.lo, a.hi, "
      "gm, gw, gu, gb, SpRow{a.sp_plan + row * kSpPlanBytes, a.tanh});")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) {")
    w("                rp[k * Z + q * ZT] = gm[k];")
    w("                gwa[k] += gw[k];")
    w("            }")
    w("        } else {")
    w("            cn_bwd_ms<DC, KIND, TIED != 0>(load_m, rp + q * ZT, Z, wv, bv, KIND == NLDPC_NEURAL || wc, a.qbit, a.lo, a.hi, "
      "gwa, gba);")
    w("        }")
    def flush_q(indent):  # this copy's wave sums, added up over the row's copies by lane 0 in LDS
        for arr, dst, off, cond in (("gwa", "a.p_cn", "0", "a.p_cn"), ("gba", "a.p_bias", "MDC", "KIND == NLDPC_NEURAL && a.p_bias")):
            w(f"{indent}if ({cond}) {{")
            w("#pragma unroll")
            w(f"{indent}    for (int k = 0; k < DC; ++k) {{")
            w(f"{indent}        const float s_ = wave_sum(dup_ ? 0.f : {arr}[k]);")
            if Q == 1:
                w(f"{indent}        if (lane0) {dst}[pc + e0 + k] = s_;")
            else:
                w(f"{indent}        if (lane0) {{")
                w(f"{indent}            if (q == 0) gacc[{off} + k] = s_;")
                w(f"{indent}            else if (q < {Q - 1}) gacc[{off} + k] = gacc[{off} + k] + s_;")
                w(f"{indent}            else {dst}[pc + e0 + k] = gacc[{off} + k] + s_;")
                w(f"{indent}        }}")
            w(f"{indent}    }}")
            w(f"{indent}}}")
    # tied CN weight (NLDPC_FLAG_CN_TIED): every edge's contribution joins the wave's running sum (one wave
    # reduction per iteration, written by bwd_p into the part's designated edge); the row's entries get 0
    def tied(indent):
        # (one wave reduction per row copy into the wave's LDS sum: a per-lane running sum across the rows,
        # no reduction inside the row loop, made the register allocator spill 5 520 VGPRs)
        w(f"{indent}if constexpr (TIED) {{")
        w(f"{indent}    float t_ = 0.f;")
        if CNBSPARSE:  # (the tied MS / QMS check node keeps its sum in gwa[0], started from +0: 0 + gwa[0] + 0 ... is gwa[0])
            w(f"{indent}    if constexpr (KIND == NLDPC_MS || KIND == NLDPC_QMS) t_ = gwa[0];")
            w(f"{indent}    else")
        w("#pragma unroll")
        w(f"{indent}    for (int k = 0; k < DC; ++k) t_ += gwa[k];")
        w(f"{indent}    const float s_ = wave_sum(dup_ ? 0.f : t_);")
        if TACC:  # (r6: the wave's running sum in a register -- no LDS read-add-write by lane 0 per row copy)
            w(f"{indent}    tacc += s_;")
        else:
            w(f"{indent}    if (lane0) gacc[0] += s_;")
        w(f"{indent}}} else {{")
    tied("        ")
    flush_q("            ")
    w("        }")
    w("        __builtin_amdgcn_sched_barrier(0);  // one check copy at a time: the state owns the registers")
    w("    }")
    w("}")
    for p in range(S.P):
        for ci, (r0, r1, e0c, e1c) in enumerate(S.chunks):
            w("template <int KIND, int TIED>")
            w(f"__device__ __forceinline__ void cnb_p{p}_c{ci}(float* lds, const char* stg, int u, const FusedBwdArgs& a, "
              "int it, rsrc_t svr, uint32_t vcw, int64_t pc, bool lane0, bool dup_, float* gacc, float& tacc) {")
            w("    asm volatile(\"\" : \"+v\"(u));")
            w("    constexpr int SB = saved_msg_bytes<KIND>();")
            # whole rows per part (untied: a row's per-edge sums add up over its copies in the wave's LDS
            # slots; tied: one wave sum per row copy; by (row, copy) units as the forward: 28.33 vs 27.87 ms,
            # profiles/r4c_ab_cfg5.txt)
            rows = sorted(S.cn_rows[ci][p], key=lambda i: -len(S.row_edges[i]))
            w("    if constexpr (!TIED) {")
            for i in rows:
                es = S.row_edges[i]
                off = (es[0] - e0c) * Z
                w(f"        cnb_row<KIND, {len(es)}, 0, 0, {Q}>(lds + {off} + u, stg + ({off} + u) * SB, u, a, it, {es[0]}, {i}, svr, "
                  "vcw, pc, lane0, dup_, gacc, tacc);")
            w("    } else {")
            for i in rows:
                es = S.row_edges[i]
                off = (es[0] - e0c) * Z
                w(f"        cnb_row<KIND, {len(es)}, 1, 0, {Q}>(lds + {off} + u, stg + ({off} + u) * SB, u, a, it, {es[0]}, {i}, "
                  "svr, vcw, pc, lane0, dup_, gacc, tacc);")
            w("    }")
            w("}")
            # the chunk's saved block -> this codeword's staging region (all threads of the workgroup)
            if SBY and p == 0:
                nb = (e1c - e0c) * Z * SBY
                W_ = S.stage_width
                w("template <int KIND>")
                # r5: 32-bit offsets into a descriptor over the block's chunk instead of 64-bit lane addresses,
                # the lane from v_mbcnt and the wave's first thread index (w0, wave-uniform) from the caller --
                # none of them kept live across the iteration (the tied kernel had spilled them and reloaded
                # them every phase: spilled VGPRs 21 -> 4, cfg5 backward 26.3 -> 25.0 ms, profiles/r5u_*)
                w(f"__device__ __forceinline__ void stage_c{ci}(const FusedBwdArgs& a, int it, int64_t blk, int nlive, "
                  "char* stg_all, int w0) {")
                w(f"    constexpr int NP = {nb // W_};  // {W_}-byte pieces")
                w("    const int lane = lane_id();")
                w(f"    const char* src = a.sv2c + ((int64_t)it * a.sv2c_stride + blk * {E * Z}) * {SBY} + {e0c * Z * SBY};")
                w("#pragma unroll")
                w(f"    for (int g = 0; g < {G}; ++g) {{")
                w("        if (g >= nlive) break;")
                w(f"        const rsrc_t sr = make_rsrc((const float*)(src + (int64_t)g * {E * Z * SBY}), {nb});")
                w(f"        char* dg = stg_all + g * {4 * S.stage_floats};")
                w(f"        for (int i = w0; i < NP; i += {S.threads}) {{")
                w(f"            if (i + lane < NP) __builtin_amdgcn_raw_ptr_buffer_load_lds(sr, (lptr_t)(dg + i * {W_}), {W_}, "
                  f"(uint32_t)(i + lane) * {W_}u, 0, 0, {2 if BWDCACHE >= 2 else 0});")
                w("        }")
                w("    }")
                w("}")

    # ---------------------------------------------------------------- per-part driver
    for p in range(S.P):
        sp = max(len(S.slots[p]), 1)
        w("template <int KIND, int TIED>")
        w(f"__device__ __forceinline__ void bwd_p{p}(const FusedBwdArgs& a, float* lds, int u, int64_t blk, int nlive, "
          f"uint32_t vo, uint32_t vm, uint32_t vcw, int slot, bool lane0, bool dup_, const char* stg, char* stg_all, "
          f"float* gacc, int wb) {{")
        for q in range(Q):
            w(f"    float g{q}[{sp}];")
        w(f"    const rsrc_t cyr = make_rsrc(a.carry ? a.carry + blk * {NZ} : nullptr, a.carry ? nlive * {4 * NZ} : 0);")
        w(f"    const rsrc_t xr = make_rsrc(a.xa + blk * {NZ}, nlive * {4 * NZ});")

        def rs(ptr_expr, esize, per_cw):
            return (f"make_rsrc((const float*)({ptr_expr} ? {ptr_expr} + blk * {per_cw} : nullptr), "
                    f"{ptr_expr} ? nlive * {per_cw * esize} : 0)")
        w("    {  // k = T-1: dL/dc2v_T = dL/dy_{T-1} * mask (no later check node)")
        w("        const float* gp_ = a.gy.p[a.T - 1];")
        w("        const uint8_t* mp_ = a.symask ? a.symask + (a.T - 1) * a.symask_stride : nullptr;")
        w(f"        const rsrc_t gr = {rs('gp_', 4, NZ)};")
        w(f"        const rsrc_t mr = {rs('mp_', 1, NZ)};")
        s0 = 0
        for j in S.reg_cols[p]:
            d = len(S.col_edges[j])
            for q in range(Q):
                w(f"        {{ const float v_ = {_GY}<KIND>(gr, mr, vo, vm, {X(j, q)});")
                for k in range(d):
                    w(f"          g{q}[{s0 + k}] = v_;")
                w("        }")
            s0 += d
        w("    }")
        w("    for (int it = a.T - 1; it >= 0; --it) {")
        w("        const float* gp_ = a.gy.p[it];")
        w("        const uint8_t* mp_ = a.symask ? a.symask + it * a.symask_stride : nullptr;")
        w(f"        const rsrc_t gr = {rs('gp_', 4, NZ)};")
        w(f"        const rsrc_t mr = {rs('mp_', 1, NZ)};")
        w("        constexpr int SB = saved_msg_bytes<KIND>();")
        w("        const char* sv_ = a.sv2c + it * a.sv2c_stride * SB;")
        w(f"        const rsrc_t svr = make_rsrc((const float*)(sv_ + blk * {E * Z} * SB), nlive * {E * Z} * SB);")
        w("        const float* sx_ = (a.sxin && it >= 1) ? a.sxin + (it - 1) * a.sxin_stride : nullptr;")
        w(f"        const rsrc_t sxp = {rs('sx_', 4, NZ)};")
        w("        const cfloat_p wvn = a.w_vn ? (cfloat_p)(a.w_vn + (int64_t)it * N) : nullptr;")
        w("        const int64_t pc = ((int64_t)it * a.nslots + slot) * E;")
        w("        const int64_t pv = ((int64_t)it * a.nslots + slot) * N;")
        def bstamp(ph):  # diagnostic stamp build: arrival of each wave at the end of a phase
            if STAMPS:
                assert ph < 16
                w(f"        stamp_store(a.stamps, {S.threads // 64}, a.T, it, {ph});")
        w("        if (TIED && lane0) gacc[0] = 0.f;  // (tied CN: the wave's sum lives in its LDS slot)")
        w("        float tacc = 0.f;  // (TACC: the tied CN's wave sum in a register instead)")
        bstamp(0)
        for ci in range(len(S.chunks)):
            if SBY:  # the chunk's saved messages start moving into LDS now and land by the barrier
                w(f"        stage_c{ci}<KIND>(a, it, blk, nlive, stg_all, wb);")
            w(f"        wrb_p{p}_c{ci}<KIND>({state_args()}, lds, u, gr, mr, vo, vm);")
            bstamp(1 + 3 * ci)
            if SBY:
                w("        asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // (LDS-DMA: not in hipcc's count)")
            w("        __syncthreads();")
            w(f"        cnb_p{p}_c{ci}<KIND, TIED>(lds, stg, u, a, it, svr, vcw, pc, lane0, dup_, gacc, tacc);")
            bstamp(2 + 3 * ci)
            w("        __syncthreads();")
            w(f"        rdb_p{p}_c{ci}<KIND, TIED>({state_args()}, lds, u, a, it, vo, xr, sxp, cyr, wvn, pv, lane0, dup_);")
            bstamp(3 + 3 * ci)
            w("        __syncthreads();")
        w("        const float* gq_ = it >= 1 ? a.gy.p[it - 1] : nullptr;  // dL/dy_{k-1}")
        w("        const uint8_t* mq_ = (a.symask && it >= 1) ? a.symask + (it - 1) * a.symask_stride : nullptr;")
        w(f"        const rsrc_t gr1 = {rs('gq_', 4, NZ)};")
        w(f"        const rsrc_t mr1 = {rs('mq_', 1, NZ)};")
        w(f"        vnb_p{p}<KIND, TIED>({state_args()}, a, it, vo, vm, gr1, mr1, xr, sxp, cyr, wvn, pv, lane0, dup_);")
        # tied weights: the wave's sums into the part's designated entries (written 0 earlier this iteration,
        # by this wave's lane 0: program order makes these the final values)
        # (the launcher zeroed the tied kernel's partials: each part's wave total goes to the part's own entry
        # p of the row -- distinct per part, and the two waves of a part have slots of their own)
        w(f"        if (TIED && a.p_cn && lane0) a.p_cn[pc + {p}] = {'tacc' if TACC else 'gacc[0]'};")

        bstamp(1 + 3 * len(S.chunks))
        w("    }")
        w("}")

    w("template <int KIND, int TIED>")
    w("__device__ __forceinline__ void bwd_body(const FusedBwdArgs& a, float* lds_sh) {")
    w("    if (a.sig != kFusedBwdArgsSig) return;  // a launcher built against another FusedBwdArgs layout")
    STF = S.stage_floats
    if SBY:
        w(f"    static_assert(saved_msg_bytes<KIND>() == {SBY}, \"kernel built for another saved-message width\");")
    GST = 2 * S.max_dc if Q > 1 else 1  # per-wave sums (lane 0): a row's copies, or the tied CN sum
    GA = GST * (S.threads // 64)
    assert 4 * (STF * S.G_lds + CF * S.G_lds + GA) <= 160 * 1024, S.tag
    w(f"    // lds_sh: [{STF * S.G_lds + CF * S.G_lds + GA}] floats, staging | images | sums (declared once in bwd_entry)")
    w(f"    char* stg_all = (char*)lds_sh;  // [G_lds][{4 * STF}] bytes: the chunk's saved messages (S.stage)")
    w(f"    float* lds_all = lds_sh + {STF * S.G_lds};")
    w(f"    float* gacc = lds_sh + {STF * S.G_lds + CF * S.G_lds} + {GST} * (threadIdx.x >> 6);  "
      "// this wave's weight-gradient sums over a row's copies (lane 0)")
    w("    const int t = threadIdx.x;")
    w(f"    const int p = __builtin_amdgcn_readfirstlane(t / {S.lanes_pad});")
    w(f"    const int r0_ = t - p * {S.lanes_pad};")
    w(f"    const bool dup_ = r0_ >= {S.lanes};  // a lane repeating a live one (Spec.lanes_pad)")
    w(f"    const int r = dup_ ? r0_ - {S.lanes} : r0_;")
    w(f"    const int g = r / {ZT};")
    w(f"    const int u = r - g * {ZT};")
    w(f"    const int64_t blk = (int64_t)blockIdx.x * {G};")
    w(f"    const int nlive = a.B - blk < {G} ? (int)(a.B - blk) : {G};")
    w(f"    const uint32_t vo = g < nlive && !dup_ ? 4u * (g * {NZ} + u) : 0x80000000u;")
    w("    const uint32_t vm = vo >> 2;")
    w(f"    const uint32_t vcw = g < nlive && !dup_ ? 4u * (g * {E * Z}) : 0x80000000u;  // codeword base in [E][Z] (CN gathers)")
    w("    const int slot = blockIdx.x * WP + __builtin_amdgcn_readfirstlane(r0_ >> 6);")
    w("    const bool lane0 = (t & 63) == 0;")
    w("    const int wb = __builtin_amdgcn_readfirstlane(t) & ~63;  // the wave's first thread index (staging)")
    if not S.padded and ZT % 64 == 0:
        # every wave lies in one codeword: its LDS regions are wave-uniform (scalar bases, nothing per lane to keep)
        w(f"    const int gw_ = __builtin_amdgcn_readfirstlane(g);")
        w(f"    float* lds = lds_all + gw_ * {CF};")
        w(f"    const char* stg = stg_all + gw_ * {4 * STF};")
    else:
        w(f"    float* lds = lds_all + (dup_ ? {G} : g) * {CF};  // (repeating lanes: their own region)")
        w(f"    const char* stg = stg_all + (dup_ ? {G} : g) * {4 * STF};")
    if SBY and S.padded:  # the repeating lanes' staging region is never filled: zeros, not stale LDS
        w(f"    for (int i = t; i < {STF}; i += {S.threads}) ((float*)(stg_all + {G * 4 * STF}))[i] = 0.f;")
    for n_, p in enumerate(PARTS or range(S.P)):  # (NLDPC_GEN_PARTS: single-part builds for the ISA budget)
        w(f"    {'if' if n_ == 0 else 'else if'} (p == {p}) bwd_p{p}<KIND, TIED>(a, lds, u, blk, nlive, vo, vm, vcw, slot, lane0, dup_, "
          "stg, stg_all, gacc, wb);")
    w("}")
    # a tied CN weight (cfg5's NW(3,0,3): one CN weight per iteration): a separate kernel (TIED = 1) reduces
    # each row copy's contributions once (one wave reduction per row copy into the wave's LDS sum) instead of
    # once per edge; the launcher takes it when the CN gradient is tied (nldpc_backward.hip).  (Both bodies behind a run-time branch in one
    # kernel: 8 994 spilled VGPRs.)
    w("template <int KIND, int TIED>")
    w("__device__ __forceinline__ void bwd_entry(const FusedBwdArgs& a) {")
    w(f"    __shared__ __attribute__((aligned(16))) float lds_sh[{STF * S.G_lds + CF * S.G_lds + GA}];")
    w("    bwd_body<KIND, TIED>(a, lds_sh);")
    w("}")
    w("template <int KIND, int TIED>")
    w(f"__global__ __launch_bounds__({S.threads}, {(S.threads + 255) // 256}) void bwd_kernel(FusedBwdArgs a) {{")
    w("    bwd_entry<KIND, TIED>(a);")
    w("}")
    w("}  // namespace")
    return "\n".join(L)


# Backward kernels by kind: bytes per staged saved message (Spec stage) and their namespace.  Neural
# stages fp32 messages (5 chunks at z=384, no spills); QMS its int8 codes (3 chunks); MS / SP gather from
# global memory (staged fp32 messages need 5 chunks, and the MS / SP kernels spill there: 2646 VGPRs)
BWD_STAGE = {0: 0, 1: 0, 2: 1, 3: 4}
BWD_NS = {0: "fusedbs", 1: "fusedbs", 2: "fusedbq", 3: "fusedb"}

MODES = (0, 1, 2, 3)  # forward kernels: decode / decode + save for backward / count-only (all-zero, LLR > 0) / count-only (general)


def jit_source(hb, Z, kind, mode):
    """One register-resident kernel for any lifted graph, compiled at run time (nldpc/jit.py: hipcc
    --genco, nldpc_graph_attach_kernel): the (graph, Z) -> geometry choice of auto_geometry, the same
    emitted code as the library's own kernels, one (kind, mode) instantiation behind an unmangled entry
    point -- nldpc_fx (MODE 0-3) or nldpc_fxb (mode 4, the backward).  Returns (source, geometry dict)."""
    hb = np.asarray(hb, dtype=np.int64)
    G, P, Q = auto_geometry(hb, Z)
    S = Spec("jit", hb, Z, G, P, Q, sched="pipe2" if mode in (0, 2, 3) else "one",  # the SAVE kernels keep one buffer
             stage=BWD_STAGE[kind] if mode == 4 else 0)  # (backward: staged saved messages)
    L = ["// GENERATED by gen_fused.py jit_source -- do not edit.", "#include <hip/hip_runtime.h>"] + \
        (["#define NLDPC_CNB_SPARSE 1"] if CNBSPARSE else []) + ['#include "nldpc_fused.h"', "namespace nldpc {", emit(S) if mode < 4 else emit_bwd(S, BWD_NS[kind]),
         "}  // namespace nldpc"]
    lb = f"__launch_bounds__({S.threads}, {(S.threads + 255) // 256})"
    if mode < 4:
        L.append(f'extern "C" __global__ {lb} void nldpc_fx(nldpc::FusedArgs a) {{ '
                 f"nldpc::fused_jit::kernel_body<{kind}, {mode}>(a); }}")
    else:
        L.append(f'extern "C" __global__ {lb} void nldpc_fxb(nldpc::FusedBwdArgs a) {{ '
                 f"nldpc::{BWD_NS[kind]}_jit::bwd_entry<{kind}, 0>(a); }}")
    # the argument layout this code object was built for: nldpc_graph_attach_kernel compares it with the
    # library's before accepting the kernel (a skewed build is refused instead of reading garbage)
    L.append(f'extern "C" __device__ uint32_t nldpc_sig = nldpc::{"kFusedBwdArgsSig" if mode == 4 else "kFusedArgsSig"};')
    return "\n".join(L) + "\n", {"G": G, "threads": S.threads, "waves_per_part": S.lanes_pad // 64,
                                 "P": P, "Q": Q, "padded": S.padded}


def main():
    """Writes OUTDIR/fused_<tag>_s<MODE>.hip (one translation unit per base graph and MODE variant,
    so make -j compiles them in parallel) and OUTDIR/fused_table.hip (the FusedSpec table)."""
    if sys.argv[1] == "--jit":  # --jit BASEGRAPH.txt Z KIND MODE OUT.hip: one run-time kernel's source
        hb = np.loadtxt(sys.argv[2], int, delimiter="\t")
        src, geo = jit_source(hb, int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
        with open(sys.argv[6], "w") as f:
            f.write(src)
        print(geo)
        return
    if sys.argv[1] == "--list":  # file names, for the Makefile
        print(" ".join([f"fused_{t[0]}_s{v}.hip" for t in SPECS for v in MODES] + [f"fused_{t[0]}_s0u.hip" for t in SPECS] +
                       [f"fused_{t[0]}_bwd.hip" for t in SPECS] + ["fused_table.hip"]))
        return
    outdir, res = sys.argv[1], sys.argv[2]
    os.makedirs(outdir, exist_ok=True)
    specs = []
    only = set(filter(None, os.environ.get("NLDPC_GEN_ONLY", "").split(",")))  # debug: subset of specs
    for tag, fname, Z, G, P, Q in SPECS:
        hb = np.loadtxt(os.path.join(res, fname), int, delimiter="\t")
        if G is None:
            G, P, Q = auto_geometry(hb, Z)
        specs.append((Spec(tag, hb, Z, G, P, Q, sched="pipe2"), Spec(tag, hb, Z, G, P, Q), not only or tag in only))
    head = ["// GENERATED by gen_fused.py from the base graphs in resources/ -- do not edit.",
            "#include <hip/hip_runtime.h>"]
    if CNBSPARSE:
        head.append("#define NLDPC_CNB_SPARSE 1")
    head += ['#include "nldpc_fused.h"', "namespace nldpc {"]
    kinds = os.environ.get("NLDPC_GEN_KINDS")  # debug: instantiate a subset of kinds
    kinds = [int(k) for k in kinds.split(",")] if kinds else [0, 1, 2, 3]

    def write(name, lines):
        path = os.path.join(outdir, name)
        text = "\n".join(lines) + "\n"
        if not os.path.exists(path) or open(path).read() != text:  # keep mtimes of unchanged units
            with open(path, "w") as f:
                f.write(text)

    for S, SB_, on in specs:
        body = emit(S) if on else ""
        # the SAVE kernels (training forward) keep the one-buffer schedule: with the pipelined one the
        # cfg5 forward went from 22.0 to 31.4 ms (r2), while inference gained 6 %.  Each MODE is its own
        # translation unit, so the two schedules never meet in one TU.
        body_save = (emit(SB_) if on else "") if S.pipe else body
        for save in MODES:
            src = list(head)
            src.append(body_save if save == 1 else body)
            src.append(f"uint32_t fused_{S.tag}_sig_s{save}() {{ return kFusedArgsSig; }}  // this unit's FusedArgs layout")
            src.append(f"void* fused_{S.tag}_kernel_s{save}(int kind) {{")
            if on:
                for k in kinds:
                    src.append(f"    if (kind == {k}) return reinterpret_cast<void*>(&fused_{S.tag}::kernel<{k}, {save}>);")
            src.append("    return nullptr;")
            src.append("}")
            if save == 1:  # (r6) the tied saving forward, MODE 5, Boosted MS / QMS
                src.append(f"void* fused_{S.tag}_kernel_s1t(int kind) {{")
                if on:
                    for k in kinds:
                        if k in (1, 2):
                            src.append(f"    if (kind == {k}) return reinterpret_cast<void*>(&fused_{S.tag}::kernel<{k}, 5>);")
                src.append("    return nullptr;")
                src.append("}")
            src.append("}  // namespace nldpc")
            write(f"fused_{S.tag}_s{save}.hip", src)
        # (r6) the decode specialised for UCN + CN / UCN / cumulative VN weights, MODE 6, MS / QMS: a unit of its own, so its
        # code object holds these two kernels only (the same kernel code placed after the generic decode kernels of
        # every kind ran 1.3 % slower, profiles/r6_ab_ucn_select.txt: instruction-cache placement)
        src = list(head)
        ucnw = on and S.tag in UCNW_TAGS and any(k in (1, 2) for k in kinds)
        src.append(body if ucnw else "")
        src.append(f"void* fused_{S.tag}_kernel_s0u(int kind) {{")
        if ucnw:
            for k in kinds:
                if k in (1, 2):
                    src.append(f"    if (kind == {k}) return reinterpret_cast<void*>(&fused_{S.tag}::kernel<{k}, 6>);")
        src.append("    return nullptr;")
        src.append("}")
        src.append("}  // namespace nldpc")
        write(f"fused_{S.tag}_s0u.hip", src)
        # backward kernels: the fp32-message kinds and QMS (int8 codes) stage their saved messages in LDS
        # beside chunk images sized for them, so they are two generated namespaces
        src = list(head)
        if on and not NOBWD:
            done = set()
            for k in kinds:
                if BWD_NS[k] not in done:
                    done.add(BWD_NS[k])
                    src.append(emit_bwd(Spec(S.tag, S.hb, S.Z, S.G, S.P, S.Q, stage=BWD_STAGE[k]), BWD_NS[k]))
        src.append(f"uint32_t fused_{S.tag}_sig_bwd() {{ return kFusedBwdArgsSig; }}  // this unit's FusedBwdArgs layout")
        src.append(f"void* fused_{S.tag}_bwd(int kind) {{")
        if on and not NOBWD:
            for k in kinds:
                nsk = BWD_NS[k]
                src.append(f"    if (kind == {k}) return reinterpret_cast<void*>(&{nsk}_{S.tag}::bwd_kernel<{k}, 0>);")
        src.append("    return nullptr;")
        src.append("}")
        src.append(f"void* fused_{S.tag}_bwd_tied(int kind) {{  // a tied CN weight (NLDPC_FLAG_CN_TIED)")
        if on and not NOBWD:
            for k in kinds:
                if k != 3:
                    src.append(f"    if (kind == {k}) return reinterpret_cast<void*>(&{BWD_NS[k]}_{S.tag}::bwd_kernel<{k}, 1>);")
        src.append("    return nullptr;")
        src.append("}")
        src.append("}  // namespace nldpc")
        write(f"fused_{S.tag}_bwd.hip", src)
    src = list(head)
    for S, _, _ in specs:
        for v in MODES:
            src.append(f"void* fused_{S.tag}_kernel_s{v}(int kind);")
        src.append(f"void* fused_{S.tag}_bwd(int kind);")
        src.append(f"void* fused_{S.tag}_bwd_tied(int kind);")
        src.append(f"void* fused_{S.tag}_kernel_s1t(int kind);")
        src.append(f"void* fused_{S.tag}_kernel_s0u(int kind);")
        for v in MODES:
            src.append(f"uint32_t fused_{S.tag}_sig_s{v}();")
        src.append(f"uint32_t fused_{S.tag}_sig_bwd();")
        src.append(f"static const int32_t basegraph_{S.tag}[{S.M * S.N}] = "
                   f"{{{', '.join(str(int(x)) for x in S.hb.reshape(-1))}}};")
    src.append("const FusedSpec* fused_specs(int* n) {")
    src.append(f"    static const FusedSpec tab[{len(specs)}] = {{")
    for S, _, _ in specs:
        ks = ", ".join("{" + ", ".join(f"fused_{S.tag}_kernel_s{v}({k})" for k in range(4)) + "}" for v in MODES)
        kb = ", ".join(f"fused_{S.tag}_bwd({k})" for k in range(4))
        kt = ", ".join(f"fused_{S.tag}_bwd_tied({k})" for k in range(4))
        sg = ", ".join([f"fused_{S.tag}_sig_s{v}()" for v in MODES] + [f"fused_{S.tag}_sig_bwd()"] * 2)
        st = ", ".join(f"fused_{S.tag}_kernel_s1t({k})" for k in range(4))
        su = ", ".join(f"fused_{S.tag}_kernel_s0u({k})" for k in range(4))
        src.append(f"        {{\"{S.tag}\", {S.M}, {S.N}, {S.Z}, {S.E}, {S.G}, {S.threads}, basegraph_{S.tag}, "
                   f"{{{ks}}}, {{{kb}}}, {S.lanes_pad // 64}, {{{kt}}}, {{{sg}}}, {{{st}}}, {{{su}}}}},")
    src.append("    };")
    src.append(f"    *n = {len(specs)};")
    src.append("    return tab;")
    src.append("}")
    src.append("}  // namespace nldpc")
    write("fused_table.hip", src)


if __name__ == "__main__":
    main()
