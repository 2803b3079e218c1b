"""Generate the register-resident fused decoder kernels (nldpc_fused_gen.hip) for known base graphs.

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

Usage: python3 gen_fused.py OUT.hip RESOURCE_DIR
"""
import os
import sys

import numpy as np

PARTS = [int(x) for x in filter(None, os.environ.get("NLDPC_GEN_PARTS", "").split(","))]  # debug
SKIP = set(filter(None, os.environ.get("NLDPC_GEN_SKIP", "").split(",")))  # debug: drop phases
LDS_BYTES = 160 * 1024 - 2048  # leave room for the compiler / alignment

# (tag, base graph file, Z, codewords per workgroup G, parts P, copies per thread Q)
SPECS = [
    ("bg2_z384", "basegraph2_set0.txt", 384, 1, 8, 3),
    ("bg2_z16", "basegraph2_set0.txt", 16, 16, 2, 1),
    ("wimax_z24", "wman_N0576_R34_z24.txt", 24, 16, 1, 1),
]


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
    def __init__(self, tag, hb, Z, G, P, Q):
        assert Z % Q == 0
        self.tag, self.hb, self.Z, self.G, self.P, self.Q = tag, hb, Z, G, P, Q
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
        self.d1_cols = balance(single, lambda j: 1, P)  # stateless degree-1 columns
        self.slots = [[e for j in cols_ for e in self.col_edges[j]] for cols_ in self.reg_cols]
        self.smax = max(1, max(len(s) for s in self.slots)) * Q
        # row chunks: contiguous row ranges whose messages (edges x Z x G) fit in LDS
        cap = (LDS_BYTES // (4 * G) - 32) // Z
        self.chunks = []  # (row_begin, row_end, edge_begin, edge_end)
        r0 = 0
        while r0 < self.M:
            e0 = self.row_edges[r0][0]
            r1 = r0
            while r1 < self.M and self.row_edges[r1][-1] - e0 + 1 <= cap:
                r1 += 1
            if r1 == r0:
                raise SystemExit(f"{tag}: a single check row does not fit in LDS")
            self.chunks.append((r0, r1, e0, self.row_edges[r1 - 1][-1] + 1))
            r0 = r1
        self.chunk_floats = max(e1 - e0 for _, _, e0, e1 in self.chunks) * Z
        if G > 1:  # codeword stride = 1 (mod 32 banks) so lanes of different codewords do not collide
            self.chunk_floats += (1 - self.chunk_floats) % 32
        self.cn_rows = [balance(list(range(r0, r1)), lambda i: len(self.row_edges[i]), P)
                        for (r0, r1, _, _) in self.chunks]
        self.lanes = G * self.ZT  # threads per part
        self.threads = P * self.lanes
        assert self.threads <= 1024 and self.lanes % 64 == 0, (tag, self.threads)
        self.max_dc = max(len(r) for r in self.row_edges)


def emit(S: Spec) -> str:
    Z, G, Q, ZT, NZ = S.Z, S.G, S.Q, S.ZT, S.N * S.Z
    L = []
    w = L.append
    CF = S.chunk_floats
    w(f"// ---- {S.tag}: M={S.M} N={S.N} E={S.E} Z={Z}; workgroup = {G} codeword(s) x {S.P} part(s) x {ZT} lanes "
      f"= {S.threads} threads, {Q} cop{'y' if Q == 1 else 'ies'} per lane; register slots/part "
      f"{[len(s) * Q for s in S.slots]}; {len(S.chunks)} LDS chunk(s) of <= {CF * G * 4} B")
    w(f"namespace fused_{S.tag} {{")
    w(f"constexpr int Z = {Z}, ZT = {ZT}, N = {S.N}, E = {S.E};")

    # Register state of part p: copies are paired (q = 0,1 / 2,3 ...) into float2 arrays so the VN's
    # additions run as packed fp32 (v_pk_add_f32: two IEEE adds per lane, same rounding); an odd
    # copy count leaves one scalar array.  The channel values a thread needs every iteration are
    # loaded once into registers (xp*/xs for its register columns, xd for its degree-1 columns).
    NPAIR, SINGLE = Q // 2, Q % 2

    def ref(q, k):
        if q < 2 * NPAIR:
            return f"cp{q // 2}[{k}].{'x' if q % 2 == 0 else 'y'}"
        return f"cs[{k}]"

    def xref(p, j, q):
        cols = S.reg_cols[p]
        if j in cols:
            n = cols.index(j)
            return f"xp{q // 2}[{n}].{'x' if q % 2 == 0 else 'y'}" if q < 2 * NPAIR else f"xs[{n}]"
        n = S.d1_cols[p].index(j)
        return f"xd[{n * Q + q}]"

    def state_params(p, const=False):
        sp = len(S.slots[p])
        c = "const " if const else ""
        ps = [f"{c}f2 (&cp{i})[{max(sp, 1)}]" for i in range(NPAIR)]
        if SINGLE:
            ps.append(f"{c}float (&cs)[{max(sp, 1)}]")
        return ", ".join(ps)

    def state_args():
        return ", ".join([f"cp{i}" for i in range(NPAIR)] + (["cs"] if SINGLE else []))

    def x_params(p):
        nr, nd = max(len(S.reg_cols[p]), 1), max(len(S.d1_cols[p]) * Q, 1)
        ps = [f"const f2 (&xp{i})[{nr}]" for i in range(NPAIR)]
        if SINGLE:
            ps.append(f"const float (&xs)[{nr}]")
        ps.append(f"const float (&xd)[{nd}]")
        return ", ".join(ps)

    def x_args():
        return ", ".join([f"xp{i}" for i in range(NPAIR)] + (["xs"] if SINGLE else []) + ["xd"])

    # ---------------------------------------------------------------- variable nodes
    # global accesses: bload/bstore(descriptor, lane byte offset vo, constant byte offset)
    def X(j, q):  # byte offset of variable copy (column j, lane copy q) in a [N][Z] codeword
        return 4 * (j * Z + q * ZT)

    def vn_group(p, n, j, s, d, final, vec, names, xin):
        """VN (or final posterior) of column j (n-th register column of part p) for one copy group:
        vec: float2 pair (names = ('cp0', 'x'/'y' copies)) or scalar."""
        T_ = "f2" if vec else "float"
        arr = names
        c = lambda k: f"{arr}[{s + k}]"  # noqa: E731
        add = (lambda x, y: f"({x} + {y})") if vec else (lambda x, y: f"fadd({x}, {y})")  # noqa: E731
        zero = "f2{0.f, 0.f}" if vec else "0.f"
        w(f"        {{  // column {j}, degree {d}, {'copies ' + xin if vec else 'copy ' + xin}")
        w(f"            {T_} P = {zero};")
        if not final:
            ch = (f"vn_channel2<KIND>({xin}, a.w_vn, N, {j}, a.vn_prefix + it + 1, a.qbit)" if vec else
                  f"vn_channel<KIND>({xin}, a.w_vn, N, {j}, a.vn_prefix + it + 1, a.qbit)")
            w(f"            const {T_} x0 = {add(zero, ch)};")
            for k in range(d):
                expr = "P"
                for m in range(k + 1, d):
                    expr = add(expr, c(m))
                # one edge at a time: the fake dependence of the running prefix on the new message
                # keeps the compiler from running the prefix chain ahead and holding every partial
                # sum in a register (dependent VALU ops issue back to back anyway)
                w(f"            {{ const {T_} S_ = {expr}; const {T_} o_ = {c(k)}; {c(k)} = {add('x0', 'S_')}; "
                  f"asm volatile(\"\" : \"+v\"(P) : \"v\"({c(k)})); P = {add('P', 'o_')}; }}")
        else:
            for k in range(d):
                w(f"            P = {add('P', c(k))};")
        return T_

    for p in range(S.P):
        cols = S.reg_cols[p]
        for final in (False, True):
            fname = f"post_p{p}" if final else f"vn_p{p}"
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void {fname}({state_params(p)}, {x_params(p)}, const FusedArgs& a, "
              f"uint32_t vo, int it, rsrc_t pr) {{")
            s = 0
            for n, j in enumerate(cols):
                d = len(S.col_edges[j])
                for i in range(NPAIR):
                    vn_group(p, n, j, s, d, final, True, f"cp{i}", f"xp{i}[{n}]")
                    w(f"            const f2 y_ = posterior2<KIND>(xp{i}[{n}], P, a);")
                    w(f"            bstore(pr, vo, {X(j, 2 * i)}, y_.x);")
                    w(f"            bstore(pr, vo, {X(j, 2 * i + 1)}, y_.y);")
                    w("        }")
                    w("        __builtin_amdgcn_sched_barrier(0);")
                if SINGLE:
                    vn_group(p, n, j, s, d, final, False, "cs", f"xs[{n}]")
                    w(f"            bstore(pr, vo, {X(j, Q - 1)}, posterior<KIND>(xs[{n}], P, a));")
                    w("        }")
                    w("        __builtin_amdgcn_sched_barrier(0);")
                s += d
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

    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            mine = [(k, e) for k, e in enumerate(S.slots[p]) if e0 <= e < e1]
            d1 = [(j, S.col_edges[j][0]) for j in S.d1_cols[p] if e0 <= S.col_edges[j][0] < e1]
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void wr_p{p}_c{ci}({state_params(p, True)}, {x_params(p)}, float* lds, "
              f"int u, const FusedArgs& a, int it) {{")
            w("    asm volatile(\"\" : \"+v\"(u));  // LDS addresses are recomputed here, not hoisted out of the loop")
            for q in range(Q):
                for k, e in mine:
                    w(f"    lds[{own(e, q, e0)}] = {ref(q, k)};")
            for j, e in d1:  # v2c = (0 + xin) + 0: no other edge in the column
                for q in range(Q):
                    w(f"    lds[{own(e, q, e0)}] = fadd(fadd(0.f, vn_channel<KIND>({xref(p, j, q)}, "
                      f"a.w_vn, N, {j}, a.vn_prefix + it + 1, a.qbit)), 0.f);")
            w("}")
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void rd_p{p}_c{ci}({state_params(p)}, {x_params(p)}, const float* lds, "
              f"int u, const FusedArgs& a, uint32_t vo, rsrc_t pr, rsrc_t cr, uint32_t vc, bool has_co) {{")
            w("    asm volatile(\"\" : \"+v\"(u));")
            for q in range(Q):
                for k, e in mine:
                    w(f"    {ref(q, k)} = lds[{own(e, q, e0)}];")
            for j, e in d1:  # this iteration's posterior right away
                for q in range(Q):
                    w(f"    bstore(pr, vo, {X(j, q)}, posterior<KIND>({xref(p, j, q)}, fadd(0.f, lds[{own(e, q, e0)}]), a));")
            if d1:
                w("    if (has_co) {  // final message state (last iteration only)")
                for j, e in d1:
                    for q in range(Q):
                        w(f"        bstore(cr, vc, {4 * (e * Z + q * ZT)}, lds[{own(e, q, e0)}]);")
                w("    }")
            w("}")

    # ---------------------------------------------------------------- check nodes (table driven)
    # LDS holds each edge's Z messages in CHECK order (the owners rotate on write/read-back), so the
    # thread of check copy h reads every edge of its row at h: one address per row, the edges at
    # immediate offsets k*Z.  Rows are grouped by degree so every loop has a compile-time degree.
    tab, groups = [], {}
    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            gl = []
            rows = S.cn_rows[ci][p]
            for dc in sorted({len(S.row_edges[i]) for i in rows}, reverse=True):
                sel = [i for i in rows if len(S.row_edges[i]) == dc]
                gl.append((dc, len(tab), len(sel)))
                tab += [S.row_edges[i][0] for i in sel]
            groups[(p, ci)] = gl
    S.cn_groups = groups
    w(f"__constant__ int32_t cn_tab[{max(1, len(tab))}] = {{{', '.join(str(x) for x in tab) or '0'}}};")
    w("template <int KIND, int DC>")
    w("__device__ __forceinline__ void cn_rows(float* lds, int u, const FusedArgs& a, int it, int t0, int n, int e0c) {")
    w("    asm volatile(\"\" : \"+v\"(u));")
    w("    for (int r = 0; r < n; ++r) {")
    w("        const int e0 = cn_tab[t0 + r];  // first edge of the row (its edges are consecutive)")
    w("        float* rp = lds + (e0 - e0c) * Z + u;")
    w("        float wv[DC], bv[DC];")
    w("        const cfloat_p wc = a.w_cn ? (cfloat_p)(a.w_cn + (int64_t)it * E + e0) : nullptr;")
    w("        const cfloat_p bs = a.bias ? (cfloat_p)(a.bias + (int64_t)it * E + e0) : nullptr;")
    w("        // whole-row scalar loads (one uniform test per row, not per edge, so the loads can merge)")
    w("        if (KIND == NLDPC_NEURAL || wc) {")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) wv[k] = wc[k];")
    w("        } else {")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) wv[k] = 1.f;")
    w("        }")
    w("        if (KIND == NLDPC_NEURAL || bs) {")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) bv[k] = bs[k];")
    w("        } else {")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) bv[k] = 0.f;")
    w("        }")
    w("#pragma unroll")
    w(f"        for (int q = 0; q < {Q}; ++q) {{  // one check copy at a time: the state owns the registers")
    w("            float m[DC];")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) m[k] = rp[k * Z + q * ZT];")
    w("            if (KIND == NLDPC_NEURAL) {")
    w("                neural_row<DC>(m, wv, bv);")
    w("            } else {")
    w("                CnCore<DC> core;")
    w("                cn_core<DC, KIND>(m, DC, a.qbit, a.lo, a.hi, core);")
    w("#pragma unroll")
    w("                for (int k = 0; k < DC; ++k)")
    w("                    m[k] = cn_epilogue<KIND, false>(core.out0[k], wv[k], 0.f, 0.f, 0.f, wc != nullptr, false, a.qbit,"
      " a.lo, a.hi).c;")
    w("            }")
    w("#pragma unroll")
    w("            for (int k = 0; k < DC; ++k) rp[k * Z + q * ZT] = m[k];")
    if Q > 1:
        w("            __builtin_amdgcn_sched_barrier(0);")
    w("        }")
    w("    }")
    w("}")

    # ---------------------------------------------------------------- the kernel
    def each_part(fmt, indent="        "):
        for p in PARTS or range(S.P):
            w(f"{indent}{'if' if p == 0 else 'else if'} (p == {p}) {fmt.format(p=p)};")

    # Each part runs its own copy of the whole iteration loop: its register state never meets another
    # part's at a control-flow join (per-phase part branches inside one loop made the register
    # allocator insert phi copies and spill).  The parts still meet at every s_barrier: a hardware
    # barrier counts waves, not program counters, and every part executes the same barrier sequence.
    for p in range(S.P):
        if PARTS and p not in PARTS:
            continue
        sp = max(len(S.slots[p]), 1)
        nr, nd = max(len(S.reg_cols[p]), 1), max(len(S.d1_cols[p]) * Q, 1)
        w("template <int KIND>")
        w(f"__device__ __forceinline__ void run_p{p}(const FusedArgs& a, float* lds, int u, int64_t blk, int nlive, "
          f"rsrc_t xr, uint32_t vo, rsrc_t cr, uint32_t vc) {{")
        for i in range(NPAIR):
            w(f"    f2 cp{i}[{sp}], xp{i}[{nr}];")
        if SINGLE:
            w(f"    float cs[{sp}], xs[{nr}];")
        w(f"    float xd[{nd}];")
        w("#pragma unroll")
        w(f"    for (int k = 0; k < {sp}; ++k) {{")
        for i in range(NPAIR):
            w(f"        cp{i}[k] = f2{{0.f, 0.f}};")
        if SINGLE:
            w("        cs[k] = 0.f;")
        w("    }")
        w("    // this thread's channel values, loaded once for all T iterations")
        for n, j in enumerate(S.reg_cols[p]):
            for i in range(NPAIR):
                w(f"    xp{i}[{n}] = f2{{bload(xr, vo, {X(j, 2 * i)}), bload(xr, vo, {X(j, 2 * i + 1)})}};")
            if SINGLE:
                w(f"    xs[{n}] = bload(xr, vo, {X(j, Q - 1)});")
        for n, j in enumerate(S.d1_cols[p]):
            for q in range(Q):
                w(f"    xd[{n * Q + q}] = bload(xr, vo, {X(j, q)});")
        w("    for (int it = 0; it < a.T; ++it) {")
        w("        const float* pp = it >= 1 ? a.outs.p[it - 1] : nullptr;  // previous iteration's posterior")
        w(f"        const rsrc_t pr = make_rsrc(pp ? pp + blk * {NZ} : a.xa, pp ? nlive * {4 * NZ} : 0);  // no output: stores dropped")
        if "vn" not in SKIP:
            w(f"        vn_p{p}<KIND>({state_args()}, {x_args()}, a, vo, it, pr);")
        w("        const float* pn = a.outs.p[it];  // this iteration's posterior (degree-1 columns)")
        w(f"        const rsrc_t nr = make_rsrc(pn ? pn + blk * {NZ} : a.xa, pn ? nlive * {4 * NZ} : 0);")
        w("        const bool co_last = a.c2v_out && it == a.T - 1;")
        for ci in range(len(S.chunks)):
            w(f"        wr_p{p}_c{ci}<KIND>({state_args()}, {x_args()}, lds, u, a, it);")
            w("        __syncthreads();")
            if "cn" not in SKIP:
                for dc, t0, n in S.cn_groups[(p, ci)]:
                    w(f"        cn_rows<KIND, {dc}>(lds, u, a, it, {t0}, {n}, {S.chunks[ci][2]});")
            w("        __syncthreads();")
            w(f"        rd_p{p}_c{ci}<KIND>({state_args()}, {x_args()}, lds, u, a, vo, nr, cr, vc, co_last);")
            w("        __syncthreads();")
        w("    }")
        w("    const float* pl = a.outs.p[a.T - 1];")
        w(f"    const rsrc_t lr = make_rsrc(pl ? pl + blk * {NZ} : a.xa, pl ? nlive * {4 * NZ} : 0);")
        w(f"    post_p{p}<KIND>({state_args()}, {x_args()}, a, vo, a.T, lr);")
        w("    if (a.c2v_out) {")
        for q in range(Q):
            for k, e in enumerate(S.slots[p]):
                w(f"        bstore(cr, vc, {4 * (e * Z + q * ZT)}, {ref(q, k)});")
        w("    }")
        w("}")
    w("template <int KIND>")
    w(f"__global__ __launch_bounds__({S.threads}, {(S.threads + 255) // 256}) void kernel(FusedArgs a) {{")
    w(f"    __shared__ float lds_all[{CF * G}];")
    w("    const int t = threadIdx.x;")
    w(f"    // every wave lies in one part ({S.lanes} threads per part): the part is wave-uniform")
    w(f"    const int p = __builtin_amdgcn_readfirstlane(t / {S.lanes});")
    w(f"    const int r = t - p * {S.lanes};")
    w(f"    const int g = r / {ZT};")
    w(f"    const int u = r - g * {ZT};")
    w(f"    const int64_t blk = (int64_t)blockIdx.x * {G};  // first codeword of the workgroup")
    w(f"    const int nlive = a.B - blk < {G} ? (int)(a.B - blk) : {G};")
    w("    // lane byte offsets into the block's codewords; a lane past the last codeword gets an offset")
    w("    // beyond every descriptor's range (its loads read 0, its stores are dropped)")
    w(f"    const uint32_t vo = g < nlive ? 4u * (g * {NZ} + u) : 0x80000000u;  // [N][Z] layouts")
    w(f"    const uint32_t vc = g < nlive ? 4u * (g * {S.E * Z} + u) : 0x80000000u;  // [E][Z] c2v state")
    w(f"    const rsrc_t xr = make_rsrc(a.xa + blk * {NZ}, nlive * {4 * NZ});")
    w(f"    const rsrc_t cr = make_rsrc(a.c2v_out ? a.c2v_out + blk * {S.E * Z} : a.xa, nlive * {4 * S.E * Z});")
    w(f"    float* lds = lds_all + g * {CF};")
    each_part("run_p{p}<KIND>(a, lds, u, blk, nlive, xr, vo, cr, vc)", indent="    ")
    w("}")
    w(f"static const int32_t basegraph[{S.M * S.N}] = {{{', '.join(str(int(x)) for x in S.hb.reshape(-1))}}};")
    w("}  // namespace")
    return "\n".join(L)


def main():
    out, res = sys.argv[1], sys.argv[2]
    specs = []
    only = set(filter(None, os.environ.get("NLDPC_GEN_ONLY", "").split(",")))  # debug: subset of specs
    for tag, fname, Z, G, P, Q in SPECS:
        if only and tag not in only:
            continue
        hb = np.loadtxt(os.path.join(res, fname), int, delimiter="\t")
        specs.append(Spec(tag, hb, Z, G, P, Q))
    src = [
        "// GENERATED by gen_fused.py from the base graphs in resources/ -- do not edit.",
        "#include <hip/hip_runtime.h>",
        '#include "nldpc_fused.h"',
        "namespace nldpc {",
    ]
    for s in specs:
        src.append(emit(s))
    src.append("template <int KIND> static void* pick(int i) {")
    kinds = os.environ.get("NLDPC_GEN_KINDS")  # debug: instantiate a subset of kinds
    if kinds:
        src.append(f"    if constexpr ({' && '.join(f'KIND != {k}' for k in kinds.split(','))}) return nullptr; else {{")
    for i, s in enumerate(specs):
        src.append(f"    if (i == {i}) return reinterpret_cast<void*>(&fused_{s.tag}::kernel<KIND>);")
    src.append("    return nullptr;")
    if kinds:
        src.append("    }")
    src.append("}")
    src.append("const FusedSpec* fused_specs(int* n) {")
    src.append(f"    static const FusedSpec tab[{len(specs)}] = {{")
    for i, s in enumerate(specs):
        src.append(f"        {{\"{s.tag}\", {s.M}, {s.N}, {s.Z}, {s.E}, {s.G}, {s.threads}, "
                   f"fused_{s.tag}::basegraph, {{pick<NLDPC_SP>({i}), pick<NLDPC_MS>({i}), pick<NLDPC_QMS>({i}), "
                   f"pick<NLDPC_NEURAL>({i})}}}},")
    src.append("    };")
    src.append(f"    *n = {len(specs)};")
    src.append("    return tab;")
    src.append("}")
    src.append("}  // namespace nldpc")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        f.write("\n".join(src) + "\n")


if __name__ == "__main__":
    main()
