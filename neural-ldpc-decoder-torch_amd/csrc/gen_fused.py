"""Generate the register-resident fused decoder kernels (nldpc_fused_gen.hip) for known base graphs.

Design (DESIGN.md §Fused kernel): one workgroup decodes G codewords for all T iterations without
touching HBM for message state.  The c2v messages of a codeword (E*Z floats, 302 KB for BG2 z=384)
live in the REGISTERS of the threads that own their variable copies: thread (part p, codeword g,
copy v) owns every edge of the columns of part p at copy v, so the variable-node update (sum of the
others, sequential fp32 in ascending check row: the reference's sgemm order) is register-only code.
The check-node update needs each row's messages at cyclically shifted copies, so per iteration the
v2c messages go through LDS in row chunks: owners write a chunk, every thread runs the check
nodes of its rows of that chunk in LDS (gather at (h + s) mod Z, update, scatter back to the same
addresses), owners read the new c2v back.  HBM traffic per codeword: the channel LLRs (re-read
from L2 every iteration) and the T posteriors the API returns.

Everything that indexes registers is emitted as straight-line code with literal indices, so the
generator needs the graph structure at build time; the per-edge arithmetic is the shared
nldpc_node.h code (cn_core / cn_epilogue / vn_channel), identical to the streaming kernels.

Usage: python3 gen_fused.py OUT.hip RESOURCE_DIR
"""
import os
import sys

import numpy as np

SKIP = set(filter(None, os.environ.get("NLDPC_GEN_SKIP", "").split(",")))  # debug: drop phases
LDS_BYTES = 160 * 1024 - 2048  # leave room for the compiler / alignment

# (tag, base graph file, Z, codewords per workgroup G, parts P)
SPECS = [
    ("bg2_z384", "basegraph2_set0.txt", 384, 1, 2),
    ("bg2_z16", "basegraph2_set0.txt", 16, 16, 2),
    ("wimax_z24", "wman_N0576_R34_z24.txt", 24, 16, 1),
]


class Spec:
    def __init__(self, tag, hb, Z, G, P):
        self.tag, self.hb, self.Z, self.G, self.P = tag, hb, Z, G, P
        self.M, self.N = hb.shape
        rows, cols = np.nonzero(hb != -1)
        self.E = len(rows)
        self.chk, self.var = rows, cols
        self.shift = hb[rows, cols] % Z
        self.row_edges = [list(np.nonzero(rows == i)[0]) for i in range(self.M)]
        self.col_edges = [list(np.nonzero(cols == j)[0]) for j in range(self.N)]
        dv = np.array([len(c) for c in self.col_edges])
        # columns -> parts, balancing edges (owner registers)
        load = [0] * P
        self.part_cols = [[] for _ in range(P)]
        for j in np.argsort(-dv, kind="stable"):
            k = int(np.argmin(load))
            self.part_cols[k].append(int(j))
            load[k] += int(dv[j])
        self.part_cols = [sorted(c) for c in self.part_cols]
        # Degree-1 columns keep no register state: their v2c is the channel value alone and their
        # c2v only enters their own posterior, which is written as soon as it is read back from LDS.
        self.reg_cols = [[j for j in c if len(self.col_edges[j]) > 1] for c in self.part_cols]
        self.d1_cols = [[j for j in c if len(self.col_edges[j]) == 1] for c in self.part_cols]
        self.slots = []  # per part: register slot -> edge (column by column, ascending check row)
        for p in range(P):
            s = []
            for j in self.reg_cols[p]:
                s += [int(e) for e in self.col_edges[j]]
            self.slots.append(s)
        self.smax = max(1, max(len(s) for s in self.slots))
        # row chunks: contiguous row ranges whose edges x Z x G fit in LDS
        cap = (LDS_BYTES // (4 * G) - 32) // Z
        self.chunks = []  # list of (row_begin, row_end, edge_begin, edge_end)
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
        # check rows of every chunk -> parts, balancing sum of degrees
        self.cn_rows = []
        for (r0, r1, _, _) in self.chunks:
            load = [0] * P
            rp = [[] for _ in range(P)]
            for i in sorted(range(r0, r1), key=lambda i: -len(self.row_edges[i])):
                k = int(np.argmin(load))
                rp[k].append(i)
                load[k] += len(self.row_edges[i])
            self.cn_rows.append([sorted(r) for r in rp])
        self.threads = P * G * Z
        assert self.threads <= 1024 and (G * Z) % 64 == 0, (tag, self.threads)
        self.max_dc = max(len(r) for r in self.row_edges)

    def chunk_of(self, e):
        for c, (_, _, e0, e1) in enumerate(self.chunks):
            if e0 <= e < e1:
                return c
        raise KeyError(e)


def emit(spec: Spec) -> str:
    S, Z, G = spec, spec.Z, spec.G
    L = []
    w = L.append
    CF = S.chunk_floats
    w(f"// ---- {S.tag}: M={S.M} N={S.N} E={S.E} Z={Z}, {G} codeword(s) x {S.P} part(s) x {Z} copies = "
      f"{S.threads} threads; slots/part {[len(s) for s in S.slots]}; "
      f"{len(S.chunks)} LDS chunk(s) of <= {CF * G * 4} B")
    w(f"namespace fused_{S.tag} {{")
    w(f"constexpr int Z = {Z}, G = {G}, N = {S.N}, E = {S.E}, SMAX = {S.smax}, CHF = {CF};")
    # VN (+ posterior of the previous iteration) per part, and the final posterior pass
    for p in range(S.P):
        cols = S.reg_cols[p]
        if not cols:
            for final in (False, True):
                w("template <int KIND>")
                w(f"__device__ __forceinline__ void {'post' if final else 'vn'}_p{p}(float (&)[SMAX], const FusedArgs&, "
                  f"const float*, int, int, float*, bool) {{}}")
            continue
        for final in (False, True):
            w("template <int KIND>")
            fname = f"post_p{p}" if final else f"vn_p{p}"
            w(f"__device__ __forceinline__ void {fname}(float (&c)[SMAX], const FusedArgs& a, const float* __restrict__ xb, "
              f"int lo, int it, float* __restrict__ post, bool live) {{")
            w("    asm volatile(\"\" : \"+v\"(lo));  // recompute per-column offsets every iteration (no hoisting)")
            s = 0
            # channel values are software-pipelined one column ahead; a scheduling barrier between
            # columns keeps the compiler from hoisting every load (and its register) to the top
            w(f"    float xnext = xb[lo + {cols[0] * Z}];")
            for n, j in enumerate(cols):
                d = len(S.col_edges[j])
                w(f"    {{  // column {j}, degree {d}")
                w("        const float xav = xnext;")
                if n + 1 < len(cols):
                    w(f"        xnext = xb[lo + {cols[n + 1] * Z}];")
                w("        float P = 0.f;")
                if not final:
                    w(f"        const float x0 = fadd(0.f, vn_channel<KIND>(xav, a.w_vn, N, {j}, a.vn_prefix + it + 1, a.qbit));")
                    for k in range(d):
                        expr = "P"
                        for m in range(k + 1, d):
                            expr = f"fadd({expr}, c[{s + m}])"
                        w(f"        {{ const float S_ = {expr}; P = fadd(P, c[{s + k}]); c[{s + k}] = fadd(x0, S_); }}")
                else:
                    for k in range(d):
                        w(f"        P = fadd(P, c[{s + k}]);")
                w(f"        if (post && live) post[lo + {j * Z}] = posterior<KIND>(xav, P, a);")
                w("    }")
                w("    __builtin_amdgcn_sched_barrier(0);")
                s += d
            w("}")
    # chunk writes / reads per part
    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            sl = [(k, e) for k, e in enumerate(S.slots[p]) if e0 <= e < e1]
            d1 = [(j, int(S.col_edges[j][0])) for j in S.d1_cols[p] if e0 <= S.col_edges[j][0] < e1]
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void wr_p{p}_c{ci}(const float (&c)[SMAX], float* lds, int v, const FusedArgs& a, "
              f"const float* __restrict__ xb, int lo, int it) {{")
            w("    asm volatile(\"\" : \"+v\"(v));")
            w("    asm volatile(\"\" : \"+v\"(lo));")
            for k, e in sl:
                w(f"    lds[{(e - e0) * Z} + v] = c[{k}];")
            for n, (j, e) in enumerate(d1):  # v2c = (0 + xin) + 0: no other edge in the column
                w(f"    lds[{(e - e0) * Z} + v] = fadd(fadd(0.f, vn_channel<KIND>(xb[lo + {j * Z}], a.w_vn, N, {j}, "
                  f"a.vn_prefix + it + 1, a.qbit)), 0.f);")
                if n % 4 == 3:
                    w("    __builtin_amdgcn_sched_barrier(0);")
            w("}")
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void rd_p{p}_c{ci}(float (&c)[SMAX], const float* lds, int v, const FusedArgs& a, "
              f"const float* __restrict__ xb, int lo, float* __restrict__ post, float* __restrict__ co, bool live) {{")
            w("    asm volatile(\"\" : \"+v\"(v));")
            w("    asm volatile(\"\" : \"+v\"(lo));")
            for k, e in sl:
                w(f"    c[{k}] = lds[{(e - e0) * Z} + v];")
            for n, (j, e) in enumerate(d1):  # posterior of this iteration right away (and the final state if asked)
                if n % 4 == 0:
                    w("    __builtin_amdgcn_sched_barrier(0);")
                w("    {")
                w(f"        const float c_ = lds[{(e - e0) * Z} + v];")
                w(f"        if (post && live) post[lo + {j * Z}] = posterior<KIND>(xb[lo + {j * Z}], fadd(0.f, c_), a);")
                w(f"        if (co && live) co[{e * Z}] = c_;")
                w("    }")
            w("}")
    # check nodes per part per chunk
    for p in range(S.P):
        for ci, (r0, r1, e0, e1) in enumerate(S.chunks):
            w("template <int KIND>")
            w(f"__device__ __forceinline__ void cn_p{p}_c{ci}(float* lds, int h, const FusedArgs& a, int it) {{")
            w("    asm volatile(\"\" : \"+v\"(h));")
            w("    const float* wc = a.w_cn ? a.w_cn + (int64_t)it * E : nullptr;")
            w("    const float* bs = a.bias ? a.bias + (int64_t)it * E : nullptr;")
            for i in S.cn_rows[ci][p]:
                es = S.row_edges[i]
                d = len(es)
                w(f"    {{  // check row {i}, degree {d}")
                w(f"        int ad[{d}];")
                w(f"        float m[{d}];")
                for k, e in enumerate(es):
                    sft = int(S.shift[e])
                    base = (e - e0) * Z
                    if sft == 0:
                        w(f"        ad[{k}] = {base} + h;")
                    else:
                        w(f"        {{ const int t_ = h + {sft}; ad[{k}] = {base} + (t_ >= Z ? t_ - Z : t_); }}")
                    w(f"        m[{k}] = lds[ad[{k}]];")
                w(f"        CnCore<{d}> core;")
                w(f"        cn_core<{d}, KIND>(m, {d}, a.qbit, a.lo, a.hi, core);")
                for k, e in enumerate(es):
                    w(f"        lds[ad[{k}]] = cn_epilogue<KIND, false>(core.out0[{k}], wc ? wc[{e}] : 1.f, 0.f, "
                      f"bs ? bs[{e}] : 0.f, 0.f, wc != nullptr, false, a.qbit, a.lo, a.hi).c;")
                w("    }")
                w("    __builtin_amdgcn_sched_barrier(0);")
            w("}")
    # the kernel
    w("template <int KIND>")
    w(f"__global__ __launch_bounds__({S.threads}, {(S.threads + 255) // 256}) void kernel(FusedArgs a) {{")
    w(f"    __shared__ float lds_all[{CF * G}];")
    w("    const int t = threadIdx.x;")
    w(f"    // every wave lies in one part ({G * Z} threads per part): make the part wave-uniform so the")
    w(f"    // per-part code is a scalar branch (a divergent one would keep two copies of the state alive)")
    w(f"    const int p = __builtin_amdgcn_readfirstlane(t / ({G * Z}));")
    w(f"    const int r = t - p * {G * Z};")
    w(f"    const int g = r / {Z};")
    w(f"    const int v = r - g * {Z};")
    w("    const int64_t blk = (int64_t)blockIdx.x * G;  // first codeword of the workgroup")
    w("    const bool live = blk + g < a.B;")
    w(f"    const int lo = (live ? g : (int)(a.B - 1 - blk)) * {S.N * Z} + v;  // lane offset in the block's codewords")
    w(f"    const float* __restrict__ xb = a.xa + blk * {S.N * Z};")
    w(f"    float* lds = lds_all + g * {CF};")
    w("    float c[SMAX];")
    w("#pragma unroll")
    w("    for (int k = 0; k < SMAX; ++k) c[k] = 0.f;")
    w("    for (int it = 0; it < a.T; ++it) {")
    w(f"        float* post = (it >= 1 && a.outs.p[it - 1]) ? a.outs.p[it - 1] + blk * {S.N * Z} : nullptr;")
    for p in range(S.P):
        if "vn" not in SKIP:
            w(f"        {'if' if p == 0 else 'else if'} (p == {p}) vn_p{p}<KIND>(c, a, xb, lo, it, post, live);")
    w(f"        float* post_now = a.outs.p[it] ? a.outs.p[it] + blk * {S.N * Z} : nullptr;  // degree-1 columns")
    w("        float* co_last = (a.c2v_out && it == a.T - 1) ? a.c2v_out + (blk + g) * (int64_t)(E * Z) + v : nullptr;")
    for ci in range(len(S.chunks)):
        for p in range(S.P):
            w(f"        {'if' if p == 0 else 'else if'} (p == {p}) wr_p{p}_c{ci}<KIND>(c, lds, v, a, xb, lo, it);")
        w("        __syncthreads();")
        for p in range(S.P):
            if "cn" not in SKIP:
                w(f"        {'if' if p == 0 else 'else if'} (p == {p}) cn_p{p}_c{ci}<KIND>(lds, v, a, it);")
        w("        __syncthreads();")
        for p in range(S.P):
            w(f"        {'if' if p == 0 else 'else if'} (p == {p}) rd_p{p}_c{ci}<KIND>(c, lds, v, a, xb, lo, post_now, co_last, live);")
        w("        __syncthreads();")
    w("    }")
    w(f"    float* post = a.outs.p[a.T - 1] ? a.outs.p[a.T - 1] + blk * {S.N * Z} : nullptr;")
    for p in range(S.P):
        w(f"    {'if' if p == 0 else 'else if'} (p == {p}) post_p{p}<KIND>(c, a, xb, lo, a.T, post, live);")
    w("    if (a.c2v_out && live) {")
    w("        float* co = a.c2v_out + (blk + g) * (int64_t)(E * Z) + v;")
    for p in range(S.P):
        w(f"        {'if' if p == 0 else 'else if'} (p == {p}) {{")
        for k, e in enumerate(S.slots[p]):
            w(f"            co[{e * Z}] = c[{k}];")
        w("        }")
    w("    }")
    w("}")
    w(f"static const int32_t basegraph[{S.M * S.N}] = {{{', '.join(str(int(x)) for x in S.hb.reshape(-1))}}};")
    w("}  // namespace")
    return "\n".join(L)


def main():
    out, res = sys.argv[1], sys.argv[2]
    specs = []
    for tag, fname, Z, G, P in SPECS:
        hb = np.loadtxt(os.path.join(res, fname), int, delimiter="\t")
        specs.append(Spec(tag, hb, Z, G, P))
    src = [
        "// GENERATED by gen_fused.py from the base graphs in resources/ -- do not edit.",
        "#include <hip/hip_runtime.h>",
        '#include "nldpc_fused.h"',
        "namespace nldpc {",
    ]
    for s in specs:
        src.append(emit(s))
    src.append("template <int KIND> static void* pick(int i) {")
    for i, s in enumerate(specs):
        src.append(f"    if (i == {i}) return reinterpret_cast<void*>(&fused_{s.tag}::kernel<KIND>);")
    src.append("    return nullptr;")
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
