// Graph construction and library-level C ABI.
//
// Replaces ConnectingMatrix / ConnectingMatrixTorch of the reference
// (src/boosted_neural_ldpc_decoder/ConnectingMatrix.py:5-163, ConnectingMatrixTorch.py:7-54).
// The reference materialises dense 0/1 routing matrices (E x E) and two (E*Z)^2 lifting
// matrices (22.9 GB each at BG2 z=384).  Here the same graph is an edge list: every base-graph
// entry Hb[i][j] != -1 is one edge, numbered in C-order (row-major), with cyclic shift
// s = Hb[i][j] mod Z.  Row (i, h) of the lifted H has its 1 at column (j, (h + s) mod Z)
// (lifting_matrix_1/2, ConnectingMatrix.py:84-99).  Columns list their edges in ascending check
// row, which is the accumulation order the reference's sgemm produces.
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <vector>

#include "nldpc_fused.h"
#include "nldpc_internal.h"

namespace nldpc {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ") at " + what;
    return NLDPC_EHIP;
}

// ---- torch.tanh table (gen_tanh_table.py): loaded once per device from next to libnldpc.so (or
// $NLDPC_TANH_TABLE), kept for the life of the process
static std::string tanh_table_path() {
    if (const char* p = std::getenv("NLDPC_TANH_TABLE")) return p;
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&tanh_ref_table), &info) && info.dli_fname) {
        std::string so = info.dli_fname;
        const size_t k = so.rfind('/');
        return (k == std::string::npos ? std::string(".") : so.substr(0, k)) + "/nldpc_tanh_ref.bin";
    }
    return "nldpc_tanh_ref.bin";
}

TanhRef tanh_ref_table(int device) {
    static std::mutex mu;
    static std::vector<std::pair<int, TanhRef>> loaded;
    std::lock_guard<std::mutex> lock(mu);
    for (auto& p : loaded)
        if (p.first == device) return p.second;
    TanhRef t{};
    std::vector<uint32_t> buf;
    if (FILE* f = std::fopen(tanh_table_path().c_str(), "rb")) {
        uint32_t h[6];
        uint32_t prov[16];  // version 2: 64 bytes of build-host provenance (gen_tanh_table.py), not used here
        if (std::fread(h, 4, 6, f) == 6 && h[0] == 0x4841544Eu && (h[1] == 1u || (h[1] == 2u && std::fread(prov, 4, 16, f) == 16))) {
            const size_t nidx = (h[3] >> h[2]) + 2, n = nidx + h[4] + 2 * (size_t)h[5];
            buf.resize(n);
            if (std::fread(buf.data(), 4, n, f) == n) {
                void* d = nullptr;
                DeviceGuard guard(device);
                if (hipMalloc(&d, n * 4) == hipSuccess && hipMemcpy(d, buf.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess) {
                    const uint32_t* b = static_cast<const uint32_t*>(d);
                    t = TanhRef{b, b + nidx, b + nidx + h[4], (int32_t)h[5], (int32_t)h[2], h[3]};
                }
            }
        }
        std::fclose(f);
    }
    loaded.emplace_back(device, t);
    return t;
}

// Product order of the SP check node.  The reference multiplies each check row's factors inside
// torch.prod(x2_abs, dim=3) over the [B, Z, E, E] tile (BoostedNeuralLDPCDecoder.py:404): the last
// axis runs over all E edges in V-order (column-major) with 1.0 everywhere outside the row.  ATen's
// CPU reduction (the order oracle/ldpc_oracle.py _prod_aten restates and pins) keeps 4 accumulators
// of 8 lanes over the first E/32*32 positions -- position p goes to accumulator (p/8)%4, lane p%8, in
// ascending p --, combines each lane as (a0*a1)*(a2*a3), the lanes left to right, then multiplies the
// remaining positions one by one.  Factors of exactly 1.0 change nothing, so only the row's own edges
// matter: per row, its edges sorted by (lane, accumulator, position), tail positions last.
// The lane width (8) is what ATen's reduction used on the machine the SP fixtures were made on (this
// container: torch 2.10.0+rocm7.0, CPU capability AVX512, measured by
// tests/test_oracle_golden.py::test_prod_order_model_matches_torch_prod); the order is a property of
// that ATen build, and a host whose ATen vectorises the product differently needs another plan (the
// device SP then stays within the SP tolerance of that host's torch, but not value for value).
static void sp_plans(int M, int E, const std::vector<int32_t>& chk, const std::vector<int32_t>& var,
                     const std::vector<int32_t>& row_ptr, std::vector<uint8_t>& plan) {
    std::vector<int32_t> vorder(E), vidx(E);
    std::iota(vorder.begin(), vorder.end(), 0);
    std::stable_sort(vorder.begin(), vorder.end(), [&](int a, int b) {
        return var[a] != var[b] ? var[a] < var[b] : chk[a] < chk[b];
    });
    for (int p = 0; p < E; ++p) vidx[vorder[p]] = p;
    const int full = E / 32 * 32;
    plan.assign((size_t)M * kSpPlanBytes, 0);
    for (int i = 0; i < M; ++i) {
        const int beg = row_ptr[i], d = row_ptr[i + 1] - beg;
        if (d > 32) continue;  // SP needs check degree <= 32 (validated at decode time)
        std::vector<int> ord(d);
        std::iota(ord.begin(), ord.end(), 0);
        auto key = [&](int k) {
            const int p = vidx[beg + k];
            return p < full ? (int64_t)((p % 8) * 4 + (p / 8) % 4) * E + p : (int64_t)32 * E + p;
        };
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return key(a) < key(b); });
        uint8_t* pl = plan.data() + (size_t)i * kSpPlanBytes;
        int prev_lane = -1;
        for (int s = 0; s < d; ++s) {
            const int k = ord[s], p = vidx[beg + k];
            pl[s] = (uint8_t)k;
            pl[32 + k] = (uint8_t)s;
            uint8_t code;
            if (p < full) {
                const int lane = p % 8;
                code = (uint8_t)(((p / 8) % 4) | (lane != prev_lane ? 4 : 0));
                prev_lane = lane;
            } else {
                code = 8;
            }
            pl[64 + s] = code;
        }
    }
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_abi_version(void) { return NLDPC_ABI_VERSION; }

extern "C" const char* nldpc_last_error(void) { return g_last_error.c_str(); }

extern "C" int nldpc_graph_create(int32_t M, int32_t N, int32_t Z, const int32_t* basegraph, int32_t device,
                                  nldpc_graph** out) {
    try {
        if (!out || !basegraph) return fail(NLDPC_EINVAL, "nldpc_graph_create: null pointer");
        *out = nullptr;
        if (M <= 0 || N <= 0 || Z <= 0) return fail(NLDPC_EINVAL, "nldpc_graph_create: M, N, Z must be positive");
        // C-order edges
        std::vector<int32_t> chk, var, shift;
        std::vector<int32_t> row_ptr(M + 1, 0), col_cnt(N, 0);
        for (int i = 0; i < M; ++i) {
            row_ptr[i] = (int32_t)chk.size();
            for (int j = 0; j < N; ++j) {
                int32_t v = basegraph[(int64_t)i * N + j];
                if (v == -1) continue;
                if (v < -1) return fail(NLDPC_EINVAL, "nldpc_graph_create: base graph entries must be >= -1");
                chk.push_back(i);
                var.push_back(j);
                shift.push_back(v % Z);
                col_cnt[j]++;
            }
        }
        row_ptr[M] = (int32_t)chk.size();
        const int32_t E = (int32_t)chk.size();
        if (E == 0) return fail(NLDPC_EINVAL, "nldpc_graph_create: base graph has no edges");
        std::vector<int32_t> col_ptr(N + 1, 0), col_edge(E), fill(N, 0);
        for (int j = 0; j < N; ++j) col_ptr[j + 1] = col_ptr[j] + col_cnt[j];
        for (int e = 0; e < E; ++e) {  // ascending e == ascending check row within a column
            int j = var[e];
            col_edge[col_ptr[j] + fill[j]++] = e;
        }
        int32_t max_dc = 0, max_dv = 0;
        for (int i = 0; i < M; ++i) max_dc = std::max(max_dc, row_ptr[i + 1] - row_ptr[i]);
        for (int j = 0; j < N; ++j) max_dv = std::max(max_dv, col_cnt[j]);
        if (deg_bucket(max_dc) < 0 || deg_bucket(max_dv) < 0)
            return fail(NLDPC_EUNSUPPORTED, "nldpc_graph_create: node degree above 64 is not supported");
        if ((int64_t)Z * 64 > (int64_t)1 << 30)
            return fail(NLDPC_EUNSUPPORTED, "nldpc_graph_create: lifting size too large");

        std::vector<uint8_t> plan;
        sp_plans(M, E, chk, var, row_ptr, plan);

        // one device blob: chk | var | shift | row_ptr | col_ptr | col_edge | sp_plan (bytes)
        std::vector<int32_t> blob;
        blob.reserve(3 * E + (M + 1) + (N + 1) + E + plan.size() / 4);
        size_t off_chk = blob.size();
        blob.insert(blob.end(), chk.begin(), chk.end());
        size_t off_var = blob.size();
        blob.insert(blob.end(), var.begin(), var.end());
        size_t off_shift = blob.size();
        blob.insert(blob.end(), shift.begin(), shift.end());
        size_t off_row = blob.size();
        blob.insert(blob.end(), row_ptr.begin(), row_ptr.end());
        size_t off_col = blob.size();
        blob.insert(blob.end(), col_ptr.begin(), col_ptr.end());
        size_t off_cole = blob.size();
        blob.insert(blob.end(), col_edge.begin(), col_edge.end());
        size_t off_plan = blob.size();
        blob.resize(blob.size() + plan.size() / 4);
        std::memcpy(blob.data() + off_plan, plan.data(), plan.size());

        DeviceGuard guard(device);
        void* d_blob = nullptr;
        NLDPC_HIP_CHECK(hipMalloc(&d_blob, blob.size() * sizeof(int32_t)));
        hipError_t e = hipMemcpy(d_blob, blob.data(), blob.size() * sizeof(int32_t), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d_blob);
            return hip_fail(e, "hipMemcpy(graph tables)");
        }
        nldpc_graph* g = new nldpc_graph();
        g->device = device;
        g->fused = -1;
        {  // a generated fused kernel for exactly this lifted graph? (same M, N, Z and edge shifts)
            int nspec = 0;
            const FusedSpec* specs = fused_specs(&nspec);
            for (int k = 0; k < nspec && g->fused < 0; ++k) {
                const FusedSpec& f = specs[k];
                if (f.M != M || f.N != N || f.Z != Z) continue;
                bool same = true;
                for (int64_t q = 0; q < (int64_t)M * N && same; ++q) {
                    const int32_t a = basegraph[q], b = f.basegraph[q];
                    same = (a == -1) == (b == -1) && (a == -1 || (a % Z) == (b % Z));
                }
                if (same) g->fused = k;
            }
        }
        g->blob = d_blob;
        const int32_t* base = static_cast<const int32_t*>(d_blob);
        g->dev = DevGraph{M, N, Z, E, max_dc, max_dv, base + off_chk, base + off_var, base + off_shift,
                          base + off_row, base + off_col, base + off_cole,
                          reinterpret_cast<const uint8_t*>(base + off_plan), tanh_ref_table(device)};
        g->h_chk = new int32_t[E];
        g->h_var = new int32_t[E];
        g->h_shift = new int32_t[E];
        std::memcpy(g->h_chk, chk.data(), E * sizeof(int32_t));
        std::memcpy(g->h_var, var.data(), E * sizeof(int32_t));
        std::memcpy(g->h_shift, shift.data(), E * sizeof(int32_t));
        *out = g;
        return NLDPC_OK;
    } catch (const std::bad_alloc&) {
        return fail(NLDPC_EINVAL, "nldpc_graph_create: host allocation failed");
    } catch (...) {
        return fail(NLDPC_EINVAL, "nldpc_graph_create: unexpected exception");
    }
}

namespace nldpc {
FusedLaunch fused_launch(const nldpc_graph* g, int mode, int kind) {
    FusedLaunch L;
    if (!g || mode < 0 || mode > 7 || kind < 0 || kind > 3) return L;
    if (g->fused >= 0) {
        int n = 0;
        const FusedSpec& f = fused_specs(&n)[g->fused];
        // a generated unit built against another argument layout than this launcher (an experiment build
        // mixing objects) would return at once and leave its outputs unwritten: no kernel, the caller reports
        // NLDPC_EUNSUPPORTED for path "fused" or decodes on the streaming kernels
        // (the tied saving forward lives in the saving unit, the specialised UCN decode in the decode unit)
        const int unit = mode == 6 ? 1 : mode == 7 ? 0 : mode;
        if (f.sig[unit] != (mode == 4 || mode == 5 ? kFusedBwdArgsSig : kFusedArgsSig)) return L;
        L.host = mode == 7 ? f.decode_ucnw[kind] : mode == 6 ? f.save_tied[kind] : mode == 5 ? f.bwd_tied[kind]
               : mode == 4 ? f.bwd[kind] : f.kernels[mode][kind];
        L.G = f.G;
        L.threads = f.threads;
        L.waves_per_part = f.waves_per_part;
    } else if (mode < 5 && g->jit_fn[mode][kind]) {  // (MODES 5 to 7: library kernels only)
        L.fn = g->jit_fn[mode][kind];
        L.G = g->jit_G;
        L.threads = g->jit_threads;
        L.waves_per_part = g->jit_wpp;
    }
    return L;
}
}  // namespace nldpc

namespace {
// The initial value of the code object's global `nldpc_sig` (gen_fused.py jit_source), read from the host copy
// of the code object: a clang offload bundle (hipcc --genco) holding the gfx950 ELF, or the ELF itself.  No device
// copy, so the check neither waits for work in flight nor touches a stream that may be capturing.
bool code_object_sig(const void* code, size_t bytes, uint32_t* sig) {
    const auto* b = static_cast<const unsigned char*>(code);
    auto rd64 = [&](size_t off, uint64_t* v) {
        if (off > bytes || bytes - off < 8) return false;
        std::memcpy(v, b + off, 8);
        return true;
    };
    static const char kBundle[] = "__CLANG_OFFLOAD_BUNDLE__";
    const unsigned char* elf = b;
    size_t elf_bytes = bytes;
    if (bytes >= 24 && std::memcmp(b, kBundle, 24) == 0) {
        uint64_t n = 0, pos = 24;
        if (!rd64(pos, &n)) return false;
        pos += 8;
        elf = nullptr;
        for (uint64_t i = 0; i < n && i < 64; ++i) {
            uint64_t off, sz, tl;
            if (!rd64(pos, &off) || !rd64(pos + 8, &sz) || !rd64(pos + 16, &tl)) return false;
            pos += 24;
            if (pos > bytes || tl > bytes - pos) return false;
            const std::string triple(reinterpret_cast<const char*>(b + pos), tl);
            pos += tl;
            if (triple.find("amdgcn") != std::string::npos && off <= bytes && sz <= bytes - off && sz >= 64) {
                elf = b + off;
                elf_bytes = sz;
                break;
            }
        }
        if (!elf) return false;
    }
    // ELF64 little endian: the symbol table, the symbol, the initialised bytes of its section
    if (elf_bytes < 64 || std::memcmp(elf, "\x7f" "ELF", 4) != 0 || elf[4] != 2 || elf[5] != 1) return false;
    auto u16 = [&](size_t o) { uint16_t v; std::memcpy(&v, elf + o, 2); return (size_t)v; };
    auto u32 = [&](size_t o) { uint32_t v; std::memcpy(&v, elf + o, 4); return (size_t)v; };
    auto u64 = [&](size_t o) { uint64_t v; std::memcpy(&v, elf + o, 8); return (size_t)v; };
    const size_t shoff = u64(0x28), shentsize = u16(0x3a), shnum = u16(0x3c);
    if (shentsize < 64 || shoff > elf_bytes || shnum > (elf_bytes - shoff) / shentsize) return false;
    auto sh = [&](size_t i, size_t field) { return shoff + i * shentsize + field; };
    for (size_t s = 0; s < shnum; ++s) {
        if (u32(sh(s, 4)) != 2 /* SHT_SYMTAB */ && u32(sh(s, 4)) != 11 /* SHT_DYNSYM */) continue;
        const size_t off = u64(sh(s, 0x18)), size = u64(sh(s, 0x20)), link = u32(sh(s, 0x28)),
                     ent = u64(sh(s, 0x38));
        if (ent < 24 || link >= shnum || off > elf_bytes || size > elf_bytes - off) return false;
        const size_t stroff = u64(sh(link, 0x18)), strsize = u64(sh(link, 0x20));
        if (stroff > elf_bytes || strsize > elf_bytes - stroff) return false;
        for (size_t k = 0; k < size / ent; ++k) {
            const size_t sym = off + k * ent, name = u32(sym);
            if (name >= strsize) continue;
            const char* nm = reinterpret_cast<const char*>(elf + stroff + name);
            if (strnlen(nm, strsize - name) != 9 || std::memcmp(nm, "nldpc_sig", 9) != 0) continue;
            const size_t shndx = u16(sym + 6), value = u64(sym + 8), symsize = u64(sym + 16);
            if (symsize != 4 || shndx == 0 || shndx >= shnum) return false;
            if (u32(sh(shndx, 4)) == 8 /* SHT_NOBITS */) {
                *sig = 0;
                return true;
            }
            const size_t saddr = u64(sh(shndx, 0x10)), soff = u64(sh(shndx, 0x18)), ssize = u64(sh(shndx, 0x20));
            if (value < saddr || value - saddr > ssize || ssize - (value - saddr) < 4) return false;
            const size_t at = soff + (value - saddr);
            if (at > elf_bytes || elf_bytes - at < 4) return false;
            std::memcpy(sig, elf + at, 4);
            return true;
        }
    }
    return false;
}
}  // namespace

extern "C" int nldpc_code_object_sig(const void* code, size_t bytes, int32_t mode, uint32_t* sig, uint32_t* expected) {
    if (!code || !bytes || !sig || !expected || mode < 0 || mode > 4)
        return fail(NLDPC_EINVAL, "nldpc_code_object_sig: null argument or mode outside 0-4");
    *expected = mode == 4 ? kFusedBwdArgsSig : kFusedArgsSig;
    if (!code_object_sig(code, bytes, sig))
        return fail(NLDPC_EINVAL, "nldpc_code_object_sig: no readable nldpc_sig in the code object");
    return NLDPC_OK;
}

extern "C" int nldpc_graph_attach_kernel(nldpc_graph* g, int32_t mode, int32_t kind, const void* code, size_t bytes,
                                         int32_t G, int32_t threads, int32_t waves_per_part) {
    if (!g || !code || !bytes) return fail(NLDPC_EINVAL, "nldpc_graph_attach_kernel: null argument");
    if (mode < 0 || mode > 4 || kind < NLDPC_SP || kind > NLDPC_NEURAL)
        return fail(NLDPC_EINVAL, "nldpc_graph_attach_kernel: mode is 0-4 and kind an nldpc kind");
    if (G <= 0 || threads <= 0 || threads > 1024 || threads % 64 || waves_per_part <= 0)
        return fail(NLDPC_EINVAL, "nldpc_graph_attach_kernel: bad geometry");
    if (g->fused >= 0) return NLDPC_OK;  // the library's own kernels serve this graph
    bool first = true;
    for (int m = 0; m < 5; ++m)
        for (int k = 0; k < 4; ++k) first = first && !g->jit_fn[m][k];
    if (!first && (G != g->jit_G || threads != g->jit_threads || waves_per_part != g->jit_wpp))
        return fail(NLDPC_EINVAL, "nldpc_graph_attach_kernel: geometry differs from the graph's attached kernels");
    if (g->jit_fn[mode][kind]) return NLDPC_OK;
    {  // the code object's argument layout (gen_fused.py jit_source: nldpc_sig) must be this library's
        uint32_t sig = 0;
        if (!code_object_sig(code, bytes, &sig) || sig != (mode == 4 ? kFusedBwdArgsSig : kFusedArgsSig))
            return fail(NLDPC_EUNSUPPORTED, "nldpc_graph_attach_kernel: the code object was built for another "
                                            "kernel argument layout (regenerate it with this library's gen_fused.py)");
    }
    DeviceGuard guard(g->device);
    hipModule_t mod = nullptr;
    NLDPC_HIP_CHECK(hipModuleLoadData(&mod, code));
    hipFunction_t fn = nullptr;
    hipError_t e = hipModuleGetFunction(&fn, mod, mode == 4 ? "nldpc_fxb" : "nldpc_fx");
    if (e != hipSuccess) {
        (void)hipModuleUnload(mod);
        return hip_fail(e, "hipModuleGetFunction(nldpc_fx)");
    }
    g->jit_mod[mode][kind] = mod;
    g->jit_fn[mode][kind] = fn;
    g->jit_G = G;
    g->jit_threads = threads;
    g->jit_wpp = waves_per_part;
    return NLDPC_OK;
}

extern "C" int nldpc_graph_kernels(const nldpc_graph* g, uint32_t* mask) {
    if (!g || !mask) return fail(NLDPC_EINVAL, "nldpc_graph_kernels: null pointer");
    uint32_t m = 0;
    for (int mode = 0; mode < 5; ++mode)
        for (int k = 0; k < 4; ++k)
            if (fused_launch(g, mode, k)) m |= 1u << (mode * 4 + k);
    *mask = m;
    return NLDPC_OK;
}

extern "C" int nldpc_graph_destroy(nldpc_graph* g) {
    if (!g) return NLDPC_OK;
    {
        DeviceGuard guard(g->device);
        if (g->blob) (void)hipFree(g->blob);
        for (auto& row : g->jit_mod)
            for (hipModule_t m : row)
                if (m) (void)hipModuleUnload(m);
    }
    delete[] g->h_chk;
    delete[] g->h_var;
    delete[] g->h_shift;
    delete g;
    return NLDPC_OK;
}

extern "C" int nldpc_graph_dims(const nldpc_graph* g, int32_t* dims) {
    if (!g || !dims) return fail(NLDPC_EINVAL, "nldpc_graph_dims: null pointer");
    dims[0] = g->dev.M;
    dims[1] = g->dev.N;
    dims[2] = g->dev.Z;
    dims[3] = g->dev.E;
    dims[4] = g->dev.max_dc;
    dims[5] = g->dev.max_dv;
    dims[6] = g->device;
    dims[7] = 0;
    return NLDPC_OK;
}

extern "C" int nldpc_graph_edges(const nldpc_graph* g, int32_t* chk, int32_t* var, int32_t* shift) {
    if (!g) return fail(NLDPC_EINVAL, "nldpc_graph_edges: null graph");
    const size_t n = (size_t)g->dev.E * sizeof(int32_t);
    if (chk) std::memcpy(chk, g->h_chk, n);
    if (var) std::memcpy(var, g->h_var, n);
    if (shift) std::memcpy(shift, g->h_shift, n);
    return NLDPC_OK;
}
