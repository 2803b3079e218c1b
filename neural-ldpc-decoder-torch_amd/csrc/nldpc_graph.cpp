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
#include <cstdlib>
#include <cstring>
#include <new>
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

        // one device blob: chk | var | shift | row_ptr | col_ptr | col_edge
        std::vector<int32_t> blob;
        blob.reserve(3 * E + (M + 1) + (N + 1) + E);
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
                          base + off_row, base + off_col, base + off_cole};
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

extern "C" int nldpc_graph_destroy(nldpc_graph* g) {
    if (!g) return NLDPC_OK;
    {
        DeviceGuard guard(g->device);
        if (g->blob) (void)hipFree(g->blob);
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
