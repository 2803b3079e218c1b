// Internal declarations shared by the translation units of libnldpc.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "nldpc.h"

namespace nldpc {

// Device edge tables of one lifted QC graph.  All arrays live in a single device allocation.
//   e_chk/e_var/e_shift [E]  C-order edges (row-major over the base graph; ConnectingMatrix.py:92-99)
//   row_ptr [M+1]            edges of check row i are the contiguous C-order range row_ptr[i]..
//   col_ptr [N+1], col_edge  edges of column j in ascending check row (== ascending C-order index)
//   sp_plan [M][96]          the sum-product check node's product order per row (nldpc_node.h
//                            sp_prod_others): ord[32] | inv[32] | code[32]
struct TanhRef {  // torch.tanh's exact fp32 results (gen_tanh_table.py); idx == nullptr: not built
    const uint32_t* idx;
    const uint32_t* ent;
    const uint32_t* ovr;
    int32_t novr, sh;
    uint32_t kmax;
};
constexpr int kSpPlanBytes = 96;
struct DevGraph {
    int32_t M, N, Z, E, max_dc, max_dv;
    const int32_t* e_chk;
    const int32_t* e_var;
    const int32_t* e_shift;
    const int32_t* row_ptr;
    const int32_t* col_ptr;
    const int32_t* col_edge;
    const uint8_t* sp_plan;
    TanhRef tanh;
};
// the process-wide device copy of lib/nldpc_tanh_ref.bin for `device` (loaded once; idx == nullptr
// when the file is missing: the SP check node then uses the rounded double tanh, within one ulp)
TanhRef tanh_ref_table(int device);

}  // namespace nldpc

struct nldpc_graph {
    nldpc::DevGraph dev;
    int32_t device;
    int32_t fused;  // index into nldpc::fused_specs() of a compiled register-resident kernel, or -1
    // register-resident kernels compiled at run time for this graph and attached by
    // nldpc_graph_attach_kernel: [MODE 0-3 | 4 = backward][kind], one code object each
    hipModule_t jit_mod[5][4];
    hipFunction_t jit_fn[5][4];
    int32_t jit_G, jit_threads, jit_wpp;  // their geometry (one per graph)
    void* blob;  // device allocation backing the tables
    // host mirrors
    int32_t* h_chk;
    int32_t* h_var;
    int32_t* h_shift;
};

namespace nldpc {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// RAII guard: make the graph's device current for the duration of a call, restore afterwards.
struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
            changed = hipSetDevice(dev) == hipSuccess;
        }
    }
    ~DeviceGuard() {
        if (changed) (void)hipSetDevice(prev);
    }
};

// Layout of the `saved` buffer nldpc_forward fills for nldpc_backward:
//   v2c   [T][B][E][Z] fp32 variable-to-check messages of every iteration
//   ymask [T][B][N][Z] uint8 clamp mask of every posterior (Boosted decoders only)
//   xin   [T][B][N][Z] fp32 channel value xin_k each iteration used (cumulative VN weighting only),
//         so neither direction re-runs the Q(x*w) chain from xa (O(T^2) over an unrolled forward)
//   (QMS with an active quantiser saves v2c as int8 codes instead, nldpc_math.h qms_code)
struct SavedLayout {
    size_t v2c_off, ymask_off, xin_off, total;
    int64_t v2c_stride, ymask_stride, xin_stride;  // elements per iteration
    bool has_ymask, has_xin, v2c_code;
};
inline bool qms_active(int q) { return q == 6 || q == 5 || q == -5 || q == 4 || q == 3; }
SavedLayout saved_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T);
int validate_cfg(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T);

// benchmark instrumentation (nldpc_profile.cpp)
enum ProfKind { PROF_VN = 0, PROF_CN = 1, PROF_POST = 2, PROF_FUSED = 3, PROF_VNB = 4, PROF_CNB = 5, PROF_FUSED_BWD = 6 };
bool prof_armed();
void prof_start(int kind, hipStream_t s);
void prof_stop(hipStream_t s);

// Pick the smallest compiled register-array bound that covers a degree.
inline int deg_bucket(int d) {
    if (d <= 8) return 8;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    if (d <= 64) return 64;
    return -1;
}

}  // namespace nldpc

#define NLDPC_HIP_CHECK(expr)                                       \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return ::nldpc::hip_fail(_e, #expr);  \
    } while (0)
