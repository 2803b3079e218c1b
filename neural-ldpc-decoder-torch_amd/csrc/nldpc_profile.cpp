// Optional per-kernel timing of the decode loop with HIP events (benchmark instrumentation).
//
// nldpc_profile_begin(capacity) arms the recorder; while armed, nldpc_forward brackets every kernel
// launch with a pair of events on the launch stream (no host synchronisation inside the loop).
// nldpc_profile_end() waits for the recorded events and returns, per kernel kind, the summed
// duration and the launch count.  Used by bench.py to measure the dominant kernel's launch time
// live, on the stream the kernels run on.
#include <vector>

#include "nldpc_internal.h"

namespace nldpc {

struct ProfRec {
    int kind;
    hipEvent_t a, b;
};

static struct {
    bool armed = false;
    size_t capacity = 0;
    std::vector<ProfRec> recs;  // recs[0..used) valid
    size_t used = 0;
    std::vector<hipEvent_t> pool;
} g_prof;

bool prof_armed() { return g_prof.armed; }

void prof_start(int kind, hipStream_t s) {
    if (!g_prof.armed || g_prof.used >= g_prof.capacity) return;
    ProfRec& r = g_prof.recs[g_prof.used];
    r.kind = kind;
    (void)hipEventRecord(r.a, s);
}

void prof_stop(hipStream_t s) {
    if (!g_prof.armed || g_prof.used >= g_prof.capacity) return;
    (void)hipEventRecord(g_prof.recs[g_prof.used].b, s);
    g_prof.used++;
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_profile_begin(int32_t capacity) {
    if (capacity <= 0) return fail(NLDPC_EINVAL, "nldpc_profile_begin: capacity must be positive");
    if ((size_t)capacity > g_prof.capacity) {
        for (auto& r : g_prof.recs) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        g_prof.recs.assign(capacity, ProfRec{0, nullptr, nullptr});
        for (auto& r : g_prof.recs) {
            NLDPC_HIP_CHECK(hipEventCreate(&r.a));
            NLDPC_HIP_CHECK(hipEventCreate(&r.b));
        }
        g_prof.capacity = capacity;
    }
    g_prof.used = 0;
    g_prof.armed = true;
    return NLDPC_OK;
}

// ms[k], count[k] for kind k in 0..nkinds-1 (0 = VN, 1 = CN, 2 = posterior, 3 = fused, 4 = VN backward,
// 5 = CN backward, 6 = fused backward)
extern "C" int nldpc_profile_end(int32_t nkinds, float* ms, int32_t* count) {
    g_prof.armed = false;
    for (int k = 0; k < nkinds; ++k) {
        ms[k] = 0.f;
        count[k] = 0;
    }
    for (size_t i = 0; i < g_prof.used; ++i) {
        ProfRec& r = g_prof.recs[i];
        NLDPC_HIP_CHECK(hipEventSynchronize(r.b));
        float t = 0.f;
        NLDPC_HIP_CHECK(hipEventElapsedTime(&t, r.a, r.b));
        if (r.kind >= 0 && r.kind < nkinds) {
            ms[r.kind] += t;
            count[r.kind]++;
        }
    }
    g_prof.used = 0;
    return NLDPC_OK;
}
