// Backward through the unrolled decoder (placeholder until the reverse kernels land).
#include <hip/hip_runtime.h>

#include "nldpc_internal.h"

using namespace nldpc;

extern "C" int nldpc_backward_workspace(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T,
                                        size_t* bytes) {
    (void)g; (void)cfg; (void)B; (void)T;
    if (bytes) *bytes = 0;
    return fail(NLDPC_EUNSUPPORTED, "nldpc_backward: not implemented yet");
}

extern "C" int nldpc_backward(const nldpc_graph*, const nldpc_cfg*, int64_t, int32_t, const float*, const float*,
                              const float*, const float*, const float*, const float* const*, const float* const*,
                              const float*, const float*, float*, float*, float*, float*, void*, size_t, void*) {
    return fail(NLDPC_EUNSUPPORTED, "nldpc_backward: not implemented yet");
}
