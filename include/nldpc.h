/*
 * nldpc.h — C ABI of the MI355X-native neural belief-propagation LDPC decoder.
 *
 * The reference (ShapeLayer/neural-ldpc-decoder-torch) has no FFI: its hot path is the Python
 * nn.Module API.  This header is the native boundary that the drop-in modules
 * (neural-ldpc-decoder-torch_amd/src/{neural_ldpc_decoder,boosted_neural_ldpc_decoder}) bind
 * through ctypes; each entry point names the reference interface it replaces.
 *
 * Conventions
 *   - int status: 0 = NLDPC_OK; anything else is an error, nldpc_last_error() gives the text
 *     (thread-local).  No C++ exception crosses this boundary.
 *   - Every tensor argument is a DEVICE pointer to contiguous fp32 (or the stated type) memory,
 *     allocated by the caller (e.g. the torch caching allocator).  Host arrays are marked "host".
 *   - All launches are stream-ordered on the `stream` argument (a hipStream_t); no entry point
 *     synchronises the device or allocates device memory, so every call is graph-capturable.
 *   - A graph handle owns only its device edge tables; it is immutable after creation and may be
 *     used from several streams at once.
 *   - Layouts: channel LLR xa [B][N][Z]; outputs [B][N*Z] (bit index j*Z+v, reference layout);
 *     message state [B][E][Z] with E in C-order (row-major over the base graph).
 */
#ifndef NLDPC_H
#define NLDPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NLDPC_ABI_VERSION 4

enum nldpc_status {
    NLDPC_OK = 0,
    NLDPC_EINVAL = 1,      /* bad argument (ValueError on the Python side) */
    NLDPC_EHIP = 2,        /* HIP runtime error */
    NLDPC_EUNSUPPORTED = 3 /* valid but not implemented configuration */
};

/* Decoder kinds.  SP/MS/QMS keep the reference DecoderType values
 * (src/boosted_neural_ldpc_decoder/struct/DecoderType.py:4-7); NEURAL is
 * src/neural_ldpc_decoder/NeuralLDPCDecoder.py. */
enum nldpc_kind { NLDPC_SP = 0, NLDPC_MS = 1, NLDPC_QMS = 2, NLDPC_NEURAL = 3 };

typedef struct nldpc_graph nldpc_graph;

/* Per-call decoder configuration (the constructor arguments of BoostedNeuralLDPCDecoder,
 * BoostedNeuralLDPCDecoder.py:15-49, reduced to what the arithmetic needs). */
typedef struct nldpc_cfg {
    int32_t kind;    /* enum nldpc_kind */
    int32_t qbit;    /* QMS quantiser: 6, 5, -5, 4, 3; anything else = identity (:187-214) */
    int32_t ucn;     /* 1: compute unsatisfied-check flags and mix w_ucn (:339-374, :436-488) */
    int32_t vn_cumulative; /* 1: xin_t = Q(xin_{t-1} * w_vn[t]) (:325-337); 0: no VN weight */
    float llr_lo;    /* allowed_llr_range.start (Clipping, :36) */
    float llr_hi;    /* allowed_llr_range.end */
    int32_t first_iter; /* absolute index of the first iteration of this call (UCN uses xin at 0) */
    int32_t c2v_in;  /* 1: read the c2v state at the start; 0: start from all-zero messages */
    int32_t vn_prefix; /* rows of w_vn applied before this call's first iteration (cumulative VN
                          weighting carried over earlier iterations of the same forward) */
    int32_t flags;   /* NLDPC_FLAG_* */
} nldpc_cfg;

/* cfg->flags */
#define NLDPC_FLAG_STREAM 1      /* force the streaming (two kernels per iteration) path */
#define NLDPC_FLAG_FUSED 2       /* require the register-resident fused path (error if ineligible) */
#define NLDPC_FLAG_NO_STATE 4    /* the caller does not need the final c2v state: c2v may be NULL
                                    when the fused path runs */
#define NLDPC_FLAG_CN_TIED 8     /* (ABI 4, nldpc_backward; r6: also a saving nldpc_forward without UCN, which then runs
                                    a kernel that reads one CN weight per iteration, w_cn[t][0]) every row of w_cn
                                    repeats one weight (sharing code 3,
                                    BoostedNeuralLDPCDecoder.py:114-124): g_w_cn may receive each iteration's total
                                    in a few entries of its row and zeros elsewhere -- only row sums are meaningful,
                                    which is all a tied weight's gradient is.  The results (every gradient) are
                                    UNDEFINED unless every row of w_cn is one value: the tied kernel derives a row's
                                    check-node masks from its first weight (the Python side sets the flag only for a
                                    stride-0 expand, nldpc.decode._honour_tied) */

/* ---- library ---------------------------------------------------------------------------- */
int nldpc_abi_version(void);
const char* nldpc_last_error(void);

/* ---- graph: replaces ConnectingMatrix(Z, basegraph) + ConnectingMatrixTorch(cm, device)
 *      (src/boosted_neural_ldpc_decoder/ConnectingMatrix.py:5-80, ConnectingMatrixTorch.py:7-54;
 *       src/neural_ldpc_decoder/ConnectingMatrix.py:4-66, ConnectingMatrixTorch.py:7-46).
 *      basegraph: host [M*N] row-major shift table, -1 = no edge; shifts are taken mod Z. ------ */
int nldpc_graph_create(int32_t M, int32_t N, int32_t Z, const int32_t* basegraph, int32_t device,
                       nldpc_graph** out);
int nldpc_graph_destroy(nldpc_graph* g);
/* dims[0..7] = M, N, Z, E, max check degree, max variable degree, device, reserved */
int nldpc_graph_dims(const nldpc_graph* g, int32_t* dims);
/* host copies of the C-order edge tables: check, variable, shift (mod Z) of every edge */
int nldpc_graph_edges(const nldpc_graph* g, int32_t* chk, int32_t* var, int32_t* shift);
/* (ABI 3) A register-resident kernel compiled at run time for this lifted graph (gen_fused.py --jit
 *      output, `hipcc --genco` for gfx950; entry point nldpc_fx, or nldpc_fxb for the backward): the
 *      library's own fused kernels cover a fixed set of (base graph, Z); any other graph gets its kernels
 *      this way, per mode (0 decode, 1 decode + save for backward, 2 / 3 count-only, 4 backward) and
 *      kind, with the geometry they were generated for (codewords per workgroup, threads, waves per
 *      part).  The graph keeps the loaded module until nldpc_graph_destroy.  No-op for a graph the
 *      library already covers.  Replaces nothing in the reference (its dense path has no per-Z code);
 *      it is what makes ConnectingMatrix(Z, basegraph) at any Z (ConnectingMatrix.py:5-53) fast.
 *      The code object's global nldpc_sig (the kernel argument layout it was generated for) must be this
 *      library's, else NLDPC_EUNSUPPORTED (r5: a skewed build is refused instead of running a kernel that
 *      leaves its outputs unwritten).  r6: the signature is read from the host copy of the code object (no
 *      device copy, no wait on work in flight).  Loading the module (hipModuleLoadData) is not a stream
 *      operation: attach a geometry's kernels -- i.e. run the first decode of a run-time geometry -- outside
 *      any stream / graph capture (nldpc.jit compiles and attaches on that first call). */
int nldpc_graph_attach_kernel(nldpc_graph* g, int32_t mode, int32_t kind, const void* code, size_t bytes,
                              int32_t G, int32_t threads, int32_t waves_per_part);
/* (r6, additive to ABI 4) The argument-layout signature a code object was generated for (its nldpc_sig, read on the host from
 *      the hipcc --genco offload bundle or a bare gfx950 ELF) and the one this library's mode needs (mode 0-3:
 *      forward kernels, 4: backward).  NLDPC_EINVAL when the object carries no readable nldpc_sig.  Lets a
 *      caller validate a cached code object before nldpc_graph_attach_kernel; no device is touched. */
int nldpc_code_object_sig(const void* code, size_t bytes, int32_t mode, uint32_t* sig, uint32_t* expected);
/* (ABI 3) *mask: bit (mode * 4 + kind) set when that fused kernel exists for the graph (modes as above) */
int nldpc_graph_kernels(const nldpc_graph* g, uint32_t* mask);

/* ---- execution path.  *eligible = 1 when nldpc_forward with these arguments runs the fused
 *      register-resident kernel: a (base graph, lifting size) compiled in, no incoming message state
 *      (c2v_in == 0; a resumed UCN segment passes app_prev instead), T <= 64, no NLDPC_FLAG_STREAM;
 *      every kind, UCN and cumulative VN weights included, saving for backward included; QMS only
 *      with an active quantiser (qbit 3, 4, 5, -5, 6: an identity quantiser decodes on the streaming
 *      kernels, r3).  Then v2c is unused, and c2v is unused too with
 *      NLDPC_FLAG_NO_STATE.  Otherwise the streaming kernels run and need both buffers. */
int nldpc_fast_path(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, int32_t saving,
                    int32_t* eligible);
/*      (ABI 3) saving = 2 / 3 asks the same for nldpc_forward_count (all-zero codeword, decoder convention /
 *      any convention or codeword), whose fused kernels are separate variants. */

/* ---- decode forward: replaces NeuralLDPCDecoder.forward (NeuralLDPCDecoder.py:44-100) and
 *      BoostedNeuralLDPCDecoder.forward (BoostedNeuralLDPCDecoder.py:260-538).
 *   T        iterations run by this call (iteration k of the call = absolute cfg->first_iter + k)
 *   xa       [B][N][Z] channel LLRs
 *   w_cn     [T][E] per-edge check-node weight, NULL = |x| (sharing code 0).  Shared codes (per
 *            check, per iteration) are expanded to per-edge by the caller.
 *   w_ucn    [T][E] per-edge UCN weight (cfg->ucn), else NULL
 *   bias     [T][E] per-edge bias (NEURAL), else NULL
 *   w_vn     [vn_prefix + T][N] per-column VN weights (cfg->vn_cumulative), else NULL; iteration k
 *            of the call uses xin = Q(..Q(xa*w_vn[0])..*w_vn[vn_prefix+k])
 *   outs     host array of T device pointers, each [B][N*Z]; NULL entries are not written
 *            (with cfg->ucn every entry but the last must be non-NULL: iteration k reads k-1)
 *   app_prev [B][N*Z] posterior of iteration first_iter-1 (UCN with first_iter > 0), else NULL
 *   c2v      [B][E][Z] message state in/out: read at the start when cfg->c2v_in (otherwise a
 *            fresh all-zero state), holds the state after the last iteration on return
 *   v2c      [B][E][Z] scratch of the streaming path (unused, may be NULL, when nldpc_fast_path
 *            reports 1; also NULL-able for a non-QMS training call, which streams through `saved`)
 *   saved    device buffer of nldpc_saved_bytes() bytes that receives what nldpc_backward needs
 *            (every iteration's variable-to-check messages -- fp32, or for QMS one int8 code per
 *            message holding Q(m) and its clip mask --, the Boosted output clamp masks, and the
 *            cumulative-VN-weight channel values), or NULL (inference); needs every `outs` entry
 *   stream   hipStream_t */
int nldpc_saved_bytes(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, size_t* bytes);
int nldpc_forward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                  const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                  float* const* outs, const float* app_prev, float* c2v, float* v2c, void* saved,
                  void* stream);

/* ---- decode backward (config 5: training through the unrolled decoder; the reference gets this
 *      from autograd over BoostedNeuralLDPCDecoder.py:320-526 / NeuralLDPCDecoder.py:54-98).
 *   outs       forward outputs (needed for UCN flags and the output clamp mask)
 *   grad_outs  host array of T device pointers [B][N*Z] (NULL entry = zero gradient)
 *   saved      as written by nldpc_forward
 *   grad_c2v_out [B][E][Z] gradient arriving at the final message state (the state a later segment
 *              of the same forward resumed from: list-valued xa, split iteration runs), or NULL
 *   grad_c2v_in  [B][E][Z] out: gradient of the incoming message state (cfg->c2v_in), or NULL
 *              (either of the two selects the streaming backward)
 *   g_w_cn, g_w_ucn, g_bias: [T][E] accumulated (+=) per-edge gradients, NULL if not wanted
 *   g_w_vn     [vn_prefix + T][N] accumulated (+=) per-column gradients, NULL if not wanted
 *   work       device scratch of nldpc_backward_workspace() bytes */
int nldpc_backward_workspace(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T,
                             size_t* bytes);
int nldpc_backward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                   const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                   const float* const* outs, const float* const* grad_outs, const float* app_prev,
                   const void* saved, const float* grad_c2v_out, float* grad_c2v_in, float* g_w_cn,
                   float* g_w_ucn, float* g_bias, float* g_w_vn, void* work, size_t work_bytes, void* stream);

/* ---- BER/FER accounting: replaces Functions.evaluate_ber_fer (Functions.py:85-102) and the
 *      per-iteration .item() loop of train/train_BoostedNeuralLDPCDecoder.py:363-383.
 *   llr [B][L]; y [B][L] uint8 bits or NULL (all-zero codeword); counts int64[2] += (bit errors,
 *   frame errors).  convention 0: bit = (LLR > 0) (decoder convention);
 *   convention 1: bit = (LLR < 0) (the reference helper's literal, inverted rule). */
int nldpc_ber_count(const float* llr, const uint8_t* y, int64_t B, int64_t L, int32_t convention,
                    int64_t* counts, void* stream);

/* ---- count-only decode (§8 F2): nldpc_forward followed by nldpc_ber_count on every iteration's
 *      output (the test loop of test/test_*.py around Functions.evaluate_ber_fer, Functions.py:85-102),
 *      fused into the decoder: each iteration's posterior is compared with the codeword bit inside
 *      the register-resident kernel and only the counts leave the chip (no T x [B][N*Z] outputs).
 *   arguments as nldpc_forward (no outs / app_prev / c2v / v2c / saved); y [B][N*Z] uint8 bits or
 *   NULL (all-zero codeword); counts int64 [T][2] device, += (bit errors, frame errors) of iteration
 *   first_iter + k in row k; convention as nldpc_ber_count.  Needs the fused path (nldpc_fast_path
 *   with saving = 0 reports 1), NLDPC_EUNSUPPORTED otherwise. */
int nldpc_forward_count(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                        const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                        const uint8_t* y, int32_t convention, int64_t* counts, void* stream);

/* ---- multi-iteration BCE loss (config 5's training loss): replaces LDPCDecoderLoss.forward with
 *      LossType.BCE over a list of outputs and one label tensor
 *      (src/boosted_neural_ldpc_decoder/LDPCDecoderLoss.py:70-108, binary_cross_entropy_with_logits
 *      per term) and its autograd backward, in one pass over the T outputs instead of a chain of
 *      elementwise ops per term.
 *   logits   host array of K device pointers, each [n] fp32 (K <= 64)
 *   coef     host [K]: weight of term k (etha^c_k / sum_k etha^c_k)
 *   target   [n] fp32 labels shared by every term, or NULL (all zero)
 *   loss     device fp32 scalar out: sum_k coef[k] * mean_i bce(logits[k][i], target[i]), with
 *            bce(x, t) = (1 - t) * x - log_sigmoid(x) (fp32 terms, fp64 fixed-order sums)
 *   work     device scratch of nldpc_bce_workspace() bytes
 *   grads    (nldpc_bce_grad) K device pointers [n]: grads[k][i] = (*gseed) * coef[k] / n *
 *            (sigmoid(logits[k][i]) - target[i]); gseed is a device fp32 scalar (dL/dloss) */
int nldpc_bce_workspace(int64_t n, int32_t K, size_t* bytes);
int nldpc_bce_loss(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                   float* loss, void* work, size_t work_bytes, void* stream);
int nldpc_bce_grad(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                   const float* gseed, float* const* grads, void* stream);
/* The training step's pair in one pass over the logits (read once for the loss and the gradients): the
 * loss as nldpc_bce_loss and grads[k] as nldpc_bce_grad would write them for *gseed == 1 (what
 * loss.backward() sends), bit for bit.  nldpc_bce_grad_unless_unit then runs at backward time with the
 * seed that arrived: it returns at once on the device when *gseed == 1 and otherwise overwrites grads
 * as nldpc_bce_grad does, so the pair equals nldpc_bce_loss + nldpc_bce_grad for any seed. */
int nldpc_bce_loss_grad(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                        float* loss, float* const* grads, void* work, size_t work_bytes, void* stream);
int nldpc_bce_grad_unless_unit(const float* const* logits, int32_t K, const float* coef, const float* target,
                               int64_t n, const float* gseed, float* const* grads, void* stream);

/* ---- synthetic AWGN channel (the step before the path; replaces the all-zero branch of
 *      AWGNPassedDatagen, boosted.../AWGNPassedDatagen.py:75-134, generated on the device):
 *   xa[b][n] = 2*(-1 + sigma*g)/sigma^2 with g ~ N(0,1) from Philox-4x32-10(seed) at counter
 *   (b_offset + b)*L + n, so a sharded run draws the same noise as a single-device run.
 *   qbit != 0 applies the QMS quantiser (Functions.Cal_MSA_Q, Functions.py:69-83). */
int nldpc_awgn_llr(float* xa, int64_t B, int64_t L, float sigma, uint64_t seed, int64_t b_offset,
                   int32_t qbit, void* stream);
/* ---- the same channel with the rest of AWGNPassedDatagen._gendata_* (AWGNPassedDatagen.py:75-134,
 *      §8 F1): y [B][L] uint8 codeword bits (NULL = all-zero), BPSK (-1)^(1-y); after the quantiser,
 *      bits [puncture_start-1, puncture_end) of every codeword are set to puncture_value (the
 *      reference: 0, or 0.001 for SP) and bits [shorten_start-1, shorten_end) to shorten_value
 *      (-|allowed_llr_range.end|); a start of 0 disables the range (Puncture(0, 0) / Shortening(0, 0)).
 *      nldpc_awgn_llr(...) == nldpc_channel_llr(..., NULL, 0, 0, 0, 0, 0, 0, stream). */
int nldpc_channel_llr(float* xa, int64_t B, int64_t L, float sigma, uint64_t seed, int64_t b_offset,
                      int32_t qbit, const uint8_t* y, int64_t puncture_start, int64_t puncture_end,
                      float puncture_value, int64_t shorten_start, int64_t shorten_end, float shorten_value,
                      void* stream);

/* ---- benchmark instrumentation: per-kernel HIP-event timing of nldpc_forward / nldpc_backward
 *   launches.  nldpc_profile_begin arms a recorder for up to `capacity` launches (not thread-safe);
 *   nldpc_profile_end synchronises on the recorded events and returns summed milliseconds and
 *   launch counts per kernel kind (0 = variable-node, 1 = check-node, 2 = final posterior,
 *   3 = fused decoder, 4 = variable-node backward, 5 = check-node backward). */
int nldpc_profile_begin(int32_t capacity);
int nldpc_profile_end(int32_t nkinds, float* ms, int32_t* count);

/* ---- benchmark instrumentation: measured HBM ceilings (SURVEY §8(d) D4 "report the measured
 *   stream-copy ceiling too").  One launch over n floats (n % 4 == 0; 16 B per lane unless stated):
 *   kind 0 = copy src -> dst, 1 = write-only fill of dst, 2 = read-only pass over src (dst receives
 *   one float4 per workgroup, 2048 workgroups), 3 = read-only with 4 B per lane (dst receives one float4 per
 *   workgroup, 8192 workgroups).  r6: kinds 0-2 keep 8 float4 loads in flight per lane, non-temporal. */
int nldpc_hbm_probe(int32_t kind, float* dst, const float* src, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NLDPC_H */
