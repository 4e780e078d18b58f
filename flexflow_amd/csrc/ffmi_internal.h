// ffmi_internal.h -- shared internals of libffmi.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/ffmi.h"

#define FFMI_HIP(expr)                                   \
  do {                                                   \
    hipError_t e_ = (expr);                              \
    if (e_ != hipSuccess) {                              \
      ffmi_set_last_error(hipGetErrorString(e_), __FILE__, __LINE__); \
      (void)hipGetLastError(); /* reset: no stale error for a later launch check */ \
      return FFMI_ERR_HIP;                               \
    }                                                    \
  } while (0)

#define FFMI_CHECK(cond, code)                                         \
  do {                                                                 \
    if (!(cond)) {                                                     \
      ffmi_set_last_error(#cond, __FILE__, __LINE__);                  \
      return (code);                                                   \
    }                                                                  \
  } while (0)

void ffmi_set_last_error(const char *msg, const char *file, int line);

namespace ffmi {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Weight fragment load.  NT (FFMI_W_STREAM launches: a model whose weights
// exceed the Infinity Cache, each weight byte read by one workgroup) puts the
// non-temporal hint on the load (MI355X_MICROARCH.md "nt-weights"), so the
// stream does not evict the KV cache, activations or the SSM's weights from
// L2 / the Infinity Cache.  A model that fits (the 68M SSM, replayed step
// after step) keeps the default policy.
template <bool NT>
__device__ __forceinline__ h8 ld_weight(const uint16_t *p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const h8 *>(p));
  else return *reinterpret_cast<const h8 *>(p);
}

// Packed activation tiles (FFMI_X_PACKED / FFMI_Y_PACKED): element (m, n) of a
// [T][K] activation lives at [m/16][n/32][lane = (m&15) + 16*((n>>3)&3)][n&7],
// i.e. each 16-row x 32-column block is one MFMA operand fragment (1 KiB,
// lane-linear), the same order the weights are packed in (weights.hip).
__host__ __device__ __forceinline__ size_t act_packed_off(int m, int n, int K) {
  return ((((size_t)(m >> 4) * (size_t)(K >> 5) + (size_t)(n >> 5)) * 64 + (m & 15) +
           16 * ((n >> 3) & 3))
          << 3) +
         (n & 7);
}

// Layout of the packed per-step metadata blob (device copy of ffmi_batch_desc):
// [header 32 B][work items, 32 B each][tokens][commits].  The work array sits
// at a FIXED offset, so a kernel's first two loads (header, its work item)
// are independent instead of a dependent chain.
struct BatchHeader {
  int32_t num_tokens, num_work, num_commits, num_mask_reqs;
  int32_t off_tokens, off_work, off_commits, off_masks;  // byte offsets
};
constexpr int kBlobWorkOffset = 32;
static_assert(sizeof(BatchHeader) == kBlobWorkOffset, "work array follows the header");

// Fused attention's LDS tail: the keys [tail0, kv_len) of a work item are
// staged in LDS, at most kTailSlots of them: the slots below the request's
// lowest written slot (< 32, chunk alignment) from the cache, every slot from
// there on written this step (its stores and TREE commits, host-checked).  At
// most kItemCommits commits per request are applied by the attention prologue.
constexpr int kTailSlots = 128;
constexpr int kItemCommits = 8;

// Device work item: the ABI item plus what the host derives for the kernels.
struct WorkDev {
  ffmi_attn_work w;
  int32_t clean;  // slots below this are not written by this step's commits
                  // or stores for the item's request (loadable before them)
  int32_t tail0;  // chunk-aligned first slot of the LDS tail (<= clean)
  int32_t ncommit;  // TREE commits of this request (cm_src / cm_depth)
  int32_t told;     // slots [tail0, tail0 + told) keep their cached K/V (< 32);
                    // every tail slot above them is written this step
  // RoPE position of each of the item's tokens (clamped to [0, 32767]; the
  // kernels clamp to their table): the table loads then depend on the work
  // item only, not on the token records
  int16_t rope_pos[FFMI_ATTN_QTILE];
  // the request's commits: staging row (previous verify batch) -> KV slot
  int16_t cm_src[kItemCommits], cm_depth[kItemCommits];
};
static_assert(sizeof(WorkDev) % 16 == 0, "16-B aligned work items");

struct BatchView {
  const BatchHeader *hdr;
  const ffmi_token_info *tokens;
  const WorkDev *work;
  const ffmi_commit_info *commits;
  const uint64_t *masks;
};

__device__ __forceinline__ BatchView batch_view(const char *blob) {
  BatchView v;
  v.hdr = reinterpret_cast<const BatchHeader *>(blob);
  v.work = reinterpret_cast<const WorkDev *>(blob + kBlobWorkOffset);
  v.tokens = reinterpret_cast<const ffmi_token_info *>(blob + v.hdr->off_tokens);
  v.commits = reinterpret_cast<const ffmi_commit_info *>(blob + v.hdr->off_commits);
  v.masks = reinterpret_cast<const uint64_t *>(blob + v.hdr->off_masks);
  return v;
}

// Split-K partial sums left in the GEMM workspace for the CONSUMER to combine
// (S fp32 slabs [S][T][NP]; value(t, n) = fp16(sum over s in order)), which
// saves the separate reduce pass.  S == 0: nothing deferred, read Y.
struct Partials {
  const float *p = nullptr;
  int S = 0, NP = 0;
};
__device__ __forceinline__ float partials_value(const float *p, int S, int NP, int T, int t,
                                                int n) {
  const size_t slab = (size_t)T * NP;
  const float *q = p + (size_t)t * NP + n;
  float acc = q[0];
  for (int s = 1; s < S; ++s) acc += q[s * slab];
  return __half2float(__float2half_rn(acc));
}

// ---- kernel launchers (defined in kernels/*.hip) ----
hipError_t launch_fill_weight(uint16_t *dst, size_t n, uint64_t key, int kind, hipStream_t s,
                              int cols = 0, uint64_t pa = 1, uint64_t pb = 0, float scale = 1.0f);
hipError_t launch_fill_weight_f32(float *dst, size_t n, uint64_t key, int kind, hipStream_t s,
                                  int cols = 0, uint64_t pa = 1, uint64_t pb = 0,
                                  float scale = 1.0f);
float weight_amp(int kind);
// ---- full-precision path (kernels/f32.hip) ----
hipError_t launch_gemm_f32(const float *X, const float *W, float *Y, int T, int N, int K,
                           hipStream_t s);
hipError_t launch_rmsnorm_f32(const float *x1, const float *x2, const float *w, float *res_out,
                              float *out, int T, int H, float eps, hipStream_t s,
                              const char *gather = nullptr);
hipError_t launch_silu_mul_f32(const float *A, const float *B, float *out, int T, int F,
                               size_t lda, size_t ldb, hipStream_t s);
hipError_t launch_kv_update_f32(const char *blob, int T, int C, const float *qkv, const float *rope,
                                int max_rope_pos, float *qbuf, float *kc, float *vc,
                                float *stage, int heads, int d, int slots, hipStream_t s);
hipError_t launch_attention_f32(const char *blob, int T, const float *qbuf, const float *kc,
                                const float *vc, float *out, int heads, int d, int slots,
                                float scale, hipStream_t s);
hipError_t launch_softmax_topk_f32(const float *logits, int T, int V, int k, int32_t *ids,
                                   float *probs, hipStream_t s);
ffmi_status attn_rope_fault(ffmi_attn *h, int from_pos);
// Packed weights (weights.hip): 1 KiB block (tile t, k-step kt) at
// t * w_tile_stride(KT) + kt * w_k_stride(P) halves, P = tiles per k-row of
// the allocation.  K-major unless FFMI_W_TILE_MAJOR=1 (A/B runs).
bool weights_kmajor();
inline size_t w_tile_stride(int KT) { return weights_kmajor() ? 512 : (size_t)KT * 512; }
inline size_t w_k_stride(int pitch) { return weights_kmajor() ? (size_t)pitch * 512 : 512; }
// Source rows [row0, row0+N) x columns [col0, col0+K) of a row-major [.][ld]
// matrix -> destination tiles tile_step * nt + tile_offset of a packed
// allocation of `pitch` tiles per k-row (gate/up: step 2, offsets 0/1; qkv:
// offsets 0, NT, 2 NT of pitch 3 NT).
hipError_t launch_pack_weight(const uint16_t *src, int ld, int row0, int col0,
                              int N, int K, uint16_t *dst, int tile_step,
                              int tile_offset, int pitch, hipStream_t s);
// defer != nullptr: a split-K plan skips its reduce pass and describes the
// slabs in *defer (the caller's next kernel combines them); otherwise / S == 1
// Y is written and defer->S = 0.  Only for FFMI_EPI_NONE.  wpitch: tiles per
// k-row of Wp's allocation (0 = the GEMM's own tile count; a column chunk of a
// wider matrix passes the full matrix's).
// Residual RMSNorm folded into the skinny GEMMs (T <= 32, unsplit), the
// reference's ResidualRMSNorm (residual_rms_norm_kernels.cu:98-131) split
// over the two GEMMs around it:
//  * producer (o / down projection, EPI 0): Y = half(res_in + half(X.W^T))
//    (Y may alias res_in) and, per row and 16-column tile, the fp32 sum of
//    squares of those fp16 values -> ss_out[T][N/16];
//  * consumer (the next qkv or gate/up): X is that residual, row-major; the
//    prologue turns the row's ss_in partials into rms = half(1/sqrt(sum/K +
//    eps)) and every X fragment becomes half(half(x * rms) * w[k]) before its
//    MFMA -- the norm kernel's arithmetic, fp16 multiplies.
struct FuseArgs {
  int kind = 0;                     // 0 none, 1 producer, 2 consumer
  const uint16_t *res_in = nullptr;  // producer: [T][N] residual
  float *ss_out = nullptr;          // producer: [T][N/16]
  const float *ss_in = nullptr;     // consumer: [T][nss]
  int nss = 0;                      // consumer: partials per row (= K/16)
  const uint16_t *wnorm = nullptr;  // consumer: norm weight [K]
  float eps = 0.f;
};
hipError_t launch_gemm(const uint16_t *X, const uint16_t *Wp, uint16_t *Y, float *ws,
                       size_t ws_bytes, int T, int N, int K, int epilogue, hipStream_t s,
                       Partials *defer = nullptr, int wpitch = 0, const FuseArgs *fuse = nullptr);
size_t gemm_workspace_bytes(int T, int N, int K, int epilogue);
// fp16 Y[T][N] (row-major) of deferred split-K slabs, summed in slab order and
// rounded once: the value every consumer of the slabs computes (tensor capture)
hipError_t launch_partials_reduce(const Partials &p, uint16_t *Y, int T, int N, hipStream_t s);
long attn_debug_stamps(long long *dst, long max_waves);
hipError_t launch_marker(int i, hipStream_t s);
void attn_stamp_gate(bool open);
long debug_markers(long long *dst, long n);
long gemm_debug_stamps(long long *dst, long max_waves);
size_t packed_act_bytes(int T, int K);
hipError_t launch_pack_act(const uint16_t *X, uint16_t *Xp, int T, int K, hipStream_t s);
hipError_t launch_rmsnorm(const uint16_t *x1, const uint16_t *x2, const uint16_t *w,
                          uint16_t *res_out, uint16_t *out, int T, int H, float eps,
                          hipStream_t s, bool out_packed = false, Partials x2p = {}, const char *gather = nullptr,
                          char *blob_dst = nullptr, size_t blob_bytes = 0,
                          const int32_t *gather_prev = nullptr);
// FFMI_FAULT_RESID_ROUND negative control (tests only; process-wide)
void set_norm_fault(bool on);
hipError_t launch_embedding(const char *blob, int T, const uint16_t *table,
                            uint16_t *out, int H, hipStream_t s);
hipError_t launch_silu_mul(const uint16_t *a, const uint16_t *b, uint16_t *out,
                           size_t n, hipStream_t s);
// softmax + argmax / top-k; with a zeroed workspace of argmax_workspace_bytes(T)
// (left zeroed) rows of a small T are split over several workgroups
hipError_t launch_argmax(const uint16_t *logits, int T, int V, int k, int32_t *ids,
                         float *probs, hipStream_t s, void *ws = nullptr, size_t ws_bytes = 0,
                         int32_t *ids2 = nullptr);  // (ids2: a second copy of the ids)
size_t argmax_workspace_bytes(int T);
// Vocab-sharded tail (norm.hip): phase 0..2 write this rank's exchange
// record ([P][T][W] floats, W >= max(4, 2k)); phase 3 merges into ids/probs.
hipError_t launch_vshard(const uint16_t *logits, int T, int Vl, int P, int rank, int k,
                         int phase, float *xch, int W, int32_t *ids, float *probs,
                         hipStream_t s);
hipError_t launch_group_sum(const void *const *bufs, int n, void *out, size_t count, int dtype,
                            hipStream_t s);

hipError_t launch_kv_update(const char *blob, int T, int W, int C, const uint16_t *qkv,
                            Partials qkvp, uint16_t *qbuf, uint16_t *kc, uint16_t *vc,
                            uint16_t *stage_wr, const uint16_t *stage_rd, const float *rope,
                            int heads, int d, int slots, int max_rope_pos, hipStream_t s);
hipError_t launch_commit(const char *blob, int C, const uint16_t *stage,
                         uint16_t *kc, uint16_t *vc, int heads, int d, int slots,
                         hipStream_t s);
// Output projection folded into the fused attention (small models, where one
// head's K-slice of Wo is a few tens of KB: the 68M SSM's is 96 KB).  Each
// (work item, head) workgroup multiplies its rounded fp16 output rows [q][d]
// by Wo[:, head*d .. head*d + d) and stores the fp32 product as slab `head`
// of [heads][T][N]; the residual norm sums the heads in order and rounds once
// (Partials), as it combines a split-K GEMM's slabs -- no o_proj launch.
struct OprojArgs {
  const uint16_t *wo = nullptr;  // packed [N][heads * d] (weights.hip)
  float *slab = nullptr;         // [heads][T][N] fp32
  int N = 0, max_T = 0;          // output width; rows the slab buffer holds
  size_t wts = 0, wks = 0;       // packed-block strides (w_tile_stride / w_k_stride)
  bool done = false;             // out: the launch projected (else run the o GEMM)
};
hipError_t launch_attention(const char *blob, int W, int max_q, uint16_t *qbuf, uint16_t *kc,
                            uint16_t *vc, uint16_t *out, int heads, int d, int slots, float scale,
                            hipStream_t s, bool out_packed, bool fused, int T, int C,
                            const uint16_t *qkv, Partials qkvp, uint16_t *stage_wr,
                            const uint16_t *stage_rd, const float *rope, int max_rope_pos,
                            const OprojArgs *opa = nullptr);

uint64_t weight_key(const char *name, uint64_t seed);

}  // namespace ffmi

// Device batch blob: pinned host staging + device copy.
struct ffmi_batch_dev {
  char *host = nullptr;  // pinned
  char *dev = nullptr;
  size_t cap = 0;
  int max_tokens = 0, max_requests = 0;
  // host-visible counts of the last upload (launch geometry)
  int num_tokens = 0, num_work = 0, num_commits = 0, num_mask_reqs = 0;
  bool commit_overlap = false;  // a commit depth is also a slot this step stores
  bool one_item_per_req = false;  // every request's tokens form one attention work item
  bool lds_tail = false;  // every item's writes fit the fused kernel's LDS tail and
                          // its commits the work item (else the two-launch path)
  int max_q = 0;                  // largest work item
  hipEvent_t uploaded = nullptr;  // guards reuse of the pinned staging
};

// Internal entry points used by the in-library model runtime (llama_gpu.cpp):
// the public ffmi_attn_* / ffmi_rmsnorm_ex with deferred split-K inputs.
namespace ffmi {
ffmi_status batch_stage(ffmi_batch_dev *b, const ffmi_batch_desc *d, size_t *bytes);
ffmi_status batch_copy(ffmi_batch_dev *b, size_t bytes, hipStream_t s, bool record_event);
// parity: which half of the TREE staging this step writes (commits read the
// other); -1 = the handle's own alternation (public API calls)
// Communicator internals for the model runtime (api.cpp): the direct xGMI
// transport when attached and the message fits its buffers.
bool comm_has_peer(const ffmi_comm *c, size_t bytes);
int comm_size(const ffmi_comm *c);
int comm_rank(const ffmi_comm *c);
// the xGMI transport is attached (whatever its capacity)
bool comm_peer_attached(const ffmi_comm *c);
// an RCCL communicator or an in-process group takes what the transport cannot
bool comm_has_fallback(const ffmi_comm *c);
// an RCCL communicator (stream-capturable all-reduce)
bool comm_is_rccl(const ffmi_comm *c);
// sum of every rank's [rows][cols] `in` into `out` (row stride ld, starting
// at column col0) over the xGMI transport; with `slabs` (f16 only) this
// rank's partial is the sum of the GEMM's deferred split-K slabs instead of
// `in` (the reduce pass folded into the copy-in)
ffmi_status comm_allreduce_cols(ffmi_comm *c, const void *in, void *out, int rows, int cols,
                                int ld, int col0, int dtype, hipStream_t s,
                                const Partials *slabs = nullptr);
// the transport takes a message of `bytes` in two shots (reduce-scatter +
// all-gather) rather than one
bool comm_two_shot(const ffmi_comm *c, size_t bytes);
// reduce-scatter by rows over the transport: rows [row0, row1) of the sum of
// every rank's [rows][cols] into out (row stride ld, column offset col0);
// must be followed by comm_allreduce_norm (two-shot) over the same rows
ffmi_status comm_reduce_rows(ffmi_comm *c, const void *in, void *out, int rows, int cols, int ld,
                             int col0, int row0, int row1, hipStream_t s,
                             const Partials *slabs = nullptr);
// all-reduce of every rank's [T][H - col0] partial (columns col0.. of the sum;
// columns < col0 from prev) fused with the residual RMSNorm after it
// (collective.h, PeerNormArgs): res += sum in place, h = norm(res) * w.
// two_shot: this rank's rows T*r/N.. only, h gathered from the other ranks
// (res valid on this rank's rows); else every row on every rank
ffmi_status comm_allreduce_norm(ffmi_comm *c, const void *in, int T, int H, int col0,
                                const uint16_t *prev, uint16_t *res, const uint16_t *w, float eps,
                                uint16_t *h, bool packed, bool two_shot, hipStream_t s,
                                const Partials *slabs = nullptr);
// FFMI_OK, or the transport's timeout error after a synchronised step
ffmi_status comm_status(ffmi_comm *c);
ffmi_status attn_forward(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv, Partials qkvp,
                         void *out, ffmi_stream stream, int parity = -1,
                         OprojArgs *opa = nullptr);
}  // namespace ffmi
