/*
 * ffmi.h -- C ABI of the MI355X-native SpecInfer hot path (libffmi.so).
 *
 * Drop-in boundary for the reference's Op/OpMeta kernel-wrapper layer
 * (hugolatendresse/FlexFlow @ 2025-01-17).  Each entry point names the
 * reference interface it replaces.  Plain C types only: device pointers,
 * sizes, an explicit hipStream_t.  Activations are caller-owned; KV caches and
 * workspaces are handle-owned (the reference's Meta objects own them too,
 * inc_multihead_self_attention.cu:1621-1807).  No exceptions cross the ABI:
 * every call returns an ffmi_status (the reference asserts instead,
 * cuda_helper.h:40-58; a caller shim may assert on != FFMI_OK).
 *
 * Threading: a handle is used by one host thread at a time, like an OpMeta
 * (one GPU task thread per processor in Legion).  All device work is ordered
 * on the stream argument.
 */
#ifndef FFMI_H_
#define FFMI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *ffmi_stream; /* == hipStream_t */

typedef enum {
  FFMI_OK = 0,
  FFMI_ERR_INVALID = 1,     /* bad argument / shape the kernels do not cover */
  FFMI_ERR_HIP = 2,         /* HIP runtime error */
  FFMI_ERR_NCCL = 3,        /* RCCL error */
  FFMI_ERR_OOM = 4,         /* device allocation failed */
  FFMI_ERR_UNSUPPORTED = 5, /* head size / mode not built */
  FFMI_ERR_NO_DEVICE = 6    /* no gfx950 device visible */
} ffmi_status;

typedef enum { FFMI_F16 = 0, FFMI_F32 = 1, FFMI_I32 = 2 } ffmi_dtype;

/* Attention mode == the reference op that the handle replaces. */
typedef enum {
  FFMI_ATTN_INC = 0,  /* IncMultiHeadSelfAttention     (inc_decoding)  */
  FFMI_ATTN_SPEC = 1, /* SpecIncMultiHeadSelfAttention (SSM beam step) */
  FFMI_ATTN_TREE = 2  /* TreeIncMultiHeadSelfAttention (LLM verify)    */
} ffmi_attn_mode;

/* ------------------------------------------------------------------------ */
/* Device batch metadata                                                     */
/* ------------------------------------------------------------------------ */
/* One packed blob per step replaces the reference's per-step H2D copies of
 * tokensInfo / requestsInfo / causalMask / committed_tokens / beam info
 * (request_manager.cu:23-159, ~83-150 KB per GPU per step): the host packs
 * only what the step uses, in the form the kernels read.                    */

typedef struct {
  int32_t token_id;   /* input token (embedding row)                         */
  int32_t pos;        /* RoPE position = abs_depth_in_request                */
  int32_t req;        /* request slot (KV-cache row)                         */
  int32_t store_slot; /* KV-cache slot this token's K/V goes to (-1: none)   */
  int32_t prefix_len; /* keys [0, prefix_len) are visible to this token      */
  int32_t tree_base;  /* first tree slot                                     */
  int32_t tree_len;   /* tree slots [tree_base, tree_base+tree_len) ...      */
  int32_t tree_bit;   /* ... visible iff mask[req][slot-tree_base] bit set   */
  uint64_t tree_vis;  /* OUTPUT of ffmi_batch_upload (input ignored): the same
                         rule transposed for this query, bit j set iff tree
                         slot tree_base+j is visible -- what kernels read */
} ffmi_token_info;

typedef struct {
  int32_t req;     /* request slot                                         */
  int32_t q_start; /* first batch token of this work item                  */
  int32_t q_count; /* tokens in the item (<= FFMI_ATTN_QTILE)              */
  int32_t kv_len;  /* keys scanned: [0, kv_len)                            */
} ffmi_attn_work;

typedef struct {
  int32_t src_token; /* token index in the PREVIOUS verify batch (staging) */
  int32_t req;       /* request slot                                       */
  int32_t depth;     /* destination KV slot (token depth)                  */
  int32_t pad;
} ffmi_commit_info;

#define FFMI_ATTN_QTILE 32
#define FFMI_MAX_TREE 64

/* Host-side description of one step (pointers into host memory). */
typedef struct {
  int32_t num_tokens;
  int32_t num_work;
  int32_t num_commits;
  int32_t num_mask_reqs;        /* rows in `masks` (indexed by req slot)    */
  const ffmi_token_info *tokens;   /* [num_tokens]                          */
  const ffmi_attn_work *work;      /* [num_work]                            */
  const ffmi_commit_info *commits; /* [num_commits]                         */
  const uint64_t *masks;           /* [num_mask_reqs][FFMI_MAX_TREE]        */
} ffmi_batch_desc;

typedef struct ffmi_batch_dev ffmi_batch_dev; /* device copy + pinned staging */

ffmi_status ffmi_batch_create(int max_tokens, int max_requests, ffmi_batch_dev **out);
void ffmi_batch_destroy(ffmi_batch_dev *b);
/* Replaces RM_LOAD_TOKENS / RM_LOAD_BATCH_CONFIG tasks
 * (request_manager.cu:23-159): one async H2D copy of the used bytes. */
ffmi_status ffmi_batch_upload(ffmi_batch_dev *b, const ffmi_batch_desc *desc,
                              ffmi_stream stream);

/* ------------------------------------------------------------------------ */
/* Attention (replaces src/ops/{inc,spec_inc,tree_inc}_multihead_self_attention) */
/* ------------------------------------------------------------------------ */
typedef struct {
  int mode;            /* ffmi_attn_mode                                     */
  int num_heads;       /* heads on this shard                                */
  int head_dim;        /* 64 or 128; 32 too in FFMI_ATTN_INC (inc...cu:911) */
  int max_requests;    /* KV rows                                            */
  int max_seq_len;     /* committed slots per request (S)                    */
  int max_tree_tokens; /* extra slots for tree / spec (S' = S + tree)        */
  int max_tokens;      /* batch capacity (staging rows for TREE commits)     */
  float qk_scale;      /* 1/sqrt(head_dim) (qk_prod_scaling)                 */
  float rope_theta;    /* HF rotate-half RoPE base                           */
  int out_layout;      /* 0: out [T][heads*head_dim] row-major;
                          1: packed activation tiles (feeds ffmi_linear with
                          FFMI_X_PACKED; heads*head_dim % 32 == 0)          */
  /* llama3 RoPE frequency scaling (inc_multihead_self_attention.cu:703-722;
   * rope_llama3 = 0: plain HF RoPE, the other fields ignored)               */
  int rope_llama3;
  float rope_factor, rope_low_freq_factor, rope_high_freq_factor;
  int rope_original_max_pos;
  /* 1: DT_FLOAT (--use-full-precision): qkv in and out fp32 row-major
   * (out_layout 0), K and V caches fp32 [req][head][slot][d] both, fp32
   * softmax (kernels/f32.hip).  0: fp16. */
  int full_precision;
} ffmi_attn_cfg;

typedef struct ffmi_attn ffmi_attn;

/* init_task -> IncMultiHeadSelfAttentionMeta ctor (inc_mha.cu:1621-1807) */
ffmi_status ffmi_attn_create(const ffmi_attn_cfg *cfg, ffmi_attn **out);
void ffmi_attn_destroy(ffmi_attn *h);
/* IncMultiHeadSelfAttention::inference_kernel_wrapper (inc_mha.h:115-119) */
ffmi_status ffmi_attn_inc(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                          void *out, ffmi_stream stream);
/* SpecIncMultiHeadSelfAttention::inference_kernel_wrapper (spec_inc_mha.h:102) */
ffmi_status ffmi_attn_spec(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                           void *out, ffmi_stream stream);
/* TreeIncMultiHeadSelfAttention::inference_kernel_wrapper (tree_inc_mha.h:104);
 * commits the previous verify batch's accepted K/V first (tree_inc...cu:583-606) */
ffmi_status ffmi_attn_tree(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                           void *out, ffmi_stream stream);
/* test hooks: raw KV cache pointers and layout ([req][head][slot][d] for K,
 * [req][head][d][slot] for V -- full precision: [req][head][slot][d] for
 * both, fp32 -- slots = max_seq_len + max_tree_tokens rounded up to 32) */
ffmi_status ffmi_attn_kv_ptrs(ffmi_attn *h, void **k, void **v, int *slots);

/* ------------------------------------------------------------------------ */
/* Linear (replaces Kernels::Linear::inference_kernel_wrapper,               */
/* linear_kernels.h:54-62; cublasGemmEx at linear_kernels.cu:510-528)        */
/* ------------------------------------------------------------------------ */
typedef enum {
  FFMI_EPI_NONE = 0,    /* Y = X W^T                                           */
  FFMI_EPI_SILU_MUL = 1 /* W = [gate;up] (2N rows): Y = silu(X Wg^T) * (X Wu^T)
                           (fuses SigmoidSiluMulti, sigmoid_silu_multi.cu:37-47) */
} ffmi_epilogue;

/* OR into `epilogue`: X is in packed activation tiles (ffmi_pack_activations)
 * instead of row-major [T][K] -- the operand-fragment order of the weights, so
 * a GEMM reads each activation fragment as one contiguous 1 KiB.  T > 64. */
#define FFMI_X_PACKED 0x10
/* OR into `epilogue`: write Y in packed activation tiles (a GEMM input of the
 * next layer; out_dim % 32 == 0). */
#define FFMI_Y_PACKED 0x20
/* OR into `epilogue`: the weights are a once-read stream (a model larger than
 * the 256 MiB Infinity Cache): their loads carry the non-temporal hint so they
 * do not evict the KV cache, activations or a small model's weights.  Long-K
 * launches of <= 64 rows then split K over 4 waves instead of 8 (faster under
 * the hint): results within the GEMM tolerance of the default policy, and
 * still independent of T within the <= 64-row regime. */
#define FFMI_W_STREAM 0x40
size_t ffmi_packed_activation_bytes(int T, int in_dim);
ffmi_status ffmi_pack_activations(const void *X, int T, int in_dim, void *X_packed,
                                  ffmi_stream stream);

/* Bytes of the MFMA-swizzled weight for an [N][K] fp16 matrix. */
size_t ffmi_linear_packed_bytes(int out_dim, int in_dim);
/* [N][K] row-major fp16 (HF layout) -> MFMA fragment order.  For
 * FFMI_EPI_SILU_MUL pass gate and up separately; they are interleaved. */
ffmi_status ffmi_linear_pack_weight(const void *W, int out_dim, int in_dim,
                                    void *W_packed, ffmi_stream stream);
ffmi_status ffmi_linear_pack_gate_up(const void *Wg, const void *Wu, int out_dim,
                                     int in_dim, void *W_packed, ffmi_stream stream);
/* Y[T][out] = X[T][in] . W^T, fp16 in/out, fp32 accumulate.  Uses a
 * library-owned split-K workspace: calls on different streams must not
 * overlap (use ffmi_linear_ws for that). */
ffmi_status ffmi_linear(const void *X, const void *W_packed, void *Y, int T,
                        int out_dim, int in_dim, int epilogue, ffmi_stream stream);
/* Linear on DT_FLOAT (linear_kernels.cu:450-582 with the full-precision
 * model's fp32 tensors): Y[T][out] = X[T][in] . W[out][in]^T, row-major fp32,
 * exact fp32 arithmetic (v_mfma_f32_16x16x4_f32: an fmaf chain per k range,
 * the k ranges of a workgroup summed in a fixed order).  in_dim % 32 == 0. */
ffmi_status ffmi_linear_f32(const float *X, const float *W, float *Y, int T, int out_dim,
                            int in_dim, ffmi_stream stream);
/* same with a caller-owned workspace of ffmi_linear_workspace_bytes() bytes */
size_t ffmi_linear_workspace_bytes(int T, int out_dim, int in_dim, int epilogue);
ffmi_status ffmi_linear_ws(const void *X, const void *W_packed, void *Y, int T,
                           int out_dim, int in_dim, int epilogue, void *workspace,
                           size_t workspace_bytes, ffmi_stream stream);

/* ------------------------------------------------------------------------ */
/* Norms (replace Kernels::RMSNorm / ResidualRMSNorm inference_kernel_wrapper, */
/* rms_norm_kernels.h:50-54, residual_rms_norm_kernels.h:53-59)              */
/* ------------------------------------------------------------------------ */
ffmi_status ffmi_rmsnorm(const void *x, const void *w, void *out, int T, int H,
                         float eps, ffmi_stream stream);
ffmi_status ffmi_residual_rmsnorm(const void *x1, const void *x2, const void *w,
                                  void *residual_out, void *out, int T, int H,
                                  float eps, ffmi_stream stream);
/* Either norm (x2 == NULL: plain RMSNorm) with flags: FFMI_Y_PACKED writes
 * `out` in packed activation tiles for a following ffmi_linear. */
ffmi_status ffmi_rmsnorm_ex(const void *x1, const void *x2, const void *w, void *residual_out,
                            void *out, int T, int H, float eps, int flags, ffmi_stream stream);

/* ------------------------------------------------------------------------ */
/* Tensor-parallel all-reduce (replaces Kernels::AllReduce::                 */
/* inference_kernel_wrapper, allreduce_kernels.h:28-31 / .cu:53-75)          */
/* ------------------------------------------------------------------------ */
typedef struct ffmi_comm ffmi_comm;
#define FFMI_UNIQUE_ID_BYTES 128
ffmi_status ffmi_comm_unique_id(void *id_out /* FFMI_UNIQUE_ID_BYTES */);
ffmi_status ffmi_comm_create(const void *id, int nranks, int rank, ffmi_comm **out);
/* In-process shard group: `nranks` (<= 8) communicators for host THREADS of
 * one process that step the TP shards of a model on one device (the
 * reference's TP-invariance tests, cpp_inference_tests.sh:203-217, on a
 * single GPU).  out[r] is rank r; destroy each with ffmi_comm_destroy. */
ffmi_status ffmi_comm_create_local(int nranks, ffmi_comm **out);
void ffmi_comm_destroy(ffmi_comm *c);
ffmi_status ffmi_allreduce(ffmi_comm *c, const void *in, void *out, size_t count,
                           int dtype, ffmi_stream stream);

/* Direct xGMI transport (replaces the NCCL data path of the same wrapper,
 * allreduce_kernels.cu:53-75, for a node's ranks).  Every rank exports one
 * exchange buffer of 4 x max_bytes (+ a 20 KiB header) as an IPC handle; the
 * caller's control plane all-gathers the handles ([nranks][64 B], rank
 * order) and every rank attaches them.  ffmi_allreduce on such a
 * communicator then runs ONE kernel per call: copy-in, a flag pushed into
 * each peer's memory, and a one-shot (every rank sums all partials) or
 * two-shot (reduce-scatter + all-gather through the peers' buffers) sum in
 * rank order -- bit-identical on every rank, graph-capturable (the epoch is
 * device-resident), never hanging (a peer silent for FFMI_PEER_TIMEOUT_S,
 * default 10, sets an error that ffmi_comm_peer_status reports).  Attach is
 * collective and ends with a checked self-test all-reduce.
 * ffmi_comm_create_peer makes a communicator with no RCCL state (the
 * transport alone: also what the multi-process tests on one GPU use). */
/* Vocab-parallel greedy / speculative tail (replaces the reference's
 * vocab-sharded lm_head + Combine, model.cc:3392-3419 / combine.cc:200-262,
 * followed by Softmax + ArgMax / ArgTopK, softmax.cu:262-288, argmax.cu:62-100,
 * arg_topk.cu:339-448).  Each rank holds logits [T][Vl] for vocabulary ids
 * [rank*Vl, (rank+1)*Vl); every rank gets the GLOBAL k best ids (k <= 4) and
 * their fp16 softmax probabilities, identical to ffmi_arg_topk on the
 * gathered [T][P*Vl] logits (same max, same float rounding of the same
 * double sum, lowest index among equal fp16 probabilities).  Three
 * exchanges of (P x T x 32 B) records over the communicator; `scratch` holds
 * ffmi_vocab_shard_scratch_bytes(P, T) device bytes. */
size_t ffmi_vocab_shard_scratch_bytes(int nranks, int T);
ffmi_status ffmi_vocab_shard_topk(ffmi_comm *c, const void *logits, int T, int Vl, int k,
                                  int32_t *ids, float *probs, void *scratch, ffmi_stream stream);

#define FFMI_PEER_HANDLE_BYTES 64
ffmi_status ffmi_comm_create_peer(int nranks, int rank, ffmi_comm **out);
ffmi_status ffmi_comm_peer_export(ffmi_comm *c, size_t max_bytes,
                                  void *handle_out /* FFMI_PEER_HANDLE_BYTES */);
ffmi_status ffmi_comm_peer_attach(ffmi_comm *c, const void *handles /* [nranks][64] */);
/* All-gather of equal-size HOST byte blocks over the communicator (any of its
 * transports): all[r * bytes ...] = rank r's block, on every rank.  Blocking;
 * for control data (the distributed SSMs' results), not the hot path. */
ffmi_status ffmi_comm_allgather(ffmi_comm *c, const void *mine, size_t bytes, void *all);
ffmi_status ffmi_comm_peer_status(ffmi_comm *c);
/* Stop using the transport (RCCL again): for a control plane that saw some
 * rank fail its attach -- every rank must take the same transport. */
ffmi_status ffmi_comm_peer_detach(ffmi_comm *c);
/* All-reduce fused with the residual RMSNorm after it (the reference's
 * AllReduce -> ResidualRMSNorm pair of every TP layer, model.cc:3421-3445,
 * allreduce_kernels.cu:53-75 + residual_rms_norm_kernels.cu:98-131), ONE
 * kernel over an attached xGMI transport: `in` is this rank's f16 partial of
 * columns [col0, H) of the [T][H] sum ([T][H - col0], contiguous); columns
 * [0, col0) of the sum are read from `prev` ([T][H], e.g. an earlier
 * ffmi_allreduce of those columns; NULL when col0 == 0).  Then, as
 * ffmi_rmsnorm_ex(residual, sum, w, residual, out, ..., flags):
 * residual = half(residual + sum) in place and out = RMSNorm(residual) * w
 * (FFMI_Y_PACKED: packed activation tiles) -- bit-identical to the unfused
 * pair.  When the transport takes T*H*2 bytes in two shots (> 2 ranks, above
 * its threshold), rank r normalises only rows [T*r/N, T*(r+1)/N) and gathers
 * every other rank's rows of `out`: `out` is complete on every rank,
 * `residual` is updated on this rank's rows only.  rows_out (optional, [2])
 * receives the updated row range. */
ffmi_status ffmi_allreduce_rmsnorm(ffmi_comm *c, const void *in, int T, int H, int col0,
                                   const void *prev, void *residual, const void *w, float eps,
                                   void *out, int flags, int *rows_out, ffmi_stream stream);

/* ------------------------------------------------------------------------ */
/* Auxiliary ops on the LLaMA greedy path                                    */
/* ------------------------------------------------------------------------ */
/* embed_forward_no_aggr (embedding_kernels.cu:233-244): ids from the batch */
ffmi_status ffmi_embedding(const ffmi_batch_dev *b, const void *table, void *out,
                           int H, ffmi_stream stream);
/* SigmoidSiluMulti standalone (sigmoid_silu_multi.cu:37-47) */
ffmi_status ffmi_silu_mul(const void *a, const void *b, void *out, size_t n,
                          ffmi_stream stream);
/* softmax (fp16 output, softmax.cu:262-288) + ArgMax (argmax.cu:62-100):
 * ids[t] = lowest index of max fp16(softmax(logits[t]))               */
ffmi_status ffmi_argmax(const void *logits, int T, int V, int32_t *ids,
                        float *probs, ffmi_stream stream);
/* softmax + ArgTopK (arg_topk.cu:339-448), k <= 4, sorted, lower index on ties */
ffmi_status ffmi_arg_topk(const void *logits, int T, int V, int k, int32_t *ids,
                          float *probs, ffmi_stream stream);
/* the same with a device workspace: rows of a small batch (the SSM's beam
 * steps, decode) are split over several workgroups that each sum 1/G of the
 * row's exp terms, identical results.  `workspace` holds
 * ffmi_arg_topk_workspace_bytes(T) bytes, zero-filled by the caller once
 * (the call leaves it zeroed); one workspace per stream in flight.  NULL or
 * too small: the one-workgroup-per-row form (ffmi_arg_topk). */
size_t ffmi_arg_topk_workspace_bytes(int T);
ffmi_status ffmi_arg_topk_ws(const void *logits, int T, int V, int k, int32_t *ids,
                             float *probs, void *workspace, size_t workspace_bytes,
                             ffmi_stream stream);
/* DT_FLOAT twins (--use-full-precision, kernels/f32.hip): RMSNorm /
 * ResidualRMSNorm (sum of squares in fp64, rounded once; fp32 residual add),
 * SigmoidSiluMulti, softmax + arg-top-k on fp32 probabilities (k <= 4, lowest
 * index among equal probabilities; k = 1 is the argmax) */
ffmi_status ffmi_rmsnorm_f32(const float *x, const float *w, float *out, int T, int H, float eps,
                             ffmi_stream stream);
ffmi_status ffmi_residual_rmsnorm_f32(const float *x1, const float *x2, const float *w,
                                      float *residual_out, float *out, int T, int H, float eps,
                                      ffmi_stream stream);
ffmi_status ffmi_silu_mul_f32(const float *a, const float *b, float *out, size_t n,
                              ffmi_stream stream);
ffmi_status ffmi_arg_topk_f32(const float *logits, int T, int V, int k, int32_t *ids,
                              float *probs, ffmi_stream stream);
/* seeded synthetic weights, identical to oracle/orc_gen_weight then fp16.
 * kind 0: matrix (uniform, std 0.02); 1: norm weight (1 +- 0.1);
 * FFMI_WKIND_DEPTH | L: o_proj / down_proj of an L-layer model under the
 * depth-scaled init (std 0.02 / sqrt(2L)) */
#define FFMI_WKIND_DEPTH 0x10000
ffmi_status ffmi_fill_weight(void *dst_f16, size_t n, const char *name,
                             uint64_t seed, int kind, ffmi_stream stream);

/* ------------------------------------------------------------------------ */
/* Serving runtime (C++ host side above the kernels; RequestManager API)     */
/* ------------------------------------------------------------------------ */
typedef struct {
  int num_layers, vocab_size, num_heads, num_kv_heads, hidden, intermediate;
  float rms_eps, rope_theta;
  /* llama3 RoPE scaling (llama.h:53-65), as in ffmi_attn_cfg */
  int rope_llama3;
  float rope_factor, rope_low_freq_factor, rope_high_freq_factor;
  int rope_original_max_pos;
} ffmi_llama_config;

typedef enum {
  FFMI_MODEL_INC = 0,  /* INC_DECODING_MODE  */
  FFMI_MODEL_BEAM = 1, /* BEAM_SEARCH_MODE (SSM) */
  FFMI_MODEL_TREE = 2  /* TREE_VERIFY_MODE (LLM) */
} ffmi_model_mode;

typedef struct {
  int mode;                  /* ffmi_model_mode                                */
  int tp_rank, tp_size;      /* tensor parallelism (heads / FFN columns)       */
  ffmi_comm *comm;           /* communicator of tp_size ranks: RCCL, xGMI
                              * transport or local group (NULL when tp_size == 1).
                              * A ONE-rank communicator without RCCL state or
                              * transport with tp_size > 1 runs shard tp_rank
                              * alone, every all-reduce the identity: the
                              * per-rank compute measurement of
                              * scripts/tp_shard_bench.py (tokens meaningless) */
  int max_requests;          /* max_requests_per_batch                         */
  int max_tokens;            /* max tokens per batch (verify capacity for TREE) */
  int max_seq_len;           /* max_sequence_length                            */
  int max_tree_tokens;       /* max_spec_tree_token_num                        */
  uint64_t weight_seed;      /* synthetic weights (orc_gen_weight spec)        */
  int use_graphs;            /* capture per-shape hipGraphs (0/1)              */
  /* Checkpoint in the reference's format (file_loader.cc:217-361,
   * serve/models/llama.py convert_hf_model): one raw fp16 or fp32 file per
   * tensor, named as the HF parameter without "model." ("embed_tokens.weight",
   * "layers.0.self_attn.q_proj.weight", ..., "norm.weight", "lm_head.weight").
   * K/V projections of GQA checkpoints are replicated to every query head as
   * the reference does (file_loader.cc:292-302).  NULL: synthetic weights. */
  const char *weights_folder;
  /* synthetic weights (no weights_folder), oracle.h orc_model_create_ex:
   * 0: every matrix uniform with std 0.02 (the bench's model);
   * 1: depth-scaled -- o_proj / down_proj at std 0.02 / sqrt(2L);
   * 2: token chain -- embeddings x 128 (x 2 per doubling of the residual
   *    noise sqrt(L (H + 2F)) over LLaMA-7B's; 65B: x 512) and lm_head = the
   *    embedding rows permuted (v -> (7919 v + 17) mod vocab): a peaked model whose greedy
   *    picks lead by margins far above fp16 rounding noise (parity tests of
   *    the reference's literal token bars; SpecInfer with full acceptance) */
  int weight_init;
  /* 1: full precision -- the reference's --use-full-precision
   * (spec_infer.cc:102, incr_decoding.cc:77): weights, activations, KV cache
   * and softmax in fp32 (runtime/llama_f32.cpp, kernels/f32.hip); lm_head
   * replicated under TP.  0: the fp16 model (the measured path). */
  int full_precision;
} ffmi_model_opts;

typedef struct ffmi_model ffmi_model;
ffmi_status ffmi_model_create(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                              ffmi_model **out);
void ffmi_model_destroy(ffmi_model *m);
/* Per-op device timing with HIP events on the model's stream (the
 * reference's --profiling, model.cc:4548-4550).  level 0: off; 1: sampled
 * (layers 0 and L/2 of every 4th step with <= 256 tokens -- FFMI_PROF_EVERY
 * sets the stride; sampled steps run eager, the others replay graphs);
 * 2: every op of every step. */
typedef struct {
  char name[32];
  long launches;
  double total_ms;
  double bytes; /* algorithmic bytes (weights + activations read/written)  */
  double flops;
} ffmi_op_stat;
ffmi_status ffmi_model_set_profiling(ffmi_model *m, int level);
int ffmi_model_op_stats(ffmi_model *m, ffmi_op_stat *out, int cap);
/* Tensor capture for alignment checks (the reference's --inference-debugging
 * per-layer dumps, operator.h:271-360, compared by
 * tests/inference/inference_alignment_test.py).  While enabled, steps run
 * eager (no graph replay) and the LAST step's tensors are kept on the device:
 *   FFMI_DBG_HIDDEN, layer l in [0, num_layers): the residual stream after
 *     decoder layer l (HF hidden_states[l + 1]); layer == num_layers: the
 *     final RMSNorm output (HF's last hidden state);
 *   FFMI_DBG_LOGITS: the lm_head output [T][V_l] (before softmax; V_l = this
 *     rank's vocab shard when the lm_head is vocab-sharded, else vocab);
 * and per op of decoder layer l, the tensors the reference's alignment test
 * compares (inference_alignment_test.py:20-370: embedding, the two norms,
 * the QKV projection with its shard re-assembly, attention output, MLP):
 *   FFMI_DBG_EMBED      [T][H]     embedding rows (layer 0 only)
 *   FFMI_DBG_ATTN_NORM  [T][H]     input_layernorm output
 *   FFMI_DBG_QKV        [T][3*H_l] qkv_proj output before RoPE, [Q_s|K_s|V_s]
 *   FFMI_DBG_ATTN_OUT   [T][H_l]   attention output (o_proj input)
 *   FFMI_DBG_O_PROJ     [T][H]     o_proj output (after the all-reduce)
 *   FFMI_DBG_FFN_NORM   [T][H]     post_attention_layernorm output
 *   FFMI_DBG_MLP_ACT    [T][F_l]   SiLU(gate) * up (down_proj input)
 *   FFMI_DBG_DOWN       [T][H]     down_proj output (after the all-reduce)
 * H_l / F_l are this rank's shard widths.  ffmi_model_debug_tensor copies one
 * as fp32 rows [T][width] into `out` (capacity `cap` floats) and returns T,
 * or -1 (nothing captured / bad argument / too small);
 * ffmi_model_debug_width returns the width (or -1). */
#define FFMI_DBG_HIDDEN 0
#define FFMI_DBG_LOGITS 1
#define FFMI_DBG_ATTN_NORM 2
#define FFMI_DBG_QKV 3
#define FFMI_DBG_ATTN_OUT 4
#define FFMI_DBG_O_PROJ 5
#define FFMI_DBG_FFN_NORM 6
#define FFMI_DBG_MLP_ACT 7
#define FFMI_DBG_DOWN 8
#define FFMI_DBG_EMBED 9
ffmi_status ffmi_model_set_debug(ffmi_model *m, int enable);
long ffmi_model_debug_tensor(ffmi_model *m, int which, int layer, float *out, long cap);
long ffmi_model_debug_width(ffmi_model *m, int which);
/* Negative-control fault injection (tests only; never set in serving): the
 * parity tests must FAIL on a model with a deliberate bug.
 *   FFMI_FAULT_ROPE_POS, layer, arg: that layer's RoPE rotates tokens at
 *     positions >= arg by position + 1 (an off-by-one position in one layer's
 *     decode phase, apply_rotary_embedding_hf inc_multihead_self_attention.cu:
 *     664-738 with a wrong abs_depth); layer -1: every layer; arg < 0
 *     clears it.
 *   FFMI_FAULT_RESID_ROUND (layer, arg ignored; fp16 models, process-wide):
 *     the residual RMSNorm kernel squares the UNROUNDED fp32 residual sum
 *     x1 + x2 where residual_rms_norm_kernels.cu:112-114 rounds it to half
 *     first -- a rounding-point bug that moves the normalised outputs by at
 *     most an ulp (the norms folded into the decode GEMMs are not faulted).
 *   FFMI_FAULT_TP_HEAD_SWAP (layer; -1: every layer; fp16 models): this
 *     model's qkv weights with the Q rows of its local heads 0 and 1
 *     exchanged -- a head-offset bug in one rank's shard (file_loader.cc:
 *     286-303 places head h's rows at h * head_dim of the rank's block).
 *   FFMI_FAULT_TP_AR_DROP (layer, arg: 0 = the all-reduce after o_proj, 1 =
 *     after down_proj; TP > 1, fp16 models): this rank's contribution to that
 *     all-reduce is zeroed (a partial sum lost, allreduce.cc:291-331).
 *   FFMI_FAULT_NONE clears every fault. */
#define FFMI_FAULT_NONE 0
#define FFMI_FAULT_ROPE_POS 1
#define FFMI_FAULT_RESID_ROUND 2
#define FFMI_FAULT_TP_HEAD_SWAP 3
#define FFMI_FAULT_TP_AR_DROP 4
ffmi_status ffmi_model_debug_fault(ffmi_model *m, int kind, int layer, int arg);
/* select the HIP device of the calling thread (one process per GPU) */
ffmi_status ffmi_set_device(int device);

typedef struct ffmi_rm ffmi_rm;
typedef struct {
  int max_requests_per_batch;
  int max_tokens_per_batch;
  int max_spec_tree_token_num;
  int max_sequence_length;
  int bos_token_id;        /* <0: none                                       */
  const int *eos_token_ids;
  int num_eos;
  const int *spec_tree_width; /* push_spec_infer_tree_width sequence         */
  int num_tree_width;
  int verbose;
  int spec_extensions;     /* FFMI_SPEC_EXT_* bits (ABI 0.3); 0: the reference's limits */
} ffmi_rm_config;
/* Flagged SpecInfer extensions beyond what the reference runs (BASELINE
 * configs C "tree width=4" and E "4x SSMs"):
 *   FFMI_SPEC_EXT_WIDTH4: tree widths and branches per layer up to 4 (the
 *     reference's MAX_BEAM_WIDTH / MAX_SPECULATIVE_TREE_BRANCHES are 3,
 *     batch_config.h:196,200, request_manager.cc:168-171); size
 *     max_spec_tree_token_num for the tree (27 tokens for widths (1,1,4));
 *   FFMI_SPEC_EXT_MULTI_SSM: more than one registered SSM; their token trees
 *     are united by path (merge_dfs_trees, request_manager.cc:2817-2878, whose
 *     reference form asserts a single SSM) and cut to max_spec_tree_token_num
 *     (<= 64) nodes in layer order. */
#define FFMI_SPEC_EXT_WIDTH4 1
#define FFMI_SPEC_EXT_MULTI_SSM 2

ffmi_status ffmi_rm_create(const ffmi_rm_config *cfg, ffmi_rm **out);
void ffmi_rm_destroy(ffmi_rm *rm);
ffmi_status ffmi_rm_register_ssm(ffmi_rm *rm, ffmi_model *ssm);
/* Config E's SSMs placed over the ranks of a TP group (the reference builds
 * each SSM as its own TP = 1 model, spec_infer.cc:381-435): SSM s runs on
 * rank s % nranks only.  Every rank registers the SSMs in the same order --
 * its own with ffmi_rm_register_ssm, the others with
 * ffmi_rm_register_remote_ssm -- and sets an exchange.  After its SSMs' beam
 * steps a rank contributes their per-step results and replays the other
 * ranks' SSMs' bookkeeping on theirs, so every rank merges the identical token
 * trees (FFMI_SPEC_EXT_MULTI_SSM).  The exchange is an all-gather of equal-
 * size host byte blocks, fn(ctx, mine, bytes, all[nranks][bytes]) returning
 * 0 on success; ffmi_rm_set_ssm_exchange_comm uses ffmi_comm_allgather. */
typedef int (*ffmi_allgather_fn)(void *ctx, const void *mine, size_t bytes, void *all);
ffmi_status ffmi_rm_register_remote_ssm(ffmi_rm *rm);
ffmi_status ffmi_rm_set_ssm_exchange(ffmi_rm *rm, int nranks, int rank, ffmi_allgather_fn fn,
                                     void *ctx);
ffmi_status ffmi_rm_set_ssm_exchange_comm(ffmi_rm *rm, ffmi_comm *comm);
/* RequestManager::register_output_filepath (request_manager.cc:246-249):
 * each completed request is appended in the reference's record format
 * (incr decoding :813-840, SpecInfer :1303-1330).  NULL or "" turns it off. */
ffmi_status ffmi_rm_register_output_filepath(ffmi_rm *rm, const char *path);
/* The text written after "token IDs:" is the reference's
 * tokenizer_->Decode(tokens) (request_manager.cc:786-789): the runtime calls
 * fn(ids, n, NULL, 0, ctx) for the byte length, then fn(ids, n, buf, len, ctx).
 * NULL fn: empty text (no tokenizer). */
typedef int (*ffmi_detokenize_fn)(const int *ids, int n, char *buf, int cap, void *ctx);
ffmi_status ffmi_rm_register_detokenizer(ffmi_rm *rm, ffmi_detokenize_fn fn, void *ctx);
/* The tokenizer is the old LLaMA SentencePiece model (the reference's
 * old_llama_tokenizer, request_manager.cc:200-211): SentencePiece drops BOS
 * when decoding, so the text of a request registered with
 * add_special_tokens whose tokens start with BOS gets a "<s> " prefix
 * (:776-781). */
ffmi_status ffmi_rm_set_old_llama_tokenizer(ffmi_rm *rm, int enable);
/* Request: prompt token ids (BOS is prepended when bos_token_id >= 0 and
 * add_special_tokens), max_length / max_new_tokens as in Request
 * (request_manager.cc:334-441).  Returns guid (> 0) or 0 on rejection. */
int64_t ffmi_rm_register_request(ffmi_rm *rm, const int *prompt, int n_prompt,
                                 int max_length, int max_new_tokens,
                                 int add_special_tokens);
/* Run the serve loop until every registered request completes
 * (serve_incr_decoding / serve_spec_infer, request_manager.cc:3012-3173). */
ffmi_status ffmi_rm_serve_incr_decoding(ffmi_rm *rm, ffmi_model *llm);
ffmi_status ffmi_rm_serve_spec_infer(ffmi_rm *rm, ffmi_model *llm);
/* GenerationResult.output_tokens; returns count (or needed size) */
int ffmi_rm_get_output(ffmi_rm *rm, int64_t guid, int *tokens, int cap);
typedef struct {
  int llm_decoding_steps, ssm_decoding_steps;
  double start_us, finish_us, registration_us, first_token_us;
  int input_len, output_len;
} ffmi_profile;
ffmi_status ffmi_rm_get_profile(ffmi_rm *rm, int64_t guid, ffmi_profile *p);
/* aggregate counters of the last serve call */
typedef struct {
  long llm_steps, ssm_steps, tokens_committed, tree_tokens_verified;
  long request_verifies; /* (request, verify step) pairs that committed tokens */
  double wall_us;
  double llm_us, ssm_us; /* wall time inside LLM / SSM steps; the rest is host scheduling */
  long ssm_phases_chained; /* speculation phases run as chained beam steps (FFMI_SSM_CHAIN) */
  double ssm_exchange_us;  /* distributed SSMs: result exchange + remote bookkeeping */
} ffmi_serve_stats;
ffmi_status ffmi_rm_get_stats(ffmi_rm *rm, ffmi_serve_stats *s);



/* Test hooks: the residual RMSNorm folded into the decode GEMMs (T <= 32,
 * the path of LLaMA-7B decode steps; residual_rms_norm_kernels.cu:98-131
 * split over the GEMMs around it).  Producer: residual[T][out] += round(X .
 * W^T) in place (fp16 add) and ss_out[T][out/16] = per 16-column tile sums of
 * squares of the new residual.  Consumer: Y = (rmsnorm(residual) from ss_in
 * [T][in/16], weight norm_w, eps) . W^T, with the epilogue (FFMI_EPI_NONE /
 * FFMI_EPI_SILU_MUL, row-major).  Row-major fp16, no split-K. */
ffmi_status ffmi_debug_fused_residual_linear(const void *X, const void *W_packed, void *residual,
                                             float *ss_out, int T, int out_dim, int in_dim,
                                             ffmi_stream stream);
ffmi_status ffmi_debug_fused_norm_linear(const void *residual, const float *ss_in,
                                         const void *norm_w, float eps, const void *W_packed,
                                         void *Y, int T, int out_dim, int in_dim, int epilogue,
                                         ffmi_stream stream);

/* Diagnostics: with FFMI_GEMM_STAMP set in the environment, M-split GEMM
 * launches record per-wave timestamps; copies the last launch's records
 * ({start, prologue done, k-loop done, end} at 100 MHz, HW_ID, XCC_ID) and
 * returns the number of waves (<= max_waves). */
long ffmi_debug_gemm_stamps(long long *dst, long max_waves);
/* Diagnostics: per-wave timeline of the last verify-size attention launch when
 * FFMI_ATTN_STAMP=1 (12 int64 per wave: start, after prologue, before the key
 * loop, after it, after the merge barrier, end, then [one-launch path] after
 * the commits, after the KV update, after its barrier, after the V^T stores
 * [100 MHz]; HW_ID, chunks). */
long ffmi_debug_attn_stamps(long long *dst, long max_waves);
/* FFMI_MARKERS=1 diagnostics: realtime-clock markers (100 MHz) enqueued
 * between the kernels of the model's last layer; copies up to n (<= 64). */
long ffmi_debug_markers(long long *dst, long n);

const char *ffmi_status_str(ffmi_status s);
/* message + file:line of the last failing check on this process */
const char *ffmi_last_error(void);
/* "ffmi 0.3 (gfx950)": 0.2 appended full_precision to ffmi_attn_cfg and
 * ffmi_model_opts (struct sizes changed) and added the *_f32 entry points;
 * 0.3 appended spec_extensions to ffmi_rm_config */
const char *ffmi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FFMI_H_ */
