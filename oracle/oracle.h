/*
 * oracle.h -- CPU restatement of the FlexFlow SpecInfer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * (or the timed CPU baseline).  The product path (libffmi.so) never links,
 * loads or calls anything in this directory.
 *
 * Every function restates the numerics of the reference kernel it names
 * (file:line into hugolatendresse/FlexFlow @ 2025-01-17).  Tensors are passed
 * as float arrays whose values are fp16-representable when `fp16 != 0`; the
 * function then rounds to fp16 at exactly the points where the reference
 * stores a half (round-to-nearest-even).  With `fp16 == 0` (the reference's
 * --use-full-precision mode) nothing is rounded.
 *
 * Parity pin: tests/golden/ holds fixtures produced by HF transformers
 * LlamaForCausalLM (the reference's own alignment oracle,
 * tests/inference/huggingface_inference.py) on identical seeded weights;
 * tests/test_oracle_golden.py checks this oracle against them.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int num_layers;
  int vocab_size;
  int num_heads;
  int num_kv_heads;
  int hidden;
  int intermediate;
  float rms_eps;
  float rope_theta;
} orc_config;

/* `fp16` argument values: 0 = full precision (--use-full-precision), 1 =
 * half storage with fp32 accumulation (the MI355X path's semantics), 2 =
 * ORC_REF16: half storage AND the reference's half compute type in the dense
 * and prompt-attention GEMMs (linear_kernels.cu:493-528,
 * inc_multihead_self_attention.cu:98-366). */
#define ORC_REF16 2

/* ---- fp16 helpers (RNE) ---- */
uint16_t orc_f2h(float f);
float orc_h2f(uint16_t h);
float orc_round16(float f);

/* ---- synthetic weights (shared spec with the GPU generator) ----
 * value i of tensor `name`: u = top-24 bits of splitmix64(seed ^ fnv1a64(name),
 * i) / 2^24; w = center + (2u-1)*amp, all in fp32, no FMA contraction.
 * kind 0: matrix / embedding (center 0, amp 0.02*sqrt(3)); kind 1: norm
 * weight (center 1, amp 0.1); kind ORC_WKIND_DEPTH | L: o_proj / down_proj of
 * an L-layer model in the depth-scaled init (amp 0.02*sqrt(3) / sqrt(2L)). */
#define ORC_WKIND_DEPTH 0x10000
void orc_gen_weight(const char *name, uint64_t seed, int kind, size_t n,
                    float *out);
float orc_weight_amp(int kind);
/* the same stream as a [n / cols][cols] tensor whose row r is row
 * (r * pa + pb) mod (n / cols) of the stream (cols == 0: no permutation),
 * amplitude times `scale` */
void orc_gen_weight_rows(const char *name, uint64_t seed, int kind, size_t n, int cols,
                         uint64_t pa, uint64_t pb, float scale, float *out);
/* token-chain init (weight_init 2): the lm_head row permutation
 * v -> (v * ORC_CHAIN_A + ORC_CHAIN_B) mod vocab (7919 is prime, so a
 * bijection for every vocabulary it does not divide) and the embedding scale:
 * 128, doubled while the random layers' residual noise (grows like
 * sqrt(L * (H + 2F))) outgrows LLaMA-7B's by the same factor -- the input
 * token's share of the final residual, and so the chain's logit margin,
 * stays at least 7B's (65B: 512).  Powers of two keep the fp16 scaling
 * exact; the GPU init computes the same (llama_gpu.cpp) */
float orc_chain_embed_scale(int num_layers, int hidden, int intermediate);
#define ORC_CHAIN_A 7919u
#define ORC_CHAIN_B 17u

/* ---- kernel-level restatements ---- */
/* Linear: Y[T][N] = X[T][K] . W[N][K]^T (linear_kernels.cu:450-582; fp32
 * accumulate -- the reference's fp16 compute type is a documented deviation) */
void orc_linear(const float *X, const float *W, float *Y, int T, int N, int K,
                int fp16);
/* MMA block (products summed in fp32 per step) of the ORC_REF16 half
 * accumulator model; default 16 */
void orc_set_ref_block(int k);
/* fp32 summation order of orc_linear (tests only): 0 = dot8 (default),
 * 1 = dot16 -- the same sums in another order, to measure how far ANY
 * reordering moves the model (the noise floor of GPU-vs-oracle drift) */
void orc_set_dot_variant(int v);
/* Prompt-phase attention of one head (inc_multihead_self_attention.cu:98-366)
 * with the reference's half compute type: q [T_new][d] at positions
 * start..start+T_new-1, K/V [start+T_new][d], out [T_new][d]. */
void orc_attention_prompt_ref16(const float *q, const float *K, const float *V, int T_new,
                                int start, int d, float *out);
/* RMSNorm (rms_norm_kernels.cu:97-124) */
void orc_rmsnorm(const float *X, const float *w, float *out, int T, int H,
                 float eps, int fp16);
/* ResidualRMSNorm (residual_rms_norm_kernels.cu:98-131) */
void orc_residual_rmsnorm(const float *X1, const float *X2, const float *w,
                          float *res_out, float *out, int T, int H, float eps,
                          int fp16);
/* SigmoidSiluMulti (sigmoid_silu_multi.cu:37-47) */
void orc_silu_mul(const float *A, const float *B, float *out, size_t n,
                  int fp16);
/* HF rotate-half RoPE on one head vector of size d at position pos
 * (inc_multihead_self_attention.cu:664-738) */
void orc_rope_head(float *x, int d, int pos, float theta, int fp16);
/* cos/sin table used by both the oracle and the GPU: tab[(pos*(d/2)+i)*2+{0,1}] */
void orc_rope_table(float *tab, int max_pos, int d, float theta);
void orc_rope_table_llama3(float *tab, int max_pos, int d, float theta, int llama3, float factor,
                           float low_ff, float high_ff, int orig_max);
/* One query row against `n_keys` key/value rows (head_dim d) with a
 * visibility vector (1 = visible).  Softmax with __expf and 1/(sum+1e-6) as
 * in compute_attention_kernel_generation_kernel (inc_..._attention.cu:372-623)
 * and the tree/spec fused kernels (tree_inc...cu:35-333). */
void orc_attention_row(const float *q, const float *K, const float *V,
                       const uint8_t *visible, int n_keys, int d, float scale,
                       float *out, int fp16);
/* argmax(softmax(logits)) with lowest-index ties (llama.cc:292-293,
 * argmax.cu:62-100); softmax output stored as fp16 when fp16 != 0 */
void orc_softmax_argmax(const float *logits, int T, int V, int fp16,
                        int *out_ids, float *out_prob);
/* ArgTopK over softmax (arg_topk.cu:339-448): sorted descending, ties ->
 * lower index */
void orc_softmax_topk(const float *logits, int T, int V, int k, int fp16,
                      int *out_ids, float *out_probs);

/* ---- model-level restatement (LLaMA, llama.cc:23-317) ---- */
typedef struct orc_model orc_model;
orc_model *orc_model_create(const orc_config *cfg, uint64_t seed, int fp16,
                            int max_requests, int max_seq);
/* weight_init 0: every matrix at amp 0.02*sqrt(3) (the bench's model);
 * 1: depth-scaled -- o_proj / down_proj at 1/sqrt(2L) of that (a residual
 * stream that does not amplify per-layer rounding; ffmi_model_opts);
 * 2: token chain -- embeddings x orc_chain_embed_scale() and lm_head = the
 * embedding rows permuted (ORC_CHAIN_A/B): a peaked model whose greedy picks
 * lead by margins far above fp16 rounding noise */
orc_model *orc_model_create_ex(const orc_config *cfg, uint64_t seed, int fp16,
                               int max_requests, int max_seq, int weight_init);
void orc_model_destroy(orc_model *m);
void orc_model_reset(orc_model *m, int req);
/* Feed T tokens of request `req` at positions start_pos..start_pos+T-1
 * (causal, KV cache kept per request).  logits: [T][V] or NULL. */
int orc_model_forward(orc_model *m, int req, const int *tokens, int T,
                      int start_pos, float *logits);
/* as orc_model_forward; prompt_phase != 0 in ORC_REF16 mode runs the
 * attention through the reference's prompt path (cuBLAS/cuDNN half
 * semantics) instead of the generation kernel's */
int orc_model_forward_ex(orc_model *m, int req, const int *tokens, int T,
                         int start_pos, float *logits, int prompt_phase);
/* Batched decode step for the CPU baseline: token t belongs to request
 * reqs[t] at position pos[t] (one token per request, caches as above); the
 * dense layers read every weight once for the whole batch. */
int orc_model_decode_batch(orc_model *m, const int *reqs, const int *tokens,
                           const int *pos, int T, float *logits);
/* R requests' token blocks in one step: block r = counts[r] tokens of request
 * reqs[r] at positions start[r].., causal inside the block (the CPU port of a
 * tree-verify / SSM beam step for the cpu_baseline; dense layers batched over
 * all tokens).  logits [sum counts][V] or NULL. */
int orc_model_forward_multi(orc_model *m, int R, const int *reqs, const int *counts,
                            const int *start, const int *tokens, float *logits);
/* hidden state (residual stream before final norm) after layer `layer` of
 * the last forward call, [T][H]; layer == num_layers gives final-normed. */
int orc_model_get_hidden(orc_model *m, int layer, float *out);
/* per-op tensor of the last forward (kind = FFMI_DBG_* of include/ffmi.h,
 * 2..9: attn_norm, qkv before RoPE [Q|K|V], attn_out, o_proj, ffn_norm,
 * mlp_act, down, embed (layer 0)); returns T or -1; out NULL: T only */
int orc_model_get_op(orc_model *m, int kind, int layer, float *out);
/* greedy incremental decoding of one request: writes n_new tokens */
int orc_model_greedy(orc_model *m, int req, const int *prompt, int n_prompt,
                     int n_new, int *out_tokens);
/* weights as packed fp16 (for uploading the identical model to the GPU in
 * tests): tensor by HF name, returns element count or -1 */
long orc_model_weight(orc_model *m, const char *name, float *out);

/* thread count used by the OpenMP loops (for the cpu_baseline report) */
int orc_num_threads(void);

#ifdef __cplusplus
}
#endif
