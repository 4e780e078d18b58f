// llama_f32.cpp -- LLaMA in full precision: the reference's
// --use-full-precision (inference/spec_infer/spec_infer.cc:102,
// incr_decoding.cc:77: the model graph of inference/models/llama.cc:23-317
// built with DT_FLOAT, so weights, activations, KV cache and softmax are
// fp32).  Same graph, modes and tensor parallelism as llama_gpu.cpp
// (model.cc:3392-3613: qkv / gate / up column-parallel, o / down
// row-parallel + sum all-reduce), on the fp32 kernels of kernels/f32.hip.
// The lm_head stays replicated per rank (every rank computes the same logits
// from the same all-reduced hidden state and picks the same tokens).
// This path exists for the reference's exact-diff invariants, which it runs
// in full precision (tests/inference/cpp_inference_tests.sh:183-217): the
// fp32 rounding noise is ~1e-7, so token-level equality binds even on the
// random-weight bench model.  It is not the measured path.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "model.h"

namespace ffmi {

namespace {

struct LayerF {
  float *in_norm = nullptr, *post_norm = nullptr;
  float *wqkv = nullptr, *wo = nullptr, *wgu = nullptr, *wd = nullptr;  // row-major [N][K]
  ffmi_attn *attn = nullptr;  // DT_FLOAT handle: fp32 KV cache, TREE staging, RoPE table
};

struct LlamaF32 : public ffmi_model {
  ffmi_llama_config c{};
  ffmi_model_opts o{};
  int token_capacity() const override { return o.max_tokens; }
  bool uses_collectives() const override { return o.tp_size > 1; }
  std::string weights_folder;
  int H = 0, F = 0, V = 0, d = 0, heads_l = 0, Hl = 0, Fl = 0, P = 1, slots = 0, Tm = 0;
  hipStream_t stream = nullptr;
  std::vector<LayerF> layers;
  float *embed = nullptr, *final_norm = nullptr, *lm = nullptr;
  float *res = nullptr, *h = nullptr, *qkv = nullptr, *att = nullptr,
        *proj = nullptr, *gu = nullptr, *mlp = nullptr, *logits = nullptr;
  int32_t *res_d = nullptr;  // [ids (T*k) | probs (T*k)] of a step
  int32_t *res_h = nullptr;  // pinned copy
  ffmi_batch_dev *batch = nullptr;
  PackedStep ps;
  std::vector<void *> allocs;
  std::map<std::tuple<int, int, int, int, size_t>, hipGraphExec_t> graphs;
  bool use_graphs = getenv("FFMI_NO_GRAPHS") == nullptr;
  int dbg = 0, dbg_T = -1;

  ~LlamaF32() override {
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto &kv : graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto &L : layers) ffmi_attn_destroy(L.attn);
    for (void *p : allocs) (void)hipFree(p);
    if (res_h) (void)hipHostFree(res_h);
    ffmi_batch_destroy(batch);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // FFMI_FAULT_ROPE_POS / FFMI_FAULT_NONE on the DT_FLOAT handles' RoPE tables
  // (the negative control of the full-precision bars; include/ffmi.h)
  ffmi_status debug_fault(int kind, int layer, int arg) override {
    if (stream) FFMI_HIP(hipStreamSynchronize(stream));
    FFMI_CHECK(kind == FFMI_FAULT_NONE ||
                   (kind == FFMI_FAULT_ROPE_POS && layer >= -1 && layer < c.num_layers),
               FFMI_ERR_INVALID);
    for (int l = 0; l < c.num_layers; ++l)
      if (kind == FFMI_FAULT_NONE || layer < 0 || l == layer) {
        ffmi_status st = ffmi::attn_rope_fault(layers[l].attn, kind == FFMI_FAULT_NONE ? -1 : arg);
        if (st != FFMI_OK) return st;
      }
    return FFMI_OK;
  }

  template <typename T>
  ffmi_status alloc(T **p, size_t elems) {
    if (hipMalloc((void **)p, elems * sizeof(T)) != hipSuccess) {
      ffmi_set_last_error("model alloc", __FILE__, __LINE__);
      return FFMI_ERR_OOM;
    }
    allocs.push_back(*p);
    return FFMI_OK;
  }

  // One tensor of a reference-format checkpoint (file_loader.cc:363-389), fp32
  // or fp16 files (full precision loads the fp32 files; half files widen
  // exactly), GQA K/V replicated per query head (:292-302)
  ffmi_status load_tensor(std::vector<float> &out, size_t n, const std::string &hf_name) {
    std::string file = hf_name.rfind("model.", 0) == 0 ? hf_name.substr(6) : hf_name;
    const bool kv = file.find("self_attn.k_proj") != std::string::npos ||
                    file.find("self_attn.v_proj") != std::string::npos;
    const int group = kv ? c.num_heads / c.num_kv_heads : 1;
    const size_t n_file = n / group;
    const std::string path = weights_folder + "/" + file;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
      ffmi_set_last_error(("weight file not found: " + path).c_str(), __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    fseek(f, 0, SEEK_END);
    const long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<float> v(n_file);
    bool ok = false;
    if (bytes == (long)(n_file * 4)) {
      ok = fread(v.data(), 4, n_file, f) == n_file;
    } else if (bytes == (long)(n_file * 2)) {
      std::vector<_Float16> h16(n_file);
      ok = fread(h16.data(), 2, n_file, f) == n_file;
      for (size_t i = 0; ok && i < n_file; ++i) v[i] = (float)h16[i];
    }
    fclose(f);
    if (!ok) {
      ffmi_set_last_error(("weight file has the wrong size: " + path).c_str(), __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    out.resize(n);
    const size_t row_block = n_file / c.num_kv_heads;
    if (group > 1) {
      for (int i = 0; i < c.num_heads; ++i)
        memcpy(out.data() + (size_t)i * row_block, v.data() + (size_t)(i / group) * row_block,
               row_block * 4);
    } else {
      memcpy(out.data(), v.data(), n * 4);
    }
    return FFMI_OK;
  }

  // the full [rows][cols] tensor into tmp: seeded synthetic (orc_gen_weight
  // spec, the oracle's fp32 values) or the checkpoint's
  ffmi_status full_tensor(float *tmp, int rows, int cols, const std::string &name, int kind,
                          int perm_cols = 0, uint64_t pa = 1, float scale = 1.0f) {
    const size_t n = (size_t)rows * cols;
    if (!weights_folder.empty()) {
      std::vector<float> v;
      ffmi_status st = load_tensor(v, n, name);
      if (st != FFMI_OK) return st;
      FFMI_HIP(hipMemcpy(tmp, v.data(), n * 4, hipMemcpyHostToDevice));
      return FFMI_OK;
    }
    FFMI_HIP(launch_fill_weight_f32(tmp, n, weight_key(name.c_str(), o.weight_seed), kind, stream,
                                    perm_cols, pa, 17, scale));
    return FFMI_OK;
  }
  // rows [r0, r0 + nr) x columns [c0, c0 + nc) of tmp ([.][ld]) -> dst [nr][nc]
  ffmi_status take(float *dst, const float *tmp, int ld, int r0, int nr, int c0, int nc) {
    FFMI_HIP(hipMemcpy2DAsync(dst, (size_t)nc * 4, tmp + (size_t)r0 * ld + c0, (size_t)ld * 4,
                              (size_t)nc * 4, nr, hipMemcpyDeviceToDevice, stream));
    return FFMI_OK;
  }

  ffmi_status init() {
    H = c.hidden, F = c.intermediate, V = c.vocab_size, P = o.tp_size;
    FFMI_CHECK(c.num_kv_heads == c.num_heads ||
                   (!weights_folder.empty() && c.num_kv_heads > 0 &&
                    c.num_heads % c.num_kv_heads == 0),
               FFMI_ERR_UNSUPPORTED);
    FFMI_CHECK(H % c.num_heads == 0 && c.num_heads % P == 0 && F % P == 0, FFMI_ERR_INVALID);
    d = H / c.num_heads;
    // (d = 32: incremental decoding only, as the reference's kernels)
    FFMI_CHECK(d == 64 || d == 128 || (d == 32 && mode == FFMI_MODEL_INC), FFMI_ERR_UNSUPPORTED);
    heads_l = c.num_heads / P;
    Hl = heads_l * d;
    Fl = F / P;
    // the fp32 GEMM's shape rule (K % 32) for every projection
    FFMI_CHECK(H % 32 == 0 && Hl % 32 == 0 && Fl % 32 == 0, FFMI_ERR_UNSUPPORTED);
    FFMI_CHECK(P == 1 || o.comm, FFMI_ERR_INVALID);
    Tm = (o.max_tokens + 15) & ~15;
    // an attached transport too small for a [Tm][H] fp32 all-reduce needs a
    // fallback (RCCL or the local group): refuse at creation, not mid-serve
    if (P > 1 && comm_peer_attached(o.comm) && !comm_has_peer(o.comm, (size_t)Tm * H * 4) &&
        !comm_has_fallback(o.comm)) {
      ffmi_set_last_error("xGMI exchange buffer smaller than max_tokens x hidden fp32 and no "
                          "RCCL communicator", __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    FFMI_CHECK(o.weight_init >= 0 && o.weight_init <= 2, FFMI_ERR_INVALID);
    FFMI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const int tree = mode == FFMI_MODEL_INC ? 0 : o.max_tree_tokens;
    slots = (o.max_seq_len + tree + 31) & ~31;  // ffmi_attn_create's slot count
    FFMI_CHECK((size_t)(d + 256 + slots) * 4 <= 64 * 1024, FFMI_ERR_UNSUPPORTED);
    ffmi_status st;
#define TRY(x) \
  do { if ((st = (x)) != FFMI_OK) return st; } while (0)
    TRY(ffmi_batch_create(Tm, o.max_requests, &batch));
    TRY(alloc(&res, (size_t)Tm * H));
    TRY(alloc(&h, (size_t)Tm * H));
    TRY(alloc(&qkv, (size_t)Tm * 3 * Hl));
    TRY(alloc(&att, (size_t)Tm * Hl));
    TRY(alloc(&proj, (size_t)Tm * H));
    TRY(alloc(&gu, (size_t)Tm * 2 * Fl));
    TRY(alloc(&mlp, (size_t)Tm * Fl));
    TRY(alloc(&logits, (size_t)Tm * V));
    TRY(alloc(&res_d, (size_t)Tm * 4 * 2));
    FFMI_HIP(hipHostMalloc((void **)&res_h, (size_t)Tm * 4 * 2 * sizeof(int32_t),
                           hipHostMallocDefault));
    // weights: full tensors through a staging buffer, this shard's rows /
    // columns copied out
    float *tmp = nullptr;
    TRY(alloc(&tmp, std::max((size_t)V * H, std::max((size_t)F * H, (size_t)H * H))));
    const bool synth = weights_folder.empty();
    const bool chain = o.weight_init == 2 && synth;
    const int kres = o.weight_init == 1 ? (FFMI_WKIND_DEPTH | c.num_layers) : 0;
    float chain_scale = 128.0f;  // oracle.h orc_chain_embed_scale
    for (long long f2 = 1; f2 * 32LL * (4096 + 2 * 11008) <
                           (long long)c.num_layers * (H + 2LL * F);
         f2 *= 4)
      chain_scale *= 2.0f;
    TRY(alloc(&embed, (size_t)V * H));
    TRY(full_tensor(embed, V, H, "model.embed_tokens.weight", 0, 0, 1, chain ? chain_scale : 1.f));
    TRY(alloc(&final_norm, H));
    TRY(full_tensor(final_norm, 1, H, "model.norm.weight", 1));
    TRY(alloc(&lm, (size_t)V * H));
    if (chain)
      TRY(full_tensor(lm, V, H, "model.embed_tokens.weight", 0, H, 7919));
    else
      TRY(full_tensor(lm, V, H, "lm_head.weight", 0));
    const int s = o.tp_rank;
    layers.resize(c.num_layers);
    for (int l = 0; l < c.num_layers; ++l) {
      LayerF &L = layers[l];
      const std::string p = "model.layers." + std::to_string(l) + ".";
      TRY(alloc(&L.in_norm, H));
      TRY(full_tensor(L.in_norm, 1, H, p + "input_layernorm.weight", 1));
      TRY(alloc(&L.post_norm, H));
      TRY(full_tensor(L.post_norm, 1, H, p + "post_attention_layernorm.weight", 1));
      // qkv: rows [Q_s; K_s; V_s] (file_loader.cc:286-303)
      TRY(alloc(&L.wqkv, (size_t)3 * Hl * H));
      const char *names[3] = {"self_attn.q_proj.weight", "self_attn.k_proj.weight",
                              "self_attn.v_proj.weight"};
      for (int q = 0; q < 3; ++q) {
        TRY(full_tensor(tmp, H, H, p + names[q], 0));
        TRY(take(L.wqkv + (size_t)q * Hl * H, tmp, H, s * Hl, Hl, 0, H));
      }
      // o_proj row-parallel: columns [s*Hl, (s+1)*Hl)
      TRY(alloc(&L.wo, (size_t)H * Hl));
      TRY(full_tensor(tmp, H, H, p + "self_attn.o_proj.weight", kres));
      TRY(take(L.wo, tmp, H, 0, H, s * Hl, Hl));
      // gate rows then up rows of this shard: one GEMM, [T][2 Fl]
      TRY(alloc(&L.wgu, (size_t)2 * Fl * H));
      TRY(full_tensor(tmp, F, H, p + "mlp.gate_proj.weight", 0));
      TRY(take(L.wgu, tmp, H, s * Fl, Fl, 0, H));
      TRY(full_tensor(tmp, F, H, p + "mlp.up_proj.weight", 0));
      TRY(take(L.wgu + (size_t)Fl * H, tmp, H, s * Fl, Fl, 0, H));
      // down row-parallel: columns [s*Fl, (s+1)*Fl) of [H][F]
      TRY(alloc(&L.wd, (size_t)H * Fl));
      TRY(full_tensor(tmp, H, F, p + "mlp.down_proj.weight", kres));
      TRY(take(L.wd, tmp, F, 0, H, s * Fl, Fl));
      // the layer's DT_FLOAT attention handle (ffmi_attn_cfg.full_precision)
      ffmi_attn_cfg ac{};
      ac.mode = mode == FFMI_MODEL_TREE ? FFMI_ATTN_TREE
                                        : (mode == FFMI_MODEL_BEAM ? FFMI_ATTN_SPEC : FFMI_ATTN_INC);
      ac.num_heads = heads_l;
      ac.head_dim = d;
      ac.max_requests = o.max_requests;
      ac.max_seq_len = o.max_seq_len;
      ac.max_tree_tokens = tree;
      ac.max_tokens = Tm;
      ac.qk_scale = 1.0f / sqrtf((float)d);
      ac.rope_theta = c.rope_theta;
      ac.rope_llama3 = c.rope_llama3;
      ac.rope_factor = c.rope_factor;
      ac.rope_low_freq_factor = c.rope_low_freq_factor;
      ac.rope_high_freq_factor = c.rope_high_freq_factor;
      ac.rope_original_max_pos = c.rope_original_max_pos;
      ac.full_precision = 1;
      TRY(ffmi_attn_create(&ac, &L.attn));
    }
    FFMI_HIP(hipStreamSynchronize(stream));
    for (auto it = allocs.begin(); it != allocs.end(); ++it)
      if (*it == tmp) {
        (void)hipFree(tmp);
        allocs.erase(it);
        break;
      }
#undef TRY
    return FFMI_OK;
  }

  ffmi_status allreduce(float *buf, size_t n) {
    if (P <= 1) return FFMI_OK;
    return ffmi_allreduce(o.comm, buf, buf, n, FFMI_F32, (ffmi_stream)stream);
  }

  // everything a step puts on the stream (llama.cc:55-295 on DT_FLOAT)
  ffmi_status enqueue(int k, size_t blob_bytes, bool record_upload) {
    const int T = (int)ps.tokens.size();
    const float eps = c.rms_eps;
    ffmi_status st;
#define TRY(x) \
  do { if ((st = (x)) != FFMI_OK) return st; } while (0)
    TRY(batch_copy(batch, blob_bytes, stream, record_upload));
    const char *blob = batch->dev;
    for (int l = 0; l < c.num_layers; ++l) {
      LayerF &L = layers[l];
      // layer 0: embedding gather into the first norm; then the residual norm
      // of the previous layer's down projection
      if (l == 0)
        FFMI_HIP(launch_rmsnorm_f32(embed, nullptr, L.in_norm, res, h, T, H, eps, stream, blob));
      else
        FFMI_HIP(launch_rmsnorm_f32(res, proj, L.in_norm, res, h, T, H, eps, stream));
      FFMI_HIP(launch_gemm_f32(h, L.wqkv, qkv, T, 3 * Hl, H, stream));
      TRY(attn_forward(L.attn, batch, qkv, Partials(), att, (ffmi_stream)stream));
      FFMI_HIP(launch_gemm_f32(att, L.wo, proj, T, H, Hl, stream));
      TRY(allreduce(proj, (size_t)T * H));
      FFMI_HIP(launch_rmsnorm_f32(res, proj, L.post_norm, res, h, T, H, eps, stream));
      FFMI_HIP(launch_gemm_f32(h, L.wgu, gu, T, 2 * Fl, H, stream));
      FFMI_HIP(launch_silu_mul_f32(gu, gu + Fl, mlp, T, Fl, 2 * (size_t)Fl, 2 * (size_t)Fl, stream));
      FFMI_HIP(launch_gemm_f32(mlp, L.wd, proj, T, H, Fl, stream));
      TRY(allreduce(proj, (size_t)T * H));
    }
    FFMI_HIP(launch_rmsnorm_f32(res, proj, final_norm, res, h, T, H, eps, stream));
    FFMI_HIP(launch_gemm_f32(h, lm, logits, T, V, H, stream));
    float *probs_d = reinterpret_cast<float *>(res_d + (size_t)T * k);
    FFMI_HIP(launch_softmax_topk_f32(logits, T, V, k, res_d, probs_d, stream));
    FFMI_HIP(hipMemcpyAsync(res_h, res_d, (size_t)T * k * 8, hipMemcpyDeviceToHost, stream));
#undef TRY
    return FFMI_OK;
  }

  ffmi_status forward(int k) {
    const int T = (int)ps.tokens.size();
    FFMI_CHECK(k >= 1 && k <= 4, FFMI_ERR_INVALID);
    ffmi_batch_desc desc;
    ps.desc(&desc);
    for (int t = 0; t < T; ++t)
      FFMI_CHECK(desc.tokens[t].token_id >= 0 && desc.tokens[t].token_id < V, FFMI_ERR_INVALID);
    size_t bytes = 0;
    ffmi_status st = batch_stage(batch, &desc, &bytes);
    if (st != FFMI_OK) return st;
    if (T == 0) return FFMI_OK;
    // graphed at TP = 1 (the host-synchronising local group and the
    // transports stay eager here: this path is not the measured one)
    const bool graph = use_graphs && !dbg && P == 1;
    if (graph) {
      const auto key = std::make_tuple(T, batch->num_work, batch->num_commits, k, bytes);
      auto it = graphs.find(key);
      if (it == graphs.end()) {
        if (graphs.size() >= 256) {
          for (auto &kv : graphs) (void)hipGraphExecDestroy(kv.second);
          graphs.clear();
        }
        hipGraph_t g = nullptr;
        FFMI_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
        st = enqueue(k, bytes, false);
        const hipError_t ce = hipStreamEndCapture(stream, &g);
        if (st != FFMI_OK || ce != hipSuccess) {
          if (g) (void)hipGraphDestroy(g);
          if (st != FFMI_OK) return st;
          FFMI_HIP(ce);
        }
        hipGraphExec_t ex = nullptr;
        const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        FFMI_HIP(ie);
        it = graphs.emplace(key, ex).first;
      }
      FFMI_HIP(hipGraphLaunch(it->second, stream));
    } else {
      st = enqueue(k, bytes, true);
      if (st != FFMI_OK) return st;
    }
    FFMI_HIP(hipStreamSynchronize(stream));
    if (P > 1 && ffmi::comm_peer_attached(o.comm) && (st = ffmi::comm_status(o.comm)) != FFMI_OK)
      return st;
    if (dbg) dbg_T = T;
    return FFMI_OK;
  }

  // --inference-debugging: the last eager step's logits (fp32, full vocab)
  long debug_width(int which) const override { return which == FFMI_DBG_LOGITS ? V : -1; }
  ffmi_status set_debug(int enable) override {
    dbg = enable ? 1 : 0;
    dbg_T = -1;
    return FFMI_OK;
  }
  long debug_tensor(int which, int layer, float *out, long cap) override {
    (void)layer;
    if (which != FFMI_DBG_LOGITS || dbg_T < 0 || cap < (long)dbg_T * V) return -1;
    if (hipMemcpy(out, logits, (size_t)dbg_T * V * 4, hipMemcpyDeviceToHost) != hipSuccess)
      return -1;
    return dbg_T;
  }

  ffmi_status run_inc(const BatchConfig &bc, InferenceResult *ir) override {
    if (mode != FFMI_MODEL_INC) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens, FFMI_ERR_INVALID);
    pack_inc(bc, o.max_requests, slots, &ps);
    ffmi_status st = forward(1);
    if (st != FFMI_OK) return st;
    memcpy(ir->token_ids, res_h, bc.num_tokens * sizeof(int32_t));
    return FFMI_OK;
  }
  ffmi_status run_tree(const TreeVerifyBatchConfig &bc, InferenceResult *ir) override {
    if (mode != FFMI_MODEL_TREE) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens, FFMI_ERR_INVALID);
    pack_tree(bc, o.max_requests, slots, &ps);
    ffmi_status st = forward(1);
    if (st != FFMI_OK) return st;
    memcpy(ir->token_ids, res_h, bc.num_tokens * sizeof(int32_t));
    return FFMI_OK;
  }
  ffmi_status run_beam(const BeamSearchBatchConfig &bc, BeamInferenceResult *ir) override {
    if (mode != FFMI_MODEL_BEAM) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens, FFMI_ERR_INVALID);
    pack_beam(bc, o.max_requests, slots, &ps);
    const int k = ps.topk;
    ffmi_status st = forward(k);
    if (st != FFMI_OK) return st;
    const size_t n = (size_t)bc.num_tokens * k;
    const float *pr = reinterpret_cast<const float *>(res_h + n);
    std::vector<int> map;
    beam_result_layout(bc, &map);
    for (size_t i = 0; i < map.size(); ++i) {
      ir->token_ids[i] = res_h[map[i]];
      ir->probs[i] = pr[map[i]];
      ir->parent_id[i] = 0;
    }
    return FFMI_OK;
  }
};

}  // namespace

ffmi_status create_llama_f32(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                             ffmi_model **out) {
  FFMI_CHECK(cfg && o && out, FFMI_ERR_INVALID);
  FFMI_CHECK(o->tp_size >= 1 && o->tp_rank >= 0 && o->tp_rank < o->tp_size, FFMI_ERR_INVALID);
  FFMI_CHECK(o->max_tokens > 0 && o->max_tokens <= BatchConfig::MAX_NUM_TOKENS, FFMI_ERR_INVALID);
  FFMI_CHECK(o->max_requests > 0 && o->max_requests <= BatchConfig::MAX_NUM_REQUESTS,
             FFMI_ERR_INVALID);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return FFMI_ERR_NO_DEVICE;
  LlamaF32 *m = new LlamaF32();
  m->mode = o->mode;
  m->c = *cfg;
  m->o = *o;
  if (o->weights_folder && o->weights_folder[0]) m->weights_folder = o->weights_folder;
  m->o.weights_folder = nullptr;
  ffmi_status st = m->init();
  if (st != FFMI_OK) {
    delete m;
    return st;
  }
  *out = m;
  return FFMI_OK;
}

}  // namespace ffmi
