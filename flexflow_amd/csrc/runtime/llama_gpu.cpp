// llama_gpu.cpp -- LLaMA on MI355X through the C-ABI kernels.
//
// Graph per layer (inference/models/llama.cc:55-252):
//   [rms_norm | residual_rms_norm] -> qkv_proj -> {Inc,Spec,Tree}IncMHA
//   -> o_proj -> AllReduce -> residual_rms_norm -> gate|up (+SiLU-mul fused)
//   -> down_proj -> AllReduce
// tail: residual_rms_norm "norm" -> lm_head -> softmax+argmax (LLM) or
// softmax+arg_top_k (SSM, llama.cc:277-295).
// Tensor parallelism (model.cc:3392-3613, linear.cc:1691-1730): qkv/gate/up
// column-parallel (heads / FFN columns of shard `tp_rank`), o/down
// row-parallel followed by a sum all-reduce -- the direct xGMI transport
// (collective.hip) or RCCL, both in two column halves overlapped on a second
// stream and captured in the step's HIP graph; norms replicated; lm_head
// vocab-sharded with the sharded softmax / top-k tail (model.cc:3392-3419).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>

#include <string>
#include <map>
#include <tuple>
#include <vector>

#include "model.h"
#include "request_manager.h"  // (now_us)

namespace ffmi {

namespace {

struct Layer {
  uint16_t *in_norm = nullptr, *post_norm = nullptr;
  uint16_t *wqkv = nullptr, *wo = nullptr, *wgu = nullptr, *wd = nullptr;
  ffmi_attn *attn = nullptr;
};

struct LlamaGPU : public ffmi_model {
  ffmi_llama_config c{};
  ffmi_model_opts o{};
  int token_capacity() const override { return o.max_tokens; }
  bool uses_collectives() const override { return o.tp_size > 1; }
  std::string weights_folder;  // reference-format checkpoint ("" = synthetic)
  int Hl = 0, Fl = 0, d = 0, heads_l = 0, slots = 0;
  // GEMM inputs (normed hidden, attention output, SiLU output) are kept in
  // packed activation tiles: every GEMM then reads its activation fragments
  // as contiguous 1 KiB blocks, like the weights (see act_packed_off)
  bool packed = false;
  // FFMI_W_STREAM on every GEMM when this rank's weights outgrow the 256 MiB
  // Infinity Cache (LLaMA-7B: 13.5 GB streamed once per step; the 68M SSM's
  // 87 MB stay cached from step to step and keep the default policy)
  int wstream = 0;
  hipStream_t stream = nullptr;
  std::vector<Layer> layers;
  uint16_t *embed = nullptr, *final_norm = nullptr, *lm = nullptr;
  // activations
  uint16_t *res = nullptr, *h = nullptr, *qkv = nullptr, *att = nullptr, *proj = nullptr,
           *mlp = nullptr, *logits = nullptr;
  int32_t *ids_d = nullptr;
  // softmax top-k workspace (the split-row form for small steps; zeroed once)
  void *topk_ws = nullptr;
  size_t topk_ws_bytes = 0;
  // vocab-sharded lm_head at TP > 1 (model.cc:3392-3419): this rank's Vl rows
  // and the [P][Tm][kXW] exchange records of the sharded softmax / top-k
  int Vl = 0;
  float *xch = nullptr;
  // TP over the direct xGMI transport (ffmi_comm_peer_attach): the
  // row-parallel GEMMs run in two column halves; each half is all-reduced on
  // comm_stream while the next half computes (allreduce.cc:291-331 runs the
  // collective as a concurrent task; here it overlaps on HIP streams)
  bool peer = false;
  // RCCL all-reduce (no transport attached, or the transport cannot hold a
  // step): the same two-half overlap and graph capture as over the transport
  // (ncclAllReduce is stream-capturable); an in-process local group is not
  // (its all-reduce synchronises the host) and runs eager and unsplit
  bool rccl = false;
  bool solo = false;  // TP shard over a 1-rank communicator without transport or RCCL
  // residual norms folded into the skinny GEMMs around them (T <= 32, TP = 1):
  // per-tile sums of squares of the residual after o (ss_o) and after down
  // (ss_d), [32][H/16] each.  Only where o/down run unsplit anyway (H/16 >=
  // 128 tiles: LLaMA-7B decode, +1.9% incr decoding -- the A/B of record is
  // profiles/r03_fused_norm_ab.log, quoted in DESIGN.md §5); the 68M SSM's
  // o/down split K over workgroups, and unsplitting them to fuse cost more
  // than the norm launches saved (SSM step +4 us).  FFMI_FUSE_NORM: 0 off,
  // 1 auto (default), 2 every width (tests)
  int fuse_norms = getenv("FFMI_FUSE_NORM") ? atoi(getenv("FFMI_FUSE_NORM")) : 1;
  float *ss_o = nullptr, *ss_d = nullptr;
  // output projection folded into the fused attention (ffmi::OprojArgs): a
  // small model (d = 64, H <= 1024 -- the 68M SSM) at TP = 1 skips its o_proj
  // launch; the attention leaves one fp32 slab per head [heads][T][H] for the
  // residual norm.  FFMI_FUSE_AO=0 turns it off (A/B, tests)
  bool fuse_ao = false;
  float *oslab = nullptr;
  int oslab_T = 0;
  // the residual norm after each all-reduce folded into it over the transport
  // (ffmi::comm_allreduce_norm; the reference's AllReduce -> ResidualRMSNorm,
  // model.cc:3421-3445): no norm launch per all-reduce, and in two-shot mode
  // each rank normalises only its T / N rows (res is then current on those
  // rows only; h is complete).  FFMI_TP_FUSED_NORM: 0 off, 1 on (not with
  // debug captures), 2 also with debug captures (tests: the h and logits
  // captures are then of the fused path; o_proj / down / hidden are not kept)
  int tp_fuse_norm = getenv("FFMI_TP_FUSED_NORM") ? atoi(getenv("FFMI_TP_FUSED_NORM")) : 1;
  int tp_chunks = 1;
  hipStream_t comm_stream = nullptr;
  uint16_t *chunk_buf = nullptr;  // [tp_chunks][Tm][H / tp_chunks]
  std::vector<hipEvent_t> ev_chunk;
  hipEvent_t ev_comm_done = nullptr;
  float *ws = nullptr;  // split-K workspace of the GEMMs
  size_t ws_bytes = 0;
  size_t ws_chunk = 0;  // per-chunk workspace of the overlapped row-parallel GEMMs
  // split-K slabs summed by the all-reduce's copy-in (FFMI_AR_SLABS=0: the
  // GEMM's own reduce pass, A/B runs)
  bool ar_slabs = !getenv("FFMI_AR_SLABS") || atoi(getenv("FFMI_AR_SLABS")) != 0;
  int32_t *ids_h = nullptr;  // [kChain slots][Tm * 4 ids | Tm * 4 probs], pinned
  // chained beam steps (beam_launch_chained): one staging blob and one result
  // slot per step of a speculation phase; the top-k also leaves each slot's
  // ids in device memory (ids_dev) for the next step's embedding gather
  static constexpr int kChain = BeamSearchBatchConfig::MAX_BEAM_DEPTH;
  ffmi_batch_dev *chain_batch[kChain] = {};
  int32_t *ids_dev = nullptr;  // [kChain][Tm * 4]
  int cur_slot = 0;
  size_t slot_results[kChain] = {};  // [T][k] ids of each slot
  std::vector<int> slot_map[kChain];  // scheduler entry -> [T][k] index (beam_result_layout)
  hipEvent_t slot_ev[kChain] = {};     // recorded behind each launched slot
  hipEvent_t chain_t0 = nullptr;       // (FFMI_STEP_TIMING: before a chain's slot 0)
  bool slot_ev_live[kChain] = {};      // slot_ev recorded for the chain in flight
  int last_slot = -1;                  // highest slot launched since the last wait
  bool chain_ok = !getenv("FFMI_SSM_CHAIN") || atoi(getenv("FFMI_SSM_CHAIN")) != 0;
  size_t slot_ints() const { return (size_t)((o.max_tokens + 15) & ~15) * 4 * 2; }
  bool result_copy = getenv("FFMI_RESULT_COPY") && atoi(getenv("FFMI_RESULT_COPY")) != 0;
  float *probs_h = nullptr;
  ffmi_batch_dev *batch = nullptr;
  PackedStep ps;
  std::vector<void *> allocs;

  // ---- per-op profiling (HIP events on `stream`) ----
  enum Cat { GEMM_QKV, GEMM_O, GEMM_GATE_UP, GEMM_DOWN, GEMM_LM_HEAD, ATTENTION, NORM,
             ALLREDUCE, SAMPLING, EMBED, NCAT };
  struct ProfRec {
    int cat;
    hipEvent_t a, b;
    double bytes, flops;
  };
  struct OpStat {
    long launches = 0;
    double ms = 0, bytes = 0, flops = 0;
  };
  int prof_level = 0;
  // level 1 samples every prof_every-th step (FFMI_PROF_EVERY, default 4):
  // event-bracketed steps run eager, and bracketing every step cost the
  // bench ~2.5 % of its tokens/s
  int prof_every = getenv("FFMI_PROF_EVERY") ? std::max(1, atoi(getenv("FFMI_PROF_EVERY"))) : 4;
  long prof_steps = 0;
  bool prof_this_step = true;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<ProfRec> recs;
  OpStat opstat[NCAT];

  hipEvent_t next_event() {
    if (ev_used == ev_pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      ev_pool.push_back(e);
    }
    return ev_pool[ev_used++];
  }
  bool prof_on(int layer, int T) const {
    if (prof_level == 2) return true;
    if (prof_level == 1)
      return prof_this_step && T <= 256 && (layer == 0 || layer == c.num_layers / 2);
    return false;
  }
  int prof_begin(bool on) {
    if (!on) return -1;
    ProfRec r;
    r.a = next_event();
    r.b = next_event();
    (void)hipEventRecord(r.a, stream);
    recs.push_back(r);
    return (int)recs.size() - 1;
  }
  void prof_end(int idx, int cat, double bytes, double flops) {
    if (idx < 0) return;
    ProfRec &r = recs[idx];
    r.cat = cat;
    r.bytes = bytes;
    r.flops = flops;
    (void)hipEventRecord(r.b, stream);
  }
  void prof_collect() {
    for (auto &r : recs) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) continue;
      OpStat &o = opstat[r.cat];
      o.launches++;
      o.ms += ms;
      o.bytes += r.bytes;
      o.flops += r.flops;
    }
    recs.clear();
    ev_used = 0;
  }
  ffmi_status set_profiling(int level) override {
    prof_level = level;
    prof_steps = 0;
    for (auto &o : opstat) o = OpStat();
    return FFMI_OK;
  }
  int op_stats(ffmi_op_stat *out, int cap) override {
    static const char *names[NCAT] = {"gemm_qkv", "gemm_o_proj", "gemm_gate_up_silu",
                                      "gemm_down", "gemm_lm_head", "attention", "rmsnorm",
                                      "rowpar_gemm_allreduce", "softmax_argmax", "embedding"};
    int n = 0;
    for (int i = 0; i < NCAT; ++i) {
      if (opstat[i].launches == 0) continue;
      if (out && n < cap) {
        snprintf(out[n].name, sizeof(out[n].name), "%s", names[i]);
        out[n].launches = opstat[i].launches;
        out[n].total_ms = opstat[i].ms;
        out[n].bytes = opstat[i].bytes;
        out[n].flops = opstat[i].flops;
      }
      ++n;
    }
    return n;
  }
  static double gemm_bytes(int T, int N_w, int N_out, int K) {
    return 2.0 * ((double)N_w * K + (double)T * K + (double)T * N_out);
  }
  double attn_bytes() const {
    // K and V of every visible slot of each request read once + qkv in + out
    std::vector<int> kv(o.max_requests, 0);
    for (const auto &w : ps.work) kv[w.req] = std::max(kv[w.req], w.kv_len);
    double b = 0;
    for (int r : kv) b += (double)r * Hl * 2 * 2;
    return b + (double)ps.tokens.size() * (3 * Hl + Hl) * 2;
  }

  // ---- tensor capture (--inference-debugging, operator.h:271-360) ----
  // kind k (FFMI_DBG_*) keeps [dbg_layers(k)][Tm][dbg_width(k)] fp16 values of
  // the last eager step; GEMM inputs are stored in their packed tile layout
  // and unpacked on readout
  static constexpr int kDbgKinds = 10;
  int dbg = 0;
  uint16_t *dbg_buf = nullptr;
  size_t dbg_off[kDbgKinds] = {};
  int dbg_T = -1;
  long debug_width(int k) const override {
    switch (k) {
      case FFMI_DBG_LOGITS: return Vl;
      case FFMI_DBG_QKV: return 3L * Hl;
      case FFMI_DBG_ATTN_OUT: return Hl;
      case FFMI_DBG_MLP_ACT: return Fl;
      case FFMI_DBG_HIDDEN: case FFMI_DBG_ATTN_NORM: case FFMI_DBG_O_PROJ:
      case FFMI_DBG_FFN_NORM: case FFMI_DBG_DOWN: case FFMI_DBG_EMBED: return c.hidden;
    }
    return -1;
  }
  int dbg_layers(int k) const {
    return k == FFMI_DBG_LOGITS ? 0 : k == FFMI_DBG_EMBED ? 1
                                    : k == FFMI_DBG_HIDDEN ? c.num_layers + 1 : c.num_layers;
  }
  // stored in the packed activation-tile layout (a GEMM input written so)
  bool dbg_is_packed(int k, int layer) const {
    if (!packed) return false;
    return k == FFMI_DBG_ATTN_NORM || k == FFMI_DBG_FFN_NORM || k == FFMI_DBG_ATTN_OUT ||
           k == FFMI_DBG_MLP_ACT || (k == FFMI_DBG_HIDDEN && layer == c.num_layers);
  }
  size_t dbg_tm() const { return (size_t)((o.max_tokens + 15) & ~15); }
  ffmi_status set_debug(int enable) override {
    if (enable && !dbg_buf) {
      size_t total = 0;
      for (int k = 0; k < kDbgKinds; ++k) {
        dbg_off[k] = total;
        total += (size_t)dbg_layers(k) * dbg_tm() * std::max(0L, debug_width(k));
      }
      if (alloc(&dbg_buf, total) != FFMI_OK) return FFMI_ERR_OOM;
    }
    dbg = enable ? 1 : 0;
    dbg_T = -1;
    return FFMI_OK;
  }
  uint16_t *dbg_slot(int k, int l) const {
    return dbg_buf + dbg_off[k] + (size_t)l * dbg_tm() * debug_width(k);
  }
  // capture src ([T][width], or packed tiles covering whole 16-row groups)
  ffmi_status dbg_copy(int k, int l, const uint16_t *src, int T) {
    const size_t rows = dbg_is_packed(k, l) ? (size_t)((T + 15) & ~15) : (size_t)T;
    FFMI_HIP(hipMemcpyAsync(dbg_slot(k, l), src, rows * debug_width(k) * 2,
                            hipMemcpyDeviceToDevice, stream));
    return FFMI_OK;
  }
  // capture a GEMM output that is either written (Y) or left as split-K slabs
  ffmi_status dbg_gemm_out(int k, int l, const uint16_t *Y, const ffmi::Partials &p, int T) {
    if (p.S > 0) {
      FFMI_HIP(ffmi::launch_partials_reduce(p, dbg_slot(k, l), T, (int)debug_width(k), stream));
      return FFMI_OK;
    }
    return dbg_copy(k, l, Y, T);
  }
  long debug_tensor(int which, int layer, float *out, long cap) override {
    if (dbg_T < 0 || (stream && hipStreamSynchronize(stream) != hipSuccess)) return -1;
    if (which < 0 || which >= kDbgKinds) return -1;
    const int T = dbg_T;
    const long width = debug_width(which);
    if (which != FFMI_DBG_LOGITS && (layer < 0 || layer >= dbg_layers(which))) return -1;
    if (cap < (long)T * width) return -1;
    const uint16_t *src = which == FFMI_DBG_LOGITS ? logits : dbg_slot(which, layer);
    const bool pk = which != FFMI_DBG_LOGITS && dbg_is_packed(which, layer);
    const size_t n = (size_t)(pk ? (T + 15) & ~15 : T) * width;
    std::vector<uint16_t> raw(n);
    if (hipMemcpy(raw.data(), src, n * 2, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (int t = 0; t < T; ++t)
      for (long j = 0; j < width; ++j) {
        const uint16_t b = raw[pk ? act_packed_off(t, (int)j, (int)width) : (size_t)t * width + j];
        _Float16 v;
        memcpy(&v, &b, 2);
        out[(size_t)t * width + j] = (float)v;
      }
    return T;
  }

  // FFMI_FAULT_TP_AR_DROP: this rank's contribution to one all-reduce zeroed
  int ar_drop_layer = -1, ar_drop_which = 0;
  bool ar_drop_now = false;  // (set around the faulted call in enqueue)
  std::vector<int> head_swapped;  // layers whose Q heads 0 / 1 are exchanged

  // pack the Q rows of layer l with local heads 0 and 1 exchanged (swap) or
  // in their places; the source rows are regenerated / reloaded
  ffmi_status pack_q_heads(int l, bool swap) {
    const int H = c.hidden, s = o.tp_rank;
    uint16_t *tmp = nullptr;
    FFMI_HIP(hipMalloc((void **)&tmp, (size_t)H * H * 2));
    const std::string p = "model.layers." + std::to_string(l) + ".self_attn.q_proj.weight";
    ffmi_status st = FFMI_OK;
    if (!weights_folder.empty()) {
      st = load_tensor(tmp, (size_t)H * H, p);
    } else if (launch_fill_weight(tmp, (size_t)H * H, ffmi::weight_key(p.c_str(), o.weight_seed),
                                  0, stream) != hipSuccess) {
      st = FFMI_ERR_HIP;
    }
    if (st == FFMI_OK) {
      const int pitch = 3 * (Hl / 16);
      const hipError_t e0 = launch_pack_weight(tmp, H, s * Hl + (swap ? d : 0), 0, d, H,
                                               layers[l].wqkv, 1, 0, pitch, stream);
      const hipError_t e1 = launch_pack_weight(tmp, H, s * Hl + (swap ? 0 : d), 0, d, H,
                                               layers[l].wqkv, 1, d / 16, pitch, stream);
      if (e0 != hipSuccess || e1 != hipSuccess || hipStreamSynchronize(stream) != hipSuccess)
        st = FFMI_ERR_HIP;
    }
    (void)hipFree(tmp);
    return st;
  }

  ffmi_status debug_fault(int kind, int layer, int arg) override {
    // the tables are rewritten with blocking copies: finish the model's
    // (non-blocking) stream first in every branch
    if (stream) FFMI_HIP(hipStreamSynchronize(stream));
    if (kind == FFMI_FAULT_TP_HEAD_SWAP) {
      FFMI_CHECK(layer >= -1 && layer < c.num_layers && heads_l >= 2 && d % 16 == 0,
                 FFMI_ERR_INVALID);
      for (int l = 0; l < c.num_layers; ++l)
        if ((layer < 0 || l == layer) &&
            std::find(head_swapped.begin(), head_swapped.end(), l) == head_swapped.end()) {
          ffmi_status st = pack_q_heads(l, true);
          if (st != FFMI_OK) return st;
          head_swapped.push_back(l);
        }
      clear_graphs();
      return FFMI_OK;
    }
    if (kind == FFMI_FAULT_TP_AR_DROP) {
      FFMI_CHECK(o.tp_size > 1 && layer >= 0 && layer < c.num_layers && (arg == 0 || arg == 1),
                 FFMI_ERR_INVALID);
      ar_drop_layer = layer;
      ar_drop_which = arg;
      clear_graphs();
      return FFMI_OK;
    }
    if (kind == FFMI_FAULT_NONE) {
      for (int l : head_swapped) {
        ffmi_status st = pack_q_heads(l, false);
        if (st != FFMI_OK) return st;
      }
      head_swapped.clear();
      ar_drop_layer = -1;
      clear_graphs();
    }
    if (kind == FFMI_FAULT_RESID_ROUND || kind == FFMI_FAULT_NONE) {
      // captured graphs hold the launches of the other norm variant
      ffmi::set_norm_fault(kind == FFMI_FAULT_RESID_ROUND);
      clear_graphs();
      if (kind == FFMI_FAULT_RESID_ROUND) return FFMI_OK;
    }
    if (kind == FFMI_FAULT_NONE) {
      for (auto &L : layers) {
        ffmi_status st = ffmi::attn_rope_fault(L.attn, -1);
        if (st != FFMI_OK) return st;
      }
      return FFMI_OK;
    }
    FFMI_CHECK(kind == FFMI_FAULT_ROPE_POS && layer >= -1 && layer < c.num_layers,
               FFMI_ERR_INVALID);
    for (int l = 0; l < c.num_layers; ++l)
      if (layer < 0 || l == layer) {
        ffmi_status st = ffmi::attn_rope_fault(layers[l].attn, arg);
        if (st != FFMI_OK) return st;
      }
    return FFMI_OK;
  }

  ~LlamaGPU() override {
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto &kv : st_sum) {
      if (kv.first < 0) {
        fprintf(stderr, "[ffmi step timing] H=%d chain of %d steps: %ld chains, gpu span %.1f us "
                "(%.1f us per step)\n", c.hidden, -kv.first, kv.second.n,
                kv.second.gpu / kv.second.n, kv.second.gpu / kv.second.n / -kv.first);
        continue;
      }
      fprintf(stderr, "[ffmi step timing] H=%d T=%d steps=%ld launch=%.1f gpu=%.1f wait=%.1f total=%.1f us\n",
              c.hidden, kv.first, kv.second.n, kv.second.launch / kv.second.n, kv.second.gpu / kv.second.n,
              kv.second.wait / kv.second.n, kv.second.total / kv.second.n);
    }
    for (auto e : st_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : slot_ev)
      if (e) (void)hipEventDestroy(e);
    if (chain_t0) (void)hipEventDestroy(chain_t0);
    clear_graphs();
    for (auto &L : layers) ffmi_attn_destroy(L.attn);
    for (auto e : ev_pool) (void)hipEventDestroy(e);
    for (auto e : ev_chunk) (void)hipEventDestroy(e);
    if (ev_comm_done) (void)hipEventDestroy(ev_comm_done);
    if (comm_stream) (void)hipStreamDestroy(comm_stream);
    for (void *p : allocs) (void)hipFree(p);
    if (ids_h) (void)hipHostFree(ids_h);
    for (int i = 1; i < kChain; ++i) ffmi_batch_destroy(chain_batch[i]);
    ffmi_batch_destroy(batch);
    if (stream) (void)hipStreamDestroy(stream);
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

  // One tensor of a reference-format checkpoint (file_loader.cc:363-389
  // load_from_file; names as convert_hf_model writes them): the HF name
  // without "model.", raw fp16 or fp32 (converted, round to nearest even).
  // k/v projections of a GQA checkpoint hold num_kv_heads * d rows; row
  // block of query head i = kv head i / (heads / kv_heads) (:292-302).
  ffmi_status load_tensor(uint16_t *dst, size_t n, const std::string &hf_name) {
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
    std::vector<uint16_t> h16(n_file);
    bool ok = false;
    if (bytes == (long)(n_file * 2)) {
      ok = fread(h16.data(), 2, n_file, f) == n_file;
    } else if (bytes == (long)(n_file * 4)) {
      std::vector<float> h32(n_file);
      ok = fread(h32.data(), 4, n_file, f) == n_file;
      for (size_t i = 0; ok && i < n_file; ++i) {
        const _Float16 v = (_Float16)h32[i];
        memcpy(&h16[i], &v, 2);
      }
    }
    fclose(f);
    if (!ok) {
      ffmi_set_last_error(("weight file has the wrong size: " + path).c_str(), __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    if (group > 1) {  // [kv_heads * d][H] -> [heads * d][H]
      const size_t row_block = n_file / c.num_kv_heads;  // d rows of one head
      std::vector<uint16_t> rep(n);
      for (int i = 0; i < c.num_heads; ++i)
        memcpy(rep.data() + (size_t)i * row_block, h16.data() + (size_t)(i / group) * row_block,
               row_block * 2);
      h16.swap(rep);
    }
    FFMI_HIP(hipMemcpy(dst, h16.data(), n * 2, hipMemcpyHostToDevice));
    return FFMI_OK;
  }

  ffmi_status init() {
    const int H = c.hidden, F = c.intermediate, V = c.vocab_size, P = o.tp_size;
    // GQA checkpoints load with K/V replicated per query head (the
    // reference's layout); synthetic weights are MHA only
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
    FFMI_CHECK(H % 32 == 0 && Hl % 32 == 0 && Fl % 32 == 0, FFMI_ERR_UNSUPPORTED);
    FFMI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const int Tm = (o.max_tokens + 15) & ~15;  // packed tiles cover 16-row groups
    packed = H % 32 == 0 && Hl % 32 == 0 && Fl % 32 == 0;
    {
      const double wbytes = 2.0 * c.num_layers * ((double)4 * Hl * H + 3.0 * Fl * H) +
                            2.0 * V * H;
      wstream = wbytes > 192.0 * (1 << 20) ? FFMI_W_STREAM : 0;
      if (const char *e = getenv("FFMI_W_STREAM"))  // A/B override: 0 / 1
        wstream = atoi(e) ? FFMI_W_STREAM : 0;
    }
    ffmi_status st;
#define TRY(x) \
  do { if ((st = (x)) != FFMI_OK) return st; } while (0)
    TRY(ffmi_batch_create(Tm, o.max_requests, &batch));
    TRY(alloc(&res, (size_t)Tm * H));
    TRY(alloc(&h, (size_t)Tm * H));
    TRY(alloc(&qkv, (size_t)Tm * 3 * Hl));
    TRY(alloc(&att, (size_t)Tm * Hl));
    TRY(alloc(&proj, (size_t)Tm * H));
    TRY(alloc(&ss_o, (size_t)2 * 32 * (H / 16)));
    ss_d = ss_o + (size_t)32 * (H / 16);
    TRY(alloc(&mlp, (size_t)Tm * Fl));
    fuse_ao = P == 1 && d == 64 && H <= 1024 && H % 16 == 0 &&
              !(getenv("FFMI_FUSE_AO") && atoi(getenv("FFMI_FUSE_AO")) == 0);
    if (fuse_ao) {  // decode / beam steps (<= 64 rows); prefill blocks run the GEMM
      oslab_T = std::min(Tm, 64);
      TRY(alloc(&oslab, (size_t)heads_l * oslab_T * H));
    }
    Vl = P > 1 && V % P == 0 && (V / P) % 16 == 0 ? V / P : V;
    if (const char *e = getenv("FFMI_VOCAB_SHARD"))  // A/B: 0 = replicated lm_head
      if (!atoi(e)) Vl = V;
    TRY(alloc(&logits, (size_t)Tm * Vl));
    if (Vl != V) TRY(alloc(&xch, (ffmi_vocab_shard_scratch_bytes(P, Tm) + 3) / 4));
    TRY(alloc(&ids_d, (size_t)Tm * 4 * 2));  // [ids | probs] of a step, one D2H copy
    topk_ws_bytes = ffmi::argmax_workspace_bytes(std::min(Tm, 256));
    TRY(alloc((char **)&topk_ws, topk_ws_bytes));
    FFMI_HIP(hipMemsetAsync(topk_ws, 0, topk_ws_bytes, stream));
    peer = P > 1 && ffmi::comm_has_peer(o.comm, (size_t)Tm * H * 2);
    // an attached transport too small for this model's largest [Tm][H]
    // all-reduce needs RCCL (or the local group) for those steps: refuse at
    // creation rather than failing mid-serve
    if (P > 1 && !peer && ffmi::comm_peer_attached(o.comm) && !ffmi::comm_has_fallback(o.comm)) {
      ffmi_set_last_error("xGMI exchange buffer smaller than max_tokens x hidden fp16 and no "
                          "RCCL communicator", __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    rccl = P > 1 && !peer && ffmi::comm_is_rccl(o.comm);
    // a shard over a one-rank communicator with no RCCL state (the per-rank
    // shard bench): every all-reduce is the identity, so o/down defer their
    // slabs to the residual norm exactly as at TP = 1
    solo = P > 1 && !peer && !rccl && ffmi::comm_size(o.comm) == 1;
    if (peer || rccl) {
      tp_chunks = 2;
      if (const char *e = getenv("FFMI_TP_OVERLAP")) tp_chunks = atoi(e) ? 2 : 1;
      if ((H / tp_chunks) % 32 != 0) tp_chunks = 1;
      FFMI_HIP(hipStreamCreateWithFlags(&comm_stream, hipStreamNonBlocking));
      ev_chunk.resize(tp_chunks);
      for (auto &e : ev_chunk) FFMI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      FFMI_HIP(hipEventCreateWithFlags(&ev_comm_done, hipEventDisableTiming));
      if (tp_chunks > 1) TRY(alloc(&chunk_buf, (size_t)Tm * H));
    }
    {
      // the split-K factor depends on the row-block count, so take the max
      // over every batch size the model can see
      for (int t = 16; t <= Tm; t += 16) {
        const size_t w1 = ffmi_linear_workspace_bytes(t, 3 * Hl, H, FFMI_EPI_NONE);
        const size_t w2 = ffmi_linear_workspace_bytes(t, H, Hl, FFMI_EPI_NONE);
        const size_t w3 = ffmi_linear_workspace_bytes(t, Fl, H, FFMI_EPI_SILU_MUL);
        const size_t w4 = ffmi_linear_workspace_bytes(t, H, Fl, FFMI_EPI_NONE);
        const size_t w5 = ffmi_linear_workspace_bytes(t, Vl, H, FFMI_EPI_NONE);
        ws_bytes = std::max(ws_bytes, std::max(std::max(std::max(w1, w2), std::max(w3, w4)), w5));
      }
      // the row-parallel column chunks over the xGMI transport defer their
      // split-K slabs to the all-reduce's copy-in on comm_stream while the
      // next chunk computes: one workspace region per chunk
      if (peer && ar_slabs && tp_chunks > 1) {
        const int Hc = H / tp_chunks;
        for (int t = 16; t <= Tm; t += 16)
          ws_chunk = std::max(ws_chunk, std::max(ffmi_linear_workspace_bytes(t, Hc, Hl, FFMI_EPI_NONE),
                                                 ffmi_linear_workspace_bytes(t, Hc, Fl, FFMI_EPI_NONE)));
        ws_chunk = (ws_chunk + 255) & ~(size_t)255;
        ws_bytes = std::max(ws_bytes, ws_chunk * tp_chunks);
      }
      if (ws_bytes) TRY(alloc(&ws, (ws_bytes + 3) / 4));
    }
    // coherent (uncached) pinned memory: the sampling kernel's stores go
    // straight over PCIe and are visible to the host once the stream has
    // synchronised, whatever HIP_HOST_COHERENT says
    FFMI_HIP(hipHostMalloc((void **)&ids_h, (size_t)kChain * Tm * 4 * 2 * sizeof(int32_t),
                           hipHostMallocCoherent | hipHostMallocMapped));
    if (mode == FFMI_MODEL_BEAM) TRY(alloc(&ids_dev, (size_t)kChain * Tm * 4));
    chain_batch[0] = batch;
    // the chained beam steps' staging batches, created here rather than on a
    // chain's first use: creating one clears its device blob on the legacy
    // stream, which fails -- and invalidates the capture -- while another
    // thread's model is capturing a graph (the TP shard threads of one
    // process, ffmi_comm_create_local, beside their SSMs)
    if (mode == FFMI_MODEL_BEAM && o.tp_size == 1)
      for (int i = 1; i < kChain; ++i)
        TRY(ffmi_batch_create((o.max_tokens + 15) & ~15, o.max_requests, &chain_batch[i]));
    // weights (seeded synthetic, orc_gen_weight spec), packed for MFMA
    uint16_t *tmp = nullptr;
    size_t tmp_elems = std::max((size_t)V * H, std::max((size_t)F * H, (size_t)H * H));
    TRY(alloc(&tmp, tmp_elems));
    // synthetic inits (ffmi_model_opts.weight_init; oracle orc_model_create_ex):
    // 1 scales o/down by 1/sqrt(2L); 2 (token chain) scales the embeddings by
    // 128, doubled while the layers' residual noise sqrt(L (H + 2F)) outgrows
    // LLaMA-7B's by the same factor (oracle.h orc_chain_embed_scale: the
    // chain's logit margin stays at least 7B's), and makes lm_head the
    // permuted unscaled embedding rows
    FFMI_CHECK(o.weight_init >= 0 && o.weight_init <= 2, FFMI_ERR_INVALID);
    const int kres = o.weight_init == 1 ? (FFMI_WKIND_DEPTH | c.num_layers) : 0;
    auto fill = [&](uint16_t *dst, size_t n, const std::string &name, int kind, int cols = 0,
                    uint64_t pa = 1, float scale = 1.0f) -> ffmi_status {
      if (!weights_folder.empty()) return load_tensor(dst, n, name);
      FFMI_CHECK(dst, FFMI_ERR_INVALID);
      FFMI_HIP(ffmi::launch_fill_weight(dst, n, ffmi::weight_key(name.c_str(), o.weight_seed), kind,
                                        stream, cols, pa, 17, scale));
      return FFMI_OK;
    };
    const bool chain = o.weight_init == 2 && weights_folder.empty();
    float chain_scale = 128.0f;
    for (long long f2 = 1; f2 * 32LL * (4096 + 2 * 11008) <
                           (long long)c.num_layers * (c.hidden + 2LL * c.intermediate);
         f2 *= 4)
      chain_scale *= 2.0f;
    TRY(alloc(&embed, (size_t)V * H));
    TRY(fill(embed, (size_t)V * H, "model.embed_tokens.weight", 0, 0, 1, chain ? chain_scale : 1.0f));
    TRY(alloc(&final_norm, H));
    TRY(fill(final_norm, H, "model.norm.weight", 1));
    TRY(alloc(&lm, ffmi_linear_packed_bytes(Vl, H) / 2));
    if (chain)
      TRY(fill(tmp, (size_t)V * H, "model.embed_tokens.weight", 0, H, 7919));
    else
      TRY(fill(tmp, (size_t)V * H, "lm_head.weight", 0));
    // vocab shard s: rows [s*Vl, (s+1)*Vl) (the whole table when replicated)
    FFMI_HIP(launch_pack_weight(tmp, H, Vl == V ? 0 : o.tp_rank * Vl, 0, Vl, H, lm, 1, 0,
                                (Vl + 15) / 16, stream));
    slots = 0;
    layers.resize(c.num_layers);
    const int s = o.tp_rank;
    for (int l = 0; l < c.num_layers; ++l) {
      Layer &L = layers[l];
      const std::string p = "model.layers." + std::to_string(l) + ".";
      TRY(alloc(&L.in_norm, H));
      TRY(fill(L.in_norm, H, p + "input_layernorm.weight", 1));
      TRY(alloc(&L.post_norm, H));
      TRY(fill(L.post_norm, H, p + "post_attention_layernorm.weight", 1));
      // qkv: [Q_s | K_s | V_s] rows of this shard (file_loader.cc:286-303)
      const size_t qkv_tiles_bytes = ffmi_linear_packed_bytes(Hl, H);
      TRY(alloc(&L.wqkv, 3 * qkv_tiles_bytes / 2));
      const char *names[3] = {"self_attn.q_proj.weight", "self_attn.k_proj.weight",
                              "self_attn.v_proj.weight"};
      for (int q = 0; q < 3; ++q) {
        TRY(fill(tmp, (size_t)H * H, p + names[q], 0));
        // one allocation of 3 NT tiles per k-row: Q, K, V tiles side by side
        FFMI_HIP(launch_pack_weight(tmp, H, s * Hl, 0, Hl, H, L.wqkv, 1, q * (Hl / 16),
                                    3 * (Hl / 16), stream));
      }
      // o_proj: row-parallel -> columns [s*Hl, (s+1)*Hl)
      TRY(alloc(&L.wo, ffmi_linear_packed_bytes(H, Hl) / 2));
      TRY(fill(tmp, (size_t)H * H, p + "self_attn.o_proj.weight", kres));
      FFMI_HIP(launch_pack_weight(tmp, H, 0, s * Hl, H, Hl, L.wo, 1, 0, H / 16, stream));
      // gate | up: column-parallel, interleaved 16-column tiles
      TRY(alloc(&L.wgu, 2 * ffmi_linear_packed_bytes(Fl, H) / 2));
      TRY(fill(tmp, (size_t)F * H, p + "mlp.gate_proj.weight", 0));
      FFMI_HIP(launch_pack_weight(tmp, H, s * Fl, 0, Fl, H, L.wgu, 2, 0, 2 * ((Fl + 15) / 16),
                                  stream));
      TRY(fill(tmp, (size_t)F * H, p + "mlp.up_proj.weight", 0));
      FFMI_HIP(launch_pack_weight(tmp, H, s * Fl, 0, Fl, H, L.wgu, 2, 1, 2 * ((Fl + 15) / 16),
                                  stream));
      // down: row-parallel -> columns [s*Fl, (s+1)*Fl) of [H][F]
      TRY(alloc(&L.wd, ffmi_linear_packed_bytes(H, Fl) / 2));
      TRY(fill(tmp, (size_t)H * F, p + "mlp.down_proj.weight", kres));
      FFMI_HIP(launch_pack_weight(tmp, F, 0, s * Fl, H, Fl, L.wd, 1, 0, H / 16, stream));
      ffmi_attn_cfg ac{};  // (zeroed: fields added to the ABI later default to 0)
      ac.mode = mode == FFMI_MODEL_TREE ? FFMI_ATTN_TREE
                                        : (mode == FFMI_MODEL_BEAM ? FFMI_ATTN_SPEC : FFMI_ATTN_INC);
      ac.num_heads = heads_l;
      ac.head_dim = d;
      ac.max_requests = o.max_requests;
      ac.max_seq_len = o.max_seq_len;
      ac.max_tree_tokens = mode == FFMI_MODEL_INC ? 0 : o.max_tree_tokens;
      ac.max_tokens = Tm;
      ac.qk_scale = 1.0f / sqrtf((float)d);
      ac.rope_theta = c.rope_theta;
      ac.rope_llama3 = c.rope_llama3;
      ac.rope_factor = c.rope_factor;
      ac.rope_low_freq_factor = c.rope_low_freq_factor;
      ac.rope_high_freq_factor = c.rope_high_freq_factor;
      ac.rope_original_max_pos = c.rope_original_max_pos;
      ac.out_layout = packed ? 1 : 0;
      TRY(ffmi_attn_create(&ac, &L.attn));
      int sl = 0;
      ffmi_attn_kv_ptrs(L.attn, nullptr, nullptr, &sl);
      slots = sl;
    }
    FFMI_HIP(hipStreamSynchronize(stream));
    // the staging buffer is not needed after init
    for (auto it = allocs.begin(); it != allocs.end(); ++it)
      if (*it == tmp) {
        (void)hipFree(tmp);
        allocs.erase(it);
        break;
      }
#undef TRY
    return FFMI_OK;
  }

  ffmi_status allreduce(uint16_t *buf, size_t n) {
    if (o.tp_size <= 1) return FFMI_OK;
    return ffmi_allreduce(o.comm, buf, buf, n, FFMI_F16, (ffmi_stream)stream);
  }

  // Row-parallel GEMM + sum all-reduce into `out` [T][H] (model.cc:3421-3445).
  // Over the xGMI transport the output columns are computed in tp_chunks
  // halves: half c goes to comm_stream for its all-reduce (strided into
  // `out`) as soon as its GEMM is done, while half c + 1 computes.
  ffmi_status rowpar_gemm_allreduce(const uint16_t *X, const uint16_t *W, int K, uint16_t *out,
                                    int T, int XP) {
    const int H = c.hidden;
    // (FFMI_FAULT_TP_AR_DROP: the GEMM's output zeroed before the all-reduce)
    const bool drop = ar_drop_now;
    if (!(peer || rccl) || tp_chunks == 1) {
      // over the transport the split-K reduce is the all-reduce's copy-in
      ffmi::Partials part;
      FFMI_HIP(ffmi::launch_gemm(X, W, out, ws, ws_bytes, T, H, K, XP, stream,
                                 peer && ar_slabs && !drop ? &part : nullptr));
      if (drop) FFMI_HIP(hipMemsetAsync(out, 0, (size_t)T * H * 2, stream));
      if (peer)
        return ffmi::comm_allreduce_cols(o.comm, out, out, T, H, H, 0, FFMI_F16, stream,
                                         part.S > 0 ? &part : nullptr);
      return allreduce(out, (size_t)T * H);
    }
    const int Hc = H / tp_chunks;
    // a chunk = Hc / 16 consecutive tiles of the H / 16 per k-row
    const size_t tiles = (size_t)(Hc / 16) * ffmi::w_tile_stride((K + 31) / 32);
    for (int ch = 0; ch < tp_chunks; ++ch) {
      uint16_t *cb = chunk_buf + (size_t)ch * T * Hc;
      // over the transport: the chunk's split-K slabs (own workspace region)
      // go to the all-reduce's copy-in, no reduce pass on this stream
      ffmi::Partials part;
      const bool def = peer && ar_slabs && !drop;
      FFMI_HIP(ffmi::launch_gemm(X, W + ch * tiles, cb,
                                 def ? (float *)((char *)ws + ch * ws_chunk) : ws,
                                 def ? ws_chunk : ws_bytes, T, Hc, K, XP, stream,
                                 def ? &part : nullptr, H / 16));
      if (drop) FFMI_HIP(hipMemsetAsync(cb, 0, (size_t)T * Hc * 2, stream));
      FFMI_HIP(hipEventRecord(ev_chunk[ch], stream));
      FFMI_HIP(hipStreamWaitEvent(comm_stream, ev_chunk[ch], 0));
      if (peer) {  // the transport reduces straight into out's columns
        ffmi_status st = ffmi::comm_allreduce_cols(o.comm, cb, out, T, Hc, H, ch * Hc, FFMI_F16,
                                                   comm_stream, part.S > 0 ? &part : nullptr);
        if (st != FFMI_OK) return st;
      } else {  // RCCL: contiguous in place, then into out's columns
        ffmi_status st = ffmi_allreduce(o.comm, cb, cb, (size_t)T * Hc, FFMI_F16,
                                        (ffmi_stream)comm_stream);
        if (st != FFMI_OK) return st;
        FFMI_HIP(hipMemcpy2DAsync(out + (size_t)ch * Hc, (size_t)H * 2, cb, (size_t)Hc * 2,
                                  (size_t)Hc * 2, T, hipMemcpyDeviceToDevice, comm_stream));
      }
    }
    FFMI_HIP(hipEventRecord(ev_comm_done, comm_stream));
    FFMI_HIP(hipStreamWaitEvent(stream, ev_comm_done, 0));
    return FFMI_OK;
  }

  // rowpar_gemm_allreduce with the residual norm after it folded into the
  // transport's all-reduce (tp_fuse_norm): res += sum (this rank's rows in
  // two-shot mode), h = RMSNorm(res) * wnorm on every rank.  Column chunks:
  // chunk 0 is reduced on comm_stream (two-shot: only this rank's rows) while
  // chunk 1 computes; chunk 1's all-reduce carries the norm, reading chunk 0's
  // columns of the sum from proj.
  ffmi_status rowpar_gemm_allreduce_norm(const uint16_t *X, const uint16_t *W, int K, int T, int XP,
                                         const uint16_t *wnorm) {
    const int H = c.hidden;
    const float eps = c.rms_eps;
    const bool drop = ar_drop_now;
    const bool two = ffmi::comm_two_shot(o.comm, (size_t)T * H * 2);
    if (tp_chunks == 1) {
      ffmi::Partials part;
      FFMI_HIP(ffmi::launch_gemm(X, W, proj, ws, ws_bytes, T, H, K, XP, stream,
                                 ar_slabs && !drop ? &part : nullptr));
      if (drop) FFMI_HIP(hipMemsetAsync(proj, 0, (size_t)T * H * 2, stream));
      return ffmi::comm_allreduce_norm(o.comm, proj, T, H, 0, nullptr, res, wnorm, eps, h, packed,
                                       two, stream, part.S > 0 ? &part : nullptr);
    }
    const int Hc = H / tp_chunks;
    const size_t tiles = (size_t)(Hc / 16) * ffmi::w_tile_stride((K + 31) / 32);
    const int nr = ffmi::comm_size(o.comm), rk = ffmi::comm_rank(o.comm);
    for (int ch = 0; ch < tp_chunks; ++ch) {
      uint16_t *cb = chunk_buf + (size_t)ch * T * Hc;
      ffmi::Partials part;
      const bool def = ar_slabs && !drop;
      FFMI_HIP(ffmi::launch_gemm(X, W + ch * tiles, cb,
                                 def ? (float *)((char *)ws + ch * ws_chunk) : ws,
                                 def ? ws_chunk : ws_bytes, T, Hc, K, XP, stream,
                                 def ? &part : nullptr, H / 16));
      if (drop) FFMI_HIP(hipMemsetAsync(cb, 0, (size_t)T * Hc * 2, stream));
      FFMI_HIP(hipEventRecord(ev_chunk[ch], stream));
      FFMI_HIP(hipStreamWaitEvent(comm_stream, ev_chunk[ch], 0));
      const ffmi::Partials *sl = part.S > 0 ? &part : nullptr;
      ffmi_status st;
      if (ch + 1 < tp_chunks) {  // columns [ch Hc, (ch+1) Hc) of the sum into proj
        st = two ? ffmi::comm_reduce_rows(o.comm, cb, proj, T, Hc, H, ch * Hc,
                                          (int)((long)T * rk / nr), (int)((long)T * (rk + 1) / nr),
                                          comm_stream, sl)
                 : ffmi::comm_allreduce_cols(o.comm, cb, proj, T, Hc, H, ch * Hc, FFMI_F16,
                                             comm_stream, sl);
      } else {
        st = ffmi::comm_allreduce_norm(o.comm, cb, T, H, ch * Hc, proj, res, wnorm, eps, h, packed,
                                       two, comm_stream, sl);
      }
      if (st != FFMI_OK) return st;
    }
    FFMI_HIP(hipEventRecord(ev_comm_done, comm_stream));
    FFMI_HIP(hipStreamWaitEvent(stream, ev_comm_done, 0));
    return FFMI_OK;
  }

  // One step over the packed batch; k = results per token.  Small batches
  // (SSM beam steps, decode) are launch-bound -- ~20 kernels of a few us
  // each -- so their whole step (metadata copy, kernels, result copies) is
  // captured once per batch shape into a HIP graph and replayed.
  struct GraphKey {
    int T, W, C, k, parity, overlap, fused, max_q, slot;
    size_t bytes;
    bool operator<(const GraphKey &o) const {
      return std::tie(T, W, C, k, parity, overlap, fused, max_q, slot, bytes) <
             std::tie(o.T, o.W, o.C, o.k, o.parity, o.overlap, o.fused, o.max_q, o.slot, o.bytes);
    }
  };
  // TREE steps write alternate halves of the attention staging (commits of
  // the next step read the half this one wrote); kept here so graph replays
  // and eager steps agree
  int tree_parity = 0;
  std::map<GraphKey, hipGraphExec_t> graphs;
  // FFMI_CHAIN_GROUP=g (>= 2): chained beam slots 1 .. kChain-2 are staged and
  // go out g per graph launch (slot kChain-1 alone, behind the collect event):
  // the boundary between two graph launches (4.9 us from one step's last
  // kernel to the next step's first, profiles/r06_ssm_gaps.log) becomes a
  // kernel boundary inside one graph.  1 = one launch per slot.  Default: all
  // six middle slots in one launch (the host stages them while slot 0 runs).
  // Same box, 3 pairs (profiles/r06_chain_group_ab.log): SSM step 95.8-97.8
  // (1 per launch) -> 93.8-94.5 (3) -> 92.9-93.9 us (6); 1325-1330 -> 1332-1336
  // tokens/s
  int chain_group = getenv("FFMI_CHAIN_GROUP") ? atoi(getenv("FFMI_CHAIN_GROUP")) : kChain - 2;
  struct PendingSlot {
    int slot, T, k;
    size_t bytes;
    GraphKey key;
  };
  std::vector<PendingSlot> pend;  // staged, not yet launched (grouped slots)
  std::map<std::vector<GraphKey>, hipGraphExec_t> group_graphs;
  bool use_graphs = getenv("FFMI_NO_GRAPHS") == nullptr;
  bool blob_fetch = !getenv("FFMI_BLOB_FETCH") || atoi(getenv("FFMI_BLOB_FETCH")) != 0;
  // largest one-item-per-request step that is graphed (FFMI_GRAPH_MAXT: A/B)
  int graph_max_t = getenv("FFMI_GRAPH_MAXT") ? atoi(getenv("FFMI_GRAPH_MAXT")) : 1024;

  // forward = forward_launch (stage the step, enqueue it) + forward_finish
  // (wait for it); SSM beam steps of several SSMs launch all, then finish
  // each (serve_spec_infer), so their latency-bound steps overlap
  bool inflight = false;
  // FFMI_STEP_TIMING=1 (diagnostics): per step, host time spent staging and
  // launching, the GPU span between events around the launch, and the
  // host's wait; summed per step size and printed at destruction
  bool step_timing = getenv("FFMI_STEP_TIMING") && atoi(getenv("FFMI_STEP_TIMING")) != 0;
  hipEvent_t st_ev[2] = {nullptr, nullptr};
  double st_t0 = 0, st_t1 = 0;
  struct StepTime { long n = 0; double launch = 0, gpu = 0, wait = 0, total = 0; };
  std::map<int, StepTime> st_sum;
  int st_T = 0;
  ffmi_status forward(int k) {
    ffmi_status st = forward_launch(k);
    if (st != FFMI_OK) return st;
    return forward_finish();
  }

  ffmi_status forward_launch(int k) {
    inflight = false;
    const int T = (int)ps.tokens.size();
    if (step_timing) {
      if (!st_ev[0]) {
        FFMI_HIP(hipEventCreate(&st_ev[0]));
        FFMI_HIP(hipEventCreate(&st_ev[1]));
      }
      st_t0 = now_us();
      st_T = T;
    }
    prof_this_step = prof_level == 1 && (prof_steps++ % prof_every) == 0;
    ffmi_batch_desc desc;
    ps.desc(&desc);
    // the embedding gather indexes the table by token id: reject bad ids on
    // the host instead of reading out of bounds on the device
    // (a chained beam step's -1 - i: entry i of the previous slot's ids,
    // themselves top-k picks in range)
    const long prev_n = cur_slot > 0 ? (long)slot_results[cur_slot - 1] : 0;
    for (int t = 0; t < T; ++t)
      FFMI_CHECK((desc.tokens[t].token_id >= 0 && desc.tokens[t].token_id < c.vocab_size) ||
                     (desc.tokens[t].token_id < 0 && -1L - desc.tokens[t].token_id < prev_n),
                 FFMI_ERR_INVALID);
    size_t bytes = 0;
    ffmi_status st = ffmi::batch_stage(batch, &desc, &bytes);
    if (st != FFMI_OK) return st;
    if (T == 0) return FFMI_OK;
    probs_h = reinterpret_cast<float *>(ids_h + cur_slot * slot_ints() + (size_t)T * k);
    // graphed: small steps, and tree-verify steps of one work item per
    // request (a fixed shape while the batch is full: T = 168 for 8 requests
    // of 21 tree tokens); prefill blocks stay eager (one-off shapes)
    const bool graph = use_graphs && !dbg && (T <= 64 || (batch->one_item_per_req && T <= graph_max_t)) &&
                       (o.tp_size == 1 || peer || rccl || ffmi::comm_size(o.comm) == 1) &&
                       !prof_on(0, T) &&
                       !prof_on(c.num_layers / 2, T);
    if (graph) {
      const GraphKey key{T, batch->num_work, batch->num_commits, k, tree_parity,
                         batch->commit_overlap ? 1 : 0,
                         (batch->one_item_per_req ? 1 : 0) | (batch->lds_tail ? 2 : 0),
                         batch->max_q, cur_slot, bytes};
      auto it = graphs.find(key);
      if (it == graphs.end()) {
        if (graphs.size() >= 512) clear_graphs();
        hipGraph_t g = nullptr;
        FFMI_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
        st = enqueue(k, bytes, false, T);
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
      if (step_timing) FFMI_HIP(hipEventRecord(st_ev[0], stream));
      FFMI_HIP(hipGraphLaunch(it->second, stream));
    } else {
      if (step_timing) FFMI_HIP(hipEventRecord(st_ev[0], stream));
      st = enqueue(k, bytes, true, T);
      if (st != FFMI_OK) return st;
    }
    if (step_timing) {
      FFMI_HIP(hipEventRecord(st_ev[1], stream));
      st_t1 = now_us();
    }
    inflight = true;
    return FFMI_OK;
  }

  // A chained slot staged for a grouped launch (chain_group): the staging
  // half of forward_launch; flush_pending captures / replays the group.
  ffmi_status stage_pending(int k, int slot) {
    const int T = (int)ps.tokens.size();
    ffmi_batch_desc desc;
    ps.desc(&desc);
    const long prev_n = slot > 0 ? (long)slot_results[slot - 1] : 0;
    for (int t = 0; t < T; ++t)
      FFMI_CHECK((desc.tokens[t].token_id >= 0 && desc.tokens[t].token_id < c.vocab_size) ||
                     (desc.tokens[t].token_id < 0 && -1L - desc.tokens[t].token_id < prev_n),
                 FFMI_ERR_INVALID);
    size_t bytes = 0;
    ffmi_status st = ffmi::batch_stage(batch, &desc, &bytes);
    if (st != FFMI_OK) return st;
    pend.push_back({slot, T, k, bytes,
                    GraphKey{T, batch->num_work, batch->num_commits, k, tree_parity,
                             batch->commit_overlap ? 1 : 0,
                             (batch->one_item_per_req ? 1 : 0) | (batch->lds_tail ? 2 : 0),
                             batch->max_q, slot, bytes}});
    return FFMI_OK;
  }
  ffmi_status flush_pending() {
    if (pend.empty()) return FFMI_OK;
    std::vector<GraphKey> keys;
    for (const auto &q : pend) keys.push_back(q.key);
    auto it = group_graphs.find(keys);
    if (it == group_graphs.end()) {
      if (group_graphs.size() >= 256) clear_graphs();
      hipGraph_t g = nullptr;
      ffmi_status st = FFMI_OK;
      FFMI_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
      for (const auto &q : pend) {
        cur_slot = q.slot;
        batch = chain_batch[q.slot];
        st = enqueue(q.k, q.bytes, false, q.T);
        if (st != FFMI_OK) break;
      }
      cur_slot = 0;
      batch = chain_batch[0];
      const hipError_t ce = hipStreamEndCapture(stream, &g);
      if (st != FFMI_OK || ce != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        pend.clear();
        if (st != FFMI_OK) return st;
        FFMI_HIP(ce);
      }
      hipGraphExec_t ex = nullptr;
      const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ie != hipSuccess) pend.clear();
      FFMI_HIP(ie);
      it = group_graphs.emplace(keys, ex).first;
    }
    pend.clear();
    FFMI_HIP(hipGraphLaunch(it->second, stream));
    inflight = true;
    return FFMI_OK;
  }

  ffmi_status forward_finish() {
    if (!inflight) return FFMI_OK;
    inflight = false;
    ffmi_status st;
    const double tw = step_timing ? now_us() : 0;
    FFMI_HIP(hipStreamSynchronize(stream));
    if (step_timing) {
      const double te = now_us();
      float ms = 0;
      (void)hipEventElapsedTime(&ms, st_ev[0], st_ev[1]);
      StepTime &q = st_sum[st_T];
      q.n++;
      q.launch += st_t1 - st_t0;
      q.gpu += ms * 1e3;
      q.wait += te - tw;
      q.total += te - st_t0;
    }
    // any attached transport (also under the RCCL path, whose chunks that fit
    // the exchange buffer still go over it) reports timeouts / errors here
    if ((peer || (o.comm && ffmi::comm_peer_attached(o.comm))) &&
        (st = ffmi::comm_status(o.comm)) != FFMI_OK)
      return st;
    if (mode == FFMI_MODEL_TREE) tree_parity ^= 1;
    if (!recs.empty()) prof_collect();
    return FFMI_OK;
  }

  void clear_graphs() {
    for (auto &kv : graphs) (void)hipGraphExecDestroy(kv.second);
    graphs.clear();
    for (auto &kv : group_graphs) (void)hipGraphExecDestroy(kv.second);
    group_graphs.clear();
  }

  // everything a step puts on the stream (no host synchronisation inside)
  ffmi_status enqueue(int k, size_t blob_bytes, bool record_upload, int T) {
    const int H = c.hidden, V = c.vocab_size;
    const float eps = c.rms_eps;
    const ffmi_stream s = (ffmi_stream)stream;
    ffmi_status st;
#define TRY(x) \
  do { if ((st = (x)) != FFMI_OK) return st; } while (0)
    // the step's blob: fetched by the first kernel from the mapped staging
    // (default), or a separate H2D copy (FFMI_BLOB_FETCH=0: A/B)
    if (!blob_fetch) TRY(ffmi::batch_copy(batch, blob_bytes, stream, record_upload));
    const bool ptail = prof_on(0, T);
    int pr = 0;
    ffmi::Partials down_part;
    // FFMI_MARKERS=<hidden>: clock markers between the last layer's kernels
    // of the model with that hidden size (diagnostics, ffmi_debug_markers)
    // (FFMI_MARKERS_T: only steps of that many tokens, e.g. 168 = a full
    // verify batch; the attention stamps then come from the same launch)
    static const int marker_h = getenv("FFMI_MARKERS") ? atoi(getenv("FFMI_MARKERS")) : 0;
    static const int marker_t = getenv("FFMI_MARKERS_T") ? atoi(getenv("FFMI_MARKERS_T")) : 0;
    int mark_i = 0;
    const bool fuse = (fuse_norms == 2 || (fuse_norms == 1 && H >= 2048)) && !dbg &&
                      o.tp_size == 1 && T <= 32 && H % 32 == 0 && Hl % 32 == 0 && H <= 4096;
    // the residual norms inside the transport's all-reduces (tp_fuse_norm)
    const bool arn = peer && !solo && o.tp_size > 1 && (tp_fuse_norm == 2 || (tp_fuse_norm == 1 && !dbg));
    for (int l = 0; l < c.num_layers; ++l) {
      Layer &L = layers[l];
      const bool on = prof_on(l, T);
      const bool mark_on = marker_h == c.hidden && l == c.num_layers - 1 && (!marker_t || T == marker_t);
      if (marker_h) ffmi::attn_stamp_gate(mark_on);
      auto mk = [&]() {
        if (mark_on) (void)ffmi::launch_marker(mark_i++, stream);
      };
      // (the marker buffer is allocated by an eager launch, never in a capture)
      if (marker_h && l == 0 && record_upload) (void)ffmi::launch_marker(63, stream);
      mk();
      // split-K GEMMs leave their partial slabs for the next kernel to combine
      // (rope-store for qkv; the residual norm for o/down when there is no
      // all-reduce in between) instead of a separate reduce pass
      const int XP = (packed ? FFMI_X_PACKED : 0) | wstream;
      // fused residual norms (see fuse_norms): from layer 1 on, the attention
      // norm is the qkv GEMM's prologue on the residual the down projection
      // left, and every post-attention norm the gate/up GEMM's
      const bool fz_in = fuse && l > 0;
      ffmi::FuseArgs fz_qkv, fz_o, fz_gu, fz_d;
      if (fuse) {
        fz_o.kind = fz_d.kind = 1;
        fz_o.res_in = fz_d.res_in = res;
        fz_o.ss_out = ss_o, fz_d.ss_out = ss_d;
        fz_qkv.kind = fz_gu.kind = 2;
        fz_qkv.ss_in = ss_d, fz_gu.ss_in = ss_o;
        fz_qkv.nss = fz_gu.nss = H / 16;
        fz_qkv.wnorm = L.in_norm, fz_gu.wnorm = L.post_norm;
        fz_qkv.eps = fz_gu.eps = eps;
      }
      if (!fz_in && !(arn && l > 0)) {  // (arn: the previous down all-reduce normalised)
        pr = prof_begin(on);
        // layer 0: the embedding lookup gathers straight into the first norm
        // (embedding_kernels.cu:233-244; res = the looked-up rows)
        FFMI_HIP(ffmi::launch_rmsnorm(l == 0 ? embed : res, l == 0 ? nullptr : proj, L.in_norm, res,
                                      h, T, H, eps, stream, packed,
                                      l == 0 ? ffmi::Partials() : down_part,
                                      l == 0 ? (blob_fetch ? batch->host : batch->dev) : nullptr,
                                      l == 0 && blob_fetch ? batch->dev : nullptr, blob_bytes,
                                      cur_slot > 0 ? ids_dev + (size_t)(cur_slot - 1) * (slot_ints() / 2)
                                                   : nullptr));
        // the staging is free for the next step once the fetch has read it
        if (l == 0 && blob_fetch && record_upload) FFMI_HIP(hipEventRecord(batch->uploaded, stream));
        prof_end(pr, NORM, (double)T * H * 2 * (l == 0 ? 3 : 4), 0);
        mk();
      }
      if (dbg) {
        // residual stream after layer l-1 (layer 0: the embedding rows; arn:
        // current on this rank's rows only, not kept)
        if (l == 0 || !arn) TRY(dbg_copy(l == 0 ? FFMI_DBG_EMBED : FFMI_DBG_HIDDEN, l == 0 ? 0 : l - 1, res, T));
        TRY(dbg_copy(FFMI_DBG_ATTN_NORM, l, h, T));
      }
      pr = prof_begin(on);
      ffmi::Partials qkv_part;
      FFMI_HIP(ffmi::launch_gemm(fz_in ? res : h, L.wqkv, qkv, (float *)ws, ws_bytes, T, 3 * Hl, H,
                                 fz_in ? wstream : XP, stream, &qkv_part, 0,
                                 fz_in ? &fz_qkv : nullptr));
      prof_end(pr, GEMM_QKV, gemm_bytes(T, 3 * Hl, 3 * Hl, H), 2.0 * T * 3 * Hl * H);
      mk();
      if (dbg) TRY(dbg_gemm_out(FFMI_DBG_QKV, l, qkv, qkv_part, T));
      pr = prof_begin(on);
      ffmi::OprojArgs oa;
      if (fuse_ao && !fuse) {
        oa.wo = L.wo, oa.slab = oslab, oa.N = H, oa.max_T = oslab_T;
        oa.wts = ffmi::w_tile_stride(Hl / 32), oa.wks = ffmi::w_k_stride(H / 16);
      }
      TRY(ffmi::attn_forward(L.attn, batch, qkv, qkv_part, att, s,
                             mode == FFMI_MODEL_TREE ? tree_parity : -1,
                             oa.wo ? &oa : nullptr));
      prof_end(pr, ATTENTION, on ? attn_bytes() : 0, 0);
      mk();
      if (dbg) TRY(dbg_copy(FFMI_DBG_ATTN_OUT, l, att, T));
      ffmi::Partials o_part;
      if (oa.done) {  // the attention projected: one slab per head
        o_part.p = oslab, o_part.S = heads_l, o_part.NP = H;
      } else if (fuse) {  // o projection + residual add (+ sums of squares): res in place
        pr = prof_begin(on);
        FFMI_HIP(ffmi::launch_gemm(att, L.wo, res, (float *)ws, ws_bytes, T, H, Hl, XP, stream,
                                   nullptr, 0, &fz_o));
        prof_end(pr, GEMM_O, gemm_bytes(T, H, H, Hl), 2.0 * T * H * Hl);
        mk();
      } else if (o.tp_size == 1 || solo) {
        pr = prof_begin(on);
        FFMI_HIP(ffmi::launch_gemm(att, L.wo, proj, (float *)ws, ws_bytes, T, H, Hl, XP, stream,
                                   H <= 8192 ? &o_part : nullptr));
        prof_end(pr, GEMM_O, gemm_bytes(T, H, H, Hl), 2.0 * T * H * Hl);
        mk();
      } else {  // GEMM + all-reduce (overlapped over xGMI): timed together
        pr = prof_begin(on);
        ar_drop_now = l == ar_drop_layer && ar_drop_which == 0;
        if (arn) TRY(rowpar_gemm_allreduce_norm(att, L.wo, Hl, T, XP, L.post_norm));
        else TRY(rowpar_gemm_allreduce(att, L.wo, Hl, proj, T, XP));
        ar_drop_now = false;
        prof_end(pr, ALLREDUCE, gemm_bytes(T, H, H, Hl), 2.0 * T * H * Hl);
        mk();
      }
      if (dbg && !arn) TRY(dbg_gemm_out(FFMI_DBG_O_PROJ, l, proj, o_part, T));
      if (!fuse && !arn) {
        pr = prof_begin(on);
        FFMI_HIP(ffmi::launch_rmsnorm(res, proj, L.post_norm, res, h, T, H, eps, stream, packed,
                                      o_part));
        prof_end(pr, NORM, (double)T * H * 2 * 4, 0);
        mk();
      }
      if (dbg) TRY(dbg_copy(FFMI_DBG_FFN_NORM, l, h, T));
      pr = prof_begin(on);
      const int YP = packed ? FFMI_Y_PACKED : 0;
      if (fuse)
        FFMI_HIP(ffmi::launch_gemm(res, L.wgu, mlp, (float *)ws, ws_bytes, T, Fl, H,
                                   FFMI_EPI_SILU_MUL | YP | wstream, stream, nullptr, 0, &fz_gu));
      else
        TRY(ffmi_linear_ws(h, L.wgu, mlp, T, Fl, H, FFMI_EPI_SILU_MUL | XP | YP, ws, ws_bytes, s));
      prof_end(pr, GEMM_GATE_UP, gemm_bytes(T, 2 * Fl, Fl, H), 2.0 * T * 2 * Fl * H);
      mk();
      if (dbg) TRY(dbg_copy(FFMI_DBG_MLP_ACT, l, mlp, T));
      if (fuse) {  // down projection + residual add (+ sums of squares)
        pr = prof_begin(on);
        FFMI_HIP(ffmi::launch_gemm(mlp, L.wd, res, (float *)ws, ws_bytes, T, H, Fl, XP, stream,
                                   nullptr, 0, &fz_d));
        prof_end(pr, GEMM_DOWN, gemm_bytes(T, H, H, Fl), 2.0 * T * H * Fl);
        mk();
        mk();
      } else if (o.tp_size == 1 || solo) {
        pr = prof_begin(on);
        FFMI_HIP(ffmi::launch_gemm(mlp, L.wd, proj, (float *)ws, ws_bytes, T, H, Fl, XP, stream,
                                   H <= 8192 ? &down_part : nullptr));
        prof_end(pr, GEMM_DOWN, gemm_bytes(T, H, H, Fl), 2.0 * T * H * Fl);
        mk();
        mk();  // (two back to back: the marker-to-marker boundary itself)
      } else {
        pr = prof_begin(on);
        ar_drop_now = l == ar_drop_layer && ar_drop_which == 1;
        // (arn: the next layer's input norm, or the final norm, rides along)
        if (arn)
          TRY(rowpar_gemm_allreduce_norm(mlp, L.wd, Fl, T, XP,
                                         l + 1 < c.num_layers ? layers[l + 1].in_norm : final_norm));
        else TRY(rowpar_gemm_allreduce(mlp, L.wd, Fl, proj, T, XP));
        ar_drop_now = false;
        prof_end(pr, ALLREDUCE, gemm_bytes(T, H, H, Fl), 2.0 * T * H * Fl);
        mk();
      }
      if (dbg && !arn) TRY(dbg_gemm_out(FFMI_DBG_DOWN, l, proj, down_part, T));
    }
    const int XP = (packed ? FFMI_X_PACKED : 0) | wstream;
    // (markers also between the tail's kernels: final norm, lm_head, sampling)
    const bool tail_mark = marker_h == c.hidden && (!marker_t || T == marker_t);
    auto mkt = [&]() {
      if (tail_mark) (void)ffmi::launch_marker(mark_i++, stream);
    };
    if (!arn) {  // (arn: the last down all-reduce applied the final norm)
      pr = prof_begin(ptail);
      if (fuse)  // res already holds the last residual add
        FFMI_HIP(ffmi::launch_rmsnorm(res, nullptr, final_norm, nullptr, h, T, H, eps, stream, packed));
      else
        FFMI_HIP(ffmi::launch_rmsnorm(res, proj, final_norm, res, h, T, H, eps, stream, packed,
                                      down_part));
      prof_end(pr, NORM, (double)T * H * 2 * 4, 0);
    }
    mkt();
    if (dbg) {
      if (!arn) TRY(dbg_copy(FFMI_DBG_HIDDEN, c.num_layers - 1, res, T));
      TRY(dbg_copy(FFMI_DBG_HIDDEN, c.num_layers, h, T));
      dbg_T = T;
    }
    pr = prof_begin(ptail);
    TRY(ffmi_linear_ws(h, lm, logits, T, Vl, H, FFMI_EPI_NONE | XP, ws, ws_bytes, s));
    prof_end(pr, GEMM_LM_HEAD, gemm_bytes(T, Vl, Vl, H), 2.0 * T * Vl * H);
    mkt();
    pr = prof_begin(ptail);
    TRY(enqueue_sampling(k, T));
    prof_end(pr, SAMPLING, (double)T * V * 2, 0);
    mkt();
#undef TRY
    return FFMI_OK;
  }

  // softmax + argmax / arg-top-k of the step's logits into the pinned results
  ffmi_status enqueue_sampling(int k, int T) {
    const int V = c.vocab_size;
    const ffmi_stream s = (ffmi_stream)stream;
    ffmi_status st;
#define TRY(x) \
  do { if ((st = (x)) != FFMI_OK) return st; } while (0)
    // ids [T*k] then probs [T*k] back to back.  The sampling kernel writes
    // them straight into the pinned host buffer (a few bytes per row over
    // PCIe, visible after the stream synchronisation like a copy kernel's
    // stores), so a step needs no result-copy launch; FFMI_RESULT_COPY=1
    // keeps the device buffer + copy (A/B runs)
    int32_t *ids_o = result_copy ? ids_d : ids_h + cur_slot * slot_ints();
    float *probs_o = reinterpret_cast<float *>(ids_o + (size_t)T * k);
    if (Vl != V) {
      // sharded softmax / top-k: three record exchanges, then the merge
      TRY(ffmi_vocab_shard_topk(o.comm, logits, T, Vl, k, ids_o, probs_o, xch, s));
    } else {
      // the ids also to device memory: the next chained beam step's
      // embedding gather reads them there
      FFMI_CHECK(k >= 1 && k <= 4 && k <= V, FFMI_ERR_INVALID);
      FFMI_HIP(ffmi::launch_argmax(logits, T, V, k, ids_o, probs_o, stream, topk_ws, topk_ws_bytes,
                                   mode == FFMI_MODEL_BEAM
                                       ? ids_dev + (size_t)cur_slot * (slot_ints() / 2)
                                       : nullptr));
    }
    if (result_copy)
      FFMI_HIP(hipMemcpyAsync(ids_h + cur_slot * slot_ints(), ids_d, (size_t)T * k * 8,
                              hipMemcpyDeviceToHost, stream));
#undef TRY
    return FFMI_OK;
  }

  ffmi_status run_inc(const BatchConfig &bc, InferenceResult *ir) override {
    if (mode != FFMI_MODEL_INC) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens, FFMI_ERR_INVALID);
    pack_inc(bc, o.max_requests, slots, &ps);
    cur_slot = 0;
    ffmi_status st = forward(1);
    if (st != FFMI_OK) return st;
    memcpy(ir->token_ids, ids_h, bc.num_tokens * sizeof(int32_t));
    return FFMI_OK;
  }
  ffmi_status run_tree(const TreeVerifyBatchConfig &bc, InferenceResult *ir) override {
    if (mode != FFMI_MODEL_TREE) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens, FFMI_ERR_INVALID);
    pack_tree(bc, o.max_requests, slots, &ps);
    cur_slot = 0;
    ffmi_status st = forward(1);
    if (st != FFMI_OK) return st;
    memcpy(ir->token_ids, ids_h, bc.num_tokens * sizeof(int32_t));
    return FFMI_OK;
  }
  ffmi_status run_beam(const BeamSearchBatchConfig &bc, BeamInferenceResult *ir) override {
    ffmi_status st = beam_launch(bc);
    if (st != FFMI_OK) return st;
    return beam_collect(ir);
  }
  ffmi_status beam_launch(const BeamSearchBatchConfig &bc) override {
    return beam_launch_chained(bc, 0);
  }
  ffmi_status beam_collect(BeamInferenceResult *ir) override { return beam_collect_chained(0, ir); }
  // an unsharded SSM, not under debug capture
  bool can_chain_beam() const override {
    return chain_ok && mode == FFMI_MODEL_BEAM && o.tp_size == 1 && !dbg && !result_copy;
  }
  ffmi_status beam_launch_chained(const BeamSearchBatchConfig &bc, int slot) override {
    if (mode != FFMI_MODEL_BEAM) return FFMI_ERR_INVALID;
    FFMI_CHECK(bc.num_tokens <= o.max_tokens && slot >= 0 && slot < kChain, FFMI_ERR_INVALID);
    FFMI_CHECK(slot == 0 || can_chain_beam(), FFMI_ERR_INVALID);
    if (!chain_batch[slot]) {
      ffmi_batch_dev *b = nullptr;
      ffmi_status st = ffmi_batch_create((o.max_tokens + 15) & ~15, o.max_requests, &b);
      if (st != FFMI_OK) return st;
      chain_batch[slot] = b;
    }
    pack_beam(bc, o.max_requests, slots, &ps);
    // a chained step's -1 - i (scheduler entry i of the previous slot) ->
    // -1 - its [T][k] index, which the gather reads from device memory
    for (auto &ti : ps.tokens)
      if (ti.token_id < 0) {
        const long i = -1L - ti.token_id;
        FFMI_CHECK(slot > 0 && i < (long)slot_map[slot - 1].size(), FFMI_ERR_INVALID);
        ti.token_id = -1 - slot_map[slot - 1][i];
      }
    const int k = ps.topk;
    if (step_timing && slot == 0) {
      if (!chain_t0) FFMI_HIP(hipEventCreate(&chain_t0));
      FFMI_HIP(hipEventRecord(chain_t0, stream));
    }
    cur_slot = slot;
    batch = chain_batch[slot];
    slot_results[slot] = (size_t)bc.num_tokens * k;
    beam_result_layout(bc, &slot_map[slot]);
    // grouped (chain_group): slots 1 .. kChain-2 staged, launched g at a time
    // (graphed shapes only; anything else first launches what is staged)
    const int Ts = (int)ps.tokens.size();
    const bool grp = chain_group >= 2 && slot >= 1 && slot <= kChain - 2 && use_graphs && !dbg &&
                     prof_level == 0 && Ts > 0 && Ts <= 64;
    ffmi_status st;
    if (grp) {
      st = stage_pending(k, slot);
      if (st == FFMI_OK && ((slot - 1) % chain_group == chain_group - 1 || slot == kChain - 2)) {
        cur_slot = 0;
        batch = chain_batch[0];
        st = flush_pending();
      }
    } else {
      cur_slot = 0;
      batch = chain_batch[0];
      st = flush_pending();
      cur_slot = slot;
      batch = chain_batch[slot];
      if (st == FFMI_OK) st = forward_launch(k);
    }
    batch = chain_batch[0];
    cur_slot = 0;
    // Events let the scheduler replay slot d's bookkeeping while later slots
    // run.  One behind every slot cost the GPU more than the replay it
    // overlapped (same-box A/B, tokens/s: 1333 with, 1342 with none, 1326
    // stepwise); FFMI_CHAIN_EVENTS: 0 none (the collect waits for the whole
    // chain), 1 every slot, 2 (default) one, behind the second-to-last slot:
    // the replays of slots 0 .. D-2 then run while slot D-1 computes
    static const int slot_events =
        getenv("FFMI_CHAIN_EVENTS") ? atoi(getenv("FFMI_CHAIN_EVENTS")) : 2;
    const bool record = slot_events == 1 || (slot_events == 2 && slot == kChain - 2);
    if (st == FFMI_OK) last_slot = slot;
    if (st == FFMI_OK && record) {
      // (so that the scheduler can collect this slot while later ones run)
      if (!slot_ev[slot])
        FFMI_HIP(hipEventCreateWithFlags(&slot_ev[slot], step_timing ? 0 : hipEventDisableTiming));
      FFMI_HIP(hipEventRecord(slot_ev[slot], stream));
      slot_ev_live[slot] = true;
      last_slot = slot;
    }
    return st;
  }
  ffmi_status beam_collect_chained(int slot, BeamInferenceResult *ir) override {
    FFMI_CHECK(slot >= 0 && slot < kChain, FFMI_ERR_INVALID);
    {  // (grouped slots still staged go out first)
      ffmi_status st = flush_pending();
      if (st != FFMI_OK) return st;
    }
    int ev = -1;  // the first live event at or after this slot, before the last
    for (int e = slot; e < last_slot && ev < 0; ++e)
      if (slot_ev_live[e] && slot_ev[e]) ev = e;
    if (ev >= 0) {
      // later slots still run: wait for this one (and those before it) only
      FFMI_HIP(hipEventSynchronize(slot_ev[ev]));
    } else {
      const int ls = last_slot;
      ffmi_status st = forward_finish();  // (every launched step: one stream)
      if (st != FFMI_OK) return st;
      for (bool &b : slot_ev_live) b = false;
      // FFMI_STEP_TIMING: the GPU span of a whole chain, from the event before
      // slot 0's launch to the one after the last slot
      if (step_timing && ls > 0 && chain_t0) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, chain_t0, slot_ev[ls]) == hipSuccess) {
          StepTime &q = st_sum[-(ls + 1)];
          q.n++;
          q.gpu += ms * 1e3;
        }
      }
      last_slot = -1;
    }
    const size_t n = slot_results[slot];
    const int32_t *ids = ids_h + slot * slot_ints();
    const float *pr = reinterpret_cast<const float *>(ids + n);
    const std::vector<int> &map = slot_map[slot];
    for (size_t i = 0; i < map.size(); ++i) {
      ir->token_ids[i] = ids[map[i]];
      ir->probs[i] = pr[map[i]];
      ir->parent_id[i] = 0;
    }
    return FFMI_OK;
  }
};

}  // namespace

ffmi_status create_llama_gpu(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                             ffmi_model **out) {
  FFMI_CHECK(cfg && o && out, FFMI_ERR_INVALID);
  FFMI_CHECK(o->tp_size >= 1 && o->tp_rank >= 0 && o->tp_rank < o->tp_size, FFMI_ERR_INVALID);
  FFMI_CHECK(o->tp_size == 1 || o->comm, FFMI_ERR_INVALID);
  FFMI_CHECK(o->max_tokens > 0 && o->max_tokens <= BatchConfig::MAX_NUM_TOKENS, FFMI_ERR_INVALID);
  FFMI_CHECK(o->max_requests > 0 && o->max_requests <= BatchConfig::MAX_NUM_REQUESTS,
             FFMI_ERR_INVALID);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return FFMI_ERR_NO_DEVICE;
  LlamaGPU *m = new LlamaGPU();
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
