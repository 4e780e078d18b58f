// api.cpp -- C ABI of the kernel-level boundary (include/ffmi.h).
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <algorithm>
#include <climits>

#include "ffmi_internal.h"
#include "collective.h"

static thread_local std::string g_last_error;

void ffmi_set_last_error(const char *msg, const char *file, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s (%s:%d)", msg, file, line);
  g_last_error = buf;
  if (getenv("FFMI_VERBOSE_ERRORS")) fprintf(stderr, "[ffmi] error: %s\n", buf);
}

extern "C" const char *ffmi_last_error(void) { return g_last_error.c_str(); }

extern "C" const char *ffmi_status_str(ffmi_status s) {
  switch (s) {
    case FFMI_OK: return "ok";
    case FFMI_ERR_INVALID: return "invalid argument";
    case FFMI_ERR_HIP: return "hip error";
    case FFMI_ERR_NCCL: return "rccl error";
    case FFMI_ERR_OOM: return "out of device memory";
    case FFMI_ERR_UNSUPPORTED: return "unsupported";
    case FFMI_ERR_NO_DEVICE: return "no gfx950 device";
  }
  return "unknown";
}

// 0.2: ffmi_attn_cfg.full_precision and ffmi_model_opts.full_precision
// appended (struct sizes changed), the *_f32 entry points added
// 0.3: ffmi_rm_config.spec_extensions
extern "C" const char *ffmi_version(void) { return "ffmi 0.3 (gfx950)"; }

// ---------------------------------------------------------------------------
// batch metadata
// ---------------------------------------------------------------------------
static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

extern "C" ffmi_status ffmi_batch_create(int max_tokens, int max_requests, ffmi_batch_dev **out) {
  FFMI_CHECK(max_tokens > 0 && max_requests > 0 && out, FFMI_ERR_INVALID);
  ffmi_batch_dev *b = new ffmi_batch_dev();
  b->max_tokens = max_tokens;
  b->max_requests = max_requests;
  // header + tokens + work (<= tokens) + commits (<= tokens) + masks
  b->cap = align16(sizeof(ffmi::BatchHeader)) + align16((size_t)max_tokens * sizeof(ffmi_token_info)) +
           align16((size_t)max_tokens * sizeof(ffmi::WorkDev)) +
           align16((size_t)max_tokens * sizeof(ffmi_commit_info)) +
           align16((size_t)max_requests * FFMI_MAX_TREE * sizeof(uint64_t)) + 64;
  // fine-grained (uncached on the device) and mapped: the model's first
  // kernel reads the step's blob straight from here (launch_rmsnorm's fetch)
  if (hipHostMalloc((void **)&b->host, b->cap, hipHostMallocCoherent | hipHostMallocMapped) !=
          hipSuccess ||
      hipMalloc((void **)&b->dev, b->cap) != hipSuccess) {
    delete b;
    ffmi_set_last_error("batch alloc", __FILE__, __LINE__);
    return FFMI_ERR_OOM;
  }
  memset(b->host, 0, b->cap);
  FFMI_HIP(hipMemset(b->dev, 0, b->cap));
  FFMI_HIP(hipEventCreateWithFlags(&b->uploaded, hipEventDisableTiming));
  *out = b;
  return FFMI_OK;
}

extern "C" void ffmi_batch_destroy(ffmi_batch_dev *b) {
  if (!b) return;
  if (b->uploaded) {
    (void)hipEventSynchronize(b->uploaded);
    (void)hipEventDestroy(b->uploaded);
  }
  if (b->host) (void)hipHostFree(b->host);
  if (b->dev) (void)hipFree(b->dev);
  delete b;
}

namespace ffmi {
// Host half of the upload: fill the pinned staging blob; returns its size.
ffmi_status batch_stage(ffmi_batch_dev *b, const ffmi_batch_desc *d, size_t *bytes) {
  FFMI_CHECK(b && d && bytes, FFMI_ERR_INVALID);
  FFMI_CHECK(d->num_tokens >= 0 && d->num_tokens <= b->max_tokens, FFMI_ERR_INVALID);
  FFMI_CHECK(d->num_work >= 0 && d->num_work <= b->max_tokens, FFMI_ERR_INVALID);
  FFMI_CHECK(d->num_commits >= 0 && d->num_commits <= b->max_tokens, FFMI_ERR_INVALID);
  FFMI_CHECK(d->num_mask_reqs >= 0 && d->num_mask_reqs <= b->max_requests, FFMI_ERR_INVALID);
  // the pinned staging may still be read by the previous async copy
  FFMI_HIP(hipEventSynchronize(b->uploaded));
  ffmi::BatchHeader h;
  h.num_tokens = d->num_tokens;
  h.num_work = d->num_work;
  h.num_commits = d->num_commits;
  h.num_mask_reqs = d->num_mask_reqs;
  size_t off = ffmi::kBlobWorkOffset;
  h.off_work = (int)off;
  {
    // lowest slot this step writes for each item's request (its stores and
    // the TREE commits): the attention kernel may load keys below it before
    // its own KV-update prologue has run
    // The fused attention stages every slot the step writes for the item's
    // request in an LDS tail [tail0, tail0 + kTailSlots) and takes the
    // request's commits from the work item (lds_tail: all items fit)
    ffmi::WorkDev *wd = reinterpret_cast<ffmi::WorkDev *>(b->host + off);
    b->lds_tail = true;
    for (int wi = 0; wi < d->num_work; ++wi) {
      ffmi::WorkDev x{};
      x.w = d->work[wi];
      int clean = INT32_MAX, hi = -1;
      for (int t = 0; t < d->num_tokens; ++t)
        if (d->tokens[t].req == x.w.req && d->tokens[t].store_slot >= 0) {
          clean = std::min(clean, (int)d->tokens[t].store_slot);
          hi = std::max(hi, (int)d->tokens[t].store_slot);
        }
      for (int c = 0; c < d->num_commits; ++c)
        if (d->commits[c].req == x.w.req && d->commits[c].depth >= 0) {
          clean = std::min(clean, (int)d->commits[c].depth);
          hi = std::max(hi, (int)d->commits[c].depth);
          if (x.ncommit < ffmi::kItemCommits && d->commits[c].src_token <= 32767 &&
              d->commits[c].depth <= 32767) {
            x.cm_src[x.ncommit] = (int16_t)d->commits[c].src_token;
            x.cm_depth[x.ncommit] = (int16_t)d->commits[c].depth;
          } else {
            b->lds_tail = false;
          }
          ++x.ncommit;
        }
      x.clean = clean;
      x.tail0 = (std::min(clean, (int)x.w.kv_len) / 32) * 32;
      x.told = std::min(clean, (int)x.w.kv_len) - x.tail0;
      const int end = std::max(hi + 1, (int)x.w.kv_len);
      if (end - x.tail0 > ffmi::kTailSlots) {
        b->lds_tail = false;
      } else if (clean < end) {  // every slot in [clean, end) written this step
        bool dense[ffmi::kTailSlots] = {};
        for (int t = 0; t < d->num_tokens; ++t)
          if (d->tokens[t].req == x.w.req && d->tokens[t].store_slot >= clean)
            dense[d->tokens[t].store_slot - clean] = true;
        for (int c = 0; c < d->num_commits; ++c)
          if (d->commits[c].req == x.w.req && d->commits[c].depth >= clean)
            dense[d->commits[c].depth - clean] = true;
        for (int sl = clean; sl < end; ++sl)
          if (!dense[sl - clean]) b->lds_tail = false;
      }
      for (int j = 0; j < FFMI_ATTN_QTILE; ++j) {
        const int t = x.w.q_start + std::min(j, std::max(x.w.q_count - 1, 0));
        const int pos = t < d->num_tokens ? d->tokens[t].pos : 0;
        // the kernels clamp to their table (rows = cache slots <= 32768)
        x.rope_pos[j] = (int16_t)std::min(std::max(pos, 0), 32767);
      }
      wd[wi] = x;
    }
  }
  off += align16(d->num_work * sizeof(ffmi::WorkDev));
  h.off_tokens = (int)off;
  {
    // kernels read the query-major visibility word; derive it here from the
    // reference's key-major per-request bitmask (the caller's value is ignored)
    ffmi_token_info *tk = reinterpret_cast<ffmi_token_info *>(b->host + off);
    memcpy(tk, d->tokens, d->num_tokens * sizeof(ffmi_token_info));
    for (int t = 0; t < d->num_tokens; ++t) {
      uint64_t v = 0;
      const int r = tk[t].req, n = tk[t].tree_len < FFMI_MAX_TREE ? tk[t].tree_len : FFMI_MAX_TREE;
      const int bit = tk[t].tree_bit;
      if (n > 0 && r >= 0 && r < d->num_mask_reqs && bit >= 0 && bit < 64) {
        const uint64_t *m = d->masks + (size_t)r * FFMI_MAX_TREE;
        for (int j = 0; j < n; ++j) v |= ((m[j] >> bit) & 1ull) << j;
      }
      tk[t].tree_vis = v;
    }
  }
  off += align16(d->num_tokens * sizeof(ffmi_token_info));
  h.off_commits = (int)off;
  if (d->num_commits) memcpy(b->host + off, d->commits, d->num_commits * sizeof(ffmi_commit_info));
  off += align16(d->num_commits * sizeof(ffmi_commit_info));
  // the bitmask table itself stays on the host (folded into tree_vis above)
  h.num_mask_reqs = 0;
  h.off_masks = (int)off;
  memcpy(b->host, &h, sizeof(h));
  FFMI_CHECK(off <= b->cap, FFMI_ERR_INVALID);
  b->num_tokens = d->num_tokens;
  b->num_work = d->num_work;
  b->num_commits = d->num_commits;
  b->num_mask_reqs = d->num_mask_reqs;
  b->max_q = 0;
  b->one_item_per_req = true;
  for (int wi = 0; wi < d->num_work; ++wi) {
    FFMI_CHECK(d->work[wi].q_count >= 0 && d->work[wi].q_count <= FFMI_ATTN_QTILE,
               FFMI_ERR_INVALID);
    b->max_q = std::max(b->max_q, (int)d->work[wi].q_count);
    if (wi > 0 && d->work[wi].req == d->work[wi - 1].req) b->one_item_per_req = false;
  }
  b->commit_overlap = false;
  for (int c = 0; c < d->num_commits && !b->commit_overlap; ++c)
    for (int t = 0; t < d->num_tokens; ++t)
      if (d->tokens[t].req == d->commits[c].req && d->tokens[t].store_slot == d->commits[c].depth) {
        b->commit_overlap = true;
        break;
      }
  *bytes = off;
  return FFMI_OK;
}

// Device half: one async H2D copy of the staged bytes (capturable in a graph;
// record_event guards the staging against the next stage call).
ffmi_status batch_copy(ffmi_batch_dev *b, size_t bytes, hipStream_t s, bool record_event) {
  FFMI_HIP(hipMemcpyAsync(b->dev, b->host, bytes, hipMemcpyHostToDevice, s));
  if (record_event) FFMI_HIP(hipEventRecord(b->uploaded, s));
  return FFMI_OK;
}
}  // namespace ffmi

extern "C" ffmi_status ffmi_batch_upload(ffmi_batch_dev *b, const ffmi_batch_desc *d,
                                         ffmi_stream stream) {
  size_t bytes = 0;
  const ffmi_status st = ffmi::batch_stage(b, d, &bytes);
  if (st != FFMI_OK) return st;
  return ffmi::batch_copy(b, bytes, (hipStream_t)stream, true);
}

// ---------------------------------------------------------------------------
// attention handles
// ---------------------------------------------------------------------------
struct ffmi_attn {
  ffmi_attn_cfg cfg;
  int slots = 0;
  uint16_t *kc = nullptr, *vc = nullptr, *qbuf = nullptr, *stage = nullptr;
  int parity = 0;  // TREE staging half written by the next public-API step
  float *rope = nullptr;
};

// cos/sin table, same arithmetic as the reference's apply_rotary_embedding_hf
// (inc_multihead_self_attention.cu:701-725): freq = pos * (1.0 /
// pow(theta, 2i/d)) in the float/double mix used there, the llama3 scaling
// branch in f32 (its wavelength is taken of pos * inv_freq, as there), and
// cos/sin in f32.
static void rope_table(std::vector<float> &tab, int max_pos, int d, const ffmi_attn_cfg *cfg) {
  const int h = d / 2;
  std::vector<double> inv(h);
  for (int i = 0; i < h; ++i) {
    volatile float ex = (float)2 * (float)i / (float)d;
    inv[i] = 1.0 / (double)powf(cfg->rope_theta, ex);
  }
  const bool l3 = cfg->rope_llama3 != 0;
  const float pi = 3.141592654f;  // CUDART_PI_F
  const float low_wl = l3 ? (float)cfg->rope_original_max_pos / cfg->rope_low_freq_factor : 0.f;
  const float high_wl = l3 ? (float)cfg->rope_original_max_pos / cfg->rope_high_freq_factor : 0.f;
  tab.resize((size_t)max_pos * d);
  for (int p = 0; p < max_pos; ++p)
    for (int i = 0; i < h; ++i) {
      volatile float freq = (float)((double)p * inv[i]);
      if (l3) {
        const float wavelen = 2 * pi / freq;
        if (wavelen < high_wl) {
        } else if (wavelen > low_wl) {
          freq = freq / cfg->rope_factor;
        } else {
          const float smooth = ((float)cfg->rope_original_max_pos / wavelen -
                                cfg->rope_low_freq_factor) /
                               (cfg->rope_high_freq_factor - cfg->rope_low_freq_factor);
          freq = (1 - smooth) * freq / cfg->rope_factor + smooth * freq;
        }
      }
      tab[((size_t)p * h + i) * 2 + 0] = cosf(freq);
      tab[((size_t)p * h + i) * 2 + 1] = sinf(freq);
    }
}

extern "C" ffmi_status ffmi_attn_create(const ffmi_attn_cfg *cfg, ffmi_attn **out) {
  FFMI_CHECK(cfg && out, FFMI_ERR_INVALID);
  // head sizes of the reference's kernels: 32 / 64 / 128 for incremental
  // decoding (inc_multihead_self_attention.cu:911-926), 64 / 128 for tree
  // verification and beam search (tree_inc...cu:562-572, spec_inc...cu:431-441)
  FFMI_CHECK(cfg->head_dim == 64 || cfg->head_dim == 128 ||
                 (cfg->head_dim == 32 && cfg->mode == FFMI_ATTN_INC),
             FFMI_ERR_UNSUPPORTED);
  FFMI_CHECK(cfg->num_heads > 0 && cfg->max_requests > 0 && cfg->max_seq_len > 0 &&
                 cfg->max_tokens > 0,
             FFMI_ERR_INVALID);
  FFMI_CHECK(cfg->out_layout == 0 || cfg->out_layout == 1, FFMI_ERR_INVALID);
  FFMI_CHECK(cfg->out_layout == 0 || (cfg->num_heads * cfg->head_dim) % 32 == 0,
             FFMI_ERR_UNSUPPORTED);
  ffmi_attn *h = new ffmi_attn();
  h->cfg = *cfg;
  h->slots = (cfg->max_seq_len + cfg->max_tree_tokens + 31) & ~31;
  const size_t Hl = (size_t)cfg->num_heads * cfg->head_dim;
  const size_t kv = (size_t)cfg->max_requests * cfg->num_heads * h->slots * cfg->head_dim;
  // element size: fp16, or fp32 for DT_FLOAT (the fp32 kernels stage one
  // TREE batch: their commits run before the step's stores, no ping-pong)
  const bool f32 = cfg->full_precision != 0;
  if (f32 && (cfg->out_layout != 0 || (size_t)(cfg->head_dim + 256 + h->slots) * 4 > 64 * 1024)) {
    delete h;
    ffmi_set_last_error("full precision: out_layout 0 and (head_dim + 256 + slots) * 4 <= 64 KiB",
                        __FILE__, __LINE__);
    return FFMI_ERR_UNSUPPORTED;
  }
  const size_t es = f32 ? 4 : 2, stage_halves = f32 ? 1 : 2;
  bool ok = hipMalloc((void **)&h->kc, kv * es) == hipSuccess &&
            hipMalloc((void **)&h->vc, kv * es) == hipSuccess &&
            hipMalloc((void **)&h->qbuf, (size_t)cfg->max_tokens * Hl * es) == hipSuccess;
  if (ok && cfg->mode == FFMI_ATTN_TREE)
    ok = hipMalloc((void **)&h->stage, (size_t)cfg->max_tokens * 2 * Hl * es * stage_halves) ==
         hipSuccess;
  std::vector<float> tab;
  rope_table(tab, h->slots, cfg->head_dim, cfg);
  if (ok) ok = hipMalloc((void **)&h->rope, tab.size() * sizeof(float)) == hipSuccess;
  if (!ok) {
    ffmi_attn_destroy(h);
    ffmi_set_last_error("attention cache alloc", __FILE__, __LINE__);
    return FFMI_ERR_OOM;
  }
  // zero the caches: masked keys are multiplied by exactly-zero weights, so
  // never-written slots must hold finite values
  FFMI_HIP(hipMemset(h->kc, 0, kv * es));
  FFMI_HIP(hipMemset(h->vc, 0, kv * es));
  if (h->stage)
    FFMI_HIP(hipMemset(h->stage, 0, (size_t)cfg->max_tokens * 2 * Hl * es * stage_halves));
  FFMI_HIP(hipMemcpy(h->rope, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice));
  *out = h;
  return FFMI_OK;
}

namespace ffmi {
// FFMI_FAULT_ROPE_POS (tests only): positions >= from_pos rotate as
// position + 1; from_pos < 0 restores the true table
ffmi_status attn_rope_fault(ffmi_attn *h, int from_pos) {
  FFMI_CHECK(h, FFMI_ERR_INVALID);
  std::vector<float> tab;
  rope_table(tab, h->slots + 1, h->cfg.head_dim, &h->cfg);
  const size_t row = (size_t)h->cfg.head_dim;
  // ascending: row p takes row p + 1 before row p + 1 itself is shifted, so
  // every position >= from_pos rotates as exactly position + 1
  if (from_pos >= 0)
    for (int p = from_pos; p < h->slots; ++p)
      memcpy(&tab[(size_t)p * row], &tab[(size_t)(p + 1) * row], row * sizeof(float));
  FFMI_HIP(hipMemcpy(h->rope, tab.data(), (size_t)h->slots * row * sizeof(float),
                     hipMemcpyHostToDevice));
  return FFMI_OK;
}
}  // namespace ffmi

extern "C" void ffmi_attn_destroy(ffmi_attn *h) {
  if (!h) return;
  (void)hipFree(h->kc);
  (void)hipFree(h->vc);
  (void)hipFree(h->qbuf);
  (void)hipFree(h->stage);
  (void)hipFree(h->rope);
  delete h;
}

extern "C" ffmi_status ffmi_attn_kv_ptrs(ffmi_attn *h, void **k, void **v, int *slots) {
  FFMI_CHECK(h, FFMI_ERR_INVALID);
  if (k) *k = h->kc;
  if (v) *v = h->vc;
  if (slots) *slots = h->slots;
  return FFMI_OK;
}

namespace ffmi {
ffmi_status attn_forward(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv, Partials qkvp,
                         void *out, ffmi_stream stream, int parity, OprojArgs *opa) {
  FFMI_CHECK(h && b && (qkv || qkvp.S > 0) && out, FFMI_ERR_INVALID);
  if (opa) opa->done = false;
  FFMI_CHECK(b->num_tokens <= h->cfg.max_tokens, FFMI_ERR_INVALID);
  const bool tree = h->cfg.mode == FFMI_ATTN_TREE;
  const hipStream_t s = (hipStream_t)stream;
  const int heads = h->cfg.num_heads, d = h->cfg.head_dim;
  if (h->cfg.full_precision) {
    // DT_FLOAT: commits (TREE), then RoPE + KV store (+ staging), then the
    // attention, each its own launch (kernels/f32.hip)
    FFMI_CHECK(qkv && qkvp.S == 0 && !(opa && opa->wo), FFMI_ERR_INVALID);
    FFMI_HIP(ffmi::launch_kv_update_f32(b->dev, b->num_tokens, tree ? b->num_commits : 0,
                                        (const float *)qkv, h->rope, h->slots, (float *)h->qbuf,
                                        (float *)h->kc, (float *)h->vc,
                                        tree ? (float *)h->stage : nullptr, heads, d, h->slots, s));
    FFMI_HIP(ffmi::launch_attention_f32(b->dev, b->num_tokens, (const float *)h->qbuf,
                                        (const float *)h->kc, (const float *)h->vc, (float *)out,
                                        heads, d, h->slots, h->cfg.qk_scale, s));
    return FFMI_OK;
  }
  uint16_t *stage_wr = nullptr, *stage_rd = nullptr;
  int C = 0;
  if (tree) {
    if (parity < 0) parity = h->parity, h->parity ^= 1;
    const size_t half = (size_t)h->cfg.max_tokens * 2 * heads * d;
    stage_wr = h->stage + (parity ? half : 0);
    stage_rd = h->stage + (parity ? 0 : half);
    C = b->num_commits;
  }
  // One work item per request (decode, SSM beam steps, tree verify): commits
  // + KV update + attention in one launch.  Otherwise (prefill blocks) the
  // separate KV-update launch first.  Commits whose depth coincides with a
  // slot this step stores go first in their own launch (the reference's
  // commit-then-store order).  FFMI_ATTN_NO_FUSE=1 forces the two-launch path
  // (A/B and parity tests).
  const bool no_fuse = getenv("FFMI_ATTN_NO_FUSE") != nullptr;
  const bool fused = b->one_item_per_req && b->lds_tail && !no_fuse;
  if (C > 0 && b->commit_overlap) {
    FFMI_HIP(ffmi::launch_commit(b->dev, C, stage_rd, h->kc, h->vc, heads, d, h->slots, s));
    C = 0;
  }
  if (!fused) {
    FFMI_HIP(ffmi::launch_kv_update(b->dev, b->num_tokens, b->num_work, C,
                                    (const uint16_t *)qkv, qkvp, h->qbuf, h->kc, h->vc, stage_wr,
                                    stage_rd, h->rope, heads, d, h->slots, h->slots, s));
    C = 0;
  }
  // the output projection rides along where its launch allows it (fused,
  // one query tile, d = 64, N <= 1024 columns); otherwise the caller runs it
  const bool oproj = opa && opa->wo && opa->slab && fused && d == 64 && b->max_q <= 16 &&
                     opa->N % 16 == 0 && opa->N <= 1024 && b->num_tokens <= opa->max_T;
  FFMI_HIP(ffmi::launch_attention(b->dev, b->num_work, b->max_q, h->qbuf, h->kc, h->vc,
                                  (uint16_t *)out, heads, d, h->slots, h->cfg.qk_scale, s,
                                  h->cfg.out_layout == 1, fused, b->num_tokens, C,
                                  (const uint16_t *)qkv, qkvp, stage_wr, stage_rd, h->rope,
                                  h->slots, oproj ? opa : nullptr));
  if (oproj) opa->done = true;
  return FFMI_OK;
}
}  // namespace ffmi

static ffmi_status attn_run(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv, void *out,
                            ffmi_stream stream, int mode) {
  FFMI_CHECK(h && qkv, FFMI_ERR_INVALID);
  FFMI_CHECK(h->cfg.mode == mode, FFMI_ERR_INVALID);  // handle made for this op
  return ffmi::attn_forward(h, b, qkv, ffmi::Partials(), out, stream);
}

extern "C" ffmi_status ffmi_attn_inc(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                                     void *out, ffmi_stream stream) {
  return attn_run(h, b, qkv, out, stream, FFMI_ATTN_INC);
}
extern "C" ffmi_status ffmi_attn_spec(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                                      void *out, ffmi_stream stream) {
  return attn_run(h, b, qkv, out, stream, FFMI_ATTN_SPEC);
}
extern "C" ffmi_status ffmi_attn_tree(ffmi_attn *h, const ffmi_batch_dev *b, const void *qkv,
                                      void *out, ffmi_stream stream) {
  FFMI_CHECK(h && h->stage, FFMI_ERR_INVALID);  // created with FFMI_ATTN_TREE
  return attn_run(h, b, qkv, out, stream, FFMI_ATTN_TREE);
}

// ---------------------------------------------------------------------------
// linear / norms / aux
// ---------------------------------------------------------------------------
extern "C" size_t ffmi_linear_packed_bytes(int out_dim, int in_dim) {
  const size_t nt = (size_t)(out_dim + 15) / 16, kt = (size_t)(in_dim + 31) / 32;
  return nt * kt * 512 * 2;
}

extern "C" ffmi_status ffmi_linear_pack_weight(const void *W, int out_dim, int in_dim,
                                               void *W_packed, ffmi_stream stream) {
  FFMI_CHECK(W && W_packed && out_dim > 0 && in_dim > 0, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_pack_weight((const uint16_t *)W, in_dim, 0, 0, out_dim, in_dim,
                                    (uint16_t *)W_packed, 1, 0, (out_dim + 15) / 16,
                                    (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_linear_pack_gate_up(const void *Wg, const void *Wu, int out_dim,
                                                int in_dim, void *W_packed, ffmi_stream stream) {
  FFMI_CHECK(Wg && Wu && W_packed && out_dim > 0 && in_dim > 0, FFMI_ERR_INVALID);
  const int pitch = 2 * ((out_dim + 15) / 16);
  FFMI_HIP(ffmi::launch_pack_weight((const uint16_t *)Wg, in_dim, 0, 0, out_dim, in_dim,
                                    (uint16_t *)W_packed, 2, 0, pitch, (hipStream_t)stream));
  FFMI_HIP(ffmi::launch_pack_weight((const uint16_t *)Wu, in_dim, 0, 0, out_dim, in_dim,
                                    (uint16_t *)W_packed, 2, 1, pitch, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" size_t ffmi_linear_workspace_bytes(int T, int out_dim, int in_dim, int epilogue) {
  if (T <= 0 || out_dim <= 0 || in_dim <= 0) return 0;
  return ffmi::gemm_workspace_bytes(T, out_dim, in_dim, epilogue);
}

extern "C" ffmi_status ffmi_linear_ws(const void *X, const void *W_packed, void *Y, int T,
                                      int out_dim, int in_dim, int epilogue, void *workspace,
                                      size_t workspace_bytes, ffmi_stream stream) {
  FFMI_CHECK(X && W_packed && Y && T >= 0 && out_dim > 0, FFMI_ERR_INVALID);
  FFMI_CHECK(in_dim > 0 && in_dim % 32 == 0, FFMI_ERR_UNSUPPORTED);
  const int epi = epilogue & ~(FFMI_X_PACKED | FFMI_W_STREAM);
  const int epi_base = epi & ~FFMI_Y_PACKED;
  FFMI_CHECK(epi_base == FFMI_EPI_NONE || epi_base == FFMI_EPI_SILU_MUL, FFMI_ERR_INVALID);
  FFMI_CHECK(!(epilogue & FFMI_Y_PACKED) || out_dim % 32 == 0, FFMI_ERR_UNSUPPORTED);
  FFMI_HIP(ffmi::launch_gemm((const uint16_t *)X, (const uint16_t *)W_packed, (uint16_t *)Y,
                             (float *)workspace, workspace_bytes, T, out_dim, in_dim, epilogue,
                             (hipStream_t)stream));
  return FFMI_OK;
}

static std::mutex g_ws_mu;
static void *g_ws = nullptr;
static size_t g_ws_bytes = 0;

extern "C" ffmi_status ffmi_linear(const void *X, const void *W_packed, void *Y, int T,
                                   int out_dim, int in_dim, int epilogue, ffmi_stream stream) {
  FFMI_CHECK(X && W_packed && Y && T >= 0 && out_dim > 0, FFMI_ERR_INVALID);
  FFMI_CHECK(in_dim > 0 && in_dim % 32 == 0, FFMI_ERR_UNSUPPORTED);
  const size_t need = ffmi_linear_workspace_bytes(T, out_dim, in_dim, epilogue);
  void *ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (need > g_ws_bytes) {
      if (g_ws) {
        FFMI_HIP(hipDeviceSynchronize());
        (void)hipFree(g_ws);
        g_ws = nullptr;
        g_ws_bytes = 0;
      }
      if (hipMalloc(&g_ws, need) != hipSuccess) return FFMI_ERR_OOM;
      g_ws_bytes = need;
    }
    ws = g_ws;
  }
  return ffmi_linear_ws(X, W_packed, Y, T, out_dim, in_dim, epilogue, ws, g_ws_bytes, stream);
}

extern "C" ffmi_status ffmi_rmsnorm(const void *x, const void *w, void *out, int T, int H,
                                    float eps, ffmi_stream stream) {
  FFMI_CHECK(x && w && out && H % 8 == 0 && H <= 16384, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_rmsnorm((const uint16_t *)x, nullptr, (const uint16_t *)w, nullptr,
                                (uint16_t *)out, T, H, eps, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_residual_rmsnorm(const void *x1, const void *x2, const void *w,
                                             void *residual_out, void *out, int T, int H,
                                             float eps, ffmi_stream stream) {
  FFMI_CHECK(x1 && x2 && w && residual_out && out && H % 8 == 0 && H <= 16384, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_rmsnorm((const uint16_t *)x1, (const uint16_t *)x2, (const uint16_t *)w,
                                (uint16_t *)residual_out, (uint16_t *)out, T, H, eps,
                                (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rmsnorm_ex(const void *x1, const void *x2, const void *w,
                                       void *residual_out, void *out, int T, int H, float eps,
                                       int flags, ffmi_stream stream) {
  FFMI_CHECK(x1 && w && out && T >= 0 && H > 0 && H % 8 == 0, FFMI_ERR_INVALID);
  FFMI_CHECK(!x2 || residual_out, FFMI_ERR_INVALID);
  FFMI_CHECK((flags & ~FFMI_Y_PACKED) == 0, FFMI_ERR_INVALID);
  const bool packed = (flags & FFMI_Y_PACKED) != 0;
  FFMI_CHECK(!packed || H % 32 == 0, FFMI_ERR_UNSUPPORTED);
  FFMI_HIP(ffmi::launch_rmsnorm((const uint16_t *)x1, (const uint16_t *)x2, (const uint16_t *)w,
                                (uint16_t *)residual_out, (uint16_t *)out, T, H, eps,
                                (hipStream_t)stream, packed));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_embedding(const ffmi_batch_dev *b, const void *table, void *out,
                                      int H, ffmi_stream stream) {
  FFMI_CHECK(b && table && out && H % 8 == 0, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_embedding(b->dev, b->num_tokens, (const uint16_t *)table,
                                  (uint16_t *)out, H, (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_silu_mul(const void *a, const void *b, void *out, size_t n,
                                     ffmi_stream stream) {
  FFMI_CHECK(a && b && out, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_silu_mul((const uint16_t *)a, (const uint16_t *)b, (uint16_t *)out, n,
                                 (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_argmax(const void *logits, int T, int V, int32_t *ids, float *probs,
                                   ffmi_stream stream) {
  FFMI_CHECK(logits && ids && V > 0, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_argmax((const uint16_t *)logits, T, V, 1, ids, probs,
                               (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_arg_topk(const void *logits, int T, int V, int k, int32_t *ids,
                                     float *probs, ffmi_stream stream) {
  FFMI_CHECK(logits && ids && V > 0 && k >= 1 && k <= 4 && k <= V, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_argmax((const uint16_t *)logits, T, V, k, ids, probs,
                               (hipStream_t)stream));
  return FFMI_OK;
}

extern "C" size_t ffmi_arg_topk_workspace_bytes(int T) { return ffmi::argmax_workspace_bytes(T); }

extern "C" ffmi_status ffmi_arg_topk_ws(const void *logits, int T, int V, int k, int32_t *ids,
                                        float *probs, void *workspace, size_t workspace_bytes,
                                        ffmi_stream stream) {
  FFMI_CHECK(logits && ids && V > 0 && k >= 1 && k <= 4 && k <= V, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_argmax((const uint16_t *)logits, T, V, k, ids, probs,
                               (hipStream_t)stream, workspace, workspace_bytes));
  return FFMI_OK;
}

// Test hooks of the residual RMSNorm folded into the decode GEMMs (the pair
// llama_gpu.cpp runs at T <= 32): the producer adds its rounded output to
// the residual in place and leaves per-(row, 16-column tile) sums of
// squares; the consumer normalises the residual from those sums in its
// prologue.  Row-major fp16 throughout.
extern "C" ffmi_status ffmi_debug_fused_residual_linear(const void *X, const void *W_packed,
                                                        void *residual, float *ss_out, int T,
                                                        int out_dim, int in_dim,
                                                        ffmi_stream stream) {
  FFMI_CHECK(X && W_packed && residual && ss_out && T > 0 && T <= 32, FFMI_ERR_INVALID);
  ffmi::FuseArgs fz;
  fz.kind = 1;
  fz.res_in = (const uint16_t *)residual;
  fz.ss_out = ss_out;
  FFMI_HIP(ffmi::launch_gemm((const uint16_t *)X, (const uint16_t *)W_packed, (uint16_t *)residual,
                             nullptr, 0, T, out_dim, in_dim, FFMI_EPI_NONE, (hipStream_t)stream,
                             nullptr, 0, &fz));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_debug_fused_norm_linear(const void *residual, const float *ss_in,
                                                    const void *norm_w, float eps,
                                                    const void *W_packed, void *Y, int T,
                                                    int out_dim, int in_dim, int epilogue,
                                                    ffmi_stream stream) {
  FFMI_CHECK(residual && ss_in && norm_w && W_packed && Y && T > 0 && T <= 32 &&
                 (epilogue == FFMI_EPI_NONE || epilogue == FFMI_EPI_SILU_MUL),
             FFMI_ERR_INVALID);
  ffmi::FuseArgs fz;
  fz.kind = 2;
  fz.ss_in = ss_in;
  fz.nss = in_dim / 16;
  fz.wnorm = (const uint16_t *)norm_w;
  fz.eps = eps;
  FFMI_HIP(ffmi::launch_gemm((const uint16_t *)residual, (const uint16_t *)W_packed, (uint16_t *)Y,
                             nullptr, 0, T, out_dim, in_dim, epilogue, (hipStream_t)stream,
                             nullptr, 0, &fz));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_fill_weight(void *dst_f16, size_t n, const char *name, uint64_t seed,
                                        int kind, ffmi_stream stream) {
  FFMI_CHECK(dst_f16 && name, FFMI_ERR_INVALID);
  FFMI_HIP(ffmi::launch_fill_weight((uint16_t *)dst_f16, n, ffmi::weight_key(name, seed), kind,
                                    (hipStream_t)stream));
  return FFMI_OK;
}

// ---------------------------------------------------------------------------
// RCCL all-reduce (RCCL over xGMI; the reference: ncclAllReduce,
// allreduce_kernels.cu:67-74)
// ---------------------------------------------------------------------------
// In-process shard group (ffmi_comm_create_local): the ranks are host
// threads of ONE process stepping their shards on one device.  All-reduce =
// barrier, rank 0 sums every rank's buffer into a group scratch, barrier, each
// rank copies the sum, barrier.  Barriers time out (a shard that failed
// mid-step returns an error to the others instead of hanging them).
struct LocalGroup {
  int n = 0;
  ffmi_status sum_status = FFMI_OK;  // rank 0's group sum, checked by every rank
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long gen = 0;
  bool broken = false;
  std::vector<const void *> bufs;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  ~LocalGroup() {
    if (tmp) (void)hipFree(tmp);
  }
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const long g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

// Direct xGMI transport (kernels/collective.hip): this rank's exchange buffer,
// every peer's mapped through its IPC handle, and a host-mapped error word.
struct PeerState {
  size_t cap = 0;
  char *own = nullptr;
  char *base[ffmi::kMaxPeers] = {};
  std::vector<void *> opened;
  int *err_h = nullptr, *err_d = nullptr;
  bool attached = false;
  uint64_t timeout_ticks = 1000000000ull;  // 10 s at 100 MHz
  size_t two_shot_min = 256 << 10;         // one-shot below (latency), two-shot above
  ~PeerState() {
    for (void *p : opened) (void)hipIpcCloseMemHandle(p);
    if (own) (void)hipFree(own);
    if (err_h) (void)hipHostFree(err_h);
  }
};

struct ffmi_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  std::shared_ptr<LocalGroup> local;
  std::unique_ptr<PeerState> peer;
  // ffmi_comm_allgather: device scratch and stream (created on first use)
  float *xg = nullptr;
  size_t xg_cap = 0;
  hipStream_t xg_stream = nullptr;
};

extern "C" ffmi_status ffmi_comm_create_local(int nranks, ffmi_comm **out) {
  FFMI_CHECK(out && nranks >= 1 && nranks <= 8, FFMI_ERR_INVALID);
  auto g = std::make_shared<LocalGroup>();
  g->n = nranks;
  g->bufs.assign(nranks, nullptr);
  for (int r = 0; r < nranks; ++r) {
    out[r] = new ffmi_comm();
    out[r]->nranks = nranks;
    out[r]->rank = r;
    out[r]->local = g;
  }
  return FFMI_OK;
}

static ffmi_status local_allreduce(ffmi_comm *c, const void *in, void *out, size_t count,
                                   int dtype, hipStream_t s) {
  LocalGroup &g = *c->local;
  const size_t bytes = count * (dtype == FFMI_F16 ? 2 : 4);
  g.bufs[c->rank] = in;
  FFMI_HIP(hipStreamSynchronize(s));  // this rank's partial is complete
  FFMI_CHECK(g.barrier(), FFMI_ERR_NCCL);
  ffmi_status st = FFMI_OK;
  if (c->rank == 0) {
    if (g.tmp_bytes < bytes) {
      if (g.tmp) (void)hipFree(g.tmp);
      g.tmp = nullptr;
      g.tmp_bytes = 0;
      if (hipMalloc(&g.tmp, bytes) == hipSuccess) g.tmp_bytes = bytes;
    }
    if (!g.tmp) {
      st = FFMI_ERR_OOM;
    } else if (ffmi::launch_group_sum(g.bufs.data(), g.n, g.tmp, count, dtype, s) != hipSuccess ||
               hipStreamSynchronize(s) != hipSuccess) {
      st = FFMI_ERR_HIP;
    }
  }
  if (c->rank == 0) g.sum_status = st;  // published by the barrier below
  if (!g.barrier() || g.sum_status != FFMI_OK) {
    // rank 0's sum failed (OOM / HIP error): no rank copies g.tmp
    std::lock_guard<std::mutex> lk(g.mu);
    g.broken = true;
    g.cv.notify_all();
    return g.sum_status != FFMI_OK ? g.sum_status : FFMI_ERR_NCCL;
  }
  FFMI_HIP(hipMemcpyAsync(out, g.tmp, bytes, hipMemcpyDeviceToDevice, s));
  FFMI_HIP(hipStreamSynchronize(s));
  FFMI_CHECK(g.barrier(), FFMI_ERR_NCCL);  // nobody reuses tmp before all copied
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_unique_id(void *id_out) {
  FFMI_CHECK(id_out, FFMI_ERR_INVALID);
  static_assert(sizeof(ncclUniqueId) == FFMI_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return FFMI_ERR_NCCL;
  memcpy(id_out, &id, sizeof(id));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_create(const void *id, int nranks, int rank, ffmi_comm **out) {
  FFMI_CHECK(id && out && nranks >= 1 && rank >= 0 && rank < nranks, FFMI_ERR_INVALID);
  ffmi_comm *c = new ffmi_comm();
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    ffmi_set_last_error(ncclGetErrorString(r), __FILE__, __LINE__);
    delete c;
    return FFMI_ERR_NCCL;
  }
  *out = c;
  return FFMI_OK;
}

extern "C" void ffmi_comm_destroy(ffmi_comm *c) {
  if (!c) return;
  if (c->xg_stream) (void)hipStreamSynchronize(c->xg_stream);
  if (c->xg) (void)hipFree(c->xg);
  if (c->xg_stream) (void)hipStreamDestroy(c->xg_stream);
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
}

// All-gather of host byte blocks as an fp32 sum all-reduce that every
// transport carries: each 16-bit half-word becomes an exact small integer in
// a float, a rank fills its own slot and zeroes the others, and x + 0 = x
// (no rounding, no -0 / denormal / NaN bit patterns in flight).
extern "C" ffmi_status ffmi_comm_allgather(ffmi_comm *c, const void *mine, size_t bytes,
                                           void *all) {
  FFMI_CHECK(c && (mine || !bytes) && (all || !bytes), FFMI_ERR_INVALID);
  const int n = c->nranks;
  if (n == 1) {
    if (bytes) memcpy(all, mine, bytes);
    return FFMI_OK;
  }
  const size_t words = (bytes + 1) / 2;  // 16-bit words per rank
  const size_t count = words * n;
  if (c->xg_cap < count) {
    if (c->xg) FFMI_HIP(hipFree(c->xg));
    c->xg = nullptr;
    c->xg_cap = 0;
    FFMI_HIP(hipMalloc((void **)&c->xg, count * sizeof(float)));
    c->xg_cap = count;
  }
  if (!c->xg_stream) FFMI_HIP(hipStreamCreateWithFlags(&c->xg_stream, hipStreamNonBlocking));
  std::vector<float> h(count, 0.0f);
  std::vector<uint16_t> w(words, 0);
  memcpy(w.data(), mine, bytes);
  for (size_t i = 0; i < words; ++i) h[(size_t)c->rank * words + i] = (float)w[i];
  FFMI_HIP(hipMemcpyAsync(c->xg, h.data(), count * sizeof(float), hipMemcpyHostToDevice,
                          c->xg_stream));
  ffmi_status st = ffmi_allreduce(c, c->xg, c->xg, count, FFMI_F32, (ffmi_stream)c->xg_stream);
  if (st != FFMI_OK) return st;
  FFMI_HIP(hipMemcpyAsync(h.data(), c->xg, count * sizeof(float), hipMemcpyDeviceToHost,
                          c->xg_stream));
  FFMI_HIP(hipStreamSynchronize(c->xg_stream));
  if (c->peer && c->peer->attached) {
    st = ffmi_comm_peer_status(c);
    if (st != FFMI_OK) return st;
  }
  std::vector<uint16_t> out(words);
  for (int r = 0; r < n; ++r) {
    for (size_t i = 0; i < words; ++i) {
      const float v = h[(size_t)r * words + i];
      if (!(v >= 0.0f && v <= 65535.0f && v == (float)(uint16_t)v)) return FFMI_ERR_NCCL;
      out[i] = (uint16_t)v;
    }
    memcpy(static_cast<char *>(all) + (size_t)r * bytes, out.data(), bytes);
  }
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_create_peer(int nranks, int rank, ffmi_comm **out) {
  FFMI_CHECK(out && nranks >= 1 && nranks <= ffmi::kMaxPeers && rank >= 0 && rank < nranks,
             FFMI_ERR_INVALID);
  ffmi_comm *c = new ffmi_comm();
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_peer_export(ffmi_comm *c, size_t max_bytes, void *handle_out) {
  FFMI_CHECK(c && handle_out && max_bytes > 0 && !c->local, FFMI_ERR_INVALID);
  FFMI_CHECK(c->nranks <= ffmi::kMaxPeers && !c->peer, FFMI_ERR_INVALID);
  static_assert(sizeof(hipIpcMemHandle_t) == FFMI_PEER_HANDLE_BYTES, "IPC handle size");
  auto p = std::make_unique<PeerState>();
  p->cap = (max_bytes + 255) & ~(size_t)255;
  if (const char *e = getenv("FFMI_PEER_TIMEOUT_S")) p->timeout_ticks = (uint64_t)(atof(e) * 1e8);
  // two ranks: two-shot moves the same bytes per rank as one-shot in two
  // signal rounds, so one-shot at every size
  if (c->nranks <= 2) p->two_shot_min = (size_t)-1;
  if (const char *e = getenv("FFMI_PEER_TWO_SHOT_MIN")) p->two_shot_min = (size_t)atoll(e);
  const size_t bytes = ffmi::peer_buffer_bytes(p->cap);
  // uncached (MTYPE UC): every rank's loads of an exchange area reach memory,
  // so a line read two epochs ago can never be served stale from an L2 --
  // neither a peer's L2 over xGMI nor another XCD's L2 of this device (the
  // multi-process test on one GPU).  FFMI_PEER_UNCACHED=0: plain hipMalloc +
  // the system-scope fences alone (A/B).
  const char *uc = getenv("FFMI_PEER_UNCACHED");
  if (uc && !atoi(uc)) FFMI_HIP(hipMalloc((void **)&p->own, bytes));
  else FFMI_HIP(hipExtMallocWithFlags((void **)&p->own, bytes, hipDeviceMallocUncached));
  FFMI_HIP(hipMemset(p->own, 0, ffmi::kDataOff));  // inboxes, counters, epoch 0
  FFMI_HIP(hipDeviceSynchronize());
  FFMI_HIP(hipHostMalloc((void **)&p->err_h, sizeof(int), hipHostMallocMapped));
  *p->err_h = 0;
  FFMI_HIP(hipHostGetDevicePointer((void **)&p->err_d, p->err_h, 0));
  hipIpcMemHandle_t h;
  FFMI_HIP(hipIpcGetMemHandle(&h, p->own));
  memcpy(handle_out, &h, sizeof(h));
  c->peer = std::move(p);
  return FFMI_OK;
}

static ffmi_status peer_run(ffmi_comm *c, const void *in, void *out, size_t rows, size_t cols,
                            size_t ld, size_t col0, int dtype, hipStream_t s,
                            const ffmi::Partials *slabs = nullptr, int rs_row0 = -1,
                            int rs_row1 = -1, const ffmi::PeerNormArgs *norm = nullptr,
                            int two_shot = -1) {
  PeerState &p = *c->peer;
  const size_t esz = dtype == FFMI_F16 ? 2 : 4;
  const size_t bytes = rows * cols * esz;
  FFMI_CHECK(bytes <= p.cap, FFMI_ERR_INVALID);
  FFMI_CHECK((cols * esz) % 16 == 0 && ((size_t)in & 15) == 0 && ((size_t)out & 15) == 0 &&
                 (ld * esz) % 16 == 0 && (col0 * esz) % 16 == 0,
             FFMI_ERR_UNSUPPORTED);
  if (slabs && slabs->S > 0)
    FFMI_CHECK(dtype == FFMI_F16 && slabs->S <= 8 && slabs->NP >= (int)cols && slabs->NP % 4 == 0 &&
                   ((size_t)slabs->p & 15) == 0,
               FFMI_ERR_UNSUPPORTED);
  ffmi::PeerArgs a;
  for (int r = 0; r < ffmi::kMaxPeers; ++r) a.base[r] = p.base[r];
  a.nranks = c->nranks;
  a.rank = c->rank;
  a.cap = p.cap;
  a.in = in;
  a.out = out;
  a.nvec = bytes / 16;
  a.vec_elems = 16 / esz;
  a.cols = cols;
  a.ld = ld;
  a.col0 = col0;
  a.esz = esz;
  a.err = p.err_d;
  a.timeout_ticks = p.timeout_ticks;
  if (slabs && slabs->S > 0) a.slabs = slabs->p, a.S = slabs->S, a.NP = slabs->NP, a.rows = rows;
  const bool ts = two_shot >= 0 ? two_shot != 0 : bytes >= p.two_shot_min;
  if (norm) FFMI_HIP(ffmi::launch_peer_allreduce_norm(a, *norm, ts, s));
  else FFMI_HIP(ffmi::launch_peer_allreduce(a, ts, s, rs_row0, rs_row1));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_peer_status(ffmi_comm *c) {
  FFMI_CHECK(c && c->peer, FFMI_ERR_INVALID);
  if (*(volatile int *)c->peer->err_h != 0) {
    ffmi_set_last_error(*(volatile int *)c->peer->err_h == 1
                            ? "xGMI all-reduce: a peer never signalled (timeout, phase 1)"
                            : "xGMI all-reduce: a peer never signalled (timeout, phase 2)",
                        __FILE__, __LINE__);
    return FFMI_ERR_NCCL;
  }
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_comm_peer_attach(ffmi_comm *c, const void *handles) {
  FFMI_CHECK(c && c->peer && handles && !c->peer->attached, FFMI_ERR_INVALID);
  PeerState &p = *c->peer;
  // one process per GPU of a node: every other device of the group must be
  // reachable over xGMI before any kernel touches a peer's buffer (a
  // refused check is an error the caller answers with RCCL, never a fault);
  // ranks sharing one device (the multi-process tests) need no peer access
  int ndev = 0, me = 0;
  FFMI_HIP(hipGetDeviceCount(&ndev));
  FFMI_HIP(hipGetDevice(&me));
  if (ndev >= c->nranks)
    for (int d = 0; d < c->nranks; ++d) {
      int can = 1;
      if (d != me) FFMI_HIP(hipDeviceCanAccessPeer(&can, me, d));
      if (!can) {
        ffmi_set_last_error("xGMI transport: a peer device is not reachable", __FILE__, __LINE__);
        return FFMI_ERR_UNSUPPORTED;
      }
    }
  for (int r = 0; r < c->nranks; ++r) {
    if (r == c->rank) {
      p.base[r] = p.own;
      continue;
    }
    hipIpcMemHandle_t h;
    memcpy(&h, (const char *)handles + (size_t)r * FFMI_PEER_HANDLE_BYTES, sizeof(h));
    void *ptr = nullptr;
    FFMI_HIP(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
    p.opened.push_back(ptr);
    p.base[r] = (char *)ptr;
  }
  // self-test (collective: every rank runs it): an exact f32 sum of small
  // integers through both kernel variants, checked on the host
  const int n = 4096 * c->nranks;
  std::vector<float> h(n), got(n);
  for (int i = 0; i < n; ++i) h[i] = (float)((c->rank + 1) * (i % 7));
  float *d = nullptr;
  FFMI_HIP(hipMalloc((void **)&d, (size_t)n * 4 * 2));
  ffmi_status st = FFMI_OK;
  p.attached = true;
  for (int pass = 0; pass < 2 && st == FFMI_OK; ++pass) {
    const size_t saved = p.two_shot_min;
    p.two_shot_min = pass == 0 ? (size_t)-1 : 0;  // one-shot, then two-shot
    if (hipMemcpy(d, h.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) st = FFMI_ERR_HIP;
    if (st == FFMI_OK) st = peer_run(c, d, d + n, 1, n, n, 0, FFMI_F32, nullptr);
    if (st == FFMI_OK && hipDeviceSynchronize() != hipSuccess) st = FFMI_ERR_HIP;
    if (st == FFMI_OK) st = ffmi_comm_peer_status(c);
    if (st == FFMI_OK &&
        hipMemcpy(got.data(), d + n, (size_t)n * 4, hipMemcpyDeviceToHost) != hipSuccess)
      st = FFMI_ERR_HIP;
    const float tri = 0.5f * c->nranks * (c->nranks + 1);
    for (int i = 0; st == FFMI_OK && i < n; ++i)
      if (got[i] != tri * (float)(i % 7)) {
        ffmi_set_last_error("xGMI all-reduce self-test: wrong sum", __FILE__, __LINE__);
        st = FFMI_ERR_NCCL;
      }
    p.two_shot_min = saved;
  }
  (void)hipFree(d);
  if (st != FFMI_OK) p.attached = false;
  return st;
}

extern "C" ffmi_status ffmi_comm_peer_detach(ffmi_comm *c) {
  FFMI_CHECK(c, FFMI_ERR_INVALID);
  if (c->peer) c->peer->attached = false;
  return FFMI_OK;
}

namespace ffmi {
bool comm_has_peer(const ffmi_comm *c, size_t bytes) {
  return c && c->peer && c->peer->attached && bytes <= c->peer->cap;
}
int comm_size(const ffmi_comm *c) { return c ? c->nranks : 1; }
int comm_rank(const ffmi_comm *c) { return c ? c->rank : 0; }
bool comm_peer_attached(const ffmi_comm *c) { return c && c->peer && c->peer->attached; }
bool comm_has_fallback(const ffmi_comm *c) { return c && (c->comm || c->local); }
bool comm_is_rccl(const ffmi_comm *c) { return c && c->comm && !c->local; }
ffmi_status comm_allreduce_cols(ffmi_comm *c, const void *in, void *out, int rows, int cols,
                                int ld, int col0, int dtype, hipStream_t s, const Partials *slabs) {
  return peer_run(c, in, out, rows, cols, ld, col0, dtype, s, slabs);
}
bool comm_two_shot(const ffmi_comm *c, size_t bytes) {
  return c && c->peer && c->peer->attached && c->nranks > 1 && bytes >= c->peer->two_shot_min;
}
ffmi_status comm_reduce_rows(ffmi_comm *c, const void *in, void *out, int rows, int cols, int ld,
                             int col0, int row0, int row1, hipStream_t s, const Partials *slabs) {
  return peer_run(c, in, out, rows, cols, ld, col0, FFMI_F16, s, slabs, row0, row1, nullptr, 1);
}
ffmi_status comm_allreduce_norm(ffmi_comm *c, const void *in, int T, int H, int col0,
                                const uint16_t *prev, uint16_t *res, const uint16_t *w, float eps,
                                uint16_t *h, bool packed, bool two_shot, hipStream_t s,
                                const Partials *slabs) {
  FFMI_CHECK(c && c->peer && c->peer->attached && res && w && h && T >= 0 && H > 0 && col0 >= 0 &&
                 col0 < H,
             FFMI_ERR_INVALID);
  if (T == 0) return FFMI_OK;
  ffmi::PeerNormArgs n;
  n.res = res, n.w = w, n.h = h, n.prev = prev, n.T = T, n.H = H, n.packed = packed ? 1 : 0;
  n.eps = eps;
  n.row0 = two_shot ? (int)((long)T * c->rank / c->nranks) : 0;
  n.row1 = two_shot ? (int)((long)T * (c->rank + 1) / c->nranks) : T;
  // (in: [T][H - col0]; out unused -- h and res are the outputs)
  return peer_run(c, in, h, T, H - col0, H - col0, col0, FFMI_F16, s, slabs, -1, -1, &n,
                  two_shot ? 1 : 0);
}
ffmi_status comm_status(ffmi_comm *c) {
  return c && c->peer && c->peer->attached ? ffmi_comm_peer_status(c) : FFMI_OK;
}
}  // namespace ffmi

// Vocab-sharded softmax + argmax / arg-top-k (model.cc:3392-3419 Combine of
// the vocab-parallel lm_head, then argmax.cu:62-100 / arg_topk.cu:339-448):
// three record exchanges over the communicator (norm.hip vshard_kernel).
static constexpr int kVshardW = 8;  // floats per (rank, row) record
extern "C" size_t ffmi_vocab_shard_scratch_bytes(int nranks, int T) {
  return nranks > 0 && T > 0 ? (size_t)nranks * T * kVshardW * sizeof(float) : 0;
}

extern "C" ffmi_status ffmi_vocab_shard_topk(ffmi_comm *c, const void *logits, int T, int Vl,
                                             int k, int32_t *ids, float *probs, void *scratch,
                                             ffmi_stream stream) {
  FFMI_CHECK(c && logits && ids && scratch && T >= 0 && Vl > 0 && k >= 1 && k <= 4,
             FFMI_ERR_INVALID);
  FFMI_CHECK(c->nranks * kVshardW <= 256 && (size_t)c->rank * Vl + Vl <= 0x7fffffffu,
             FFMI_ERR_UNSUPPORTED);
  if (T == 0) return FFMI_OK;
  const hipStream_t s = (hipStream_t)stream;
  const int P = c->nranks;
  float *x = (float *)scratch;
  for (int phase = 0; phase < 3; ++phase) {
    FFMI_HIP(ffmi::launch_vshard((const uint16_t *)logits, T, Vl, P, c->rank, k, phase, x,
                                 kVshardW, nullptr, nullptr, s));
    const ffmi_status st = ffmi_allreduce(c, x, x, (size_t)P * T * kVshardW, FFMI_F32, stream);
    if (st != FFMI_OK) return st;
  }
  FFMI_HIP(ffmi::launch_vshard((const uint16_t *)logits, T, Vl, P, c->rank, k, 3, x, kVshardW,
                               ids, probs, s));
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_allreduce(ffmi_comm *c, const void *in, void *out, size_t count,
                                      int dtype, ffmi_stream stream) {
  FFMI_CHECK(c && in && out, FFMI_ERR_INVALID);
  if (c->nranks > 1 && c->peer && c->peer->attached && dtype != FFMI_I32) {
    const size_t esz = dtype == FFMI_F16 ? 2 : 4;
    if (count * esz <= c->peer->cap)
      return peer_run(c, in, out, 1, count, count, 0, dtype, (hipStream_t)stream);
    // larger than the exchange buffers: RCCL or the local group takes it
    if (!c->comm && !c->local) {
      ffmi_set_last_error("all-reduce larger than the xGMI exchange buffer and no RCCL "
                          "communicator to fall back to", __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
  }
  FFMI_CHECK(c->local || c->comm || c->nranks == 1, FFMI_ERR_INVALID);
  if (c->local && c->nranks > 1)
    return local_allreduce(c, in, out, count, dtype, (hipStream_t)stream);
  if (c->nranks == 1 && !c->comm) {
    if (in != out) {
      const size_t esz = dtype == FFMI_F16 ? 2 : 4;
      FFMI_HIP(hipMemcpyAsync(out, in, count * esz, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    }
    return FFMI_OK;
  }
  ncclDataType_t t = dtype == FFMI_F16 ? ncclHalf : (dtype == FFMI_F32 ? ncclFloat : ncclInt32);
  ncclResult_t r = ncclAllReduce(in, out, count, t, ncclSum, c->comm, (hipStream_t)stream);
  if (r != ncclSuccess) {
    ffmi_set_last_error(ncclGetErrorString(r), __FILE__, __LINE__);
    return FFMI_ERR_NCCL;
  }
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_allreduce_rmsnorm(ffmi_comm *c, const void *in, int T, int H,
                                              int col0, const void *prev, void *residual,
                                              const void *w, float eps, void *out, int flags,
                                              int *rows_out, ffmi_stream stream) {
  FFMI_CHECK(c && in && residual && w && out && T >= 0 && H > 0 && col0 >= 0 && col0 < H &&
                 (col0 == 0 || prev) && (flags & ~FFMI_Y_PACKED) == 0,
             FFMI_ERR_INVALID);
  if (!(c->nranks > 1 && c->peer && c->peer->attached)) {
    ffmi_set_last_error("ffmi_allreduce_rmsnorm needs an attached xGMI transport of >= 2 ranks",
                        __FILE__, __LINE__);
    return FFMI_ERR_UNSUPPORTED;
  }
  FFMI_CHECK(H % 8 == 0 && col0 % 8 == 0 && H / 8 <= 4096 &&
                 (!(flags & FFMI_Y_PACKED) || H % 32 == 0),
             FFMI_ERR_UNSUPPORTED);
  FFMI_CHECK((size_t)T * H * 2 <= c->peer->cap, FFMI_ERR_INVALID);
  const bool two = ffmi::comm_two_shot(c, (size_t)T * H * 2);
  if (rows_out) {
    rows_out[0] = two ? (int)((long)T * c->rank / c->nranks) : 0;
    rows_out[1] = two ? (int)((long)T * (c->rank + 1) / c->nranks) : T;
  }
  return ffmi::comm_allreduce_norm(c, in, T, H, col0, (const uint16_t *)prev,
                                   (uint16_t *)residual, (const uint16_t *)w, eps, (uint16_t *)out,
                                   (flags & FFMI_Y_PACKED) != 0, two, (hipStream_t)stream);
}

extern "C" long ffmi_debug_gemm_stamps(long long *dst, long max_waves) {
  return ffmi::gemm_debug_stamps(dst, max_waves);
}

extern "C" long ffmi_debug_attn_stamps(long long *dst, long max_waves) {
  return ffmi::attn_debug_stamps(dst, max_waves);
}

extern "C" long ffmi_debug_markers(long long *dst, long n) { return ffmi::debug_markers(dst, n); }

extern "C" size_t ffmi_packed_activation_bytes(int T, int in_dim) {
  return T > 0 && in_dim > 0 ? ffmi::packed_act_bytes(T, in_dim) : 0;
}

extern "C" ffmi_status ffmi_pack_activations(const void *X, int T, int in_dim, void *X_packed,
                                             ffmi_stream stream) {
  FFMI_CHECK(X && X_packed && T >= 0 && in_dim > 0, FFMI_ERR_INVALID);
  FFMI_CHECK(in_dim % 32 == 0, FFMI_ERR_UNSUPPORTED);
  FFMI_HIP(ffmi::launch_pack_act((const uint16_t *)X, (uint16_t *)X_packed, T, in_dim,
                                 (hipStream_t)stream));
  return FFMI_OK;
}
