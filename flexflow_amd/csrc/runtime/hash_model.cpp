// hash_model.cpp -- scheduler test double (no GPU, TEST USE ONLY).
//
// Emulates exactly what the attention kernels see: token ids are stored into
// per-request cache rows at the packed store slots, TREE commits copy from
// the previous batch's staging, and each query's "context" is the sequence of
// cached ids at its visible slots (packed prefix / tree-bitmask rule), in
// slot order.  The next token is a hash of that context, so:
//   * incremental decoding yields next = f(prompt + generated so far);
//   * SpecInfer must reproduce the same tokens (the reference's own
//     invariant, tests/inference/cpp_inference_tests.sh:183-189) -- any error
//     in batching, tree build, bitmask, verification or commit lists changes a
//     context and therefore a token.
// The SSM flavour ranks f(ctx) first with probability (100-disagree)%.
#include <algorithm>
#include <array>
#include <memory>
#include <vector>

#include "model.h"
#include "../../../include/ffmi_test.h"

namespace ffmi {

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct HashModel : public ffmi_model {
  int vocab, max_requests, slots;
  uint64_t salt;
  int disagree;
  std::vector<int> cache;  // [max_requests][slots]
  std::vector<int> stage;  // previous batch token ids (TREE commits)
  int cap = -1;            // tokens per step (-1: unbounded), as a GPU model's max_tokens
  int token_capacity() const override { return cap; }
  // chained beam steps (model.h), run eagerly: a step's -1 - i token ids are
  // filled in from the previous slot's results, as the GPU model's gather does
  static constexpr int kChain = BeamSearchBatchConfig::MAX_BEAM_DEPTH;
  std::vector<int> slot_ids[kChain];
  std::vector<float> slot_probs[kChain];
  size_t last_results = 0;  // scheduler entries of the last beam step
  bool can_chain_beam() const override { return mode == FFMI_MODEL_BEAM; }
  ffmi_status beam_launch_chained(const BeamSearchBatchConfig &bc, int slot) override {
    if (slot < 0 || slot >= kChain) return FFMI_ERR_INVALID;
    std::unique_ptr<BeamSearchBatchConfig> b(new BeamSearchBatchConfig(bc));
    for (int t = 0; t < b->num_tokens; ++t) {
      int &id = b->tokensInfo[t].token_id;
      if (id >= 0) continue;
      if (slot == 0 || -1L - id >= (long)slot_ids[slot - 1].size()) return FFMI_ERR_INVALID;
      id = slot_ids[slot - 1][-1 - id];
    }
    std::unique_ptr<BeamInferenceResult> r(new BeamInferenceResult());
    const ffmi_status st = run_beam(*b, r.get());
    if (st != FFMI_OK) return st;
    const size_t n = last_results;  // (scheduler entries: the layout the placeholders index)
    slot_ids[slot].assign(r->token_ids, r->token_ids + n);
    slot_probs[slot].assign(r->probs, r->probs + n);
    return FFMI_OK;
  }
  ffmi_status beam_collect_chained(int slot, BeamInferenceResult *ir) override {
    if (slot < 0 || slot >= kChain) return FFMI_ERR_INVALID;
    const size_t n = slot_ids[slot].size();
    std::copy(slot_ids[slot].begin(), slot_ids[slot].end(), ir->token_ids);
    std::copy(slot_probs[slot].begin(), slot_probs[slot].end(), ir->probs);
    for (size_t i = 0; i < n; ++i) ir->parent_id[i] = 0;
    return FFMI_OK;
  }

  int slot_of(int r, int s) const { return r * slots + s; }

  // returns context hash for each token; -1 entries poison the hash
  void contexts(const PackedStep &ps, std::vector<uint64_t> *hs) {
    for (const auto &c : ps.commits) {
      int v = (c.src_token >= 0 && c.src_token < (int)stage.size()) ? stage[c.src_token] : -7;
      if (c.depth >= 0 && c.depth < slots) cache[slot_of(c.req, c.depth)] = v;
    }
    stage.assign(ps.tokens.size(), -1);
    for (size_t t = 0; t < ps.tokens.size(); ++t) {
      const auto &ti = ps.tokens[t];
      stage[t] = ti.token_id;
      if (ti.store_slot >= 0) cache[slot_of(ti.req, ti.store_slot)] = ti.token_id;
    }
    hs->resize(ps.tokens.size());
    for (size_t t = 0; t < ps.tokens.size(); ++t) {
      const auto &ti = ps.tokens[t];
      const int end = std::max(ti.prefix_len, ti.tree_base + ti.tree_len);
      uint64_t h = 0x243F6A8885A308D3ull;
      for (int s = 0; s < end; ++s) {
        bool vis = s < ti.prefix_len;
        if (!vis && s >= ti.tree_base && s < ti.tree_base + ti.tree_len)
          vis = (ti.tree_vis >> (s - ti.tree_base)) & 1ull;
        if (!vis) continue;
        h = mix64(h + (uint64_t)(int64_t)cache[slot_of(ti.req, s)] + 1);
      }
      (*hs)[t] = h;
    }
  }

  int next_token(uint64_t h) const { return (int)((h >> 17) % (uint64_t)vocab); }

  ffmi_status run_inc(const BatchConfig &bc, InferenceResult *ir) override {
    if (cap >= 0 && bc.num_tokens > cap) return FFMI_ERR_INVALID;
    // (as the GPU model: ids outside the vocabulary are rejected, so a
    // scheduler read past a step's results cannot pass unnoticed)
    for (int t = 0; t < bc.num_tokens; ++t)
      if (bc.tokensInfo[t].token_id < 0 || bc.tokensInfo[t].token_id >= vocab)
        return FFMI_ERR_INVALID;
    PackedStep ps;
    pack_inc(bc, max_requests, slots, &ps);
    std::vector<uint64_t> hs;
    contexts(ps, &hs);
    for (size_t t = 0; t < hs.size(); ++t) ir->token_ids[t] = next_token(hs[t]);
    return FFMI_OK;
  }
  ffmi_status run_tree(const TreeVerifyBatchConfig &bc, InferenceResult *ir) override {
    if (cap >= 0 && bc.num_tokens > cap) return FFMI_ERR_INVALID;
    // (as the GPU model: ids outside the vocabulary are rejected, so a
    // scheduler read past a step's results cannot pass unnoticed)
    for (int t = 0; t < bc.num_tokens; ++t)
      if (bc.tokensInfo[t].token_id < 0 || bc.tokensInfo[t].token_id >= vocab)
        return FFMI_ERR_INVALID;
    PackedStep ps;
    pack_tree(bc, max_requests, slots, &ps);
    std::vector<uint64_t> hs;
    contexts(ps, &hs);
    for (size_t t = 0; t < hs.size(); ++t) ir->token_ids[t] = next_token(hs[t]);
    return FFMI_OK;
  }
  ffmi_status run_beam(const BeamSearchBatchConfig &bc, BeamInferenceResult *ir) override {
    if (cap >= 0 && bc.num_tokens > cap) return FFMI_ERR_INVALID;
    // (as the GPU model: ids outside the vocabulary are rejected, so a
    // scheduler read past a step's results cannot pass unnoticed)
    for (int t = 0; t < bc.num_tokens; ++t)
      if (bc.tokensInfo[t].token_id < 0 || bc.tokensInfo[t].token_id >= vocab)
        return FFMI_ERR_INVALID;
    PackedStep ps;
    pack_beam(bc, max_requests, slots, &ps);
    std::vector<uint64_t> hs;
    contexts(ps, &hs);
    const int k = ps.topk;
    // [T][k] as the GPU model's top-k writes it, then the scheduler's layout
    std::vector<int> ids(hs.size() * k);
    std::vector<float> prs(hs.size() * k);
    for (size_t t = 0; t < hs.size(); ++t) {
      const uint64_t h = hs[t];
      const int c0 = next_token(h);
      const int c1 = (int)((c0 + 1 + (h >> 40) % 7) % (uint64_t)vocab);
      const int c2 = (int)((c1 + 1 + (h >> 45) % 7) % (uint64_t)vocab);
      const int c3 = (int)((c2 + 1 + (h >> 50) % 7) % (uint64_t)vocab);  // k = 4 (width 4)
      const bool agree = (int)(mix64(h ^ salt) % 100) >= disagree;
      std::array<int, 4> rank = agree ? std::array<int, 4>{c0, c1, c2, c3}
                                      : std::array<int, 4>{c1, c0, c2, c3};
      for (int j = 0; j < k; ++j) {
        ids[t * k + j] = rank[j % 4];
        prs[t * k + j] = 1.0f / (float)(1 << j);
      }
    }
    std::vector<int> map;
    beam_result_layout(bc, &map);
    for (size_t i = 0; i < map.size(); ++i) {
      ir->token_ids[i] = ids[map[i]];
      ir->probs[i] = prs[map[i]];
      ir->parent_id[i] = 0;
    }
    // entries past the step's results: out of the vocabulary (see above)
    for (size_t i = map.size(); i < map.size() + 4 * hs.size() + 4; ++i) ir->token_ids[i] = -7777;
    last_results = map.size();
    return FFMI_OK;
  }
};

ffmi_status create_hash_model(int vocab, int mode, int max_requests, int max_seq,
                              int max_tree, uint64_t salt, int disagree_pct,
                              ffmi_model **out) {
  if (vocab < 32 || max_requests <= 0 || max_seq <= 0) return FFMI_ERR_INVALID;
  HashModel *m = new HashModel();
  m->mode = mode;
  m->vocab = vocab;
  m->max_requests = max_requests;
  m->slots = max_seq + max_tree;
  m->salt = salt;
  m->disagree = disagree_pct;
  m->cache.assign((size_t)max_requests * m->slots, -1);
  *out = m;
  return FFMI_OK;
}

}  // namespace ffmi

// Built into libffmi_testmodel.so (tests only), never into libffmi.so.
extern "C" ffmi_status ffmi_test_hash_model_create(int vocab, int mode, int max_requests,
                                                   int max_seq, int max_tree, uint64_t salt,
                                                   int disagree_pct, ffmi_model **out) {
  if (!out) return FFMI_ERR_INVALID;
  return ffmi::create_hash_model(vocab, mode, max_requests, max_seq, max_tree, salt,
                                 disagree_pct, out);
}

extern "C" ffmi_status ffmi_test_hash_model_set_capacity(ffmi_model *m, int max_tokens) {
  ffmi::HashModel *h = dynamic_cast<ffmi::HashModel *>(m);
  if (!h) return FFMI_ERR_INVALID;
  h->cap = max_tokens;
  return FFMI_OK;
}
