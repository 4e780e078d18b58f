// pack.cpp -- BatchConfig -> per-token KV-slot / visibility metadata.
//
// This is where the reference's three attention ops differ; the device
// kernels (kernels/attention.hip) only evaluate the packed rule.  The scheduler
// test double (hash_model.cpp) consumes the SAME packed metadata, so CPU tests
// of the RequestManager also check these rules.
#include <algorithm>

#include "model.h"

namespace ffmi {

void PackedStep::desc(ffmi_batch_desc *d) const {
  d->num_tokens = (int)tokens.size();
  d->num_work = (int)work.size();
  d->num_commits = (int)commits.size();
  d->num_mask_reqs = num_mask_reqs;
  d->tokens = tokens.data();
  d->work = work.data();
  d->commits = commits.data();
  d->masks = masks.data();
}

static void build_work(PackedStep *ps) {
  ps->work.clear();
  const int T = (int)ps->tokens.size();
  int t = 0;
  while (t < T) {
    const int req = ps->tokens[t].req;
    ffmi_attn_work w;
    w.req = req;
    w.q_start = t;
    w.q_count = 0;
    w.kv_len = 0;
    while (t < T && ps->tokens[t].req == req && w.q_count < FFMI_ATTN_QTILE) {
      const ffmi_token_info &ti = ps->tokens[t];
      w.kv_len = std::max(w.kv_len, std::max(ti.prefix_len, ti.tree_base + ti.tree_len));
      ++w.q_count;
      ++t;
    }
    ps->work.push_back(w);
  }
}

// transpose the request's key-major bitmask into the query's visibility word
static void fill_tree_vis(PackedStep *ps) {
  for (auto &ti : ps->tokens) {
    ti.tree_vis = 0;
    if (ti.tree_len <= 0 || ps->num_mask_reqs == 0) continue;
    const uint64_t *m = &ps->masks[(size_t)ti.req * FFMI_MAX_TREE];
    const int n = std::min(ti.tree_len, FFMI_MAX_TREE);
    for (int j = 0; j < n; ++j) ti.tree_vis |= ((m[j] >> ti.tree_bit) & 1ull) << j;
  }
}

static void clamp_slots(PackedStep *ps, int slots) {
  for (auto &ti : ps->tokens) {
    if (ti.store_slot >= slots) ti.store_slot = -1;
    ti.prefix_len = std::min(ti.prefix_len, slots);
    if (ti.tree_base + ti.tree_len > slots) ti.tree_len = std::max(0, slots - ti.tree_base);
  }
}

static void copy_masks(const BatchConfig &bc, int max_requests, PackedStep *ps) {
  ps->num_mask_reqs = max_requests;
  ps->masks.assign((size_t)max_requests * FFMI_MAX_TREE, 0ull);
  for (int r = 0; r < max_requests && r < BatchConfig::MAX_NUM_REQUESTS; ++r) {
    if (bc.request_completed[r]) continue;
    std::copy(bc.causalMask[r].mask, bc.causalMask[r].mask + FFMI_MAX_TREE,
              ps->masks.begin() + (size_t)r * FFMI_MAX_TREE);
  }
}

void pack_inc(const BatchConfig &bc, int max_requests, int slots, PackedStep *ps) {
  ps->tokens.resize(bc.num_tokens);
  ps->commits.clear();
  ps->masks.clear();
  ps->num_mask_reqs = 0;
  ps->topk = 1;
  for (int t = 0; t < bc.num_tokens; ++t) {
    const auto &tk = bc.tokensInfo[t];
    ffmi_token_info &ti = ps->tokens[t];
    ti.token_id = tk.token_id;
    ti.pos = tk.abs_depth_in_request;
    ti.req = tk.request_index;
    ti.store_slot = tk.abs_depth_in_request;  // store_kv_cache: tok_id = abs depth
    ti.prefix_len = tk.abs_depth_in_request + 1;  // causal incl. self
    ti.tree_base = 0;
    ti.tree_len = 0;
    ti.tree_bit = 0;
    ti.tree_vis = 0;
  }
  (void)max_requests;
  clamp_slots(ps, slots);
  build_work(ps);
}

void pack_tree(const TreeVerifyBatchConfig &bc, int max_requests, int slots, PackedStep *ps) {
  ps->tokens.resize(bc.num_tokens);
  ps->topk = 1;
  ps->commits.resize(bc.num_tokens_to_commit);
  for (int c = 0; c < bc.num_tokens_to_commit; ++c) {
    ps->commits[c].src_token = bc.committed_tokens[c].token_index;
    ps->commits[c].req = bc.committed_tokens[c].request_index;
    ps->commits[c].depth = bc.committed_tokens[c].token_depth;
    ps->commits[c].pad = 0;
  }
  copy_masks(bc, max_requests, ps);
  for (int t = 0; t < bc.num_tokens; ++t) {
    const auto &tk = bc.tokensInfo[t];
    const int r = tk.request_index;
    const auto &R = bc.requestsInfo[r];
    const int local = t - R.first_token_offset_in_batch;
    ffmi_token_info &ti = ps->tokens[t];
    ti.token_id = tk.token_id;
    ti.pos = tk.abs_depth_in_request;
    ti.req = r;
    ti.store_slot = R.first_token_depth_in_request + local;
    if (R.prompt_phase) {
      ti.prefix_len = R.first_token_depth_in_request + local + 1;
      ti.tree_base = ti.tree_len = ti.tree_bit = 0;
    } else {
      const int ntcs = bc.causalMask[r].non_tree_cache_size;
      const int tlength = R.first_token_depth_in_request + R.num_tokens_in_batch;
      ti.prefix_len = std::min(ntcs, tlength);
      ti.tree_base = ntcs;
      ti.tree_len = std::max(0, tlength - ntcs);
      ti.tree_bit = local;
    }
  }
  clamp_slots(ps, slots);
  fill_tree_vis(ps);
  build_work(ps);
}

int beam_step_topk(const BeamSearchBatchConfig &bc) {
  int k = 1;
  for (int t = 0; t < bc.num_tokens; ++t)
    k = std::max(k, bc.beamRequestsInfo[bc.tokensInfo[t].request_index].beam_size);
  return k;
}

void beam_result_layout(const BeamSearchBatchConfig &bc, std::vector<int> *map) {
  const int k = beam_step_topk(bc);
  map->clear();
  for (int t = 0; t < bc.num_tokens; ++t) {
    const int w = bc.beamRequestsInfo[bc.tokensInfo[t].request_index].beam_size;
    for (int j = 0; j < w && j < k; ++j) map->push_back(t * k + j);
  }
}

void pack_beam(const BeamSearchBatchConfig &bc, int max_requests, int slots,
               PackedStep *ps) {
  ps->tokens.resize(bc.num_tokens);
  ps->commits.clear();
  copy_masks(bc, max_requests, ps);
  // the top-k of every token for the widest request of the step (the
  // reference's ArgTopK computes MAX_BEAM_WIDTH for every token and asserts
  // that all requests but the last share one width, arg_topk.cu:403-420);
  // beam_result_layout hands each request its own width's entries
  ps->topk = beam_step_topk(bc);
  for (int t = 0; t < bc.num_tokens; ++t) {
    const auto &tk = bc.tokensInfo[t];
    const int r = tk.request_index;
    const auto &R = bc.requestsInfo[r];
    const auto &M = bc.causalMask[r];
    const int local = t - R.first_token_offset_in_batch;
    ffmi_token_info &ti = ps->tokens[t];
    ti.token_id = tk.token_id;
    ti.pos = tk.abs_depth_in_request;
    ti.req = r;
    ti.store_slot = M.prompt_size + M.non_tree_cache_size + M.tree_size - 1 -
                    M.this_layer_size + local;
    const bool gen = bc.request_running[r] && !R.prompt_phase;
    if (!gen) {
      ti.prefix_len = R.first_token_depth_in_request + local + 1;
      ti.tree_base = ti.tree_len = ti.tree_bit = 0;
    } else {
      const int ntcs = M.non_tree_cache_size;
      const int total = ntcs + M.tree_size + M.prompt_size - 1;
      const int branches = bc.beamRequestsInfo[r].sub_request_num;
      ti.prefix_len = ntcs;
      ti.tree_base = ntcs;
      ti.tree_len = std::max(0, total - ntcs);
      ti.tree_bit = M.prompt_size + M.tree_size - 1 - branches + local;
    }
  }
  clamp_slots(ps, slots);
  fill_tree_vis(ps);
  build_work(ps);
}

}  // namespace ffmi
