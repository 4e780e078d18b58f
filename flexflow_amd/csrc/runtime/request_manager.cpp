// request_manager.cpp -- continuous batching and the SpecInfer token-tree
// scheduler, restated from src/runtime/request_manager.cc (reference
// @2025-01-17).  Each function cites the reference lines whose behaviour it
// reproduces.  Deliberate differences (documented in DESIGN.md):
//  * bit operations on BitMask words are 64-bit (1ull << j); the reference's
//    `1 << j` on int breaks for trees deeper than 31 tokens (quirk 6);
//  * no tokenizer: requests carry token ids (the parity unit);
//  * no PEFT / finetuning requests;
//  * flagged extensions (FFMI_SPEC_EXT_*, off by default, where the reference
//    asserts): tree width / branches 4 (request_manager.cc:168-171 allows 3),
//    and N SSMs whose trees merge_dfs_trees unites (the reference asserts one
//    SSM, :2823-2827, ahead of a merge it never runs);
//  * the verify step walks the tree by parent links (traverse_verify_tree):
//    identical to the reference's layer-slot walk on every tree it admits,
//    and correct on trees that branch twice or are merged.
#include "request_manager.h"

#include <assert.h>
#include <stdio.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>

void ffmi_set_last_error(const char *msg, const char *file, int line);  // api.cpp

namespace ffmi {

double now_us() {
  using namespace std::chrono;
  return (double)duration_cast<nanoseconds>(steady_clock::now().time_since_epoch()).count() *
         1e-3;
}

static BatchLimits g_limits;
BatchLimits &batch_limits() { return g_limits; }
int BatchConfig::max_requests_per_batch() { return g_limits.max_requests_per_batch; }
int BatchConfig::max_tokens_per_batch() { return g_limits.max_tokens_per_batch; }
int BatchConfig::max_spec_tree_token_num() { return g_limits.max_spec_tree_token_num; }
int BatchConfig::max_sequence_length() { return g_limits.max_sequence_length; }
int BatchConfig::max_verify_tokens_per_batch() {
  return g_limits.max_tokens_per_batch +
         g_limits.max_spec_tree_token_num * g_limits.max_requests_per_batch;
}

BatchConfig::BatchConfig() {
  for (int i = 0; i < MAX_NUM_REQUESTS; ++i) {
    request_completed[i] = true;
    request_running[i] = false;
  }
}

int BatchConfig::num_active_requests() const {
  int n = 0;
  for (int i = 0; i < max_requests_per_batch(); ++i) n += !request_completed[i];
  return n;
}

RequestManager::RequestManager() {}

void RequestManager::apply_limits() const {
  g_limits.max_requests_per_batch = max_requests_per_batch;
  g_limits.max_tokens_per_batch = max_tokens_per_batch;
  g_limits.max_spec_tree_token_num = max_spec_tree_token_num;
  g_limits.max_sequence_length = max_sequence_length;
}

int RequestManager::max_beam_width() const {
  return spec_extensions & FFMI_SPEC_EXT_WIDTH4 ? BeamSearchBatchConfig::MAX_BEAM_WIDTH
                                                : BeamSearchBatchConfig::REFERENCE_MAX_BEAM_WIDTH;
}
int RequestManager::max_tree_branches() const {
  return spec_extensions & FFMI_SPEC_EXT_WIDTH4
             ? BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES
             : BeamSearchBatchConfig::REFERENCE_MAX_SPECULATIVE_TREE_BRANCHES;
}

// request_manager.cc:168-171
bool RequestManager::push_spec_infer_tree_width(int w) {
  if (w > max_beam_width() || w < 1) return false;
  // nodes per tree layer = product of the widths so far; the reference
  // asserts it stays <= MAX_SPECULATIVE_TREE_BRANCHES at run time
  // (request_manager.cc:1685-1687) -- reject such a sequence up front
  int nodes = w;
  for (int x : spec_infer_tree_width) nodes *= x;
  if (nodes > max_tree_branches()) return false;
  spec_infer_tree_width.push_back(w);
  return true;
}

// request_manager.cc:334-441 (tokenizer replaced by token ids)
RequestManager::RequestGuid RequestManager::register_new_request(
    const std::vector<int> &prompt, int max_length, int max_new_tokens,
    bool add_special_tokens) {
  Request request;
  request.status = Request::PENDING;
  request.guid = next_available_guid++;
  request.max_length = max_length;
  request.max_new_tokens = max_new_tokens;
  request.add_special_tokens = add_special_tokens;
  if (request.max_length == -1 && request.max_new_tokens == -1)
    request.max_length = max_sequence_length - 1;
  if (request.max_length != -1 && request.max_new_tokens != -1) request.max_length = -1;
  if (bos_token_id >= 0 && request.add_special_tokens) request.tokens.push_back(bos_token_id);
  if (request.max_new_tokens != -1)
    request.max_length = (int)prompt.size() + request.max_new_tokens;
  if ((int)prompt.size() >= max_sequence_length) return 0;
  if (request.max_length >= max_sequence_length) return 0;
  request.tokens.insert(request.tokens.end(), prompt.begin(), prompt.end());
  request.initial_len = (int)request.tokens.size();
  if (!ssm_models.empty()) request.beam_trees.resize(ssm_models.size());
  pending_infr_request_queue.push_back(request);
  all_requests[request.guid] = request;
  GenerationResult gr;
  gr.guid = request.guid;
  gr.input_tokens = request.tokens;
  gr.output_tokens = request.tokens;
  request_generation_results[request.guid] = gr;
  ProfileInfo pi;
  pi.registration_time = now_us();
  profiling_requests[request.guid] = pi;
  return request.guid;
}

bool RequestManager::is_eos_token(int token_id) const {
  for (int e : eos_token_ids)
    if (e == token_id) return true;
  return false;
}

// request_manager.cc:645-657
bool RequestManager::check_inf_req_completion(const BatchConfig &old_bc, int i) {
  Request &request = all_requests[old_bc.requestsInfo[i].request_guid];
  if ((int)request.tokens.size() >= old_bc.requestsInfo[i].max_length) return true;
  return is_eos_token(request.tokens.back());
}

void RequestManager::complete_request(Request &request, bool spec) {
  request.status = Request::COMPLETED;
  GenerationResult &gr = request_generation_results[request.guid];
  gr.output_tokens = request.tokens;
  ProfileInfo &pi = profiling_requests[request.guid];
  pi.finish_time = now_us();
  num_processed_requests++;
  if (verbose)
    printf("[ffmi] guid(%lld) done: len %zu llm_steps %d latency %.1f us\n",
           (long long)request.guid, request.tokens.size(), pi.llm_decoding_steps,
           pi.finish_time - pi.start_time);
  if (!output_filepath.empty()) write_output_record(request, spec);
}

std::string RequestManager::decode(const std::vector<int> &ids) const {
  if (!detok) return std::string();
  const int n = detok(ids.data(), (int)ids.size(), nullptr, 0, detok_ctx);
  if (n <= 0) return std::string();
  std::string out((size_t)n, '\0');
  const int m = detok(ids.data(), (int)ids.size(), &out[0], n, detok_ctx);
  out.resize((size_t)std::max(0, std::min(m, n)));
  return out;
}

std::string RequestManager::decode_request(const Request &request) const {
  std::string text = decode(request.tokens);
  if (detok && old_llama_tokenizer && request.add_special_tokens && !request.tokens.empty() &&
      request.tokens[0] == bos_token_id)
    text = "<s> " + text;
  return text;
}

// The reference's per-request output record, appended on completion:
// incremental decoding request_manager.cc:813-840 ("[Profile] guid(..)
// llm_decoding_steps(..) latency(..) ttft(..)"), SpecInfer :1303-1330 (no
// ttft); then "token IDs: a,b,...", a newline and the decoded text, which the
// reference writes without a trailing newline.  Times in microseconds with 3
// decimals.  Warmup requests do not exist here, so the tag is always Profile.
void RequestManager::write_output_record(const Request &request, bool spec) const {
  FILE *f = fopen(output_filepath.c_str(), "a");
  if (!f) {
    fprintf(stderr, "Unable to open the output file: %s\n", output_filepath.c_str());
    return;
  }
  const ProfileInfo &pi = profiling_requests.at(request.guid);
  fprintf(f, "[Profile] guid(%lld) llm_decoding_steps(%d) latency(%.3f)", (long long)request.guid,
          pi.llm_decoding_steps, pi.finish_time - pi.start_time);
  if (!spec) fprintf(f, " ttft(%.3f)", pi.first_token_time - pi.registration_time);
  fputs("\ntoken IDs: ", f);
  for (size_t i = 0; i < request.tokens.size(); ++i)
    fprintf(f, i + 1 < request.tokens.size() ? "%d," : "%d", request.tokens[i]);
  fputc('\n', f);
  const std::string text = decode_request(request);
  fwrite(text.data(), 1, text.size(), f);
  fclose(f);
}

// request_manager.cc:713-1135 (inference requests only)
BatchConfig RequestManager::prepare_next_batch(const BatchConfig &old_bc,
                                               const InferenceResult &result) {
  // Step 1: append the result of the previous step
  for (int i = 0; i < old_bc.num_tokens; i++) {
    const RequestGuid guid = old_bc.requestsInfo[old_bc.tokensInfo[i].request_index].request_guid;
    Request &request = all_requests[guid];
    if (old_bc.tokensInfo[i].abs_depth_in_request + 1 < (int)request.tokens.size()) continue;
    assert(old_bc.tokensInfo[i].abs_depth_in_request + 1 == (int)request.tokens.size());
    ProfileInfo &pi = profiling_requests[guid];
    if (!pi.first_token_time_set) {
      pi.first_token_time = now_us();
      pi.first_token_time_set = true;
    }
    request.tokens.push_back(result.token_ids[i]);
  }
  // Step 2: carry on running requests
  BatchConfig new_bc;
  int num_generation_tokens = 0;
  int num_active_req = -1;
  const int batch_size = max_requests_per_batch;
  for (int i = 0; i < batch_size; i++) {
    if (old_bc.request_completed[i]) continue;
    Request &request = all_requests[old_bc.requestsInfo[i].request_guid];
    const int processed = old_bc.requestsInfo[i].first_token_depth_in_request +
                          old_bc.requestsInfo[i].num_tokens_in_batch;
    assert(processed < (int)request.tokens.size());
    if (check_inf_req_completion(old_bc, i)) {
      if (is_eos_token(request.tokens.back())) request.tokens.pop_back();
      complete_request(request);
      continue;
    }
    auto &R = new_bc.requestsInfo[i];
    new_bc.request_completed[i] = false;
    R.first_token_depth_in_request = processed;
    R.first_token_offset_in_batch = new_bc.num_tokens;
    R.request_guid = old_bc.requestsInfo[i].request_guid;
    R.max_length = old_bc.requestsInfo[i].max_length;
    num_active_req++;
    new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
    if (R.first_token_depth_in_request + 1 == (int)request.tokens.size()) {
      R.num_tokens_in_batch = 1;  // decoding
      num_generation_tokens++;
      R.prompt_phase = false;
    } else {
      // prompt chunk; keep room for the decoding requests behind it (:866-890)
      int space_for_incr_dec_requests = 0;
      for (int ii = i + 1; ii < batch_size; ii++) {
        if (old_bc.request_completed[ii]) continue;
        if (!check_inf_req_completion(old_bc, ii)) space_for_incr_dec_requests++;
      }
      R.num_tokens_in_batch = std::min(
          max_tokens_per_batch - new_bc.num_tokens - space_for_incr_dec_requests,
          (int)request.tokens.size() - R.first_token_depth_in_request);
      R.prompt_phase = true;
    }
    for (int j = 0; j < R.num_tokens_in_batch; j++) {
      const int depth = R.first_token_depth_in_request + j;
      new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
      new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = depth;
      new_bc.tokensInfo[new_bc.num_tokens].token_id = request.tokens[depth];
      new_bc.num_tokens++;
    }
    profiling_requests[R.request_guid].llm_decoding_steps++;
  }
  new_bc.num_generation_tokens = num_generation_tokens;
  // Step 3: admit new requests into free slots (:910-963)
  for (int i = 0; i < batch_size; i++) {
    if (!new_bc.request_completed[i]) continue;
    if (pending_infr_request_queue.empty() || new_bc.num_tokens >= max_tokens_per_batch) continue;
    Request new_request = pending_infr_request_queue.front();
    pending_infr_request_queue.pop_front();
    auto &R = new_bc.requestsInfo[i];
    R.first_token_depth_in_request = 0;
    R.first_token_offset_in_batch = new_bc.num_tokens;
    R.request_guid = new_request.guid;
    R.num_tokens_in_batch = std::min(max_tokens_per_batch - new_bc.num_tokens,
                                     (int)new_request.tokens.size());
    R.max_length = new_request.max_length;
    R.prompt_phase = true;
    new_bc.request_completed[i] = false;
    num_active_req++;
    new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
    ProfileInfo &pi = profiling_requests[new_request.guid];
    pi.llm_decoding_steps = 1;
    pi.start_time = now_us();
    for (int j = 0; j < R.num_tokens_in_batch; j++) {
      new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
      new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = j;
      new_bc.tokensInfo[new_bc.num_tokens].token_id = new_request.tokens[j];
      new_bc.num_tokens++;
    }
    if (new_bc.num_tokens == max_tokens_per_batch) break;
  }
  return new_bc;
}

// ---------------------------------------------------------------------------
// SpecInfer: request init phase (request_manager.cc:1170-1579)
// ---------------------------------------------------------------------------
BeamSearchBatchConfig RequestManager::prepare_next_batch_init(
    const TreeVerifyBatchConfig &old_bc, const InferenceResult &result, int model_id) {
  BeamSearchBatchConfig new_bc;
  new_bc.num_tokens = 0;
  new_bc.model_id = model_id;
  int result_index = 0;
  int num_active_req = -1;
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (old_bc.request_completed[i]) continue;
    const RequestGuid guid = old_bc.requestsInfo[i].request_guid;
    Request &request = all_requests[guid];
    std::vector<TokenDepth> tree_outputs;
    committed_tokens[guid].clear();
    const int root_abs_depth = (int)request.tokens.size() - 1;
    while (result_index < old_bc.num_tokens &&
           old_bc.tokensInfo[result_index].request_index == i) {
      const int abs_depth = old_bc.tokensInfo[result_index].abs_depth_in_request;
      const int token_id = result.token_ids[result_index];
      if (request.status == Request::PENDING) {
        committed_tokens[guid].emplace_back(abs_depth, result_index);
      } else if (abs_depth >= root_abs_depth) {
        tree_outputs.emplace_back(token_id, abs_depth + 1);
        committed_tokens[guid].emplace_back(abs_depth, result_index);
      }
      result_index++;
    }
    if (request.status == Request::RUNNING) {
      std::vector<TokenDepth> verified_tokens =
          traverse_verify_tree(guid, dfs_tree_inputs.at(guid), tree_outputs);
      stats.tokens_committed += (long)verified_tokens.size();
      stats.request_verifies++;
      // The reference keeps no SpecInfer ttft (its output record has none,
      // :1303-1311); recorded here for the Python results only.
      ProfileInfo &pi = profiling_requests[guid];
      if (!pi.first_token_time_set) {
        pi.first_token_time = now_us();
        pi.first_token_time_set = true;
      }
      if ((int)(verified_tokens.size() + request.tokens.size()) >= request.max_length) {
        for (const auto &tp : verified_tokens)
          if (tp.second < request.max_length) request.tokens.push_back(tp.first);
        complete_request(request, true);
        new_bc.request_completed[i] = true;
        new_bc.request_running[i] = false;
        dfs_tree_inputs.erase(guid);
        dfs_tree_parents.erase(guid);
      } else {
        new_bc.request_completed[i] = false;
        new_bc.request_running[i] = true;
        num_active_req++;
        auto &R = new_bc.requestsInfo[i];
        R.first_token_depth_in_request = verified_tokens.front().second;
        R.first_token_offset_in_batch = new_bc.num_tokens;
        R.request_guid = guid;
        R.max_length = old_bc.requestsInfo[i].max_length;
        R.num_tokens_in_batch = (int)verified_tokens.size();
        new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
        const int new_max_depth =
            R.max_length - R.first_token_depth_in_request - (int)verified_tokens.size();
        auto &B = new_bc.beamRequestsInfo[i];
        B.current_depth = 1;
        profiling_requests[guid].ssm_decoding_steps = 0;
        R.prompt_phase = true;
        B.beam_size = spec_infer_tree_width.size() > 0 ? spec_infer_tree_width[0] : 1;
        B.max_depth = std::min(new_max_depth, BeamSearchBatchConfig::MAX_BEAM_DEPTH);
        for (int j = 0; j < BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES; j++) {
          B.parent_id[j] = 0;
          B.probs[j] = 1;
        }
        B.sub_request_num = 1;
        new_bc.sub_requests[i] = 1;
        updateBitMask(new_bc.causalMask[i], (int)verified_tokens.size(),
                      (int)request.tokens.size());
        for (size_t j = 0; j < verified_tokens.size(); j++) {
          const auto &tk = verified_tokens[j];
          new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
          new_bc.tokensInfo[new_bc.num_tokens].token_id = tk.first;
          new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = tk.second;
          new_bc.beamTokenInfo[new_bc.num_tokens].sub_request_index = 0;
          new_bc.num_tokens++;
          request.tokens.push_back(tk.first);
          // (the reference breaks here once the batch holds
          // max_tokens_per_batch tokens, :1402-1404: the rest of this
          // request's verified tokens never reach request.tokens although
          // the LLM committed them, and later requests' tokens go past the
          // limit anyway.  Every verified token is kept: an init batch holds
          // at most max_requests x (MAX_BEAM_DEPTH + 1) tokens, which the SSM
          // models are sized for, and a model smaller than that reports
          // FFMI_ERR_INVALID instead of dropping tokens.)
        }
      }
    } else if (request.status == Request::PENDING) {
      new_bc.request_completed[i] = false;
      new_bc.request_running[i] = false;
      num_active_req++;
      // The reference asserts here (:1425): a prompt the SSM could not load
      // within one init + MAX_BEAM_DEPTH beam batches while the LLM still
      // loads it in chunks.  Reported as an error, not an abort.
      if (request.ssm_cache_size != request.initial_len) ssm_prompt_behind = true;
      auto &R = new_bc.requestsInfo[i];
      R.first_token_depth_in_request = request.ssm_cache_size;
      R.first_token_offset_in_batch = new_bc.num_tokens;
      R.request_guid = guid;
      R.max_length = old_bc.requestsInfo[i].max_length;
      R.num_tokens_in_batch = 0;
      new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
      auto &B = new_bc.beamRequestsInfo[i];
      B.current_depth = 1;
      const int steps = profiling_requests[guid].ssm_decoding_steps;
      B.beam_size = (int)spec_infer_tree_width.size() > steps ? spec_infer_tree_width[steps] : 1;
      B.max_depth = 0;
      for (int j = 0; j < BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES; j++) {
        B.parent_id[j] = 0;
        B.probs[j] = 1;
      }
      B.sub_request_num = 1;
      new_bc.sub_requests[i] = 1;
    } else {
      assert(false && "request status is not RUNNING or PENDING");
    }
  }
  // admit new requests (:1497-1571)
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (!new_bc.request_completed[i]) continue;
    if (pending_infr_request_queue.empty() || new_bc.num_tokens >= max_tokens_per_batch) continue;
    Request new_request = pending_infr_request_queue.front();
    pending_infr_request_queue.pop_front();
    num_active_req++;
    auto &R = new_bc.requestsInfo[i];
    R.first_token_depth_in_request = 0;
    R.first_token_offset_in_batch = new_bc.num_tokens;
    R.request_guid = new_request.guid;
    R.num_tokens_in_batch =
        std::min(max_tokens_per_batch - new_bc.num_tokens, (int)new_request.tokens.size());
    R.max_length = new_request.max_length;
    new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
    ProfileInfo &pi = profiling_requests[new_request.guid];
    pi.llm_decoding_steps = 0;
    pi.ssm_decoding_steps = 0;
    pi.start_time = now_us();
    auto &B = new_bc.beamRequestsInfo[i];
    B.beam_size = spec_infer_tree_width.size() > 0 ? spec_infer_tree_width[0] : 1;
    B.current_depth = 1;
    B.max_depth = std::min(BeamSearchBatchConfig::MAX_BEAM_DEPTH,
                           max_tokens_per_batch - R.num_tokens_in_batch - 1);
    for (int j = 0; j < BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES; j++) {
      B.parent_id[j] = 0;
      B.probs[j] = 1;
    }
    new_bc.request_completed[i] = false;
    R.prompt_phase = true;
    B.sub_request_num = 1;
    new_bc.sub_requests[i] = 1;
    for (int j = 0; j < R.num_tokens_in_batch; j++) {
      new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
      new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = j;
      new_bc.tokensInfo[new_bc.num_tokens].token_id = new_request.tokens[j];
      new_bc.beamTokenInfo[new_bc.num_tokens].sub_request_index = 0;
      new_bc.num_tokens++;
    }
    initBitMask(new_bc.causalMask[i], R.num_tokens_in_batch);
    all_requests[new_request.guid].status = Request::PENDING;
    all_requests[new_request.guid].ssm_cache_size = R.num_tokens_in_batch;
    new_bc.request_running[i] = false;
    if (new_bc.num_tokens == max_tokens_per_batch) break;
  }
  new_bc.num_generation_tokens = 0;
  return new_bc;
}

// ---------------------------------------------------------------------------
// SpecInfer: beam (SSM) phase (request_manager.cc:1610-1892)
// ---------------------------------------------------------------------------
BeamSearchBatchConfig RequestManager::prepare_next_batch_beam(
    const BeamSearchBatchConfig &old_bc, const BeamInferenceResult &result) {
  store_beam_metadata(old_bc, result);
  BeamSearchBatchConfig new_bc;
  new_bc.model_id = old_bc.model_id;
  int num_generation_tokens = 0;
  int num_active_req = -1;
  // running requests first
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (old_bc.request_completed[i] || !old_bc.request_running[i]) continue;
    num_active_req++;
    Request &request = all_requests[old_bc.requestsInfo[i].request_guid];
    const int processed = old_bc.requestsInfo[i].first_token_depth_in_request +
                          old_bc.requestsInfo[i].num_tokens_in_batch;
    auto &R = new_bc.requestsInfo[i];
    auto &B = new_bc.beamRequestsInfo[i];
    const auto &OB = old_bc.beamRequestsInfo[i];
    new_bc.request_completed[i] = false;
    R.first_token_depth_in_request = processed;
    R.first_token_offset_in_batch = new_bc.num_tokens;
    R.request_guid = old_bc.requestsInfo[i].request_guid;
    R.max_length = old_bc.requestsInfo[i].max_length;
    ++profiling_requests[request.guid].ssm_decoding_steps;
    // the reference indexes the widths by ssm_decoding_steps, reset to 0 at
    // init and counted per beam batch (:1680-1683): with one SSM that is
    // the beam depth reached, OB.current_depth.  With N SSMs the counter runs
    // on through every SSM's steps, so the depth is used.
    const int steps = OB.current_depth;
    new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
    B.beam_size = (int)spec_infer_tree_width.size() > steps ? spec_infer_tree_width[steps] : 1;
    B.max_depth = OB.max_depth;
    new_bc.sub_requests[i] = old_bc.sub_requests[i] * B.beam_size;
    B.sub_request_num = OB.sub_request_num * OB.beam_size;
    assert(B.sub_request_num <= BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES);
    assert(request.status == Request::RUNNING);
    B.current_depth = OB.current_depth + 1;
    new_bc.request_running[i] = true;
    update_beam_metadata(new_bc, old_bc, request.beam_trees.at(old_bc.model_id), i);
    if (R.first_token_depth_in_request >= (int)request.tokens.size())
      R.num_tokens_in_batch = 1;
    new_bc.causalMask[i] = old_bc.causalMask[i];
    appendBitMask(new_bc.causalMask[i], B.sub_request_num, OB.beam_size, OB.sub_request_num,
                  request.beam_trees[old_bc.model_id], OB.current_depth);
    for (int j = 0; j < R.num_tokens_in_batch; j++) {
      const int depth = R.first_token_depth_in_request + j;
      for (int k = 0; k < B.sub_request_num; k++) {
        new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
        new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = depth;
        new_bc.tokensInfo[new_bc.num_tokens].token_id = B.tokens[k];
        new_bc.beamTokenInfo[new_bc.num_tokens].sub_request_index = k;
        new_bc.num_tokens++;
        num_generation_tokens++;
      }
    }
  }
  new_bc.speculative_request_num = num_active_req + 1;
  // pending (prompt-loading) requests
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (old_bc.request_completed[i] || old_bc.request_running[i]) continue;
    num_active_req++;
    Request &request = all_requests[old_bc.requestsInfo[i].request_guid];
    const int processed = old_bc.requestsInfo[i].first_token_depth_in_request +
                          old_bc.requestsInfo[i].num_tokens_in_batch;
    auto &R = new_bc.requestsInfo[i];
    auto &B = new_bc.beamRequestsInfo[i];
    const auto &OB = old_bc.beamRequestsInfo[i];
    new_bc.request_completed[i] = false;
    R.first_token_depth_in_request = processed;
    R.first_token_offset_in_batch = new_bc.num_tokens;
    R.request_guid = old_bc.requestsInfo[i].request_guid;
    R.max_length = old_bc.requestsInfo[i].max_length;
    new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
    B.beam_size = 1;
    B.max_depth = OB.max_depth;
    new_bc.sub_requests[i] = 1;
    B.sub_request_num = OB.sub_request_num;
    assert(request.status == Request::PENDING);
    B.current_depth = OB.current_depth;
    new_bc.request_running[i] = false;
    new_bc.causalMask[i] = old_bc.causalMask[i];
    R.prompt_phase = true;
    if (R.first_token_depth_in_request >= (int)request.tokens.size()) {
      R.num_tokens_in_batch = 0;
      new_bc.causalMask[i].this_layer_size = 0;
      B.sub_request_num = 0;
      B.beam_size = 1;
    } else if (max_tokens_per_batch - new_bc.num_tokens - max_requests_per_batch + i <= 0) {
      // the running requests' beams took the batch: no prompt chunk in this
      // beam step (the reference asserts in appendPendingRequest, :2431);
      // a prompt that falls behind the LLM this way is reported as
      // ssm_prompt_behind at the next init, as any other
      R.num_tokens_in_batch = 0;
      new_bc.causalMask[i].this_layer_size = 0;
    } else {
      R.num_tokens_in_batch =
          std::min(max_tokens_per_batch - new_bc.num_tokens - max_requests_per_batch + i,
                   (int)request.tokens.size() - R.first_token_depth_in_request);
      // every SSM loads the same prompt chunk; count it once
      if (old_bc.model_id == 0) request.ssm_cache_size += R.num_tokens_in_batch;
      appendPendingRequest(new_bc.causalMask[i], R.num_tokens_in_batch);
    }
    for (int j = 0; j < R.num_tokens_in_batch; j++) {
      const int depth = R.first_token_depth_in_request + j;
      for (int k = 0; k < B.sub_request_num; k++) {
        new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
        new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = depth;
        new_bc.tokensInfo[new_bc.num_tokens].token_id =
            request.tokens[request.tokens.size() - R.num_tokens_in_batch + j];
        new_bc.beamTokenInfo[new_bc.num_tokens].sub_request_index = k;
        new_bc.num_tokens++;
      }
    }
  }
  new_bc.num_generation_tokens = num_generation_tokens;
  return new_bc;
}

// ---------------------------------------------------------------------------
// SpecInfer: verify (LLM) phase (request_manager.cc:1923-2215)
// ---------------------------------------------------------------------------
TreeVerifyBatchConfig RequestManager::prepare_next_batch_verify(
    const std::vector<BeamSearchBatchConfig> &old_batches) {
  assert(!old_batches.empty());
  TreeVerifyBatchConfig new_bc;
  new_bc.num_tokens_to_commit = 0;
  new_bc.num_tokens = 0;
  const int max_verify = get_max_verify_tokens_per_batch();
  int max_prompt_load_size = max_verify;
  const BeamSearchBatchConfig &b0 = old_batches.at(0);
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (b0.request_completed[i]) continue;
    if (b0.request_running[i])
      max_prompt_load_size -= (BeamSearchBatchConfig::MAX_BEAM_DEPTH + 1);
    else
      max_prompt_load_size -= 1;
  }
  // later[i]: active requests after slot i.  Each keeps one token slot
  // (a root or a prompt token), so a request's tree or prompt chunk never
  // takes the last slots a later request needs.  The reference budgets
  // MAX_BEAM_DEPTH + 1 tokens per running request (:1938-1946) although its
  // trees hold up to ~21 and merged trees up to 64, and asserts when the batch
  // overflows (:2137-2147); this only changes batches it would abort on.
  std::vector<int> later(max_requests_per_batch, 0);
  for (int i = max_requests_per_batch - 2; i >= 0; i--)
    later[i] = later[i + 1] + (b0.request_completed[i + 1] ? 0 : 1);
  int num_active_req = -1;
  for (int i = 0; i < max_requests_per_batch; i++) {
    if (b0.request_completed[i]) continue;
    num_active_req++;
    const RequestGuid guid = b0.requestsInfo[i].request_guid;
    Request &request = all_requests[guid];
    const int limit = max_verify - later[i];
    profiling_requests[guid].llm_decoding_steps += 1;
    auto &R = new_bc.requestsInfo[i];
    if (request.status == Request::RUNNING) {
      new_bc.request_running[i] = true;
      std::vector<std::vector<TokenDepth>> all_dfs_trees;
      for (size_t j = 0; j < old_batches.size(); j++)
        all_dfs_trees.push_back(
            traverse_beam_tree(old_batches.at(j), i, (int)request.tokens.size() - 1));
      std::vector<TokenDepth> tree =
          merge_dfs_trees(all_dfs_trees, (int)request.tokens.size() - 1, guid);
      const std::vector<int> &parent = dfs_tree_parents.at(guid);
      R.first_token_depth_in_request = tree.front().second;
      R.first_token_offset_in_batch = new_bc.num_tokens;
      R.request_guid = guid;
      R.max_length = b0.requestsInfo[i].max_length;
      new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
      new_bc.causalMask[i] = b0.causalMask[i];
      R.num_tokens_in_batch = 0;
      new_bc.request_completed[i] = false;
      auto it = committed_tokens.find(guid);
      if (it != committed_tokens.end()) {
        for (const auto &ct : it->second) {
          auto &c = new_bc.committed_tokens[new_bc.num_tokens_to_commit];
          c.token_index = ct.second;
          c.request_index = i;
          c.token_depth = ct.first;
          new_bc.num_tokens_to_commit++;
          request.llm_cache_size++;
        }
      }
      // the root: the last verified token
      new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
      new_bc.tokensInfo[new_bc.num_tokens].token_id = request.tokens.back();
      new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request =
          (int)request.tokens.size() - 1;
      new_bc.num_tokens++;
      R.num_tokens_in_batch++;
      assert(new_bc.num_tokens <= limit);
      R.first_token_depth_in_request = (int)request.tokens.size() - 1;
      bool cutLayer = false;
      for (size_t j = 1; j < tree.size(); j++) {
        // the batch is full with tree tokens left: drop the partially
        // included last layer (:2055-2091).  Checked before placing token j:
        // the root itself can take the last slot of `limit`, and then there
        // is no tree layer to drop (the request verifies its root alone)
        if (new_bc.num_tokens == limit) {
          cutLayer = j > 1;
          break;
        }
        new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
        new_bc.tokensInfo[new_bc.num_tokens].token_id = tree[j].first;
        new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = tree[j].second;
        new_bc.num_tokens++;
        R.num_tokens_in_batch++;
      }
      if (cutLayer) {  // drop the partially included last layer
        const int total_tokens = new_bc.num_tokens;
        for (int j = total_tokens - 1; j >= 1; j--) {
          new_bc.num_tokens--;
          R.num_tokens_in_batch--;
          if (new_bc.tokensInfo[j].abs_depth_in_request !=
              new_bc.tokensInfo[j - 1].abs_depth_in_request)
            break;
        }
      }
      // the verify bitmask of the tree as placed (a layer-order prefix of it
      // after cutLayer).  With one SSM this is the mask its beam steps built
      // (appendBitMask, :2426-2476); a merged tree needs its own.
      tree_bitmask(parent, R.num_tokens_in_batch, new_bc.causalMask[i]);
      stats.tree_tokens_verified += R.num_tokens_in_batch;
    } else if (request.status == Request::PENDING) {
      new_bc.request_running[i] = false;
      auto it = committed_tokens.find(guid);
      if (it != committed_tokens.end()) {
        for (const auto &ct : it->second) {
          auto &c = new_bc.committed_tokens[new_bc.num_tokens_to_commit];
          c.token_index = ct.second;
          c.request_index = i;
          c.token_depth = ct.first;
          new_bc.num_tokens_to_commit++;
          request.llm_cache_size++;
        }
      }
      new_bc.causalMask[i] = b0.causalMask[i];
      R.first_token_depth_in_request = request.llm_cache_size;
      R.first_token_offset_in_batch = new_bc.num_tokens;
      R.request_guid = guid;
      R.max_length = b0.requestsInfo[i].max_length;
      new_bc.requestsInfo[num_active_req].batch_config_request_id = i;
      new_bc.request_completed[i] = false;
      R.num_tokens_in_batch = std::max(
          0, std::min({max_prompt_load_size, limit - new_bc.num_tokens,
                       request.initial_len - R.first_token_depth_in_request}));
      max_prompt_load_size -= R.num_tokens_in_batch;
      if (request.llm_cache_size < request.initial_len) {
        for (int j = 0; j < R.num_tokens_in_batch; j++) {
          new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
          new_bc.tokensInfo[new_bc.num_tokens].token_id = request.tokens[request.llm_cache_size + j];
          new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request = request.llm_cache_size + j;
          new_bc.num_tokens++;
        }
        assert(new_bc.num_tokens <= limit);
        if (R.num_tokens_in_batch + request.llm_cache_size >= request.initial_len) {
          request.status = Request::RUNNING;
          new_bc.request_running[i] = true;
          R.prompt_phase = true;
          dfs_tree_inputs[guid] = std::vector<TokenDepth>{
              TokenDepth(request.tokens.back(), (int)request.tokens.size() - 1)};
          dfs_tree_parents[guid] = std::vector<int>{-1};
        }
      } else if (limit - new_bc.num_tokens > 0) {
        // whole prompt cached: launch the request with its last token
        request.status = Request::RUNNING;
        new_bc.request_running[i] = true;
        new_bc.tokensInfo[new_bc.num_tokens].request_index = i;
        new_bc.tokensInfo[new_bc.num_tokens].token_id = request.tokens.back();
        new_bc.tokensInfo[new_bc.num_tokens].abs_depth_in_request =
            (int)request.tokens.size() - 1;
        new_bc.num_tokens++;
        R.num_tokens_in_batch++;
        R.prompt_phase = true;
        dfs_tree_inputs[guid] = std::vector<TokenDepth>{
            TokenDepth(request.tokens.back(), (int)request.tokens.size() - 1)};
        dfs_tree_parents[guid] = std::vector<int>{-1};
      }
    } else {
      assert(false && "request status is not RUNNING or PENDING");
    }
  }
  return new_bc;
}

// request_manager.cc:2217-2325
void RequestManager::store_beam_metadata(const BeamSearchBatchConfig &old_bc,
                                         const BeamInferenceResult &result) {
  if (old_bc.num_tokens <= 0) return;
  RequestGuid guid = old_bc.requestsInfo[old_bc.tokensInfo[0].request_index].request_guid;
  int start_depth = old_bc.tokensInfo[0].abs_depth_in_request;
  int result_index = 0;
  for (int i = 0; i <= old_bc.num_tokens; i++) {
    if (i == old_bc.num_tokens ||
        old_bc.requestsInfo[old_bc.tokensInfo[i].request_index].request_guid != guid) {
      const int index = old_bc.tokensInfo[i - 1].request_index;
      const int beam_size = old_bc.beamRequestsInfo[index].beam_size;
      const int leaf_node_num = old_bc.beamRequestsInfo[index].sub_request_num * beam_size;
      const int depth = old_bc.beamRequestsInfo[index].current_depth;
      result_index += (old_bc.tokensInfo[i - 1].abs_depth_in_request - start_depth) * beam_size;
      Request &request = all_requests[old_bc.requestsInfo[index].request_guid];
      if (old_bc.requestsInfo[index].num_tokens_in_batch == 0) continue;
      auto &tree = request.beam_trees.at(old_bc.model_id);
      if (depth == 1) {
        tree.treeLayers[0].tokens[0] = request.tokens.back();
        tree.treeLayers[0].probs[0] = 1;
        tree.treeLayers[0].parent_ids[0] = -1;
        tree.treeLayers[0].nodes_num_this_layer = 1;
      }
      tree.treeLayers[depth].nodes_num_this_layer = leaf_node_num;
      for (int beam_id = 0; beam_id < leaf_node_num; beam_id++) {
        tree.treeLayers[depth].tokens[beam_id] = result.token_ids[result_index];
        tree.treeLayers[depth].probs[beam_id] = result.probs[result_index];
        tree.treeLayers[depth].parent_ids[beam_id] = result.parent_id[result_index];
        result_index += 1;
      }
      if (i < old_bc.num_tokens) {
        guid = old_bc.requestsInfo[old_bc.tokensInfo[i].request_index].request_guid;
        start_depth = old_bc.tokensInfo[i].abs_depth_in_request;
      }
    }
  }
}

// request_manager.cc:2327-2380
void RequestManager::update_beam_metadata(BeamSearchBatchConfig &new_bc,
                                          const BeamSearchBatchConfig &old_bc,
                                          Request::BeamTree &tree, int request_index) {
  (void)old_bc;
  const int depth = new_bc.beamRequestsInfo[request_index].current_depth - 1;
  const int leaf_node_num = new_bc.beamRequestsInfo[request_index].sub_request_num;
  if (new_bc.beamRequestsInfo[request_index].current_depth == 1) return;
  for (int j = 0; j < leaf_node_num; j++) {
    new_bc.beamRequestsInfo[request_index].parent_id[j] = tree.treeLayers[depth].parent_ids[j];
    new_bc.beamRequestsInfo[request_index].probs[j] = tree.treeLayers[depth].probs[j];
    new_bc.beamRequestsInfo[request_index].tokens[j] = tree.treeLayers[depth].tokens[j];
  }
}

// request_manager.cc:2382-2390
void RequestManager::initBitMask(BatchConfig::BitMask &bitmask, int initLength) {
  assert(initLength > 0);
  bitmask.non_tree_cache_size = 0;
  bitmask.tree_size = 1;
  bitmask.prompt_size = initLength;
  bitmask.this_layer_size = initLength;
}

// request_manager.cc:2393-2412
void RequestManager::updateBitMask(BatchConfig::BitMask &bitmask, int initLength,
                                   int non_tree_size) {
  assert(initLength <= BatchConfig::MAX_SPEC_TREE_TOKEN_NUM);
  assert(initLength >= 1);
  bitmask.non_tree_cache_size = non_tree_size + initLength - 1;
  bitmask.tree_size = 1;
  bitmask.this_layer_size = initLength;
  bitmask.prompt_size = 1;
  for (int i = 0; i < bitmask.prompt_size; i++)
    for (int j = i; j < bitmask.prompt_size; j++) bitmask.mask[i] |= (1ull << j);
}

// request_manager.cc:2415-2423
void RequestManager::appendPendingRequest(BatchConfig::BitMask &bitmask, int initLength) {
  assert(initLength > 0);
  bitmask.non_tree_cache_size = 0;
  bitmask.tree_size = 1;
  bitmask.prompt_size += initLength;
  bitmask.this_layer_size = initLength;
}

// request_manager.cc:2426-2476
void RequestManager::appendBitMask(BatchConfig::BitMask &bitmask, int newNodes,
                                   int preBeamSize, int old_sub_num,
                                   const Request::BeamTree &tree, int currentDepth) {
  (void)preBeamSize;
  (void)old_sub_num;
  const int pre_tree_size = bitmask.tree_size;
  bitmask.tree_size += newNodes;
  bitmask.this_layer_size = newNodes;
  assert(bitmask.tree_size <= BatchConfig::MAX_SPEC_TREE_TOKEN_NUM);
  for (int i = 0; i < bitmask.prompt_size; i++)
    for (int j = pre_tree_size; j < bitmask.tree_size; j++) bitmask.mask[i] |= (1ull << j);
  int token_idx = bitmask.prompt_size;
  int new_nodes_start_idx = pre_tree_size;
  for (int i = 1; i < currentDepth; i++) {
    new_nodes_start_idx = pre_tree_size;
    const int nodes_this_layer = tree.treeLayers[i].nodes_num_this_layer;
    for (int j = 0; j < nodes_this_layer; j++) {
      const int group_size = newNodes / nodes_this_layer;
      for (int k = 0; k < group_size; k++) {
        bitmask.mask[token_idx] |= (1ull << new_nodes_start_idx);
        new_nodes_start_idx += 1;
      }
      token_idx += 1;
    }
  }
  assert(token_idx == pre_tree_size);
  assert(currentDepth <= 1 || new_nodes_start_idx == bitmask.tree_size);
  for (int i = token_idx; i < bitmask.tree_size; i++) bitmask.mask[i] |= (1ull << i);
}

// request_manager.cc:2583-2741: greedy path acceptance; returns the
// verified (token, depth) list and rewrites the request's commit list to the
// accepted nodes.  output[i] is the LLM's pick at tree node i.  Node c is
// accepted when its parent is the last accepted node and its token is the
// LLM's pick there.  The reference walks the layer-order list instead and,
// once a node of a branching layer matched, accepts only the same slot of
// every later layer (:2665-2700); on the trees it admits (widths whose
// product is <= 3: one branching layer, chains below it) that slot IS the
// accepted node's only child, so both walks accept the same nodes.  Trees that
// branch twice (widths (2, 2) under FFMI_SPEC_EXT_WIDTH4) and merged trees
// need the parent links.
std::vector<RequestManager::TokenDepth> RequestManager::traverse_verify_tree(
    size_t guid, const std::vector<TokenDepth> &input, const std::vector<TokenDepth> &output) {
  std::vector<TokenDepth> verifiedTree;
  std::vector<std::pair<int, int>> new_committed_tokens;
  assert(input.size() >= output.size());
  const RequestGuid g = (RequestGuid)guid;
  auto pit = dfs_tree_parents.find(g);
  const std::vector<int> parent = pit != dfs_tree_parents.end() && pit->second.size() == input.size()
                                      ? pit->second
                                      : layer_order_parents(input);
  const auto &ct = committed_tokens.at(g);
  if (!output.empty()) {
    assert(ct.at(0).first == input.at(0).second);
    verifiedTree.push_back(output[0]);
    new_committed_tokens.push_back(std::make_pair(input[0].second, ct.at(0).second));
    int last = 0;
    for (size_t c = 1; c < output.size(); ++c) {
      if (parent[c] != last) continue;
      if (input[c].first != verifiedTree.back().first ||
          input[c].second != verifiedTree.back().second)
        continue;
      assert(ct.at(c).first == input[c].second);
      verifiedTree.push_back(output[c]);
      new_committed_tokens.push_back(std::make_pair(input[c].second, ct.at(c).second));
      last = (int)c;
    }
  }
  committed_tokens[g] = new_committed_tokens;
  return verifiedTree;
}

// request_manager.cc:2743-2815: layer-order serialization of the beam tree
std::vector<RequestManager::TokenDepth> RequestManager::traverse_beam_tree(
    const BeamSearchBatchConfig &old_bc, int request_index, int first_token_depth) {
  const RequestGuid guid = old_bc.requestsInfo[request_index].request_guid;
  Request &request = all_requests[guid];
  const auto &tree = request.beam_trees.at(old_bc.model_id);
  std::vector<TokenDepth> serializedTree;
  for (int i = 0; i <= old_bc.beamRequestsInfo[request_index].max_depth; i++)
    for (int j = 0; j < tree.treeLayers[i].nodes_num_this_layer; j++)
      serializedTree.push_back(std::make_pair(tree.treeLayers[i].tokens[j], i));
  for (auto &p : serializedTree) p.second += first_token_depth;
  return serializedTree;
}

std::vector<int> RequestManager::layer_order_parents(const std::vector<TokenDepth> &tree) {
  std::vector<int> parent(tree.size(), -1);
  size_t prev_start = 0, prev_n = 0;
  for (size_t i = 0; i < tree.size();) {
    size_t j = i;
    while (j < tree.size() && tree[j].second == tree[i].second) ++j;
    const size_t n = j - i;
    if (i > 0)  // n_d = n_{d-1} * width: equal groups (store_beam_metadata, :2304-2316)
      for (size_t k = 0; k < n; ++k) parent[i + k] = (int)(prev_start + k * prev_n / n);
    prev_start = i;
    prev_n = n;
    i = j;
  }
  return parent;
}

void RequestManager::tree_bitmask(const std::vector<int> &parent, int n,
                                  BatchConfig::BitMask &m) {
  assert(n <= BatchConfig::MAX_SPEC_TREE_TOKEN_NUM && n <= (int)parent.size());
  std::fill(m.mask, m.mask + BatchConfig::MAX_SPEC_TREE_TOKEN_NUM, 0ull);
  for (int q = 0; q < n; ++q)
    for (int a = q; a >= 0; a = parent[a]) m.mask[a] |= 1ull << q;
  m.tree_size = n;
}

// request_manager.cc:2817-2878.  One SSM: its tree is used as is (the
// reference's path).  N SSMs (FFMI_SPEC_EXT_MULTI_SSM): the reference's merge
// after its assert gives every node the id token * 10000 + depth, records
// each node under curr_path[depth - 1] as its parent's child and emits the
// union depth-first from the root.  Restated here with two corrections: a
// node's identity is its PATH from the root (the <token, depth> id joins two
// different nodes that carry the same token at the same depth, giving the
// union node two parents, whose KV contexts differ), and the parent of a node
// comes from the layer-order grouping its SSM built (curr_path presumes the
// depth-first serialisation traverse_beam_tree no longer produces).  The union
// is emitted in layer order (depth, then first-seen: SSM 0's nodes, then new
// nodes of SSM 1, ...), the order the verify step, its bitmask and the commit
// lists use, and is cut to the root + max_spec_tree_token_num nodes (<= 64,
// the bitmask's width): a layer-order prefix, so every kept node keeps its
// ancestors.
std::vector<RequestManager::TokenDepth> RequestManager::merge_dfs_trees(
    const std::vector<std::vector<TokenDepth>> &trees, int root_depth, RequestGuid guid) {
  (void)root_depth;
  assert(!trees.empty());
  // root + max_spec_tree_token_num nodes: the root's KV slot lies in the
  // committed range, so the models' tail of max_spec_tree_token_num slots
  // per request holds that many nodes below it (the reference places a
  // widths (1,1,3) tree of 21 nodes whole under its default budget of 20)
  const int cap = std::max(1, std::min(max_spec_tree_token_num + 1,
                                       (int)BatchConfig::MAX_SPEC_TREE_TOKEN_NUM));
  if (trees.size() == 1) {
    // (cut to the cap like a merged tree: a tree larger than the models' KV
    // tail -- max_seq_len + max_spec_tree_token_num slots per request -- has
    // nowhere to store its last nodes; e.g. widths (4,) grow 1 + 4 x 8 = 33
    // nodes.  The reference places such a tree whole.  A layer-order prefix
    // keeps every node's ancestors.)
    std::vector<TokenDepth> t = trees[0];
    std::vector<int> par = layer_order_parents(t);
    if ((int)t.size() > cap) t.resize(cap), par.resize(cap);
    dfs_tree_inputs[guid] = t;
    dfs_tree_parents[guid] = par;
    return t;
  }
  struct Node {
    TokenDepth td;
    int parent;
  };
  std::vector<Node> nodes;
  std::map<std::pair<int, int>, int> child;  // (parent id, token) -> node id
  const TokenDepth root = trees[0].at(0);
  nodes.push_back(Node{root, -1});
  for (const auto &tree : trees) {
    assert(!tree.empty() && tree[0] == root);  // all trees share the root
    const std::vector<int> par = layer_order_parents(tree);
    std::vector<int> id(tree.size(), 0);
    for (size_t i = 1; i < tree.size(); ++i) {
      const int p = id[par[i]];
      auto ins = child.emplace(std::make_pair(p, tree[i].first), (int)nodes.size());
      if (ins.second) nodes.push_back(Node{tree[i], p});
      id[i] = ins.first->second;
    }
  }
  std::vector<int> order(nodes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return nodes[a].td.second < nodes[b].td.second;
  });
  if ((int)order.size() > cap) order.resize(cap);
  std::vector<int> pos(nodes.size(), -1);
  for (size_t i = 0; i < order.size(); ++i) pos[order[i]] = (int)i;
  std::vector<TokenDepth> merged;
  std::vector<int> mparent;
  for (int id : order) {
    merged.push_back(nodes[id].td);
    mparent.push_back(nodes[id].parent < 0 ? -1 : pos[nodes[id].parent]);
  }
  dfs_tree_inputs[guid] = merged;
  dfs_tree_parents[guid] = mparent;
  return merged;
}

bool RequestManager::all_done() const {
  if (!pending_infr_request_queue.empty()) return false;
  for (const auto &kv : all_requests)
    if (kv.second.status != Request::COMPLETED) return false;
  return true;
}

const GenerationResult *RequestManager::get_generation_result(RequestGuid guid) const {
  auto it = request_generation_results.find(guid);
  return it == request_generation_results.end() ? nullptr : &it->second;
}

const RequestManager::ProfileInfo *RequestManager::get_profile(RequestGuid guid) const {
  auto it = profiling_requests.find(guid);
  return it == profiling_requests.end() ? nullptr : &it->second;
}

// request_manager.cc:3012-3080 (synchronous: one batch in flight)
ffmi_status RequestManager::serve_incr_decoding(ffmi_model *llm) {
  if (!llm) return FFMI_ERR_INVALID;
  apply_limits();
  stats = Stats();
  const double t0 = now_us();
  BatchConfig *bc = new BatchConfig();
  InferenceResult *ir = new InferenceResult();
  ffmi_status st = FFMI_OK;
  while (!all_done()) {
    BatchConfig *next = new BatchConfig(prepare_next_batch(*bc, *ir));
    delete bc;
    bc = next;
    if (bc->num_tokens == 0) {
      if (all_done()) break;
      st = FFMI_ERR_INVALID;  // nothing schedulable but requests remain
      break;
    }
    const double tl = now_us();
    st = llm->run_inc(*bc, ir);
    stats.llm_us += now_us() - tl;
    if (st != FFMI_OK) break;
    stats.llm_steps++;
  }
  delete bc;
  delete ir;
  stats.wall_us = now_us() - t0;
  return st;
}

// Does a beam batch staged from placeholder results (`spec`: the previous
// step's top-k id i appears as token id -1 - i) describe the batch built from
// the real results (`real`)?  Everything but those token ids must agree, and
// each placeholder must name the real id.
static bool same_beam_batch(const BeamSearchBatchConfig &spec, const BeamSearchBatchConfig &real,
                            const BeamInferenceResult &prev, int max_requests) {
  if (spec.num_tokens != real.num_tokens || spec.model_id != real.model_id) return false;
  for (int t = 0; t < real.num_tokens; ++t) {
    const auto &a = spec.tokensInfo[t], &b = real.tokensInfo[t];
    if (a.request_index != b.request_index || a.abs_depth_in_request != b.abs_depth_in_request ||
        spec.beamTokenInfo[t].sub_request_index != real.beamTokenInfo[t].sub_request_index)
      return false;
    const int id = a.token_id < 0 ? prev.token_ids[-1 - a.token_id] : a.token_id;
    if (id != b.token_id) return false;
  }
  for (int r = 0; r < max_requests && r < BatchConfig::MAX_NUM_REQUESTS; ++r) {
    if (spec.request_completed[r] != real.request_completed[r] ||
        spec.request_running[r] != real.request_running[r])
      return false;
    if (real.request_completed[r]) continue;
    const auto &a = spec.requestsInfo[r], &b = real.requestsInfo[r];
    if (a.first_token_depth_in_request != b.first_token_depth_in_request ||
        a.first_token_offset_in_batch != b.first_token_offset_in_batch ||
        a.num_tokens_in_batch != b.num_tokens_in_batch || a.prompt_phase != b.prompt_phase)
      return false;
    const auto &ma = spec.causalMask[r], &mb = real.causalMask[r];
    if (ma.non_tree_cache_size != mb.non_tree_cache_size || ma.tree_size != mb.tree_size ||
        ma.this_layer_size != mb.this_layer_size || ma.prompt_size != mb.prompt_size ||
        memcmp(ma.mask, mb.mask, sizeof ma.mask) != 0)
      return false;
    const auto &ba = spec.beamRequestsInfo[r], &bb = real.beamRequestsInfo[r];
    if (ba.beam_size != bb.beam_size || ba.current_depth != bb.current_depth ||
        ba.max_depth != bb.max_depth || ba.sub_request_num != bb.sub_request_num)
      return false;
  }
  return true;
}

// The speculation phase with chained beam steps.  What a beam step's batch
// holds -- sizes, positions, KV slots, bitmasks -- follows from the tree
// widths, depths and prompt lengths; only its generation tokens' ids come from
// the previous step's results (B.tokens, store_beam_metadata /
// update_beam_metadata).  So the 8 steps of each SSM are prepared up front
// from placeholder results whose entry i reads -1 - i, and launched back to
// back: the device puts the previous step's top-k id i in place of -1 - i
// (the embedding gather), with no host round trip between steps.  The
// scheduler state those placeholder preparations touched is then restored and
// the same prepare_next_batch_beam calls are replayed, in the order the
// stepwise loop makes them, on the real results -- so beam trees, counters and
// the final batches are exactly the stepwise ones -- and every staged batch is
// checked against the replayed one (same_beam_batch; a mismatch is an error,
// never a silent divergence).
ffmi_status RequestManager::run_ssm_phase_chained(std::vector<BeamSearchBatchConfig> *beam_vec,
                                                  BeamInferenceResult *beam_ir) {
  const std::vector<int> &loc = ssm_local;  // (the SSMs this rank runs)
  const size_t n = loc.size();
  const int D = BeamSearchBatchConfig::MAX_BEAM_DEPTH;
  const double ts = now_us();
  double prep_us = 0, t_last = ts;
  ffmi_status st = FFMI_OK;
  // step 0 of every SSM (its tokens are known)
  size_t launched0 = 0;
  for (size_t i = 0; i < n && st == FFMI_OK; ++i) {
    st = ssm_models[loc[i]]->beam_launch_chained((*beam_vec)[loc[i]], 0);
    if (st == FFMI_OK) ++launched0;
  }
  // the state prepare_next_batch_beam writes, saved for the replay
  struct Saved {
    std::vector<Request::BeamTree> trees;
    int ssm_cache_size;
  };
  std::map<RequestGuid, Saved> saved;
  for (const auto &kv : all_requests)
    saved[kv.first] = Saved{kv.second.beam_trees, kv.second.ssm_cache_size};
  std::map<RequestGuid, int> saved_steps;
  for (const auto &kv : profiling_requests) saved_steps[kv.first] = kv.second.ssm_decoding_steps;
  // steps 1 .. D-1 prepared from placeholders while step 0 runs: spec[s * D + d]
  std::vector<BeamSearchBatchConfig> &spec = chain_spec;
  spec.resize(n * D);
  if (!chain_ph) {
    chain_ph.reset(new BeamInferenceResult());
    for (int i = 0;
         i < BatchConfig::MAX_NUM_TOKENS * BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES; ++i) {
      chain_ph->token_ids[i] = -1 - i;
      chain_ph->probs[i] = 1.0f;
      chain_ph->parent_id[i] = 0;
    }
  }
  // a placeholder must name an entry the previous step produces (its
  // tokens' top-w entries, beam_result_layout); otherwise the phase runs
  // step by step
  std::vector<int> layout;
  auto results_of = [&](const BeamSearchBatchConfig &bc) -> long {
    beam_result_layout(bc, &layout);
    return (long)layout.size();
  };
  bool chainable = st == FFMI_OK;
  const double tp0 = now_us();
  chain_t[0] += tp0 - ts;
  for (size_t i = 0; i < n && chainable; ++i) {
    spec[i * D] = (*beam_vec)[loc[i]];
    for (int d = 1; d < D && chainable; ++d) {
      spec[i * D + d] = prepare_next_batch_beam(spec[i * D + d - 1], *chain_ph);
      const long have = results_of(spec[i * D + d - 1]);
      const BeamSearchBatchConfig &b = spec[i * D + d];
      for (int t = 0; t < b.num_tokens; ++t)
        if (b.tokensInfo[t].token_id < 0 && -1L - b.tokensInfo[t].token_id >= have)
          chainable = false;
    }
  }
  for (auto &kv : all_requests) {  // restore
    auto it = saved.find(kv.first);
    if (it == saved.end()) continue;
    kv.second.beam_trees = it->second.trees;
    kv.second.ssm_cache_size = it->second.ssm_cache_size;
  }
  for (auto &kv : profiling_requests) {
    auto it = saved_steps.find(kv.first);
    if (it != saved_steps.end()) kv.second.ssm_decoding_steps = it->second;
  }
  prep_us += now_us() - tp0;
  chain_t[1] += now_us() - tp0;
  // launch steps 1 .. D-1 back to back (chainable), or nothing more yet
  if (chainable) stats.ssm_phases_chained++;
  size_t launched = launched0;
  const double tl0 = now_us();
  for (int d = 1; d < D && chainable && st == FFMI_OK; ++d)
    for (size_t i = 0; i < n && st == FFMI_OK; ++i) {
      st = ssm_models[loc[i]]->beam_launch_chained(spec[i * D + d], d);
      if (st == FFMI_OK) ++launched;
    }
  chain_t[2] += now_us() - tl0;
  chain_t[4] += 1;
  // collect in the stepwise loop's order, replaying the bookkeeping on the
  // real results; unchained: collect, prepare, launch the next step (slot 0)
  for (int d = 0; d < D; ++d)
    for (size_t i = 0; i < n; ++i) {
      const int s = loc[i];
      const bool was_launched = chainable ? (size_t)d * n + i < launched
                                          : (d == 0 ? i < launched0 : st == FFMI_OK);
      if (!was_launched) continue;
      const ffmi_status cs = ssm_models[s]->beam_collect_chained(chainable ? d : 0, beam_ir);
      t_last = now_us();
      if (st == FFMI_OK) st = cs;
      if (st != FFMI_OK) continue;  // (collect the rest: nothing left in flight)
      stats.ssm_steps++;
      const double tp = now_us();
      record_step(s, d, (*beam_vec)[s], *beam_ir);
      (*beam_vec)[s] = prepare_next_batch_beam((*beam_vec)[s], *beam_ir);
      if (chainable && d + 1 < D &&
          !same_beam_batch(spec[i * D + d + 1], (*beam_vec)[s], *beam_ir, max_requests_per_batch)) {
        ffmi_set_last_error("chained SSM beam steps: a staged batch differs from the one its "
                            "results give (FFMI_SSM_CHAIN=0 runs the steps one by one)",
                            __FILE__, __LINE__);
        st = FFMI_ERR_INVALID;
      }
      prep_us += now_us() - tp;
      if (!chainable && st == FFMI_OK && d + 1 < D)
        st = ssm_models[s]->beam_launch_chained((*beam_vec)[s], 0);
    }
  // first launch to last result: the staging and the replay of every step
  // but the last overlap the device's work; what follows the last result is
  // host scheduling, as in the stepwise loop
  (void)prep_us;
  stats.ssm_us += t_last - ts;
  chain_t[3] += t_last - ts;
  return st;
}

// Distributed SSMs (set_ssm_exchange).  A local SSM's results of each step,
// in the scheduler's layout (beam_result_layout: what store_beam_metadata
// reads), are kept for the exchange.
void RequestManager::record_step(int s, int depth, const BeamSearchBatchConfig &bc,
                                 const BeamInferenceResult &ir) {
  if (xch_world <= 1) return;
  std::vector<int> layout;
  beam_result_layout(bc, &layout);
  StepRecord &r = phase_rec.at(s).at(depth);
  r.ids.assign(ir.token_ids, ir.token_ids + layout.size());
  r.probs.assign(ir.probs, ir.probs + layout.size());
}

// After the local SSMs' speculation phase: every rank's records, then each
// remote SSM's MAX_BEAM_DEPTH prepare_next_batch_beam calls replayed on its
// results from the same init batch.  prepare_next_batch_beam of SSM s writes
// only SSM s's beam trees, plus counters that commute (ssm_decoding_steps) or
// belong to SSM 0 alone (ssm_cache_size), so the order of SSMs does not
// matter: every rank ends with the trees, counters and batches of a run with
// every SSM local.  Records are int32 words: [k SSMs] then per SSM [s, then
// per depth n_d, n_d ids, n_d probs (float bits)]; one all-gather of the
// sizes, one of the records padded to the largest.
ffmi_status RequestManager::exchange_and_replay(std::vector<BeamSearchBatchConfig> *beam_vec,
                                                BeamInferenceResult *beam_ir) {
  const int D = BeamSearchBatchConfig::MAX_BEAM_DEPTH;
  const int W = xch_world;
  std::vector<int32_t> mine;
  mine.push_back((int32_t)ssm_local.size());
  for (int s : ssm_local) {
    mine.push_back(s);
    for (int d = 0; d < D; ++d) {
      const StepRecord &r = phase_rec[s][d];
      mine.push_back((int32_t)r.ids.size());
      mine.insert(mine.end(), r.ids.begin(), r.ids.end());
      for (float p : r.probs) {
        int32_t b;
        memcpy(&b, &p, 4);
        mine.push_back(b);
      }
    }
  }
  int64_t len = (int64_t)mine.size();
  std::vector<int64_t> lens(W, 0);
  if (xch_fn(xch_ctx, &len, sizeof len, lens.data()) != 0) {
    ffmi_set_last_error("SSM exchange (sizes) failed", __FILE__, __LINE__);
    return FFMI_ERR_NCCL;
  }
  int64_t mx = 0;
  for (int64_t l : lens) mx = std::max(mx, l);
  if (mx <= 0 || mx > (int64_t)1 << 26) return FFMI_ERR_INVALID;
  mine.resize((size_t)mx, 0);
  std::vector<int32_t> all((size_t)mx * W);
  if (xch_fn(xch_ctx, mine.data(), (size_t)mx * 4, all.data()) != 0) {
    ffmi_set_last_error("SSM exchange (records) failed", __FILE__, __LINE__);
    return FFMI_ERR_NCCL;
  }
  std::vector<bool> have(ssm_models.size(), false);
  for (int s : ssm_local) have[s] = true;
  std::vector<int> layout;
  for (int r = 0; r < W; ++r) {
    if (r == xch_rank) continue;
    const int32_t *p = all.data() + (size_t)r * mx;
    const int32_t *end = p + lens[r];
    auto take = [&]() -> int32_t { return p < end ? *p++ : INT32_MIN; };
    const int k = take();
    for (int j = 0; j < k; ++j) {
      const int s = take();
      FFMI_CHECK(s >= 0 && s < (int)ssm_models.size() && !ssm_models[s] && !have[s],
                 FFMI_ERR_INVALID);
      have[s] = true;
      for (int d = 0; d < D; ++d) {
        const int nd = take();
        beam_result_layout((*beam_vec)[s], &layout);
        FFMI_CHECK(nd == (int)layout.size() && end - p >= 2L * nd, FFMI_ERR_INVALID);
        for (int i = 0; i < nd; ++i) {
          beam_ir->token_ids[i] = p[i];
          memcpy(&beam_ir->probs[i], &p[nd + i], 4);
          beam_ir->parent_id[i] = 0;
        }
        p += 2 * nd;
        (*beam_vec)[s] = prepare_next_batch_beam((*beam_vec)[s], *beam_ir);
      }
    }
  }
  for (size_t s = 0; s < ssm_models.size(); ++s)
    if (!have[s]) {
      ffmi_set_last_error("SSM exchange: no rank ran one of the registered SSMs", __FILE__,
                          __LINE__);
      return FFMI_ERR_INVALID;
    }
  return FFMI_OK;
}

// request_manager.cc:3083-3173
ffmi_status RequestManager::serve_spec_infer(ffmi_model *llm) {
  if (!llm) return FFMI_ERR_INVALID;
  if (ssm_models.empty()) return FFMI_ERR_INVALID;
  // the reference asserts one SSM (merge_dfs_trees :2823-2827)
  if (ssm_models.size() > 1 && !(spec_extensions & FFMI_SPEC_EXT_MULTI_SSM)) {
    ffmi_set_last_error("SpecInfer with more than one SSM needs FFMI_SPEC_EXT_MULTI_SSM",
                        __FILE__, __LINE__);
    return FFMI_ERR_UNSUPPORTED;
  }
  // every SSM step must fit its model: an init batch holds every running
  // request's verified tokens (up to MAX_BEAM_DEPTH + 1 each) or prompt
  // chunks up to max_tokens_per_batch, a beam step every request's beams
  // (up to MAX_SPECULATIVE_TREE_BRANCHES each) or prompt chunks up to the
  // same budget.  Checked here rather than failing partway through a serve
  // placement: SSM s runs on rank s % nranks (set_ssm_exchange); without an
  // exchange every SSM is local
  ssm_local.clear();
  for (size_t s = 0; s < ssm_models.size(); ++s) {
    const bool mine = xch_world <= 1 || (int)(s % xch_world) == xch_rank;
    if (mine != (ssm_models[s] != nullptr) || (xch_world > 1 && !xch_fn)) {
      ffmi_set_last_error("SpecInfer: SSM s must be a model on rank s % nranks and a remote "
                          "placeholder on the other ranks (set_ssm_exchange)", __FILE__, __LINE__);
      return FFMI_ERR_INVALID;
    }
    if (mine) ssm_local.push_back((int)s);
  }
  if (xch_world > 1)
    phase_rec.assign(ssm_models.size(),
                     std::vector<StepRecord>(BeamSearchBatchConfig::MAX_BEAM_DEPTH));
  {
    const int need = std::max(max_tokens_per_batch,
                              max_requests_per_batch *
                                  std::max(BeamSearchBatchConfig::MAX_BEAM_DEPTH + 1,
                                           (int)BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES));
    for (int s : ssm_local) {
      const int cap = ssm_models[s]->token_capacity();
      if (cap >= 0 && cap < need) {
        char msg[256];
        snprintf(msg, sizeof msg,
                 "SpecInfer: SSM %zu holds %d tokens per step, the scheduler can build %d "
                 "(max(max_tokens_per_batch, max_requests x %d)): create it with max_tokens >= %d",
                 (size_t)s, cap, need,
                 std::max(BeamSearchBatchConfig::MAX_BEAM_DEPTH + 1,
                          (int)BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES),
                 need);
        ffmi_set_last_error(msg, __FILE__, __LINE__);
        return FFMI_ERR_INVALID;
      }
    }
  }
  // requests registered before the last SSM was: one beam tree per SSM
  for (auto &kv : all_requests)
    if (kv.second.beam_trees.size() < ssm_models.size())
      kv.second.beam_trees.resize(ssm_models.size());
  for (auto &r : pending_infr_request_queue)
    if (r.beam_trees.size() < ssm_models.size()) r.beam_trees.resize(ssm_models.size());
  // SSMs whose steps run collectives (TP-sharded) are stepped one at a time:
  // their steps' all-reduces must reach every rank in the same order
  bool overlap_ssms = true;
  for (int s : ssm_local)
    if (ssm_models[s]->uses_collectives()) overlap_ssms = false;
  // chained beam steps where every SSM supports them (FFMI_SSM_CHAIN=0: off)
  bool chain = overlap_ssms && !(getenv("FFMI_SSM_CHAIN") && atoi(getenv("FFMI_SSM_CHAIN")) == 0);
  for (int s : ssm_local)
    if (!ssm_models[s]->can_chain_beam()) chain = false;
  apply_limits();
  stats = Stats();
  const double t0 = now_us();
  TreeVerifyBatchConfig *tree_bc = new TreeVerifyBatchConfig();
  InferenceResult *tree_ir = new InferenceResult();
  BeamInferenceResult *beam_ir = new BeamInferenceResult();
  std::vector<BeamSearchBatchConfig> *beam_vec = new std::vector<BeamSearchBatchConfig>();
  ffmi_status st = FFMI_OK;
  while (!all_done()) {
    ssm_prompt_behind = false;
    beam_vec->assign(ssm_models.size(), prepare_next_batch_init(*tree_bc, *tree_ir, 0));
    // each SSM builds its own beam tree (the reference hands every SSM the
    // init batch of model 0, :3147-3150, so all would write beam_trees[0])
    for (size_t s = 0; s < beam_vec->size(); ++s) (*beam_vec)[s].model_id = (int)s;
    if (ssm_prompt_behind) {
      ffmi_set_last_error(
          "SpecInfer: the SSM loaded less of a prompt than the LLM (prompt longer than one "
          "init + MAX_BEAM_DEPTH beam batches can hold; raise max_tokens_per_batch)",
          __FILE__, __LINE__);
      st = FFMI_ERR_UNSUPPORTED;
      break;
    }
    if (all_done()) break;
    // MAX_BEAM_DEPTH beam steps per SSM (:3147-3159).  The reference runs
    // SSM 0's steps, then SSM 1's ...; the SSMs are independent, so here
    // their latency-bound steps overlap on their streams: every SSM's step 0
    // is launched, then each SSM's step d + 1 goes out as soon as its step d
    // is collected and its next batch prepared, while the other SSMs' steps
    // d are still running (identical batches and results: each SSM's chain
    // of steps is unchanged)
    if (chain) {
      st = run_ssm_phase_chained(beam_vec, beam_ir);
    } else {
      const std::vector<int> &loc = ssm_local;
      const size_t n = ssm_models.size();
      const double ts = now_us();
      double prep_us = 0;
      std::vector<bool> inflight(n, false);
      if (!overlap_ssms) {
        // one step in flight at a time, SSM by SSM (the reference's order)
        for (size_t i = 0; i < loc.size() && st == FFMI_OK; i++)
          for (int depth = 0; depth < BeamSearchBatchConfig::MAX_BEAM_DEPTH && st == FFMI_OK;
               depth++) {
            const int s = loc[i];
            st = ssm_models[s]->beam_launch((*beam_vec)[s]);
            if (st == FFMI_OK) st = ssm_models[s]->beam_collect(beam_ir);
            if (st != FFMI_OK) break;
            stats.ssm_steps++;
            const double tp = now_us();
            record_step(s, depth, (*beam_vec)[s], *beam_ir);
            (*beam_vec)[s] = prepare_next_batch_beam((*beam_vec)[s], *beam_ir);
            prep_us += now_us() - tp;
          }
      }
      for (size_t i = 0; i < loc.size() && st == FFMI_OK && overlap_ssms; i++) {
        st = ssm_models[loc[i]]->beam_launch((*beam_vec)[loc[i]]);
        inflight[loc[i]] = st == FFMI_OK;
      }
      for (int depth = 0; depth < BeamSearchBatchConfig::MAX_BEAM_DEPTH && overlap_ssms; depth++) {
        for (int s : loc) {
          if (!inflight[s]) continue;
          inflight[s] = false;
          const ffmi_status cs = ssm_models[s]->beam_collect(beam_ir);
          if (st == FFMI_OK) st = cs;
          if (st != FFMI_OK) continue;  // collect the rest: no step left in flight
          stats.ssm_steps++;
          const double tp = now_us();  // (host scheduling: not SSM step time)
          record_step(s, depth, (*beam_vec)[s], *beam_ir);
          (*beam_vec)[s] = prepare_next_batch_beam((*beam_vec)[s], *beam_ir);
          prep_us += now_us() - tp;
          if (depth + 1 < BeamSearchBatchConfig::MAX_BEAM_DEPTH) {
            st = ssm_models[s]->beam_launch((*beam_vec)[s]);
            inflight[s] = st == FFMI_OK;
          }
        }
      }
      stats.ssm_us += now_us() - ts - prep_us;
    }
    if (st != FFMI_OK) break;
    if (xch_world > 1) {  // the other ranks' SSMs (config E placement)
      const double tx = now_us();
      st = exchange_and_replay(beam_vec, beam_ir);
      stats.ssm_exchange_us += now_us() - tx;
      if (st != FFMI_OK) break;
    }
    *tree_bc = prepare_next_batch_verify(*beam_vec);
    if (tree_bc->num_tokens == 0 && !all_done()) {
      st = FFMI_ERR_INVALID;
      break;
    }
    const double tl = now_us();
    st = llm->run_tree(*tree_bc, tree_ir);
    stats.llm_us += now_us() - tl;
    if (st != FFMI_OK) break;
    stats.llm_steps++;
  }
  delete tree_bc;
  delete tree_ir;
  delete beam_ir;
  delete beam_vec;
  stats.wall_us = now_us() - t0;
  if (getenv("FFMI_STEP_TIMING") && chain_t[4] > 0)
    fprintf(stderr, "[ffmi chain timing] %.0f phases: launch step 0 %.1f us, stage steps 1-7 %.1f us, "
            "launch steps 1-7 %.1f us, phase to last result %.1f us\n", chain_t[4],
            chain_t[0] / chain_t[4], chain_t[1] / chain_t[4], chain_t[2] / chain_t[4],
            chain_t[3] / chain_t[4]);
  return st;
}

}  // namespace ffmi
