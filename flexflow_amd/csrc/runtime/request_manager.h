// request_manager.h -- continuous batching + SpecInfer token-tree scheduler.
//
// API-compatible restatement of include/flexflow/request_manager.h:119-358
// (RequestManager) without Legion: the prepare_next_batch* functions take
// and return the BatchConfig structs directly, and the serve loops run in the
// caller's thread until every registered request has completed (the
// reference runs the same loop as a background Legion task and generate()
// blocks on per-request promises, request_manager.cc:2880-2989).
#pragma once
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "batch_config.h"
#include "model.h"

namespace ffmi {

struct Request {
  enum Status { PENDING = 101, RUNNING = 102, COMPLETED = 103, FINISHING = 104 };
  BatchConfig::RequestGuid guid = 0;
  int max_length = -1;
  int max_new_tokens = -1;
  bool add_special_tokens = true;
  int initial_len = 0;
  int ssm_cache_size = 0;
  int llm_cache_size = 0;
  Status status = PENDING;
  std::vector<BatchConfig::TokenId> tokens;
  struct BeamTree {
    struct Layer {
      BatchConfig::TokenId tokens[BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
      int parent_ids[BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
      float probs[BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
      int nodes_num_this_layer = 0;
    };
    Layer treeLayers[BeamSearchBatchConfig::MAX_BEAM_DEPTH + 1];
  };
  std::vector<BeamTree> beam_trees;
};

struct GenerationResult {
  BatchConfig::RequestGuid guid = 0;
  std::vector<BatchConfig::TokenId> input_tokens, output_tokens;
};

class RequestManager {
 public:
  using RequestGuid = BatchConfig::RequestGuid;
  using TokenId = BatchConfig::TokenId;
  using TokenDepth = std::pair<TokenId, int>;

  RequestManager();
  void set_max_requests_per_batch(int n) { max_requests_per_batch = n; }
  void set_max_tokens_per_batch(int n) { max_tokens_per_batch = n; }
  void set_max_spec_tree_token_num(int n) { max_spec_tree_token_num = n; }
  void set_max_sequence_length(int n) { max_sequence_length = n; }
  int get_max_requests_per_batch() const { return max_requests_per_batch; }
  int get_max_tokens_per_batch() const { return max_tokens_per_batch; }
  int get_max_spec_tree_token_num() const { return max_spec_tree_token_num; }
  int get_max_sequence_length() const { return max_sequence_length; }
  int get_max_verify_tokens_per_batch() const {
    return max_tokens_per_batch + max_spec_tree_token_num * max_requests_per_batch;
  }
  bool push_spec_infer_tree_width(int w);
  // Flagged extensions beyond what the reference runs (include/ffmi.h
  // FFMI_SPEC_EXT_*): tree width / branches up to 4 per layer, and more than
  // one SSM with their trees merged (merge_dfs_trees).  Set before widths are
  // pushed.
  void set_spec_extensions(int flags) { spec_extensions = flags; }
  int get_spec_extensions() const { return spec_extensions; }
  int max_beam_width() const;
  int max_tree_branches() const;
  void register_tokenizer(int bos, const std::vector<int> &eos) {
    bos_token_id = bos;
    eos_token_ids = eos;
  }
  // m == nullptr: an SSM that runs on another rank of the TP group
  // (set_ssm_exchange); every rank registers the same SSMs in the same order
  int register_ssm_model(ffmi_model *m) {
    ssm_models.push_back(m);
    return (int)ssm_models.size() - 1;
  }
  // Config E's SSMs placed over the ranks of a TP group: SSM s runs on rank
  // s % nranks only (the reference builds each SSM as its own TP = 1 model,
  // spec_infer.cc:381-435).  After its SSMs' beam steps each rank contributes
  // their per-step results through `fn` (an all-gather of equal-size byte
  // blocks: fn(ctx, mine, bytes, all[nranks][bytes]) == 0 on success) and
  // replays the other ranks' SSMs' bookkeeping on theirs, so every rank
  // merges the identical trees.
  typedef int (*AllGather)(void *ctx, const void *mine, size_t bytes, void *all);
  void set_ssm_exchange(int nranks, int rank, AllGather fn, void *ctx) {
    xch_world = nranks, xch_rank = rank, xch_fn = fn, xch_ctx = ctx;
  }
  size_t get_num_ssms() const { return ssm_models.size(); }
  // register_output_filepath (request_manager.cc:246-249): every completed
  // request is appended to the file in the reference's record format
  void register_output_filepath(const std::string &path) { output_filepath = path; }
  // the reference's tokenizer_->Decode(request.tokens) (request_manager.cc:
  // 786-789): a caller-supplied detokenizer (none: the text is empty)
  typedef int (*Detokenizer)(const int *ids, int n, char *buf, int cap, void *ctx);
  void register_detokenizer(Detokenizer fn, void *ctx) { detok = fn, detok_ctx = ctx; }
  std::string decode(const std::vector<int> &ids) const;
  // the text of a completed request: decode(tokens), with the "<s> " prefix
  // of the old LLaMA tokenizer for requests that asked for special tokens
  // (request_manager.cc:776-781)
  std::string decode_request(const Request &request) const;
  void set_old_llama_tokenizer(bool v) { old_llama_tokenizer = v; }
  void set_verbose(bool v) { verbose = v; }

  RequestGuid register_new_request(const std::vector<int> &prompt, int max_length,
                                   int max_new_tokens, bool add_special_tokens);

  // bitmask helpers (request_manager.cc:2382-2517)
  void initBitMask(BatchConfig::BitMask &bitmask, int initLength);
  void appendPendingRequest(BatchConfig::BitMask &bitmask, int initLength);
  void appendBitMask(BatchConfig::BitMask &bitmask, int newNodes, int preBeamSize,
                     int old_sub_num, const Request::BeamTree &tree, int currentDepth);
  void updateBitMask(BatchConfig::BitMask &bitmask, int initLength, int non_tree_size);

  bool is_eos_token(int token_id) const;
  bool check_inf_req_completion(const BatchConfig &old_bc, int i);

  BatchConfig prepare_next_batch(const BatchConfig &bc, const InferenceResult &result);
  BeamSearchBatchConfig prepare_next_batch_init(const TreeVerifyBatchConfig &old_bc,
                                                const InferenceResult &result, int model_id);
  BeamSearchBatchConfig prepare_next_batch_beam(const BeamSearchBatchConfig &old_bc,
                                                const BeamInferenceResult &result);
  TreeVerifyBatchConfig prepare_next_batch_verify(
      const std::vector<BeamSearchBatchConfig> &old_batches);

  void store_beam_metadata(const BeamSearchBatchConfig &old_bc,
                           const BeamInferenceResult &result);
  void update_beam_metadata(BeamSearchBatchConfig &new_bc, const BeamSearchBatchConfig &old_bc,
                            Request::BeamTree &tree, int request_index);
  std::vector<TokenDepth> traverse_beam_tree(const BeamSearchBatchConfig &old_bc,
                                             int request_index, int first_token_depth);
  std::vector<TokenDepth> merge_dfs_trees(const std::vector<std::vector<TokenDepth>> &trees,
                                          int root_depth, RequestGuid guid);
  std::vector<TokenDepth> traverse_verify_tree(size_t guid,
                                               const std::vector<TokenDepth> &input,
                                               const std::vector<TokenDepth> &output);
  // parent index of every node of a layer-order serialised beam tree (layer
  // d's nodes are equal groups, group j the children of node j of layer d-1)
  static std::vector<int> layer_order_parents(const std::vector<TokenDepth> &tree);
  // the verify step's key-major bitmask of a tree given by parent indices:
  // mask[k] bit q <=> node k is node q or one of its ancestors
  static void tree_bitmask(const std::vector<int> &parent, int n, BatchConfig::BitMask &m);

  ffmi_status serve_incr_decoding(ffmi_model *llm);
  ffmi_status serve_spec_infer(ffmi_model *llm);
  // the speculation phase as chained beam steps (model.h): every SSM's
  // MAX_BEAM_DEPTH steps staged and launched up front, the bookkeeping
  // replayed on the results (identical batches and trees)
  ffmi_status run_ssm_phase_chained(std::vector<BeamSearchBatchConfig> *beam_vec,
                                    BeamInferenceResult *beam_ir);
  // distributed SSMs: keep a local SSM's step results / exchange them and
  // replay the remote SSMs' prepare_next_batch_beam chains
  void record_step(int s, int depth, const BeamSearchBatchConfig &bc,
                   const BeamInferenceResult &ir);
  ffmi_status exchange_and_replay(std::vector<BeamSearchBatchConfig> *beam_vec,
                                  BeamInferenceResult *beam_ir);

  bool all_done() const;
  const GenerationResult *get_generation_result(RequestGuid guid) const;

  struct ProfileInfo {
    int llm_decoding_steps = 0;
    int ssm_decoding_steps = 0;
    double start_time = 0, finish_time = 0;
    double registration_time = 0, first_token_time = 0;
    bool first_token_time_set = false;
  };
  const ProfileInfo *get_profile(RequestGuid guid) const;
  struct Stats {
    long llm_steps = 0, ssm_steps = 0, tokens_committed = 0, tree_tokens_verified = 0;
    long request_verifies = 0;
    double wall_us = 0;
    double llm_us = 0, ssm_us = 0;  // wall time inside the model steps (incl. sync)
    long ssm_phases_chained = 0;
    double ssm_exchange_us = 0;  // distributed SSMs: exchange + replay
  } stats;

 private:
  void complete_request(Request &request, bool spec = false);
  void write_output_record(const Request &request, bool spec) const;
  void apply_limits() const;

  int max_requests_per_batch = 8;
  int max_tokens_per_batch = 128;
  int max_spec_tree_token_num = 23;
  int max_sequence_length = 512;
  std::vector<int> spec_infer_tree_width;
  int bos_token_id = 1;
  std::vector<int> eos_token_ids;
  bool verbose = false;
  // set by prepare_next_batch_init when a pending request's SSM prompt load
  // fell behind the LLM's (the reference asserts there, request_manager.cc:1425)
  bool ssm_prompt_behind = false;
  std::string output_filepath;
  Detokenizer detok = nullptr;
  void *detok_ctx = nullptr;
  bool old_llama_tokenizer = false;

  std::deque<Request> pending_infr_request_queue;
  std::map<RequestGuid, Request> all_requests;
  std::map<RequestGuid, GenerationResult> request_generation_results;
  RequestGuid next_available_guid = 1000000;
  std::unordered_map<RequestGuid, std::vector<TokenDepth>> dfs_tree_inputs;
  // parent index of each node of dfs_tree_inputs[guid] (-1 for the root)
  std::unordered_map<RequestGuid, std::vector<int>> dfs_tree_parents;
  int spec_extensions = 0;
  std::unordered_map<RequestGuid, std::vector<std::pair<int, int>>> committed_tokens;
  std::vector<ffmi_model *> ssm_models;
  std::map<RequestGuid, ProfileInfo> profiling_requests;
  size_t num_processed_requests = 0;
  std::vector<BeamSearchBatchConfig> chain_spec;  // staged chained beam batches
  std::unique_ptr<BeamInferenceResult> chain_ph;   // placeholder results (-1 - i)
  double chain_t[5] = {};  // (FFMI_STEP_TIMING: host-side phase timings, count)
  // distributed SSMs (set_ssm_exchange)
  int xch_world = 1, xch_rank = 0;
  AllGather xch_fn = nullptr;
  void *xch_ctx = nullptr;
  std::vector<int> ssm_local;  // indices of the SSMs this rank runs
  struct StepRecord {
    std::vector<int> ids;
    std::vector<float> probs;
  };
  std::vector<std::vector<StepRecord>> phase_rec;  // [ssm][depth] of the phase
};

double now_us();

}  // namespace ffmi
