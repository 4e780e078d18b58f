// batch_config.h -- BatchConfig / TreeVerifyBatchConfig / BeamSearchBatchConfig.
//
// Same field names and meaning as include/flexflow/batch_config.h:53-240 of
// the reference (so RequestManager logic and callers read the same), minus
// Legion futures and the PEFT fields.  Capacities are compile-time like the
// reference's MAX_NUM_* constants; MAX_NUM_TOKENS is raised to 2048 so that
// max_tokens_per_batch = 1024 plus a full token tree per request fits the
// verify batch (the reference's 1024 would overflow there).
#pragma once
#include <stdint.h>
#include <string.h>

namespace ffmi {

enum InferenceMode { INC_DECODING_MODE = 0, BEAM_SEARCH_MODE = 1, TREE_VERIFY_MODE = 2 };

class BatchConfig {
 public:
  using RequestGuid = int64_t;
  using TokenId = int;
  static constexpr int MAX_NUM_REQUESTS = 65;
  static constexpr int MAX_NUM_TOKENS = 2048;
  static constexpr int MAX_SPEC_TREE_TOKEN_NUM = 64;

  BatchConfig();
  virtual ~BatchConfig() {}
  virtual InferenceMode get_mode() const { return INC_DECODING_MODE; }
  int num_active_requests() const;
  int num_active_tokens() const { return num_tokens; }
  int num_active_infr_tokens() const { return num_tokens; }

  // run-time limits (set by RequestManager, like the reference's statics)
  static int max_requests_per_batch();
  static int max_tokens_per_batch();
  static int max_verify_tokens_per_batch();
  static int max_spec_tree_token_num();
  static int max_sequence_length();

  int num_tokens = 0;
  int num_generation_tokens = 0;

  struct PerRequestInfo {
    int first_token_depth_in_request = 0;
    int first_token_offset_in_batch = 0;
    int num_tokens_in_batch = 0;
    int max_length = 0;
    int batch_config_request_id = -1;
    bool prompt_phase = false;
    RequestGuid request_guid = 0;
  };
  struct PerTokenInfo {
    int abs_depth_in_request = 0;
    int request_index = 0;
    TokenId token_id = 0;
  };
  struct BitMask {
    uint64_t mask[MAX_SPEC_TREE_TOKEN_NUM] = {0};
    int non_tree_cache_size = 0;  // tokens before the tree
    int tree_size = 0;            // current tree size
    int this_layer_size = 0;
    int prompt_size = 0;          // input length -> prompt / root
  };

  BitMask causalMask[MAX_NUM_REQUESTS];
  PerRequestInfo requestsInfo[MAX_NUM_REQUESTS];
  PerTokenInfo tokensInfo[MAX_NUM_TOKENS];
  bool request_completed[MAX_NUM_REQUESTS];
  bool request_running[MAX_NUM_REQUESTS];
};

class TreeVerifyBatchConfig : public BatchConfig {
 public:
  InferenceMode get_mode() const override { return TREE_VERIFY_MODE; }
  struct CommittedTokensInfo {
    int token_index;    // index of the token in the previous batch
    int request_index;  // request index in the batch
    int token_depth;    // position of the token in the request's sequence
  };
  int num_tokens_to_commit = 0;
  CommittedTokensInfo committed_tokens[MAX_NUM_TOKENS];
};

struct InferenceResult {
  static constexpr int MAX_NUM_TOKENS = BatchConfig::MAX_NUM_TOKENS;
  BatchConfig::TokenId token_ids[MAX_NUM_TOKENS];
};

class BeamSearchBatchConfig : public BatchConfig {
 public:
  InferenceMode get_mode() const override { return BEAM_SEARCH_MODE; }
  int max_beam_depth_all_requests() const;
  int current_depth_all_requests() const;
  int get_speculative_request_num() const { return speculative_request_num; }

  // Capacities.  The reference's limits are 3 and 3 (batch_config.h:196,200,
  // enforced by push_spec_infer_tree_width, request_manager.cc:168-171); the
  // arrays here hold 4 so that the flagged tree-width-4 extension
  // (FFMI_SPEC_EXT_WIDTH4, BASELINE config C) fits.  RequestManager enforces
  // the reference's 3 unless that flag is set.
  static constexpr int MAX_BEAM_WIDTH = 4;
  static constexpr int MAX_BEAM_DEPTH = 8;
  static constexpr int MAX_SPECULATIVE_TREE_BRANCHES = 4;
  static constexpr int REFERENCE_MAX_BEAM_WIDTH = 3;
  static constexpr int REFERENCE_MAX_SPECULATIVE_TREE_BRANCHES = 3;

  int speculative_request_num = 0;
  int model_id = 0;
  struct BeamSearchPerRequestInfo {
    int beam_size = 1;
    int current_depth = -1;
    int max_depth = MAX_BEAM_DEPTH;
    TokenId tokens[MAX_SPECULATIVE_TREE_BRANCHES] = {};
    float probs[MAX_SPECULATIVE_TREE_BRANCHES] = {};
    int parent_id[MAX_SPECULATIVE_TREE_BRANCHES] = {};
    int sub_request_num = 0;
  };
  struct BeamSearchPerTokenInfo {
    int sub_request_index = 0;
  };
  BeamSearchPerRequestInfo beamRequestsInfo[MAX_NUM_REQUESTS];
  BeamSearchPerTokenInfo beamTokenInfo[MAX_NUM_TOKENS];
  int sub_requests[MAX_NUM_REQUESTS] = {0};
};

struct BeamInferenceResult {
  static constexpr int MAX_NUM_TOKENS = BatchConfig::MAX_NUM_TOKENS;
  BatchConfig::TokenId
      token_ids[MAX_NUM_TOKENS * BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
  float probs[MAX_NUM_TOKENS * BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
  int parent_id[MAX_NUM_TOKENS * BeamSearchBatchConfig::MAX_SPECULATIVE_TREE_BRANCHES];
};

// process-wide limits (RequestManager setters write them)
struct BatchLimits {
  int max_requests_per_batch = 8;
  int max_tokens_per_batch = 128;
  int max_spec_tree_token_num = 23;
  int max_sequence_length = 512;
};
BatchLimits &batch_limits();

}  // namespace ffmi
