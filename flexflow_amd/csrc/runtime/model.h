// model.h -- model handles behind the RequestManager (C handle ffmi_model).
//
// The reference builds a Legion operator graph per InferenceMode
// (inference/models/llama.cc:23-317) and runs it with
// InferenceManager::inference (inference_manager.cc:408-468).  Here a model
// is a C++ object that owns its weights and per-layer attention handles and
// runs one step of a BatchConfig through the C-ABI kernels in graph order.
#pragma once
#include <vector>

#include "../ffmi_internal.h"
#include "batch_config.h"

namespace ffmi {

// Per-step device metadata derived from a BatchConfig (what the kernels read).
struct PackedStep {
  std::vector<ffmi_token_info> tokens;
  std::vector<ffmi_attn_work> work;
  std::vector<ffmi_commit_info> commits;
  std::vector<uint64_t> masks;  // [num_mask_reqs][FFMI_MAX_TREE]
  int num_mask_reqs = 0;
  int topk = 1;  // BEAM: results per token (beam width)
  void desc(ffmi_batch_desc *d) const;
};

// KV-slot / visibility packing, one per reference attention op:
//  INC  : store_kv_cache, inc_multihead_self_attention.cu:35-61 (slot = depth),
//         causal visibility (generation + prompt paths)
//  TREE : update_tree_branch_kv_cache_fused, tree_inc...cu:433-478 (slot =
//         first_depth + local), commit list tree_inc...cu:335-396, bitmask
//         visibility tree_inc...cu:150-170 / prompt causal :166-168
//  BEAM : spec_inc_store_kv_cache, spec_inc...cu:311-358 (slot = prompt_size
//         + non_tree + tree_size - 1 - this_layer_size + local), bitmask
//         visibility with query_token = prompt_size+tree_size-1-branches+qi
//         (spec_inc...cu:145-170), causal prompt path :461-679
void pack_inc(const BatchConfig &bc, int max_requests, int slots, PackedStep *out);
void pack_tree(const TreeVerifyBatchConfig &bc, int max_requests, int slots, PackedStep *out);
void pack_beam(const BeamSearchBatchConfig &bc, int max_requests, int slots, PackedStep *out);
// A beam step's results as the scheduler reads them (store_beam_metadata,
// request_manager.cc:2217-2325): each token's top-w entries, w its request's
// beam width, back to back in token order.  The step computes the top-k of
// every token for k = beam_step_topk (the widest request) into [T][k]; map[i]
// is the [T][k] index of scheduler entry i (the identity when every request
// has the same width).
int beam_step_topk(const BeamSearchBatchConfig &bc);
void beam_result_layout(const BeamSearchBatchConfig &bc, std::vector<int> *map);

}  // namespace ffmi

struct ffmi_model {
  int mode = FFMI_MODEL_INC;
  virtual ~ffmi_model() {}
  virtual ffmi_status run_inc(const ffmi::BatchConfig &bc, ffmi::InferenceResult *ir) = 0;
  virtual ffmi_status run_tree(const ffmi::TreeVerifyBatchConfig &bc,
                               ffmi::InferenceResult *ir) = 0;
  virtual ffmi_status run_beam(const ffmi::BeamSearchBatchConfig &bc,
                               ffmi::BeamInferenceResult *ir) = 0;
  // A beam step in two halves, so that several SSMs' steps run at once
  // (serve_spec_infer launches every SSM's step, then collects each):
  // beam_launch enqueues the step of `bc` (which stays alive until the
  // collect), beam_collect waits for it and writes the results.  Default:
  // the synchronous run_beam at collect time.
  virtual ffmi_status beam_launch(const ffmi::BeamSearchBatchConfig &bc) {
    pending_beam = &bc;
    return FFMI_OK;
  }
  virtual ffmi_status beam_collect(ffmi::BeamInferenceResult *ir) {
    if (!pending_beam) return FFMI_ERR_INVALID;
    const ffmi::BeamSearchBatchConfig *bc = pending_beam;
    pending_beam = nullptr;
    return run_beam(*bc, ir);
  }
  const ffmi::BeamSearchBatchConfig *pending_beam = nullptr;
  // Chained beam steps (serve_spec_infer): the 8 beam steps of a speculation
  // phase are launched back to back without waiting for results.  Step
  // `slot` > 0 carries token id -1 - i where its token is entry i of step
  // slot - 1's top-k ids (the device fills it in); the results of every slot
  // are kept until the next phase.  The scheduler's state does not depend on
  // the token values beyond those ids, so it stages all 8 steps up front and
  // replays its bookkeeping once the results are in (request_manager.cpp).
  virtual bool can_chain_beam() const { return false; }
  virtual ffmi_status beam_launch_chained(const ffmi::BeamSearchBatchConfig &bc, int slot) {
    (void)bc;
    (void)slot;
    return FFMI_ERR_UNSUPPORTED;
  }
  virtual ffmi_status beam_collect_chained(int slot, ffmi::BeamInferenceResult *ir) {
    (void)slot;
    (void)ir;
    return FFMI_ERR_UNSUPPORTED;
  }
  // tokens one step can hold (-1: unknown), checked by serve_spec_infer
  // against the largest batch the scheduler can build for an SSM
  virtual int token_capacity() const { return -1; }
  // a TP-sharded model: its steps run collectives on a communicator, so two
  // such models' steps must not be in flight at once (their collectives
  // could pair up across ranks in different orders)
  virtual bool uses_collectives() const { return false; }
  virtual ffmi_status set_profiling(int level) {
    (void)level;
    return FFMI_ERR_UNSUPPORTED;
  }
  virtual int op_stats(ffmi_op_stat *out, int cap) {
    (void)out;
    (void)cap;
    return 0;
  }
  virtual ffmi_status set_debug(int enable) {
    (void)enable;
    return FFMI_ERR_UNSUPPORTED;
  }
  virtual long debug_tensor(int which, int layer, float *out, long cap) {
    (void)which;
    (void)layer;
    (void)out;
    (void)cap;
    return -1;
  }
  virtual ffmi_status debug_fault(int kind, int layer, int arg) {
    (void)kind;
    (void)layer;
    (void)arg;
    return FFMI_ERR_UNSUPPORTED;
  }
  virtual long debug_width(int which) const {
    (void)which;
    return -1;
  }
};

namespace ffmi {
ffmi_status create_llama_gpu(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                             ffmi_model **out);
// full precision (--use-full-precision): runtime/llama_f32.cpp
ffmi_status create_llama_f32(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                             ffmi_model **out);
ffmi_status create_hash_model(int vocab, int mode, int max_requests, int max_seq,
                              int max_tree, uint64_t salt, int disagree_pct,
                              ffmi_model **out);
}  // namespace ffmi
