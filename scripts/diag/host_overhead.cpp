// Host-side cost of the SpecInfer scheduler per verify cycle, no GPU: the
// bench's workload (8 requests, 128-token prompts, 128 new tokens, widths
// (1,1,3), 23-token trees, max_tokens_per_batch 1024) served by null models
// that pack every step as the GPU model does (pack_beam / pack_tree) and
// return fixed tokens (the SSM never agrees: one token per verify, as with
// random weights).  Chained (FFMI_SSM_CHAIN default) and stepwise.
//   /opt/rocm/bin/hipcc -O2 -std=c++17 -I flexflow_amd/csrc -I include \
//     scripts/diag/host_overhead.cpp -L flexflow_amd -lffmi \
//     -Wl,-rpath,$PWD/flexflow_amd -o /tmp/host_overhead && /tmp/host_overhead
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "runtime/request_manager.h"

using namespace ffmi;

struct NullModel : public ffmi_model {
  int tok;
  PackedStep ps;
  std::vector<int> slot_n[8];
  explicit NullModel(int mode_, int tok_) : tok(tok_) { mode = mode_; }
  ffmi_status run_inc(const BatchConfig &bc, InferenceResult *ir) override {
    pack_inc(bc, 8, 544, &ps);
    for (int t = 0; t < bc.num_tokens; ++t) ir->token_ids[t] = tok;
    return FFMI_OK;
  }
  ffmi_status run_tree(const TreeVerifyBatchConfig &bc, InferenceResult *ir) override {
    pack_tree(bc, 8, 544, &ps);
    for (int t = 0; t < bc.num_tokens; ++t) ir->token_ids[t] = tok;
    return FFMI_OK;
  }
  ffmi_status run_beam(const BeamSearchBatchConfig &bc, BeamInferenceResult *ir) override {
    pack_beam(bc, 8, 544, &ps);
    std::vector<int> map;
    beam_result_layout(bc, &map);
    for (size_t i = 0; i < map.size(); ++i) {
      ir->token_ids[i] = tok + (int)(i % 3);
      ir->probs[i] = 0.5f;
      ir->parent_id[i] = 0;
    }
    return FFMI_OK;
  }
  bool can_chain_beam() const override { return true; }
  std::unique_ptr<BeamInferenceResult> res[8];
  ffmi_status beam_launch_chained(const BeamSearchBatchConfig &bc, int slot) override {
    if (!res[slot]) res[slot].reset(new BeamInferenceResult());
    BeamSearchBatchConfig b = bc;  // (the patch the device gather does)
    for (int t = 0; t < b.num_tokens; ++t)
      if (b.tokensInfo[t].token_id < 0) b.tokensInfo[t].token_id = tok;
    return run_beam(b, res[slot].get());
  }
  ffmi_status beam_collect_chained(int slot, BeamInferenceResult *ir) override {
    *ir = *res[slot];
    return FFMI_OK;
  }
};

int main() {
  for (int chain = 1; chain >= 0; --chain) {
    setenv("FFMI_SSM_CHAIN", chain ? "1" : "0", 1);
    double best = 1e30;
    long cycles = 0;
    for (int rep = 0; rep < 5; ++rep) {
      RequestManager rm;
      rm.set_max_requests_per_batch(8);
      rm.set_max_tokens_per_batch(1024);
      rm.set_max_spec_tree_token_num(23);
      rm.set_max_sequence_length(512);
      for (int w : {1, 1, 3}) rm.push_spec_infer_tree_width(w);
      NullModel llm(FFMI_MODEL_TREE, 5), ssm(FFMI_MODEL_BEAM, 7);
      rm.register_ssm_model(&ssm);
      for (int r = 0; r < 8; ++r) {
        std::vector<int> p(127);
        for (int i = 0; i < 127; ++i) p[i] = 3 + (r * 131 + i * 17) % 31997;
        rm.register_new_request(p, 256, -1, true);
      }
      const auto t0 = std::chrono::steady_clock::now();
      if (rm.serve_spec_infer(&llm) != FFMI_OK) return 1;
      const double us =
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      cycles = rm.stats.llm_steps;
      if (us < best) best = us;
    }
    printf("%s: %ld verify cycles, host %.1f us per cycle (%.2f ms per generate)\n",
           chain ? "chained" : "stepwise", cycles, best / cycles, best / 1e3);
  }
  return 0;
}
