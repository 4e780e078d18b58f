// capi.cpp -- C ABI of the serving runtime (models + RequestManager).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "request_manager.h"

struct ffmi_rm {
  ffmi::RequestManager rm;
};

extern "C" ffmi_status ffmi_model_create(const ffmi_llama_config *cfg, const ffmi_model_opts *o,
                                         ffmi_model **out) {
  if (o && o->full_precision) return ffmi::create_llama_f32(cfg, o, out);
  return ffmi::create_llama_gpu(cfg, o, out);
}

extern "C" void ffmi_model_destroy(ffmi_model *m) { delete m; }

extern "C" ffmi_status ffmi_model_set_profiling(ffmi_model *m, int level) {
  if (!m || level < 0 || level > 2) return FFMI_ERR_INVALID;
  return m->set_profiling(level);
}

extern "C" int ffmi_model_op_stats(ffmi_model *m, ffmi_op_stat *out, int cap) {
  if (!m) return -1;
  return m->op_stats(out, cap);
}

extern "C" ffmi_status ffmi_model_set_debug(ffmi_model *m, int enable) {
  if (!m) return FFMI_ERR_INVALID;
  return m->set_debug(enable);
}

extern "C" long ffmi_model_debug_tensor(ffmi_model *m, int which, int layer, float *out,
                                        long cap) {
  if (!m || !out || cap <= 0) return -1;
  return m->debug_tensor(which, layer, out, cap);
}

extern "C" long ffmi_model_debug_width(ffmi_model *m, int which) {
  if (!m) return -1;
  return m->debug_width(which);
}

extern "C" ffmi_status ffmi_model_debug_fault(ffmi_model *m, int kind, int layer, int arg) {
  if (!m) return FFMI_ERR_INVALID;
  return m->debug_fault(kind, layer, arg);
}

extern "C" ffmi_status ffmi_set_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return FFMI_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return FFMI_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return FFMI_ERR_HIP;
  // FFMI_SYNC=spin|yield|block: how a host thread waits in hipStreamSynchronize
  // (A/B of the per-step host round trip; left to HIP's default otherwise).
  // Only before the device's context is live; later calls report an error.
  if (const char *e = getenv("FFMI_SYNC")) {
    const unsigned f = !strcmp(e, "spin") ? hipDeviceScheduleSpin
                       : !strcmp(e, "yield") ? hipDeviceScheduleYield
                       : !strcmp(e, "block") ? hipDeviceScheduleBlockingSync : 0u;
    if (!f || hipSetDeviceFlags(f) != hipSuccess)
      fprintf(stderr, "ffmi: FFMI_SYNC=%s not applied (spin, yield or block, before first use)\n", e);
  }
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_create(const ffmi_rm_config *cfg, ffmi_rm **out) {
  if (!cfg || !out) return FFMI_ERR_INVALID;
  if (cfg->max_requests_per_batch <= 0 ||
      cfg->max_requests_per_batch > ffmi::BatchConfig::MAX_NUM_REQUESTS ||
      cfg->max_tokens_per_batch <= 0 || cfg->max_sequence_length <= 0 ||
      cfg->max_spec_tree_token_num < 0 ||
      cfg->max_spec_tree_token_num > ffmi::BatchConfig::MAX_SPEC_TREE_TOKEN_NUM)
    return FFMI_ERR_INVALID;
  if (cfg->max_tokens_per_batch + cfg->max_spec_tree_token_num * cfg->max_requests_per_batch >
      ffmi::BatchConfig::MAX_NUM_TOKENS)
    return FFMI_ERR_INVALID;
  ffmi_rm *r = new ffmi_rm();
  r->rm.set_max_requests_per_batch(cfg->max_requests_per_batch);
  r->rm.set_max_tokens_per_batch(cfg->max_tokens_per_batch);
  r->rm.set_max_spec_tree_token_num(cfg->max_spec_tree_token_num);
  r->rm.set_max_sequence_length(cfg->max_sequence_length);
  std::vector<int> eos;
  for (int i = 0; i < cfg->num_eos; ++i) eos.push_back(cfg->eos_token_ids[i]);
  r->rm.register_tokenizer(cfg->bos_token_id, eos);
  if (cfg->spec_extensions & ~(FFMI_SPEC_EXT_WIDTH4 | FFMI_SPEC_EXT_MULTI_SSM)) {
    delete r;
    return FFMI_ERR_INVALID;
  }
  r->rm.set_spec_extensions(cfg->spec_extensions);
  for (int i = 0; i < cfg->num_tree_width; ++i)
    if (!r->rm.push_spec_infer_tree_width(cfg->spec_tree_width[i])) {
      delete r;
      return FFMI_ERR_INVALID;  // tree_width <= MAX_BEAM_WIDTH (request_manager.cc:168-171),
                                // 4 under FFMI_SPEC_EXT_WIDTH4
    }
  r->rm.set_verbose(cfg->verbose != 0);
  *out = r;
  return FFMI_OK;
}

extern "C" void ffmi_rm_destroy(ffmi_rm *rm) { delete rm; }

extern "C" ffmi_status ffmi_rm_register_ssm(ffmi_rm *rm, ffmi_model *ssm) {
  if (!rm || !ssm || ssm->mode != FFMI_MODEL_BEAM) return FFMI_ERR_INVALID;
  rm->rm.register_ssm_model(ssm);
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_register_remote_ssm(ffmi_rm *rm) {
  if (!rm) return FFMI_ERR_INVALID;
  rm->rm.register_ssm_model(nullptr);
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_set_ssm_exchange(ffmi_rm *rm, int nranks, int rank,
                                                ffmi_allgather_fn fn, void *ctx) {
  if (!rm || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !fn))
    return FFMI_ERR_INVALID;
  rm->rm.set_ssm_exchange(nranks, rank, fn, ctx);
  return FFMI_OK;
}

static int comm_allgather_cb(void *ctx, const void *mine, size_t bytes, void *all) {
  return ffmi_comm_allgather(static_cast<ffmi_comm *>(ctx), mine, bytes, all) == FFMI_OK ? 0 : 1;
}

extern "C" ffmi_status ffmi_rm_set_ssm_exchange_comm(ffmi_rm *rm, ffmi_comm *comm) {
  if (!rm || !comm) return FFMI_ERR_INVALID;
  rm->rm.set_ssm_exchange(ffmi::comm_size(comm), ffmi::comm_rank(comm), comm_allgather_cb, comm);
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_register_output_filepath(ffmi_rm *rm, const char *path) {
  if (!rm) return FFMI_ERR_INVALID;
  rm->rm.register_output_filepath(path ? path : "");
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_register_detokenizer(ffmi_rm *rm, ffmi_detokenize_fn fn,
                                                    void *ctx) {
  if (!rm) return FFMI_ERR_INVALID;
  rm->rm.register_detokenizer(fn, ctx);
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_set_old_llama_tokenizer(ffmi_rm *rm, int enable) {
  if (!rm) return FFMI_ERR_INVALID;
  rm->rm.set_old_llama_tokenizer(enable != 0);
  return FFMI_OK;
}

extern "C" int64_t ffmi_rm_register_request(ffmi_rm *rm, const int *prompt, int n_prompt,
                                            int max_length, int max_new_tokens,
                                            int add_special_tokens) {
  if (!rm || (n_prompt > 0 && !prompt) || n_prompt < 0) return 0;
  std::vector<int> p(prompt, prompt + n_prompt);
  return rm->rm.register_new_request(p, max_length, max_new_tokens, add_special_tokens != 0);
}

extern "C" ffmi_status ffmi_rm_serve_incr_decoding(ffmi_rm *rm, ffmi_model *llm) {
  if (!rm || !llm || llm->mode != FFMI_MODEL_INC) return FFMI_ERR_INVALID;
  return rm->rm.serve_incr_decoding(llm);
}

extern "C" ffmi_status ffmi_rm_serve_spec_infer(ffmi_rm *rm, ffmi_model *llm) {
  if (!rm || !llm || llm->mode != FFMI_MODEL_TREE) return FFMI_ERR_INVALID;
  return rm->rm.serve_spec_infer(llm);
}

extern "C" int ffmi_rm_get_output(ffmi_rm *rm, int64_t guid, int *tokens, int cap) {
  if (!rm) return -1;
  const ffmi::GenerationResult *gr = rm->rm.get_generation_result(guid);
  if (!gr) return -1;
  const int n = (int)gr->output_tokens.size();
  for (int i = 0; i < n && i < cap && tokens; ++i) tokens[i] = gr->output_tokens[i];
  return n;
}

extern "C" ffmi_status ffmi_rm_get_profile(ffmi_rm *rm, int64_t guid, ffmi_profile *p) {
  if (!rm || !p) return FFMI_ERR_INVALID;
  const auto *pi = rm->rm.get_profile(guid);
  const ffmi::GenerationResult *gr = rm->rm.get_generation_result(guid);
  if (!pi || !gr) return FFMI_ERR_INVALID;
  p->llm_decoding_steps = pi->llm_decoding_steps;
  p->ssm_decoding_steps = pi->ssm_decoding_steps;
  p->start_us = pi->start_time;
  p->finish_us = pi->finish_time;
  p->registration_us = pi->registration_time;
  p->first_token_us = pi->first_token_time;
  p->input_len = (int)gr->input_tokens.size();
  p->output_len = (int)gr->output_tokens.size();
  return FFMI_OK;
}

extern "C" ffmi_status ffmi_rm_get_stats(ffmi_rm *rm, ffmi_serve_stats *s) {
  if (!rm || !s) return FFMI_ERR_INVALID;
  s->llm_steps = rm->rm.stats.llm_steps;
  s->ssm_steps = rm->rm.stats.ssm_steps;
  s->tokens_committed = rm->rm.stats.tokens_committed;
  s->tree_tokens_verified = rm->rm.stats.tree_tokens_verified;
  s->request_verifies = rm->rm.stats.request_verifies;
  s->llm_us = rm->rm.stats.llm_us;
  s->ssm_us = rm->rm.stats.ssm_us;
  s->wall_us = rm->rm.stats.wall_us;
  s->ssm_phases_chained = rm->rm.stats.ssm_phases_chained;
  s->ssm_exchange_us = rm->rm.stats.ssm_exchange_us;
  return FFMI_OK;
}
