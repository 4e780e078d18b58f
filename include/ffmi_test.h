/* ffmi_test.h -- test doubles, exported by libffmi_testmodel.so (built
 * next to libffmi.so, linked against it) and NEVER by the product library. */
#ifndef FFMI_TEST_H
#define FFMI_TEST_H
#include "ffmi.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Scheduler test double (no GPU): a deterministic hash "model" whose next
 * token is a function of the exact token context each query sees through the
 * KV-slot / bitmask rules, so the RequestManager's batching, tree build,
 * verification and commit lists can be checked on CPU.  TEST USE ONLY. */
ffmi_status ffmi_test_hash_model_create(int vocab, int mode, int max_requests,
                                        int max_seq, int max_tree, uint64_t salt,
                                        int disagree_pct, ffmi_model **out);
/* Give the hash model a token capacity per step, as a GPU model's
 * max_tokens: larger steps fail with FFMI_ERR_INVALID, and the scheduler's
 * up-front SSM capacity check sees it.  TEST USE ONLY. */
ffmi_status ffmi_test_hash_model_set_capacity(ffmi_model *m, int max_tokens);

#ifdef __cplusplus
}
#endif
#endif
