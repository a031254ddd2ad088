/*
 * ksg_oracle.h -- PARITY ORACLE C API (test infrastructure only).
 *
 * A CPU restatement of kube-scheduler's node-evaluation path (see oracle.cpp for the
 * reference file:line of every step).  It has the same shape as include/ksg.h with a
 * ksgo_ prefix so tests drive the product and the oracle with the identical event and
 * pod sequence.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load liboracle; the product never links it.
 */
#ifndef KSG_ORACLE_H_
#define KSG_ORACLE_H_
#include "../include/ksg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ksgo_ctx ksgo_ctx;

ksgo_ctx *ksgo_create(const char *config_json, size_t len);
const char *ksgo_create_error(void);
void ksgo_destroy(ksgo_ctx *ctx);
const char *ksgo_last_error(const ksgo_ctx *ctx);
int ksgo_upsert_namespace(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_upsert_object(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_remove_object(ksgo_ctx *ctx, const char *kind, const char *ns, const char *name);
int ksgo_add_node(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_update_node(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_remove_node(ksgo_ctx *ctx, const char *name);
int ksgo_add_pod(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_remove_pod(ksgo_ctx *ctx, const char *uid);
int ksgo_num_nodes(const ksgo_ctx *ctx);
int ksgo_node_name(const ksgo_ctx *ctx, int32_t index, char *buf, size_t cap);
int ksgo_pod_compile(ksgo_ctx *ctx, const char *json, size_t len, int32_t *handle);
int ksgo_pod_release(ksgo_ctx *ctx, int32_t handle);
int ksgo_schedule_one(ksgo_ctx *ctx, int32_t handle, uint32_t flags, ksg_result *result,
                      ksg_eval_out *eval);
int ksgo_schedule_batch(ksgo_ctx *ctx, const int32_t *handles, int32_t n, uint32_t flags,
                        ksg_result *results);
int ksgo_forget(ksgo_ctx *ctx, int32_t handle);
/* the nominator, same contract as ksg_add_nominated_pod / ksg_delete_nominated_pod (include/ksg.h) */
int ksgo_add_nominated_pod(ksgo_ctx *ctx, const char *json, size_t len);
int ksgo_delete_nominated_pod(ksgo_ctx *ctx, const char *uid);
/* CPU-baseline breakdown: microseconds per cycle section since the last call (see oracle.cpp) */
int ksgo_debug_profile(ksgo_ctx *ctx, double *out, int n);
int ksgo_run_filter_plugin(ksgo_ctx *ctx, int32_t handle, int32_t plugin, int32_t *prefilter_code,
                           uint8_t *codes, uint32_t *reasons);
int ksgo_run_score_plugin(ksgo_ctx *ctx, int32_t handle, int32_t plugin, const uint8_t *nodes,
                          int32_t *status_code, int64_t *raw, int64_t *normalized);

/* DefaultPreemption PostFilter, same contract as ksg_preempt (include/ksg.h). */
int ksgo_preempt(ksgo_ctx *ctx, int32_t handle, const char *args_json, size_t args_len, ksg_preempt_result *result,
                 char *detail, size_t detail_cap, size_t *detail_len);

/* Go math.Log restatement (exposed so tests can compare it with libm). */
double ksgo_go_log(double x);
/* time.Now() of the following scheduling cycles (OpportunisticBatching's maxBatchAge); 0: the wall clock */
int ksgo_set_clock(ksgo_ctx *ctx, int64_t now_ns);
int ksgo_debug_clock_step(ksgo_ctx *ctx, int64_t step_ns);
/* one TestBatchBasic case through the OpportunisticBatch restatement (oracle.cpp) */
int ksgo_debug_batch_basic(const char *json, size_t len, char *out, size_t cap);
int ksgo_debug_pod_resources(const char *json, size_t len, int64_t *out, int32_t cap);
/* SignPod of one pod under one profile, as ksg_debug_pod_signature (1 signed, 0 nil) */
int ksgo_debug_pod_signature(const char *cfg, size_t cfg_len, const char *json, size_t len, char *out, size_t cap,
                             size_t *out_len);
/* container/heap Init over (score) with nodeScoreHeap.Less, returns index of the root. */
int32_t ksgo_heap_root(const int64_t *scores, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
