#include <algorithm>
// capi.cpp -- the extern "C" boundary declared in include/ksg.h.
//
// Every entry point catches C++ exceptions and maps them to KSG_E* codes; nothing here falls
// back to a CPU evaluation -- a missing/broken device is KSG_EDEVICE.
#include <cstring>
#include <memory>
#include <new>
#include <string>

#include "comm.hpp"
#include "host.hpp"

using namespace ksg;

struct ksg_ctx {
  std::unique_ptr<Cluster> cluster;
  std::unique_ptr<Engine> engine;
  std::string err;
};

static thread_local std::string g_create_error;

#define GUARD(body)                                   \
  try {                                               \
    body                                              \
  } catch (const std::bad_alloc&) {                   \
    ctx->err = "out of memory";                       \
    return KSG_ENOMEM;                                \
  } catch (const std::exception& e) {                 \
    ctx->err = e.what();                              \
    return KSG_EINVAL;                                \
  }

// The resident single-pod loop holds the stream and node cores in LDS: it ends before any other use
// of the device and before any change to the cache it mirrors (Engine::schedule_resident)
static int with_err(ksg_ctx* ctx, int rc);
static int quiesce(ksg_ctx* ctx) { return with_err(ctx, ctx->engine->resident_stop()); }

// A call that succeeded may still leave a message: a loop give-up recovered over the all-reduce path
// ("recovered: ..." with give_up_detail's missing participants, Engine::run_batch_api) is kept too.
static int with_err(ksg_ctx* ctx, int rc) {
  if (rc != KSG_OK || !ctx->cluster->err.empty()) {
    if (!ctx->cluster->err.empty()) ctx->err = ctx->cluster->err;
    ctx->cluster->err.clear();
  }
  return rc;
}

extern "C" {

ksg_ctx* ksg_create(const char* config_json, size_t len) {
  try {
    Config cfg;
    std::string err;
    if (config_json && len && !decode_config(config_json, len, &cfg, &err)) {
      g_create_error = err;
      return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
      g_create_error = "no HIP device visible (the engine has no CPU fallback)";
      return nullptr;
    }
    if (cfg.device < 0 || cfg.device >= ndev) {
      g_create_error = "device index out of range";
      return nullptr;
    }
    auto* ctx = new ksg_ctx();
    ctx->cluster.reset(new Cluster(cfg));
    if (!ctx->cluster->err.empty()) {
      g_create_error = ctx->cluster->err;
      delete ctx;
      return nullptr;
    }
    ctx->engine.reset(new Engine(ctx->cluster.get()));
    if (!ctx->cluster->err.empty()) {  // the kernels' code object did not load
      g_create_error = ctx->cluster->err;
      delete ctx;
      return nullptr;
    }
    if (cfg.sharded()) {  // node-sharded: join the exchange group (collective across the ranks)
      if (ctx->engine->ob_acting()) {  // before the collective: every rank has the same profile, so all fail here
        g_create_error = "OpportunisticBatching acts in this profile (PodTopologySpread without default constraints) "
                         "and the node-sharded scheduler does not run it: set featureGates.OpportunisticBatching false";
        delete ctx;
        return nullptr;
      }
      std::string err;
      ctx->engine->comm = make_comm(cfg, &err);
      if (!ctx->engine->comm) {
        g_create_error = err;
        delete ctx;
        return nullptr;
      }
    }
    return ctx;
  } catch (const std::exception& e) {
    g_create_error = e.what();
    return nullptr;
  }
}

const char* ksg_create_error(void) { return g_create_error.c_str(); }

void ksg_destroy(ksg_ctx* ctx) {
  if (!ctx) return;
  ctx->engine.reset();
  ctx->cluster.reset();
  delete ctx;
}

const char* ksg_last_error(const ksg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int ksg_upsert_namespace(ksg_ctx* ctx, const char* ns_json, size_t len) {
  if (!ctx || !ns_json) return KSG_EINVAL;
  GUARD({
    NamespaceSpec ns;
    if (!decode_namespace(ns_json, len, &ns, &ctx->err)) return KSG_EINVAL;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->upsert_namespace(ns));
  })
}

int ksg_upsert_object(ksg_ctx* ctx, const char* obj_json, size_t len) {
  if (!ctx || !obj_json) return KSG_EINVAL;
  GUARD({
    SelectorObj o;
    if (!decode_selector_obj(obj_json, len, &o, &ctx->err)) return KSG_EINVAL;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->upsert_object(std::move(o)));
  })
}

int ksg_remove_object(ksg_ctx* ctx, const char* kind, const char* ns, const char* name) {
  if (!ctx || !kind || !name) return KSG_EINVAL;
  GUARD({
    const int k = obj_kind(kind);
    if (k < 0) {
      ctx->err = std::string("unsupported kind ") + kind;
      return KSG_EINVAL;
    }
    const std::string n = (ns && *ns) ? ns : "default";
    if (const int rs = quiesce(ctx)) return rs;
    const int rc = ctx->cluster->remove_object(k, n, name);
    if (rc == KSG_ENOTFOUND) ctx->err = std::string(kind) + " " + n + "/" + name + " not found";
    return with_err(ctx, rc);
  })
}

int ksg_add_node(ksg_ctx* ctx, const char* node_json, size_t len) {
  if (!ctx || !node_json) return KSG_EINVAL;
  GUARD({
    NodeSpec n;
    if (!decode_node(node_json, len, &n, &ctx->err)) return KSG_EINVAL;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->add_node(std::move(n)));
  })
}

int ksg_update_node(ksg_ctx* ctx, const char* node_json, size_t len) {
  if (!ctx || !node_json) return KSG_EINVAL;
  GUARD({
    NodeSpec n;
    if (!decode_node(node_json, len, &n, &ctx->err)) return KSG_EINVAL;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->update_node(std::move(n)));
  })
}

int ksg_remove_node(ksg_ctx* ctx, const char* name) {
  if (!ctx || !name) return KSG_EINVAL;
  GUARD({
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->remove_node(name));
  })
}

int ksg_add_pod(ksg_ctx* ctx, const char* pod_json, size_t len) {
  if (!ctx || !pod_json) return KSG_EINVAL;
  GUARD({
    PodSpec p;
    if (!decode_pod(pod_json, len, &p, &ctx->err)) return KSG_EINVAL;
    if (p.node_name.empty()) {
      ctx->err = "ksg_add_pod: pod is not bound (spec.nodeName empty)";
      return KSG_EINVAL;
    }
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->add_pod(p));
  })
}

int ksg_remove_pod(ksg_ctx* ctx, const char* uid) {
  if (!ctx || !uid) return KSG_EINVAL;
  GUARD({
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->remove_pod(uid));
  })
}

int ksg_num_nodes(const ksg_ctx* ctx) {
  if (!ctx) return KSG_EINVAL;
  return (int)const_cast<ksg_ctx*>(ctx)->cluster->order().size();
}

int ksg_node_name(const ksg_ctx* ctx, int32_t index, char* buf, size_t cap) {
  if (!ctx) return KSG_EINVAL;
  const auto& o = const_cast<ksg_ctx*>(ctx)->cluster->order();
  if (index < 0 || (size_t)index >= o.size()) return KSG_ENOTFOUND;
  const std::string& s = o[(size_t)index];
  if (buf && cap) {
    size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)s.size();
}

int ksg_pod_compile(ksg_ctx* ctx, const char* pod_json, size_t len, int32_t* handle) {
  if (!ctx || !pod_json || !handle) return KSG_EINVAL;
  GUARD({
    PodSpec p;
    if (!decode_pod(pod_json, len, &p, &ctx->err)) return KSG_EINVAL;
    if (!p.unsupported.empty()) {  // declined, not mis-evaluated: the caller schedules it on the CPU path
      ctx->err = "pod " + p.ns + "/" + p.name + ": " + p.unsupported;
      return KSG_ENOTSUP;
    }
    if (p.needs_features) {  // NodeDeclaredFeatures' PreFilter would not Skip (nodedeclaredfeatures.go:86-104)
      ctx->err = "pod " + p.ns + "/" + p.name + ": needs a declared node feature (NodeDeclaredFeatures), which runs "
                 "outside the device path";
      return KSG_ENOTSUP;
    }
    if (!p.nominated_node.empty() && ctx->engine->comm) {  // evaluateNominatedNode runs on one device's mirror
      ctx->err = "pod " + p.ns + "/" + p.name + ": status.nominatedNodeName on a node-sharded context (the nominated "
                 "node's single-node pass is not sharded)";
      return KSG_ENOTSUP;
    }
    // the pod's pod-table entry (labels, affinity terms) compiled once, as NewPodInfo does at enqueue
    ctx->cluster->pod_table_precompile(p);
    const int32_t h = ctx->engine->next_handle++;
    ctx->engine->queue[h] = std::move(p);
    *handle = h;
    return KSG_OK;
  })
}

int ksg_pod_release(ksg_ctx* ctx, int32_t handle) {
  if (!ctx) return KSG_EINVAL;
  return ctx->engine->queue.erase(handle) ? KSG_OK : KSG_ENOTFOUND;
}

int ksg_schedule_one(ksg_ctx* ctx, int32_t handle, uint32_t flags, ksg_result* result, ksg_eval_out* eval) {
  if (!ctx || !result) return KSG_EINVAL;
  GUARD({
    auto it = ctx->engine->queue.find(handle);
    if (it == ctx->engine->queue.end()) return KSG_ENOTFOUND;
    if (const int rn = ctx->engine->check_nominations({&it->second})) return with_err(ctx, rn);
    if (!eval && (flags & KSG_FLAG_ASSUME)) {  // a resident loop (k_sched_loop / k_agg_loop), else the launch path
      bool handled = false;
      const int rc = ctx->engine->schedule_resident(it->second, handle, result, &handled);
      if (handled) return with_err(ctx, rc);
    }
    if (const int rs = quiesce(ctx)) return rs;
    std::vector<const PodSpec*> pods{&it->second};
    std::vector<int32_t> hs{handle};
    return with_err(ctx, ctx->engine->run_batch_api(pods, hs, (flags & KSG_FLAG_ASSUME) != 0, result, eval));
  })
}

int ksg_schedule_batch(ksg_ctx* ctx, const int32_t* handles, int32_t n, uint32_t flags, ksg_result* results) {
  if (!ctx || n < 0 || (n && (!handles || !results))) return KSG_EINVAL;
  GUARD({
    if (const int rs = quiesce(ctx)) return rs;
    ctx->engine->api_t0_ = std::chrono::steady_clock::now();  // loopStamps: the handle lookups' share
    std::vector<const PodSpec*> pods;
    std::vector<int32_t> hs(handles, handles + n);
    pods.reserve((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
      auto it = ctx->engine->queue.find(handles[i]);
      if (it == ctx->engine->queue.end()) return KSG_ENOTFOUND;
      pods.push_back(&it->second);
    }
    if (const int rn = ctx->engine->check_nominations(pods)) return with_err(ctx, rn);
    return with_err(ctx, ctx->engine->run_batch_api(pods, hs, (flags & KSG_FLAG_ASSUME) != 0, results, nullptr));
  })
}

int ksg_forget(ksg_ctx* ctx, int32_t handle) {  // Cache.ForgetPod (backend/cache/cache.go:412-434)
  if (!ctx) return KSG_EINVAL;
  GUARD({
    auto it = ctx->engine->assumed.find(handle);
    if (it == ctx->engine->assumed.end()) return KSG_ENOTFOUND;
    if (const int rs = quiesce(ctx)) return rs;
    std::string uid = it->second;
    ctx->engine->assumed.erase(it);
    return with_err(ctx, ctx->cluster->remove_pod(uid));
  })
}

int ksg_add_nominated_pod(ksg_ctx* ctx, const char* pod_json, size_t len) {  // nominator.go:60-103
  if (!ctx || !pod_json) return KSG_EINVAL;
  GUARD({
    PodSpec p;
    if (!decode_pod(pod_json, len, &p, &ctx->err)) return KSG_EINVAL;
    if (p.uid.empty()) {
      ctx->err = "ksg_add_nominated_pod: metadata.uid is empty";
      return KSG_EINVAL;
    }
    ctx->engine->nominated.erase(p.uid);  // deleteUnlocked: at most one nomination per uid
    if (!p.nominated_node.empty()) ctx->engine->nominated[p.uid] = std::make_pair(p.nominated_node, p.priority);
    return KSG_OK;
  })
}

int ksg_delete_nominated_pod(ksg_ctx* ctx, const char* uid) {  // nominator.go:138-...
  if (!ctx || !uid) return KSG_EINVAL;
  ctx->engine->nominated.erase(uid);
  return KSG_OK;
}

int ksg_run_filter_plugin(ksg_ctx* ctx, int32_t handle, int32_t plugin, int32_t* prefilter_code, uint8_t* codes,
                          uint32_t* reasons) {
  if (!ctx || !prefilter_code || plugin < 0 || plugin > KSG_PLUGIN_INTER_POD_AFFINITY) return KSG_EINVAL;
  GUARD({
    auto it = ctx->engine->queue.find(handle);
    if (it == ctx->engine->queue.end()) return KSG_ENOTFOUND;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->engine->run_plugin(it->second, Engine::FILTER_ONE, plugin, nullptr, prefilter_code,
                                                 codes, reasons, nullptr, nullptr));
  })
}

int ksg_preempt(ksg_ctx* ctx, int32_t handle, const char* args_json, size_t args_len, ksg_preempt_result* result,
                char* detail, size_t detail_cap, size_t* detail_len) {
  if (!ctx || !result) return KSG_EINVAL;
  GUARD({
    auto it = ctx->engine->queue.find(handle);
    if (it == ctx->engine->queue.end()) return KSG_ENOTFOUND;
    // node-sharded contexts: every rank holds the whole mirror and pod table, so each rank runs the
    // PostFilter over every node by itself (no exchange) and returns the identical choice
    // (SelectVictimsOnNode filters with the nominated pods too: refused likewise)
    if (const int rn = ctx->engine->check_nominations({&it->second})) return with_err(ctx, rn);
    if (const int rs = quiesce(ctx)) return rs;
    std::string d;
    const int rc = ctx->engine->preempt(it->second, args_json, args_len, result, detail ? &d : nullptr);
    if (rc) return with_err(ctx, rc);
    if (detail_len) *detail_len = d.size();
    if (detail) {
      if (d.size() + 1 > detail_cap) {
        ctx->err = "detail buffer too small";
        return KSG_ENOMEM;
      }
      std::memcpy(detail, d.c_str(), d.size() + 1);
    }
    return KSG_OK;
  })
}

int ksg_run_score_plugin(ksg_ctx* ctx, int32_t handle, int32_t plugin, const uint8_t* nodes, int32_t* status_code,
                         int64_t* raw, int64_t* normalized) {
  if (!ctx || !status_code) return KSG_EINVAL;
  if (plugin != KSG_PLUGIN_TAINT_TOLERATION && plugin != KSG_PLUGIN_NODE_AFFINITY &&
      plugin != KSG_PLUGIN_NODE_RESOURCES_FIT && plugin != KSG_PLUGIN_POD_TOPOLOGY_SPREAD &&
      plugin != KSG_PLUGIN_INTER_POD_AFFINITY && plugin != KSG_PLUGIN_BALANCED_ALLOCATION &&
      plugin != KSG_PLUGIN_IMAGE_LOCALITY)
    return KSG_EINVAL;
  GUARD({
    auto it = ctx->engine->queue.find(handle);
    if (it == ctx->engine->queue.end()) return KSG_ENOTFOUND;
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->engine->run_plugin(it->second, Engine::SCORE_ONE, plugin, nodes, status_code, nullptr,
                                                 nullptr, raw, normalized));
  })
}

int ksg_comm_unique_id(char* buf, size_t cap) {
  try {
    std::string hex, err;
    int rc = comm_unique_id(&hex, &err);
    if (rc) {
      g_create_error = err;
      return rc;
    }
    if (!buf || cap < hex.size() + 1) return KSG_EINVAL;
    std::memcpy(buf, hex.c_str(), hex.size() + 1);
    return (int)hex.size();
  } catch (const std::exception& e) {
    g_create_error = e.what();
    return KSG_EINVAL;
  }
}

int ksg_shard_range(const ksg_ctx* ctx, int32_t* first_node, int32_t* num_nodes) {
  if (!ctx || !first_node || !num_nodes) return KSG_EINVAL;
  int32_t b0 = 0, nb = 0;
  const int32_t n = (int32_t)ctx->cluster->order().size();
  ctx->engine->shard_range(n, &b0, &nb);
  const int32_t lo = std::min<int32_t>(b0 * kBlock, n), hi = std::min<int32_t>((b0 + nb) * kBlock, n);
  *first_node = lo;
  *num_nodes = hi - lo;
  return KSG_OK;
}

int ksg_last_batch_kernel_stats(const ksg_ctx* ctx, double* avg_kernel_ms, double* bytes_per_launch,
                                int32_t* launches, int32_t* kernel) {
  if (!ctx) return KSG_EINVAL;
  if (kernel) *kernel = ctx->engine->last_kernel;
  if (avg_kernel_ms) *avg_kernel_ms = ctx->engine->last_kernel_ms;
  if (bytes_per_launch) *bytes_per_launch = ctx->engine->last_bytes;
  if (launches) *launches = ctx->engine->last_launches;
  return KSG_OK;
}

int ksg_debug_compare_mirror(ksg_ctx* ctx, int32_t sync, int32_t* ndiff, int32_t* first) {
  if (!ctx || !ndiff || !first) return KSG_EINVAL;
  GUARD({
    if (const int rs = quiesce(ctx)) return rs;
    return with_err(ctx, ctx->cluster->compare_mirror(sync != 0, ndiff, first));
  })
}

int ksg_debug_relayouts(const ksg_ctx* ctx, uint64_t* full, uint64_t* gather) {
  if (!ctx || !full || !gather) return KSG_EINVAL;
  *full = ctx->cluster->relayouts_full;
  *gather = ctx->cluster->relayouts_gather;
  return KSG_OK;
}

int ksg_set_clock(ksg_ctx* ctx, int64_t now_ns) {
  if (!ctx) return KSG_EINVAL;
  ctx->engine->ob_clock_ = now_ns;
  return KSG_OK;
}

int ksg_debug_clock_step(ksg_ctx* ctx, int64_t step_ns) {
  if (!ctx || step_ns < 0) return KSG_EINVAL;
  ctx->engine->ob_clock_step_ = step_ns;
  return KSG_OK;
}

int ksg_debug_batching(const ksg_ctx* ctx, uint64_t* hinted, uint64_t* cycles) {
  if (!ctx || !hinted || !cycles) return KSG_EINVAL;
  *hinted = ctx->engine->ob_hinted_;
  *cycles = (uint64_t)ctx->engine->ob_cycle_;
  return KSG_OK;
}

int ksg_debug_loop_stats(const ksg_ctx* ctx, uint64_t* give_ups, uint64_t* retries) {
  if (!ctx || !give_ups || !retries) return KSG_EINVAL;
  *give_ups = ctx->engine->loop_give_ups_;
  *retries = ctx->engine->loop_retries_;
  return KSG_OK;
}

int ksg_debug_log_table(double* out, int32_t n) {
  if (!out || n < 0) return KSG_EINVAL;
  for (int32_t k = 0; k < n; ++k) out[k] = ksg::go_log((double)k);  // as Cluster::upload_pod_table builds it
  return n;
}

int ksg_generation(const ksg_ctx* ctx, uint64_t* list_gen, uint64_t* events) {
  if (!ctx) return KSG_EINVAL;
  ctx->cluster->order();  // a pending node-list rebuild counts now
  if (list_gen) *list_gen = ctx->cluster->list_gen;
  if (events) *events = ctx->cluster->events;
  return KSG_OK;
}

int ksg_debug_schedule_calls(ksg_ctx* ctx, const int32_t* handles, int32_t n, uint32_t flags, ksg_result* results,
                             double* us_per_call) {
  if (!ctx || n < 0 || (n && (!handles || !results)) || !us_per_call) return KSG_EINVAL;
  const auto t0 = std::chrono::steady_clock::now();
  for (int32_t k = 0; k < n; ++k)
    if (const int rc = ksg_schedule_one(ctx, handles[k], flags, results + k, nullptr)) return rc;
  *us_per_call = n ? std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n : 0.0;
  return KSG_OK;
}

int ksg_debug_pod_resources(const char* pod_json, size_t len, int64_t* out, int32_t cap) {
  using namespace ksg;
  if (!pod_json || !out || cap < 8) return KSG_EINVAL;
  PodSpec p;
  std::string err;
  if (!decode_pod(pod_json, len, &p, &err)) return KSG_EINVAL;
  const PodResources r = calc_resources(p), f = calc_fit_request(p);
  const int64_t v[8] = {r.cpu, r.mem, r.eph, r.nz_cpu, r.nz_mem, f.cpu, f.mem, f.eph};
  for (int k = 0; k < 8; ++k) out[k] = v[k];
  return 8;
}

int ksg_debug_pod_signature(const char* config_json, size_t config_len, const char* pod_json, size_t pod_len, char* out,
                            size_t cap, size_t* out_len) {
  using namespace ksg;
  if (!pod_json || !out || !out_len) return KSG_EINVAL;
  try {
    Config cfg;
    PodSpec p;
    std::string err, sig;
    if (config_json && config_len && !decode_config(config_json, config_len, &cfg, &err)) return KSG_EINVAL;
    if (!decode_pod(pod_json, pod_len, &p, &err)) return KSG_EINVAL;
    // the request Fit signs: the spec's (fit.go:317-325), as the cycle compile takes it
    const PodResources fit = p.has_status_res ? calc_fit_request(p) : calc_resources(p);
    if (!sign_text(cfg, p, fit, &sig)) {
      *out_len = 0;
      if (cap) out[0] = 0;
      return 0;
    }
    if (sig.size() + 1 > cap) return KSG_EINVAL;
    std::memcpy(out, sig.c_str(), sig.size() + 1);
    *out_len = sig.size();
    return 1;
  } catch (const std::exception&) {
    return KSG_EINVAL;
  }
}

int ksg_debug_exchange_layout(int32_t* out, int32_t cap) {
  using namespace ksg;
  const int32_t v[] = {kMaxShards, XA_CNT,   XA_BELOW, XA_NONIGN,  XA_MAX_TAINT, XA_MAX_NA,   XA_MAX_IPA,
                       XA_NMIN_IPA, XA_END,  XA_PROC,  XA_WORDS,   XB_KEY,       XB_NODE,     XB_WORDS,
                       XP_MAX_PTS, XP_NMIN_PTS, XP_WORDS, XS_CNT,   XS_BELOW,     XS_WORDS,    kPreBits};
  const int32_t n = (int32_t)(sizeof v / sizeof v[0]);
  if (!out || cap < n) return KSG_EINVAL;
  for (int32_t k = 0; k < n; ++k) out[k] = v[k];
  return n;
}

uint64_t ksg_debug_pack_best(int64_t total, uint32_t pos) { return ksg::pack_best(total, pos); }

uint64_t ksg_debug_gran_a(int32_t which, uint32_t count, uint32_t below, int64_t max_taint, int64_t max_na) {
  return which == 0 ? ksg::gran_a_counts(count, below)
                    : ksg::gran_a_maxima(count, ksg::enc_i64(max_taint), ksg::enc_i64(max_na));
}

int ksg_debug_gran_a_decode(uint64_t g0, uint64_t g1, uint32_t* count, uint32_t* below, int64_t* taint_p1,
                            int64_t* na_p1) {
  if (!count || !below || !taint_p1 || !na_p1) return KSG_EINVAL;
  *count = ksg::gran_a_count(g0);
  *below = ksg::gran_a_below(g0);
  *taint_p1 = (int64_t)ksg::gran_a_tp1(g1);
  *na_p1 = (int64_t)ksg::gran_a_np1(g1);
  return KSG_OK;
}

}  // extern "C"
