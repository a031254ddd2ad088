// engine.cpp -- per-pod compilation into PodDesc programs and batched kernel execution.
//
// compile() does, once per pod and on the host, exactly the O(pod) work the reference's
// PreFilter/PreScore plugins do (cycle-state construction), but against interned cluster
// tables so the per-node work left for the GPU is table lookups:
//   NodeResourcesFit  PreFilter/PreScore  fit.go:136-153,317-335; resource_allocation.go:236-267
//   BalancedAllocation PreScore            balanced_allocation.go:78-100
//   TaintToleration   tolerations -> bitmaps over distinct taints (taint_toleration.go:102-175)
//   NodeAffinity      PreFilter/PreScore  node_affinity.go:148-256 -> selector programs
//   NodePorts         PreFilter            node_ports.go:73-82 -> conflict bitmap over port ids
//   ImageLocality     per-image scaled scores (image_locality.go:141-148)
// run_batch() then launches k_filter_score + k_select per pod on one stream with no host
// round trip inside the batch (device-side AssumePod), and reads the results back once.
#include <algorithm>
#include <unordered_set>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <cstddef>

#include "comm.hpp"
#include "host.hpp"

namespace ksg {

// KSG_HOST_TRACE=1: each rank thread's host steps inside run_batch (microseconds since the process's first
// mark), printed to stderr when the call returns -- where a thread waited while its peers' loops spun.
static bool htrace_on() {
  static const bool on = [] { const char* e = std::getenv("KSG_HOST_TRACE"); return e && *e == '1'; }();
  return on;
}
static thread_local std::string g_htrace;
static void htrace(const char* what, long a = -1) {
  if (!htrace_on()) return;
  static const auto t0 = std::chrono::steady_clock::now();
  char b[96];
  std::snprintf(b, sizeof b, " %.0f:%s%s%ld", std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(),
                what, a >= 0 ? "=" : "", a >= 0 ? a : 0L);
  g_htrace += b;
}
static void htrace_flush(int rank) {
  if (!htrace_on() || g_htrace.empty()) return;
  std::fprintf(stderr, "[htrace rank %d]%s\n", rank, g_htrace.c_str());
  g_htrace.clear();
}

hipError_t launch_filter_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, hipEvent_t t0,
                               hipEvent_t t1, int blk0, int nblk, bool lds);
hipError_t launch_select(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, bool lds);
hipError_t launch_sample(const MirrorView& m, const BatchView& b, int pod, bool cut, hipStream_t s);
hipError_t launch_aggregate(const MirrorView& m, const BatchView& b, int pod, const PodDesc& d, hipStream_t s);
hipError_t launch_eval_pack(const BatchView& b, int n, int cap, int lo, int hi, unsigned long long* g, hipStream_t s);
hipError_t launch_pts_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, int blk0 = 0,
                            int nblk = -1);
hipError_t launch_xpack_a(const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
hipError_t launch_sample_shard_a(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
hipError_t launch_sample_shard_b(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, bool cut,
                                 hipStream_t s);
hipError_t launch_unpack_pts(const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
hipError_t launch_xpack_p(const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
hipError_t launch_select_shard(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
hipError_t launch_commit(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s);
#ifdef KSG_DIAG
hipError_t set_diag(unsigned long long* p);
#endif
hipError_t launch_sched_loop(const MirrorView& m, const BatchView& b, const LoopView& lv, hipStream_t s,
                             hipEvent_t t0, hipEvent_t t1, int unit);
hipError_t launch_agg_loop(const MirrorView& m, const BatchView& b, const AggView& av, hipStream_t s, hipEvent_t t0,
                           hipEvent_t t1);
hipError_t launch_put_group_arg(const LoopGroupArg& a, LoopGroupArg* dst, hipStream_t s);
hipError_t launch_put_group_arg(const AggGroupArg& a, AggGroupArg* dst, hipStream_t s);
hipError_t launch_sched_loop_group(const LoopGroupArg* ga, int world, int nwg, hipStream_t s, hipEvent_t t0,
                                   hipEvent_t t1, int unit);
hipError_t launch_agg_loop_group(const AggGroupArg* ga, int world, int nwg, hipStream_t s, hipEvent_t t0, hipEvent_t t1);
hipError_t warm_kernels();
hipError_t warm_aggregate();
hipError_t launch_ob_hint(const MirrorView& m, const BatchView& b, int pod, hipStream_t s);
hipError_t launch_nominated(const MirrorView& m, const BatchView& b, int pod, hipStream_t s);
hipError_t launch_ob_store(const BatchView& b, int pod, hipStream_t s);
hipError_t launch_ob_remap(ObState* st, ObEnt* h, const int32_t* map, int nold, int maxlen, hipStream_t s);
hipError_t loop_occupancy(int (&occ)[4]);

#define HIPCHK(x)                                               \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      c->err = std::string(#x) + ": " + hipGetErrorString(e_); \
      return KSG_EDEVICE;                                       \
    }                                                           \
  } while (0)

enum : int { P_UNSCHED = 0, P_NODENAME = 1, P_TAINT = 2, P_NA = 3, P_PORTS = 4, P_FIT = 5, P_PTS = 6,
             P_IPA = 7, P_BAL = 8, P_IMG = 9 };

// ---- blob builder ------------------------------------------------------------------------------
// The header is kept outside the byte vector (put() may reallocate it) and copied in by finish().
struct Blob {
  PodDesc hdr;
  std::vector<uint8_t> b;
  Blob() {
    std::memset(&hdr, 0, sizeof(hdr));
    b.resize((sizeof(PodDesc) + 15) & ~size_t(15), 0);
  }
  PodDesc& d() { return hdr; }
  template <typename T>
  int32_t put(const T* p, size_t n) {
    size_t off = (b.size() + 7) & ~size_t(7);
    b.resize(off + sizeof(T) * n, 0);
    if (n) std::memcpy(b.data() + off, p, sizeof(T) * n);
    return (int32_t)off;
  }
  template <typename T>
  int32_t put(const std::vector<T>& v) { return put(v.data(), v.size()); }
  void finish() {
    b.resize((b.size() + 15) & ~size_t(15), 0);
    hdr.blob_bytes = (uint32_t)b.size();
    std::memcpy(b.data(), &hdr, sizeof(hdr));
  }
};

// selector-program builder (labels.Requirement semantics, apimachinery/pkg/labels/selector.go)
struct SelBuilder {
  Cluster* c;
  std::vector<SelReq> reqs;
  std::vector<SelTerm> terms;
  std::vector<int32_t> vals;
  int rc = KSG_OK;

  int32_t slot_of(const std::string& key) {
    int32_t k = c->key_id(key);
    int r = c->ensure_label_slot(k);
    if (r) rc = r;
    return c->keys[k].slot;
  }
  void add_in(SelReq& r, const std::string& key, const std::vector<std::string>& values) {
    int32_t k = c->key_id(key);
    r.vals_off = (int32_t)vals.size();
    for (auto& v : values) {
      int32_t id = c->keys[k].values.find(v);
      if (id >= 0) vals.push_back(id);
    }
    r.nvals = (int32_t)vals.size() - r.vals_off;
  }
  // one labels.Requirement; returns false on a NewRequirement validation error
  bool label_req(const Expr& e, std::vector<SelReq>* out) {
    SelReq r{};
    r.slot = slot_of(e.key);
    bool ok = valid_label_key(e.key);
    if (e.op == "In" || e.op == "NotIn") {
      r.op = e.op == "In" ? SEL_IN : SEL_NOTIN;
      ok = ok && !e.values.empty();
      add_in(r, e.key, e.values);
    } else if (e.op == "Exists" || e.op == "DoesNotExist") {
      r.op = e.op == "Exists" ? SEL_EXISTS : SEL_DNE;
      ok = ok && e.values.empty();
    } else if (e.op == "Gt" || e.op == "Lt") {
      r.op = e.op == "Gt" ? SEL_GT : SEL_LT;
      ok = ok && e.values.size() == 1 && parse_go_int(e.values[0], &r.num);
    } else {
      return false;
    }
    for (auto& v : e.values) ok = ok && valid_label_value(v);
    out->push_back(r);
    return ok;
  }
  // nodeaffinity.newNodeSelectorTerm + nodeSelectorTerm.match (nodeaffinity.go:170-201)
  SelTerm node_term(const NSTerm& t, int32_t weight) {
    SelTerm st{};
    st.weight = weight;
    std::vector<SelReq> rs;
    bool ok = true;
    for (auto& e : t.exprs) ok = label_req(e, &rs) && ok;
    for (auto& f : t.fields) {
      if ((f.op != "In" && f.op != "NotIn") || f.values.size() != 1) { ok = false; continue; }
      SelReq r{};
      const bool in = f.op == "In";
      if (f.key == "metadata.name") {
        r.op = in ? SEL_NODE_EQ : SEL_NODE_NE;
        r.num = c->index_of(f.values[0]);  // -1: no such node, never equal
      } else {  // fields.Set{"metadata.name"}.Get(other) == ""
        const bool eq = f.values[0].empty();
        r.op = (in ? eq : !eq) ? SEL_TRUE : SEL_FALSE;
      }
      rs.push_back(r);
    }
    st.req_off = (int32_t)reqs.size();
    st.nreq = (int32_t)rs.size();
    st.parse_err = ok ? 0 : 1;
    reqs.insert(reqs.end(), rs.begin(), rs.end());
    return st;
  }
};

static bool empty_term(const NSTerm& t) { return t.exprs.empty() && t.fields.empty(); }

// ---- compile ---------------------------------------------------------------------------------------
int Engine::compile(const PodSpec& p, Mode mode, int plugin, bool assume, bool eval, CompiledPod* out,
                    const uint8_t* node_list) {
  const Config& cfg = c->cfg;
  using pclk = std::chrono::steady_clock;
  pclk::time_point pt = cfg.loop_stamps ? pclk::now() : pclk::time_point{};
  auto mark = [&](int k) {
    if (!cfg.loop_stamps) return;
    const pclk::time_point t = pclk::now();
    cprof_[k] += std::chrono::duration<double, std::micro>(t - pt).count();
    pt = t;
  };
  const int32_t N = (int32_t)c->order().size();
  Blob B;
  PodDesc& D = B.d();
  D.node_name = -1;
  D.rot_start = 0;
  D.prefilter_plugin = 15;
  for (int i = 0; i < kNumPlugins; ++i) D.weight[i] = cfg.weight[i];
  *out = CompiledPod{};
  out->num_all = N;

  // ---- which plugins run (PreFilter/PreScore Skip, framework.go:960-962,1324-1327)
  // fmask/smask start as "would run" and lose the plugins whose PreFilter/PreScore Skips;
  // the profile's enabled set is applied per mode at the end.
  uint32_t fmask = (1u << (P_IPA + 1)) - 1u, smask = 0;
  for (int q : {P_TAINT, P_NA, P_FIT, P_PTS, P_IPA, P_BAL, P_IMG}) smask |= 1u << q;

  SelBuilder sb{c};
  // NodeAffinity PreFilter (node_affinity.go:148-198)
  const bool noNA = !p.has_required_na;
  if (noNA && !cfg.has_added_required && !p.has_node_selector) fmask &= ~(1u << P_NA);
  std::vector<int32_t> subset;
  bool restricted = false, conflict = false;
  // (only when the profile runs NodeAffinity: a disabled plugin's PreFilter neither restricts
  // the node list nor rejects, RunPreFilterPlugins framework.go:934-990)
  if (cfg.enabled[P_NA] && !noNA && !p.required_na.empty()) {
    std::set<std::string> names;
    bool namesNil = true, allNodes = false;
    for (auto& t : p.required_na) {
      bool termNil = true;
      std::set<std::string> tn;
      for (auto& r : t.fields)
        if (r.key == "metadata.name" && r.op == "In") {
          std::set<std::string> s(r.values.begin(), r.values.end());
          if (termNil) { tn = s; termNil = false; }
          else {
            std::set<std::string> x;
            for (auto& n : tn)
              if (s.count(n)) x.insert(n);
            tn = x;
          }
        }
      if (termNil) { allNodes = true; break; }
      namesNil = false;
      names.insert(tn.begin(), tn.end());
    }
    if (!allNodes) {
      if (!namesNil && names.empty()) conflict = true;
      else if (!names.empty()) {
        restricted = true;
        for (auto& n : names) {
          int32_t ix = c->index_of(n);
          if (ix >= 0) subset.push_back(ix);
        }
        std::sort(subset.begin(), subset.end());
      }
    }
  }
  if (cfg.has_added_required) {
    std::vector<SelTerm> ts;
    for (auto& t : cfg.added_required)
      if (!empty_term(t)) ts.push_back(sb.node_term(t, 0));
    D.flags |= DF_HAS_ADDED_NA;
    D.na_added.nterm = (int32_t)ts.size();
    D.na_added.term_off = (int32_t)sb.terms.size();
    sb.terms.insert(sb.terms.end(), ts.begin(), ts.end());
  }
  if (!p.node_selector.empty()) {  // labels.SelectorFromSet (no validation)
    SelTerm st{};
    st.req_off = (int32_t)sb.reqs.size();
    for (auto& kv : p.node_selector) {
      SelReq r{};
      r.slot = sb.slot_of(kv.first);
      r.op = SEL_IN;
      sb.add_in(r, kv.first, {kv.second});
      sb.reqs.push_back(r);
    }
    st.nreq = (int32_t)p.node_selector.size();
    D.flags |= DF_HAS_SELECTOR;
    D.na_selector.term_off = (int32_t)sb.terms.size();
    D.na_selector.nterm = 1;
    sb.terms.push_back(st);
  }
  if (p.has_required_na) {
    std::vector<SelTerm> ts;
    for (auto& t : p.required_na)
      if (!empty_term(t)) ts.push_back(sb.node_term(t, 0));
    D.flags |= DF_HAS_REQUIRED_NA;
    D.na_required.term_off = (int32_t)sb.terms.size();
    D.na_required.nterm = (int32_t)ts.size();
    sb.terms.insert(sb.terms.end(), ts.begin(), ts.end());
  }
  // NodeAffinity PreScore (node_affinity.go:242-256): preferred terms, Skip when none
  bool pref_err = false;
  auto pref_prog = [&](const std::vector<std::pair<int32_t, NSTerm>>& in, SelProg* prog, bool pod_terms) {
    std::vector<SelTerm> ts;
    for (auto& t : in) {
      if (t.first == 0 || empty_term(t.second)) continue;
      SelTerm st = sb.node_term(t.second, t.first);
      if (st.parse_err) pref_err |= pod_terms;  // config terms are validated at create
      else ts.push_back(st);
    }
    prog->term_off = (int32_t)sb.terms.size();
    prog->nterm = (int32_t)ts.size();
    sb.terms.insert(sb.terms.end(), ts.begin(), ts.end());
  };
  if (cfg.has_added_pref) {
    D.flags |= DF_HAS_ADDED_PREF;
    pref_prog(cfg.added_pref, &D.na_added_pref, false);
  }
  if (p.has_preferred_na) {
    D.flags |= DF_HAS_PREF_NA;
    pref_prog(p.preferred_na, &D.na_preferred, true);
  }
  if (!p.has_preferred_na && !cfg.has_added_pref) smask &= ~(1u << P_NA);
  if (sb.rc) return sb.rc;

  mark(0);
  // NodeName (node_name.go:67-83)
  if (!p.node_name.empty()) {
    int32_t ix = c->index_of(p.node_name);
    D.node_name = ix >= 0 ? ix : -2;
  }
  // evaluateNominatedNode (schedule_one.go:657-669,714-745): a status.nominatedNodeName in the snapshot is tried
  // alone first (k_nominated); one that is not is an error the reference logs before the full pass
  if (mode == CYCLE && !p.nominated_node.empty()) {
    const int32_t ix = c->index_of(p.nominated_node);
    if (ix >= 0) {
      D.flags |= DF_NOMINATED;
      D.nominated_node = ix;
    }
  }

  // TaintToleration: per distinct taint, "not tolerated" bits (taint_toleration.go:102-196)
  bool any_intol = false;  // some PreferNoSchedule taint of the cluster is not tolerated (raw scores can be > 0)
  {
    const size_t T = c->taints.size();
    const int32_t words = (int32_t)((T + 31) / 32);
    std::vector<uint32_t> untol(words, 0), intol(words, 0);
    std::vector<const Tol*> pref;
    for (auto& t : p.tolerations)
      if (t.effect.empty() || t.effect == "PreferNoSchedule") pref.push_back(&t);
    for (size_t id = 0; id < T; ++id) {
      const TaintRec& tr = c->taints[id];
      if (tr.effect == "NoSchedule" || tr.effect == "NoExecute") {
        bool ok = false;
        for (auto& t : p.tolerations) ok = ok || tolerates(t, tr.key, tr.value, tr.effect, cfg.taint_cmp_ops);
        if (!ok) untol[id / 32] |= 1u << (id % 32);
      } else if (tr.effect == "PreferNoSchedule") {
        bool ok = false;
        for (auto* t : pref) ok = ok || tolerates(*t, tr.key, tr.value, tr.effect, cfg.taint_cmp_ops);
        if (!ok) intol[id / 32] |= 1u << (id % 32);
      }
    }
    D.n_taint_words = words;
    D.untol_ns_off = B.put(untol);
    D.intol_pns_off = B.put(intol);
    for (uint32_t x : intol) any_intol = any_intol || x != 0;
    for (auto& t : p.tolerations)  // NodeUnschedulable (node_unschedulable.go:133-138)
      if (tolerates(t, "node.kubernetes.io/unschedulable", "", "NoSchedule", cfg.taint_cmp_ops)) D.flags |= DF_TOLERATES_UNSCHED;
  }

  // NodePorts PreFilter (node_ports.go:73-82) -> conflict bitmap over distinct port ids
  std::vector<HostPort> want;
  for (auto& k : p.init_containers)
    if (k.sidecar)
      for (auto& hp : k.ports)
        if (hp.port > 0) want.push_back(hp);
  for (auto& k : p.containers)
    for (auto& hp : k.ports)
      if (hp.port > 0) want.push_back(hp);
  if (want.empty()) fmask &= ~(1u << P_PORTS);
  std::vector<uint32_t> own;
  for (auto& hp : want) own.push_back(c->port_id(hp.ip, hp.proto, hp.port));
  {
    const size_t P = c->ports.size();
    const int32_t words = (int32_t)((P + 31) / 32);
    std::vector<uint32_t> conf(words, 0);
    for (size_t id = 0; id < P; ++id) {
      const PortRec& pr = c->ports[id];
      bool hit = false;
      for (auto& w : want) {  // HostPortInfo.CheckConflict (kube-scheduler/framework/types.go:603-631)
        std::string ip = w.ip.empty() ? "0.0.0.0" : w.ip, proto = w.proto.empty() ? "TCP" : w.proto;
        if (proto != pr.proto || w.port != pr.port) continue;
        if (ip == "0.0.0.0" || pr.ip == "0.0.0.0" || pr.ip == ip) hit = true;
      }
      if (hit) conf[id / 32] |= 1u << (id % 32);
    }
    D.n_port_words = words;
    D.port_conflict_off = B.put(conf);
    std::sort(own.begin(), own.end());
    own.erase(std::unique(own.begin(), own.end()), own.end());
    D.n_pod_ports = (int32_t)own.size();
    D.pod_ports_off = B.put(own);
  }

  mark(1);
  // NodeResourcesFit PreFilter (fit.go:317-335: the spec's requests) and the assume payload
  // (CalculateResource, framework/types.go:1035-1076: a resized pod's status resources count too; the
  // two differ only for a pod that carries status resources)
  const PodResources res = calc_resources(p);
  const PodResources fit = p.has_status_res ? calc_fit_request(p) : res;
  out->res = res;
  if (mode == CYCLE && ob_acting()) {  // SignPod: the pod takes part in OpportunisticBatching
    out->sig = sign(p, fit);
    if (out->sig >= 0) D.flags |= DF_OB;
  }
  out->port_ids = own;
  D.req_cpu = fit.cpu;
  D.req_mem = fit.mem;
  D.req_eph = fit.eph;
  std::vector<ScalarReq> fsr, asr;
  for (auto& s : res.scalar) {
    int32_t slot = c->scalar_slot(s.first);
    if (slot < 0) { c->err = "too many extended resources"; return KSG_ENOTSUP; }
    asr.push_back({slot, 0, s.second});
  }
  for (auto& s : fit.scalar) {
    int32_t slot = c->scalar_slot(s.first);
    if (slot < 0) { c->err = "too many extended resources"; return KSG_ENOTSUP; }
    if (s.second == 0) continue;
    const bool extended = s.first.find('/') != std::string::npos && s.first.find("kubernetes.io/") == std::string::npos;
    if (extended) {
      std::string prefix = s.first.substr(0, s.first.find('/'));
      if (cfg.ignored_res.count(s.first) || cfg.ignored_groups.count(prefix)) continue;
    }
    fsr.push_back({slot, 0, s.second});
  }
  D.fit_any = (fit.cpu > 0 || fit.mem > 0 || fit.eph > 0 || !fit.scalar.empty()) ? 1 : 0;
  D.n_scalar = (int32_t)fsr.size();
  D.scalar_off = B.put(fsr);
  D.a_cpu = res.cpu;
  D.a_mem = res.mem;
  D.a_eph = res.eph;
  D.a_nz_cpu = res.nz_cpu;
  D.a_nz_mem = res.nz_mem;
  D.n_a_scalar = (int32_t)asr.size();
  D.a_scalar_off = B.put(asr);

  // NodeResourcesFit / BalancedAllocation PreScore (resource_allocation.go:167-267)
  auto score_res = [&](const std::vector<std::pair<std::string, int64_t>>& specs, bool useRequested,
                       bool* best_effort) {
    std::vector<ScoreRes> v;
    ResVec nm;
    if (!useRequested) nm = {{"cpu", 100}, {"memory", 200LL * 1024 * 1024 * 1000}};
    const ResVec reqs = pod_requests(p, useRequested ? nullptr : &nm, true);  // resource_allocation.go:236-259
    *best_effort = true;
    for (auto& sp : specs) {
      ScoreRes r{};
      r.weight = sp.second;
      int64_t m = 0;
      for (auto& x : reqs)
        if (x.name == sp.first) m = x.milli;
      r.pod_req = sp.first == "cpu" ? m : milli_ceil(m);
      if (r.pod_req != 0) *best_effort = false;
      if (sp.first == "cpu") r.kind = RES_CPU;
      else if (sp.first == "memory") r.kind = RES_MEM;
      else if (sp.first == "ephemeral-storage") r.kind = RES_EPH;
      else if (scalar_resource(sp.first)) {
        if (r.pod_req == 0) r.kind = RES_SKIP;
        else {
          int32_t slot = c->scalar_slot(sp.first);
          r.kind = slot >= 0 ? RES_SCALAR : RES_SKIP;
          r.slot = slot;
        }
      } else {
        r.kind = RES_SKIP;  // no such allocatable: (0, 0) -> skipped
      }
      v.push_back(r);
    }
    return v;
  };
  bool be_fit, be_bal;
  std::vector<ScoreRes> fr = score_res(cfg.fit_res, false, &be_fit);
  std::vector<ScoreRes> br = score_res(cfg.bal_res, true, &be_bal);
  if (br.size() > 8 || fr.size() > 64) { c->err = "too many scoring resources"; return KSG_ENOTSUP; }
  D.fit_strategy = cfg.fit_strategy;
  D.n_fit_res = (int32_t)fr.size();
  D.fit_res_off = B.put(fr);
  D.n_bal_res = (int32_t)br.size();
  D.bal_res_off = B.put(br);
  std::vector<int64_t> shape;
  for (auto& pt : cfg.rtcr) { shape.push_back(pt.first); shape.push_back(pt.second); }
  D.n_rtcr = (int32_t)cfg.rtcr.size();
  D.rtcr_off = B.put(shape);
  if (be_bal) smask &= ~(1u << P_BAL);  // balanced_allocation.go:80-85

  // ImageLocality (image_locality.go:70-152)
  {
    std::vector<std::string> names;
    for (auto& k : p.init_containers) names.push_back(k.image);
    for (auto& k : p.containers) names.push_back(k.image);
    for (auto& v : p.image_volumes) names.push_back(v);
    std::vector<ImageTerm> terms;
    for (auto& nm : names) {
      std::string n = nm;  // normalizedImageName (:154-159)
      auto colon = n.rfind(':'), slash = n.rfind('/');
      long lc = colon == std::string::npos ? -1 : (long)colon, ls = slash == std::string::npos ? -1 : (long)slash;
      if (lc <= ls) n += ":latest";
      auto st = c->image_states.find(n);
      if (st == c->image_states.end()) continue;
      int32_t id = c->image_ix.find(n);
      auto it = std::find_if(terms.begin(), terms.end(), [&](const ImageTerm& t) { return t.image == id; });
      if (it != terms.end()) { it->mult++; continue; }
      const double spread = (double)(int64_t)st->second.nodes.size() / (double)N;
      terms.push_back({id, 1, (int64_t)((double)st->second.size * spread)});
    }
    D.n_img = (int32_t)terms.size();
    D.img_off = B.put(terms);
    D.img_count = (int64_t)names.size();
  }

  mark(2);
  // PodTopologySpread / InterPodAffinity: per-domain aggregation programs
  {
    const int rc = compile_topology(p, mode, plugin, N, &B, &D, &fmask, &smask, out);
    if (rc) return rc;
  }
  mark(3);

  // selector program pools
  D.req_off = B.put(sb.reqs);
  D.vals_off = B.put(sb.vals);
  const int32_t term_base = B.put(sb.terms);
  for (SelProg* pr : {&D.na_required, &D.na_selector, &D.na_added, &D.na_preferred, &D.na_added_pref})
    pr->term_off = term_base + pr->term_off * (int32_t)sizeof(SelTerm);
  // selector terms hold req offsets in units of SelReq; vals_off in units of int32 (kernel indexes arrays)

  // ---- mode-specific masks
  // PreScore/Score errors: NodeAffinity preferred-term parse error (node_affinity.go:243-246),
  // NodeResourcesFit with no scoring resources (resource_allocation.go:149-151)
  const bool score_err = (pref_err && cfg.enabled[P_NA]) || (cfg.enabled[P_FIT] && cfg.fit_res.empty());
  if (mode == CYCLE) {
    for (int q = 0; q < kNumPlugins; ++q)
      if (!cfg.enabled[q]) { fmask &= ~(1u << q); smask &= ~(1u << q); }
    bool any_score = false;
    for (int q : {P_TAINT, P_NA, P_FIT, P_PTS, P_IPA, P_BAL, P_IMG}) any_score |= cfg.enabled[q];
    // percentageOfNodesToScore / a profile without score plugins: nextStartNodeIndex then depends
    // on where the filter pass stopped, so it lives on the device (DF_ROTDEV, k_sample_find)
    if (!any_score) D.flags |= DF_NO_SCORE;
    if (rotdev()) D.flags |= DF_ROTDEV;
    if (score_err) D.flags |= DF_SCORE_ERROR;
    if (conflict || (!out->prefilter_error && out->ipa_parse_error)) {
      // PreFilter UnschedulableAndUnresolvable (NodeAffinity conflict, InterPodAffinity parse):
      // every node gets it (schedule_one.go:635-648)
      const int32_t pl = conflict ? P_NA : P_IPA;
      D.flags |= DF_PREFILTER_REJECT;
      D.prefilter_code = 3;
      D.prefilter_plugin = pl;
      out->prefilter_reject = true;
      out->prefilter_code = 3;
      out->prefilter_plugin = pl;
      out->prefilter_error = false;
    } else if (out->prefilter_error) {
      // PodTopologySpread PreFilter Error: the cycle errors before filtering (run_batch)
    } else if (restricted) {
      D.flags |= DF_SUBSET;
      D.subset_cnt = (int32_t)subset.size();
      D.subset_off = B.put(subset);
      out->num_all = (int32_t)subset.size();
      if (!subset.empty()) D.rot_start = subset[(size_t)(c->next_start % (int64_t)subset.size())];
    } else {
      D.rot_start = N ? (int32_t)(c->next_start % N) : 0;
    }
    // numFeasibleNodesToFind (schedule_one.go:778-782,858-884) over len(nodes)
    const int32_t num_all = out->num_all;
    int64_t k = num_all;
    if (num_all >= 100) {
      int64_t pct = cfg.pct;
      if (pct == 0) pct = std::max<int64_t>(5, 50 - num_all / 125);
      k = std::max<int64_t>(100, (int64_t)num_all * pct / 100);
    }
    if (!any_score) k = 1;
    D.num_to_find = (int32_t)std::min<int64_t>(k, INT32_MAX);
    if ((D.flags & DF_ROTDEV) && k < num_all && !(D.flags & DF_PREFILTER_REJECT)) D.flags |= DF_SAMPLE;
  } else if (mode == FILTER_ONE) {
    fmask &= 1u << plugin;
    if ((plugin == P_PTS && out->prefilter_error) || (plugin == P_IPA && out->ipa_parse_error)) {
      out->prefilter_reject = true;
      out->prefilter_code = plugin == P_PTS ? 1 : 3;
      out->prefilter_plugin = plugin;
    }
    if (plugin == P_NA && conflict) {
      out->prefilter_reject = true;
      out->prefilter_code = 3;
      out->prefilter_plugin = P_NA;
    }
    smask = 0;
    eval = true;
  } else {  // SCORE_ONE
    if ((plugin == P_NA && pref_err) || (plugin == P_FIT && cfg.fit_res.empty()) || out->topo_score_error)
      out->error = true;
    fmask = 0;
    smask &= 1u << plugin;
    for (int i = 0; i < kNumPlugins; ++i) D.weight[i] = 1;
    D.flags |= DF_ALL_FEASIBLE;
    if (node_list) {
      std::vector<uint32_t> bm((size_t)(N + 31) / 32, 0);
      for (int32_t i = 0; i < N; ++i)
        if (node_list[i]) bm[(size_t)i / 32] |= 1u << (i % 32);
      D.flags |= DF_NODE_LIST;
      D.node_list_off = B.put(bm);
    }
    eval = true;
  }
  D.filter_mask = fmask;
  D.score_mask = smask;
  out->score_mask = smask;
  // raw TaintToleration / NodeAffinity scores are 0 on every node: nothing intolerable to count, no terms to weigh
  if ((!((smask >> P_TAINT) & 1u) || !any_intol) &&
      (!((smask >> P_NA) & 1u) || (D.na_preferred.nterm == 0 && D.na_added_pref.nterm == 0)))
    D.flags |= DF_RAW0;
  if (assume) {
    D.flags |= DF_ASSUME;
    // live once k_select's assume writes its node index; a pipelined batch reserved it up front
    D.slot = next_slot_ >= 0 ? next_slot_ : c->pod_table_put(p, -1);
    out->slot = D.slot;
    // the pod's own affinity terms: k_agg_loop's owner of its node adds them when it is assumed
    const std::vector<int32_t>& own = c->pt_terms[(size_t)D.slot];
    D.n_own_terms = (int32_t)own.size();
    D.own_terms_off = B.put(own);
    out->own_terms = D.n_own_terms;
  }
  if (eval) D.flags |= DF_EVAL_OUT;
  // DF_FAST: the straight-line default-plugin evaluation (kernels.hip eval_node_fast)
  {
    const uint32_t topo = (1u << P_PTS) | (1u << P_IPA);
    const bool shape = fr.size() == 2 && fr[0].kind == RES_CPU && fr[1].kind == RES_MEM && br.size() == 2 &&
                       br[0].kind == RES_CPU && br[1].kind == RES_MEM && (cfg.fit_strategy == 0 || cfg.fit_strategy == 1);
    // PodTopologySpread / InterPodAffinity filters with nothing to check (no constraints, no terms,
    // no existing anti-affinity) leave their mask bits set but never reject: not a reason to leave
    const bool topo_filter = D.n_ptsf > 0 || D.n_raff > 0 || D.n_ranti > 0 || (D.ipa_flags & IPA_EXIST_FILTER);
    if (mode == CYCLE && shape && D.n_scalar == 0 && !topo_filter && !(smask & topo) &&
        !(D.flags & (DF_PREFILTER_REJECT | DF_SUBSET | DF_ALL_FEASIBLE | DF_AGGREGATE | DF_SCORE_ERROR)) &&
        c->alloc_bound < ((int64_t)1 << 52) / 100)
      D.flags |= DF_FAST;
    if (mode == CYCLE && shape && D.n_scalar == 0 &&
        !(D.flags & (DF_PREFILTER_REJECT | DF_SUBSET | DF_ALL_FEASIBLE | DF_SCORE_ERROR | DF_ROTDEV)) &&
        c->alloc_bound < ((int64_t)1 << 52) / 100)
      D.flags |= DF_LFAST;
  }
  if (p.terminating) D.flags |= DF_TERMINATING;
  B.finish();
  out->blob = std::move(B.b);
  mark(4);
  return KSG_OK;
}

// ---- PodTopologySpread / InterPodAffinity compilation ----------------------------------------------------
// The O(pod) half of calPreFilterState / initPreScoreState (podtopologyspread/filtering.go:237-311,
// scoring.go:61-115) and of the InterPodAffinity PreFilter/PreScore (interpodaffinity/filtering.go:286-321,
// scoring.go:128-221): constraints and terms become selector programs over interned labels, and every
// per-domain map of the reference becomes an arena histogram indexed by the topology key's value id.
int Engine::compile_topology(const PodSpec& p, Mode mode, int plugin, int32_t N, Blob* Bp, PodDesc* Dp,
                             uint32_t* fmask, uint32_t* smask, CompiledPod* out) {
  Blob& B = *Bp;
  PodDesc& D = *Dp;
  const Config& cfg = c->cfg;
  using pclk = std::chrono::steady_clock;
  pclk::time_point pt = cfg.loop_stamps ? pclk::now() : pclk::time_point{};
  auto mark = [&](int k) {
    if (!cfg.loop_stamps) return;
    const pclk::time_point t = pclk::now();
    cprof_[k] += std::chrono::duration<double, std::micro>(t - pt).count();
    pt = t;
  };
  // the plugins this evaluation actually runs (profile in CYCLE mode, the one plugin otherwise)
  uint32_t* const fmask_caller = fmask;
  uint32_t* const smask_caller = smask;
  uint32_t fm = *fmask, sm = *smask;
  if (mode == CYCLE) {
    for (int q = 0; q < kNumPlugins; ++q)
      if (!cfg.enabled[q]) { fm &= ~(1u << q); sm &= ~(1u << q); }
  } else if (mode == FILTER_ONE) {
    fm &= 1u << plugin;
    sm = 0;
  } else {
    fm = 0;
    sm &= 1u << plugin;
  }
  const uint32_t fm_in = fm, sm_in = sm;
  fmask = &fm;
  smask = &sm;
  std::vector<int32_t> pool;  // selector programs + namespace id lists
  int32_t arena = 0;
  struct HistRec { int32_t base, n, key; bool pres; };
  std::vector<HistRec> hists;  // every histogram of the arena (k_agg_loop's placement below)
  auto alloc = [&](int32_t n, int32_t key, bool pres) {
    const int32_t b = arena;
    arena += n;
    hists.push_back({b, n, key, pres});
    return b;
  };
  auto nvals = [&](int32_t key) { return (int32_t)c->keys[key].values.strs.size(); };
  auto slot_of = [&](int32_t key) -> int32_t {
    c->ensure_label_slot(key);
    return c->keys[key].slot;
  };
  const std::vector<unsigned long long> podset = c->label_set(p.labels);
  D.ns_id = c->ns_id(p.ns);
  D.slot = -1;

  // ---------------- PodTopologySpread (filterTopologySpreadConstraints, common.go:87-128)
  // A pod without constraints of its own gets the plugin's default constraints (getConstraints,
  // filtering.go:220-235; buildDefaultConstraints, common.go:59-75), whose selector is
  // helper.DefaultSelector over the Services / RCs / RSs / StatefulSets selecting the pod; an Empty
  // selector means no constraint at all.
  const bool use_defaults = p.spreads.empty() && !cfg.pts_defaults.empty();
  LabelSel dsel;
  bool dsel_done = false, dsel_ok = false;
  // requireAllTopologies = len(pod.Spec.TopologySpreadConstraints) > 0 || !systemDefaulted (scoring.go:141-144):
  // system-defaulted scoring ignores no node, and a node without the key is in the "" domain
  const bool anytopo = use_defaults && cfg.pts_system_defaulted;
  auto build_cons = [&](const char* action, std::vector<PtsCons>* cons, bool score) -> bool {
    const std::vector<Spread>& src = use_defaults ? cfg.pts_defaults : p.spreads;
    for (auto& sp : src) {
      if (sp.when != action) continue;
      PtsCons pc{};
      if (use_defaults) {
        if (!dsel_done) {
          dsel_ok = c->default_selector(p, &dsel);
          dsel_done = true;
        }
        if (!dsel_ok) return true;  // selector.Empty(): no default constraints (common.go:65-67)
        if (!c->compile_lsel(dsel, nullptr, &pool, &pc.sel, true)) return false;
      } else {
        StrMap ml;
        for (auto& k : sp.match_label_keys)  // MatchLabelKeysInPodTopologySpread (on by default)
          for (auto& kv : p.labels)
            if (kv.first == k) ml.push_back(kv);
        std::sort(ml.begin(), ml.end());
        if (!c->compile_lsel(sp.sel, sp.sel.present ? &ml : nullptr, &pool, &pc.sel)) return false;
      }
      const int32_t key = c->key_id(sp.key);
      pc.slot = slot_of(key);
      pc.max_skew = sp.max_skew;
      pc.min_domains = sp.min_domains;
      pc.self_match = lsel_match(pool.data() + pc.sel, podset.data(), (int32_t)podset.size()) ? 1 : 0;
      pc.aff_honor = sp.aff_honor ? 1 : 0;
      pc.taint_honor = sp.taint_honor ? 1 : 0;
      pc.hostname = (score && sp.key == "kubernetes.io/hostname") ? 1 : 0;
      pc.nvals = pc.hostname ? N : nvals(key);
      pc.absent = -1;
      if (score && anytopo && !pc.hostname) {
        // a node without the key counts in the "" domain: its value id if some node carries key="",
        // else one extra histogram entry past the interned values
        const int32_t e = c->keys[key].values.find("");
        pc.absent = e >= 0 ? e : pc.nvals++;
      }
      pc.hist_base = alloc(pc.nvals, key, false);
      pc.pres_base = pc.hostname ? -1 : alloc(pc.nvals, key, true);
      cons->push_back(pc);
    }
    return true;
  };
  std::vector<PtsCons> ptsf, ptss;
  if (*fmask & (1u << P_PTS)) {
    if (!build_cons("DoNotSchedule", &ptsf, false)) {  // PreFilter Error (filtering.go:146-148)
      out->prefilter_error = true;
      ptsf.clear();
    }
    if (ptsf.empty()) *fmask &= ~(1u << P_PTS);  // PreFilter Skip: no hard constraints
  }
  if (*smask & (1u << P_PTS)) {
    if (!build_cons("ScheduleAnyway", &ptss, true)) {
      out->topo_score_error = true;  // PreScore Error (scoring.go:132-134)
      D.flags |= DF_SCORE_ERROR;
      ptss.clear();
    }
    if (ptss.empty() || N == 0) *smask &= ~(1u << P_PTS);
    if (!ptss.empty() && anytopo) D.flags |= DF_PTS_ANYTOPO;
  }
  if (ptsf.size() > (size_t)kMaxCons || ptss.size() > (size_t)kMaxCons) {
    c->err = "more topology spread constraints than the device path supports";
    return KSG_ENOTSUP;
  }

  mark(5);
  // ---------------- InterPodAffinity (framework.NewPodInfo for the incoming pod)
  const bool ipa_f = (*fmask >> P_IPA) & 1u, ipa_s = (*smask >> P_IPA) & 1u;
  std::vector<IpaTerm> raff, ranti, paff, panti;
  std::map<int32_t, int32_t> aff_base, anti_base, topo_base, exanti_base;
  bool parse_ok = true;
  auto own_terms = [&](const std::vector<PATerm>& in, std::vector<IpaTerm>* o, std::map<int32_t, int32_t>* bases,
                       bool pref) {
    for (auto& t : in) {
      IpaTerm it{};
      it.weight = t.weight;
      int32_t nssel;
      if (!c->compile_lsel(t.sel, nullptr, &pool, &it.sel) || !c->compile_lsel(t.ns_sel, nullptr, &pool, &nssel)) {
        parse_ok = false;
        return;
      }
      static const unsigned long long kNone = 0;
      it.all_ns = lsel_match(pool.data() + nssel, &kNone, 0) ? 1 : 0;
      // namespaces (types.go:422-448) merged with the namespaces the selector matches
      // (mergeAffinityTermNamespacesIfNotEmpty, interpodaffinity/plugin.go:134-147)
      std::vector<int32_t> ns;
      if (t.namespaces.empty() && !t.ns_sel.present) ns.push_back(c->ns_id(p.ns));
      else
        for (auto& n : t.namespaces) ns.push_back(c->ns_id(n));
      if (!lsel_empty(pool.data() + nssel))
        for (auto& kv : c->namespaces) {
          const auto nl = c->label_set(kv.second.labels);
          if (lsel_match(pool.data() + nssel, nl.data(), (int32_t)nl.size())) ns.push_back(c->ns_id(kv.first));
        }
      it.ns_off = (int32_t)pool.size();
      it.ns_cnt = (int32_t)ns.size();
      pool.insert(pool.end(), ns.begin(), ns.end());
      const int32_t key = c->key_id(t.topo);
      it.slot = slot_of(key);
      auto b = bases->find(key);
      if (b == bases->end()) b = bases->emplace(key, alloc(nvals(key), key, false)).first;
      it.hist_base = b->second;
      it.nvals = nvals(key);
      (void)pref;
      o->push_back(it);
    }
  };
  const bool hasConstraints =
      (p.has_pod_affinity && !p.aff_pref.empty()) || (p.has_pod_anti && !p.anti_pref.empty());  // scoring.go:148-150
  if (ipa_f || ipa_s) {
    std::vector<IpaTerm> tmp;
    std::map<int32_t, int32_t> scratch;
    // parse check of every category first (NewPodInfo fails as a whole)
    if (p.has_pod_affinity) own_terms(p.aff_req, &raff, &aff_base, false);
    if (p.has_pod_anti) own_terms(p.anti_req, &ranti, &anti_base, false);
    if (p.has_pod_affinity) own_terms(p.aff_pref, &paff, &topo_base, true);
    if (p.has_pod_anti) own_terms(p.anti_pref, &panti, &topo_base, true);
    if (!parse_ok) {
      raff.clear(); ranti.clear(); paff.clear(); panti.clear();
      if (ipa_f) out->ipa_parse_error = true;  // PreFilter UnschedulableAndUnresolvable (filtering.go:294-296)
      if (ipa_s) {                             // PreScore Error (scoring.go:176-179)
        D.flags |= DF_SCORE_ERROR;
        out->topo_score_error = true;
      }
    }
    if (raff.size() > (size_t)kMaxPodTerms || ranti.size() > (size_t)kMaxPodTerms ||
        paff.size() > (size_t)kMaxPodTerms || panti.size() > (size_t)kMaxPodTerms) {
      c->err = "more pod (anti-)affinity terms than the device path supports";
      return KSG_ENOTSUP;
    }
    out->ipa_own_req = !raff.empty() || !ranti.empty();
    bool self_all = !raff.empty();
    for (auto& t : raff)
      self_all = self_all && (t.all_ns || id_in(pool.data() + t.ns_off, t.ns_cnt, D.ns_id)) &&
                 lsel_match(pool.data() + t.sel, podset.data(), (int32_t)podset.size());
    if (self_all) D.ipa_flags |= IPA_SELF_ALL;
    if (!ipa_f) { raff.clear(); ranti.clear(); }
    if (ipa_f && parse_ok && !c->exanti_keys.empty()) {
      D.ipa_flags |= IPA_EXIST_FILTER;
      for (auto& kv : c->exanti_keys) exanti_base[kv.first] = alloc(nvals(kv.first), kv.first, false);
    }
    // PreScore: IgnorePreferredTermsOfExistingPods && !hasConstraints -> Skip (scoring.go:152-156)
    if (ipa_s && cfg.ignore_pref_existing && !hasConstraints) *smask &= ~(1u << P_IPA);
    if ((*smask >> P_IPA) & 1u) {
      if (hasConstraints && parse_ok) D.ipa_flags |= IPA_PREF;
      else { paff.clear(); panti.clear(); }
      std::set<int32_t> ekeys;
      if (cfg.hard_weight > 0)
        for (auto& kv : c->score_keys_req) ekeys.insert(kv.first);
      for (auto& kv : c->score_keys_pref) ekeys.insert(kv.first);
      if (!ekeys.empty() && parse_ok) D.ipa_flags |= IPA_EXIST_SCORE;
      for (int32_t k : ekeys)
        if (!topo_base.count(k)) topo_base[k] = alloc(nvals(k), k, false);
      // Neither the pod's preferred terms nor any existing pod's scoring terms can add to
      // topologyScore, so it stays empty and PreScore returns Skip (scoring.go:207-209) -- known
      // here without counting anything on the device.
      if (!(D.ipa_flags & (IPA_PREF | IPA_EXIST_SCORE)) && !(D.flags & DF_SCORE_ERROR)) *smask &= ~(1u << P_IPA);
    } else {
      paff.clear();
      panti.clear();
    }
  }
  D.hard_weight = cfg.hard_weight;
  mark(6);

  // k_agg_loop's placement of every histogram (AggRef, desc.h): a key whose values are each on one
  // node only keeps per-node counts with the node's owner workgroup (its presence flags are not
  // needed: every eligible node is its own domain); any other key's histogram goes to the pod's
  // compact shared region, summed over workgroups.  A pod that does not fit takes the launch path.
  std::unordered_map<int32_t, int32_t> ref;  // arena base -> AggRef
  int32_t gwords = 0, nlocal = 0;
  for (auto& h : hists) {
    const bool uniq = c->key_unique(h.key);
    if (uniq && h.pres) ref[h.base] = -1 - kAggLocal;  // never read
    else if (uniq) ref[h.base] = -1 - nlocal++;
    else {
      ref[h.base] = gwords;
      gwords += h.n;
    }
  }
  auto aref = [&](int32_t b) { return b < 0 ? 0 : ref.at(b); };
  int32_t local_cons = 0, nlc = 0;
  for (size_t k = 0; k < ptsf.size(); ++k) {
    ptsf[k].lref = aref(ptsf[k].hist_base);
    ptsf[k].pref = aref(ptsf[k].pres_base);
    if (ptsf[k].lref < 0) {
      local_cons |= 1 << k;
      ++nlc;
    }
  }
  for (auto* v : {&raff, &ranti, &paff, &panti})
    for (auto& t : *v) t.lref = aref(t.hist_base);
  for (auto& pc : ptss) {
    pc.lref = aref(pc.hist_base);
    pc.pref = aref(pc.pres_base);
  }
  D.agg_gwords = gwords;
  D.agg_nlocal = nlocal;
  D.agg_local_cons = local_cons;
  // ScheduleAnyway constraints in k_agg_loop: per-node counts of at most kAggScoreCons constraints in LDS,
  // their domains as presence bits in exchange A, raw scores < 2^24 in exchange PX
  bool pts_loop = ptss.size() <= (size_t)kAggScoreCons;
  {
    int32_t bits = 0;
    double raw_bound = 0;
    const double cnt_bound = (double)c->pt_node.size() + (double)kLoopMaxPods + 1.0;
    for (auto& pc : ptss) {
      pc.pbit = pc.hostname ? -1 : bits;
      bits += pc.hostname ? 0 : pc.nvals;
      raw_bound += cnt_bound * go_log((double)N + 3.0) + (double)pc.max_skew;
    }
    pts_loop = pts_loop && bits <= kAggPresBits && raw_bound < (double)kAggPtsRawMax;
  }
  out->agg_ok = pts_loop && nlocal <= kAggLocal && gwords <= kAggGWords && nlc <= kAggLocalCons &&
                ptsf.size() <= (size_t)kAggMaxCons && raff.size() <= (size_t)kAggMaxTerms &&
                ranti.size() <= (size_t)kAggMaxTerms && paff.size() <= (size_t)kAggMaxTerms &&
                panti.size() <= (size_t)kAggMaxTerms;

  // key table for the existing-term pass: {label slot, existing-anti base, topology-score base, AggRefs}
  std::vector<int32_t> keytab;
  if (!exanti_base.empty() || ((D.ipa_flags & IPA_EXIST_SCORE) != 0)) {
    const int32_t nk = (int32_t)c->label_keys.strs.size();
    keytab.assign((size_t)nk * kKeytabStride, -1);
    for (auto& kv : exanti_base) {
      keytab[(size_t)kv.first * kKeytabStride] = slot_of(kv.first);
      keytab[(size_t)kv.first * kKeytabStride + 1] = kv.second;
      keytab[(size_t)kv.first * kKeytabStride + 3] = aref(kv.second);
    }
    for (auto& kv : topo_base) {
      keytab[(size_t)kv.first * kKeytabStride] = slot_of(kv.first);
      keytab[(size_t)kv.first * kKeytabStride + 2] = kv.second;
      keytab[(size_t)kv.first * kKeytabStride + 4] = aref(kv.second);
    }
    D.n_keytab = nk;
  }
  std::vector<KeyHist> exkeys, topokeys;
  for (auto& kv : exanti_base) exkeys.push_back({c->keys[kv.first].slot, kv.second, aref(kv.second), 0});
  for (auto& kv : topo_base) topokeys.push_back({c->keys[kv.first].slot, kv.second, aref(kv.second), 0});

  const bool agg = !ptsf.empty() || !ptss.empty() || !raff.empty() || !ranti.empty() || !exkeys.empty() ||
                   ((*smask >> P_IPA) & 1u);
  if (agg) D.flags |= DF_AGGREGATE;
  D.n_lbl = (int32_t)podset.size();
  D.lbl_off = B.put(podset);
  {
    std::vector<unsigned long long> nsl;
    auto it = c->namespaces.find(p.ns);  // GetNamespaceLabelsSnapshot (interpodaffinity/plugin.go:150-159)
    if (it != c->namespaces.end()) nsl = c->label_set(it->second.labels);
    D.n_nslbl = (int32_t)nsl.size();
    D.nslbl_off = B.put(nsl);
  }
  D.sel_pool_off = B.put(pool);
  D.n_ptsf = (int32_t)ptsf.size();
  D.ptsf_off = B.put(ptsf);
  D.n_ptss = (int32_t)ptss.size();
  D.ptss_off = B.put(ptss);
  D.n_raff = (int32_t)raff.size();
  D.raff_off = B.put(raff);
  D.n_ranti = (int32_t)ranti.size();
  D.ranti_off = B.put(ranti);
  D.n_paff = (int32_t)paff.size();
  D.paff_off = B.put(paff);
  D.n_panti = (int32_t)panti.size();
  D.panti_off = B.put(panti);
  D.keytab_off = B.put(keytab);
  D.n_exkeys = (int32_t)exkeys.size();
  D.exkeys_off = B.put(exkeys);
  D.n_topokeys = (int32_t)topokeys.size();
  D.topokeys_off = B.put(topokeys);
  D.arena_words = arena;
  out->arena_words = arena;
  // Skips decided here propagate to the caller's masks (PTS without constraints, IPA ignore rule)
  for (int q : {P_PTS, P_IPA}) {
    if (((fm_in >> q) & 1u) && !((fm >> q) & 1u)) *fmask_caller &= ~(1u << q);
    if (((sm_in >> q) & 1u) && !((sm >> q) & 1u)) *smask_caller &= ~(1u << q);
  }
  mark(7);
  return KSG_OK;
}

// ---- batch execution ---------------------------------------------------------------------------------
Engine::Engine(Cluster* cl) : c(cl) {
  (void)hipEventCreate(&ev0);
  (void)hipEventCreate(&ev1);
  if (hipDeviceGetAttribute(&cu_count, hipDeviceAttributeMultiprocessorCount, c->cfg.device) != hipSuccess)
    cu_count = 0;
  // every kernel's code object loaded before the first batch (see warm_kernels)
  if (c->err.empty() && (warm_kernels() != hipSuccess || warm_aggregate() != hipSuccess))
    c->err = "cannot load the kernels' code object on HIP device " + std::to_string(c->cfg.device);
  if (c->err.empty() && loop_occupancy(loop_occ) != hipSuccess)
    c->err = "cannot query the persistent loops' occupancy on HIP device " + std::to_string(c->cfg.device);
}

// A pod the persistent loop evaluates: node-local plugins only (no pod-table aggregation, no
// PodTopologySpread / InterPodAffinity scores, no per-node evaluation output).
// No extended-resource requests anywhere in the pod (the batch pipeline's compile-cannot-fail test).
static bool calc_scalar_free(const PodSpec& p) {  // decided once per pod at decode (ksg_pod_compile)
  return p.scalar_free >= 0 ? p.scalar_free != 0 : pod_scalar_free(p);
}

bool Engine::rotdev() const {
  bool any_score = false;
  for (int q : {P_TAINT, P_NA, P_FIT, P_PTS, P_IPA, P_BAL, P_IMG}) any_score |= c->cfg.enabled[q];
  // (OpportunisticBatching: a hinted pod leaves nextStartNodeIndex alone, which only the device knows; so does
  // a pod placed on its nominated node, and one whose nominated node failed may count that node once more)
  return c->cfg.pct != 100 || !any_score || ob_acting() || nom_batch_;
}

// ---- OpportunisticBatching (framework/runtime/batch.go:31-242) --------------------------
// Signatures exist only when PodTopologySpread refuses none on profile grounds: disabled, or List
// defaulting without default constraints (podtopologyspread/plugin.go:92-102); every in-tree plugin of
// the profile implements SignPlugin and there are no extenders (framework.go:832-876).
bool Engine::ob_acting() const {
  const Config& k = c->cfg;
  return k.ob_gate && (!k.enabled[P_PTS] || (!k.pts_system_defaulted && k.pts_defaults.empty()));
}

// frameworkImpl.SignPod (framework.go:884-924): the fragments of the profile's plugins keyed by signer
// name, nil (-1) when a plugin refuses; equal texts <=> equal json.Marshal bytes.  Interned per context.
int32_t Engine::sign(const PodSpec& p, const PodResources& fit) {
  std::string o;
  if (!sign_text(c->cfg, p, fit, &o)) return -1;
  auto it = ob_sigs_.find(o);
  if (it != ob_sigs_.end()) return it->second;
  const int32_t id = (int32_t)ob_sigs_.size();
  ob_sigs_.emplace(std::move(o), id);
  return id;
}

// The signature text itself: one "|key=value" per signer key the profile's plugins contribute (each key once,
// as the reference's fragment map holds it), false for a nil signature (a plugin refused: SignPod returns nil).
bool sign_text(const Config& k, const PodSpec& p, const PodResources& fit, std::string* out) {
  const PodSpec::Sign& f = p.sign;
  std::string o = "sched=" + f.sched;
  if (k.enabled[P_FIT] || k.enabled[P_BAL]) {  // Fit / BalancedAllocation: computePodResourceRequest
    o += "|res=" + std::to_string(fit.cpu) + "," + std::to_string(fit.mem) + "," + std::to_string(fit.eph) + ",0";
    if (fit.scalar.empty()) {
      o += ",null";
    } else {
      std::vector<std::pair<std::string, int64_t>> sc(fit.scalar.begin(), fit.scalar.end());
      std::sort(sc.begin(), sc.end());
      o += ",{";
      for (auto& x : sc) o += x.first + "=" + std::to_string(x.second) + ";";
      o += "}";
    }
  }
  if (k.enabled[P_TAINT] || k.enabled[P_UNSCHED]) o += "|tol=" + f.tols;
  if (k.enabled[P_IPA]) {  // interpodaffinity/plugin.go:62-78
    if (p.has_pod_affinity || p.has_pod_anti) return false;
    if (!k.ignore_pref_existing) o += "|lbl=" + f.labels;
  }
  if (k.enabled[P_PORTS]) o += "|ports=" + f.ports;
  if (k.enabled[P_PTS] && (!p.spreads.empty() || k.pts_system_defaulted || !k.pts_defaults.empty())) return false;
  if (k.enabled[P_NA]) o += "|na=" + f.na + "|nsel=" + f.nsel;
  if (k.enabled[P_NODENAME]) o += "|nn=" + p.node_name;
  if (k.enabled[P_IMG]) o += "|img=" + f.images;
  o += "|vol=" + f.vols;  // the four volume plugins
  if (f.claims) return false;  // DynamicResources
  o += "|feat=";               // NodeDeclaredFeatures: nothing required (else the pod is refused at compile)
  *out = std::move(o);
  return true;
}

int64_t Engine::ob_now() {
  if (ob_clock_) {  // ksg_set_clock's value; ksg_debug_clock_step advances it by a step per read (cycle)
    const int64_t v = ob_clock_;
    ob_clock_ += ob_clock_step_;
    return v;
  }
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One scheduling cycle of this context (every pod of a call, in queue order): its SchedulingCycle count, its
// clock and whether GetNodeHint may find the state usable -- the previous cycle was a pod of the same
// signature without a nominated node (batch.go:183-200); the device checks the rest (k_ob_hint).
int Engine::ob_sequence(CompiledPod& cp, const PodSpec& p, int64_t now) {
  const int64_t cycle = ++ob_cycle_;
  if (cp.blob.size() < sizeof(PodDesc) || cp.error) {
    ob_prev_sig_ = -1;
    return KSG_OK;
  }
  PodDesc& D = *reinterpret_cast<PodDesc*>(cp.blob.data());
  if (D.flags & DF_OB) {
    D.ob_cycle = cycle;
    D.ob_now = now;
    D.ob_hint = (ob_prev_sig_ == cp.sig && p.nominated_node.empty()) ? 1 : 0;
  }
  ob_prev_sig_ = (D.flags & DF_OB) ? cp.sig : -1;
  return KSG_OK;
}

void Engine::ob_invalidate() {
  ob_prev_sig_ = -1;
  if (d_ob.p) (void)hipMemsetAsync(d_ob.p, 0, sizeof(ObState), c->stream);  // len 0: stateEmpty
}

// The device state exists (zeroed once), its heap holds cap entries, and its node indices follow the
// snapshot's node list: after UpdateSnapshot rebuilt the list (cache.go:273-283) every stored index is mapped
// to the node's new one (-1: removed -- GetNodeInPlacement fails for it and the full pass runs).
int Engine::ob_sync(hipStream_t s) {
  int rc_ob_ = KSG_OK;
  const size_t cap = (size_t)std::max(c->view.cap, 1);
  if (!d_ob.p) {
    if ((rc_ob_ = ensure(d_ob, sizeof(ObState)))) return rc_ob_;
    HIPCHK(hipMemsetAsync(d_ob.p, 0, sizeof(ObState), s));
  }
  if (d_ob_heap.bytes < cap * sizeof(ObEnt)) {  // grown: keep the stored heap
    DevBuf old = d_ob_heap;
    d_ob_heap = DevBuf{};
    if ((rc_ob_ = ensure(d_ob_heap, cap * sizeof(ObEnt)))) return rc_ob_;
    if (old.p) {
      HIPCHK(hipMemcpyAsync(d_ob_heap.p, old.p, old.bytes, hipMemcpyDeviceToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
      (void)hipFree(old.p);
    }
  }
  const std::vector<std::string>& order = c->order();
  if (ob_list_gen_ != c->list_gen || ob_order_.size() != order.size()) {
    if (!ob_order_.empty()) {
      std::vector<int32_t> map(ob_order_.size());
      for (size_t i = 0; i < ob_order_.size(); ++i) map[i] = c->index_of(ob_order_[i]);
      if ((rc_ob_ = ensure(d_ob_map, map.size() * 4))) return rc_ob_;
      HIPCHK(hipMemcpyAsync(d_ob_map.p, map.data(), map.size() * 4, hipMemcpyHostToDevice, s));
      HIPCHK(launch_ob_remap((ObState*)d_ob.p, (ObEnt*)d_ob_heap.p, (const int32_t*)d_ob_map.p, (int)map.size(),
                             (int)map.size(), s));
      HIPCHK(hipStreamSynchronize(s));  // the host map buffer goes out of scope
    }
    ob_order_ = order;
    ob_list_gen_ = c->list_gen;
  }
  return KSG_OK;
}

bool Engine::loop_ok(const CompiledPod& p) const {
  if (p.error) return false;
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(p.blob.data());
  if (d.flags & (DF_AGGREGATE | DF_EVAL_OUT | DF_SCORE_ERROR | DF_ALL_FEASIBLE | DF_EARLY)) return false;
  if (d.score_mask & ((1u << P_PTS) | (1u << P_IPA))) return false;
  // percentageOfNodesToScore / no-score profiles: the loop cuts the list and carries nextStartNodeIndex
  // itself (k_sched_loop), unsharded, over the whole snapshot (no PreFilterResult)
  if ((d.flags & DF_ROTDEV) && (comm || (d.flags & (DF_SUBSET | DF_PREFILTER_REJECT)))) return false;
  return loop_bounds_ok(p);
}
// A pod k_agg_loop takes: any CYCLE pod without evaluation output, PreFilter outcomes or sampling, whose
// histograms and PodTopologySpread score constraints fit the loop's placement (CompiledPod::agg_ok).
bool Engine::agg_loop_ok(const CompiledPod& p) const {
  if (p.error || !p.agg_ok || p.blob.size() > (size_t)kAggBlobLds) return false;
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(p.blob.data());
  if (d.flags & (DF_EVAL_OUT | DF_SCORE_ERROR | DF_ALL_FEASIBLE | DF_ROTDEV | DF_PREFILTER_REJECT | DF_SUBSET | DF_EARLY))
    return false;
  // the fold plan holds <= 8 items per kind of the next pod's constraints / terms plus one per own
  // term of the pod just placed (kFoldMax = 80 in k_agg_loop)
  if (d.n_own_terms > 4 * kAggMaxTerms) return false;
  // raw InterPodAffinity scores ride the granules biased by 2^46: every existing term and pod adds
  // at most 100 per matching term of the pod
  const double ipa_bound = ((double)c->tt.size() + (double)c->pt_node.size() + 1.0) * 100.0 * (4.0 * kAggMaxTerms + 1.0);
  if (ipa_bound >= (double)kAggIpaBias) return false;
  return loop_bounds_ok(p);
}
bool Engine::loop_bounds_ok(const CompiledPod& p) const {
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(p.blob.data());
  if (p.blob.size() > (size_t)kBlobLds) return false;
  // the exchange granules carry raw TaintToleration counts and raw NodeAffinity sums (+1) in 24
  // bits each and the packed key in 48: bound the pod's possible values
  int64_t wsum = 0;
  for (int q = 0; q < kNumPlugins; ++q) {
    if (d.weight[q] < 0) return false;
    wsum += (d.score_mask >> q) & 1u ? d.weight[q] : 0;
  }
  if (wsum * 100 >= ((int64_t)1 << 19)) return false;  // TotalScore <= 100 * wsum < 2^19, key < 2^48
  int64_t pref = 0;
  for (SelProg pg : {d.na_preferred, d.na_added_pref}) {
    const SelTerm* t = reinterpret_cast<const SelTerm*>(p.blob.data() + pg.term_off);
    for (int k = 0; k < pg.nterm; ++k) pref += t[k].weight < 0 ? -(int64_t)t[k].weight : t[k].weight;
  }
  return pref < ((int64_t)1 << 24) - 1;
}
// Algorithmic HBM bytes of one k_filter_score launch: every SoA field the pod's active plugins
// must read for a node, plus what the launch writes, each counted once per node.
double Engine::algo_bytes(const PodDesc& d) const {
  const double N = (double)c->view.n;
  const uint32_t fm = d.filter_mask, sm = d.score_mask;
  double b = 4.0 + 1.0 / 8.0;                              // status word + feasibility bit
  if (fm & (1u << P_UNSCHED)) b += 4;                      // flags
  b += 4 + 4 * c->taint_ids_per_node;                      // taint CSR offset + ids (TaintToleration)
  if (fm & (1u << P_NA)) {
    b += 4.0 * (d.na_required.nterm + d.na_selector.nterm + d.na_added.nterm);  // one label column per term (lower bound)
  }
  if (fm & (1u << P_PORTS)) b += 4.0 * c->view.port_slots;
  if (fm & (1u << P_FIT)) {
    b += 4 + 4;                                            // alloc pods, pod count
    if (d.fit_any) {
      b += d.req_cpu > 0 ? 16 : 0;                         // alloc + requested milliCPU
      b += d.req_mem > 0 ? 16 : 0;
      b += d.req_eph > 0 ? 16 : 0;
      b += 16.0 * d.n_scalar;
    }
  }
  if (sm & ((1u << P_FIT) | (1u << P_BAL))) b += 16;       // NonZeroRequested cpu/mem (alloc/requested reused)
  if (sm & (1u << P_NA)) b += 4.0 * (d.na_preferred.nterm + d.na_added_pref.nterm);
  if ((sm & (1u << P_IMG)) && d.n_img) b += 4 + 4 * c->img_ids_per_node;
  if (sm & ((1u << P_FIT) | (1u << P_BAL) | (1u << P_IMG))) b += 8;  // weighted fixed-score sum
  if (sm & (1u << P_TAINT)) b += 8;                        // raw TaintToleration score
  if (sm & (1u << P_NA)) b += 8;                           // raw NodeAffinity score
  return b * N;
}

// Algorithmic bytes of one pod's pod-table pass (k_aggregate / k_agg_loop's aggregation): every
// existing pod's node, namespace, flags, label range and labels, every existing term's record.
double Engine::agg_bytes(const PodDesc& d) const {
  if (!(d.flags & DF_AGGREGATE)) return 0;
  const bool pod_work = d.n_ptsf || d.n_ptss || d.n_raff || d.n_ranti || (d.ipa_flags & IPA_PREF);
  const bool term_work = (d.ipa_flags & (IPA_EXIST_FILTER | IPA_EXIST_SCORE)) != 0;
  const double pods = (double)c->view.pods_hw;
  const double lbl = pods > 0 ? (double)c->pt_pool.size() / pods : 0.0;
  double b = 0;
  if (pod_work) b += pods * (20.0 + 8.0 * lbl);
  if (term_work) b += (double)c->view.n_terms * (double)sizeof(DTerm);
  return b;
}

Engine::~Engine() {
  (void)resident_stop();
  if (ring_) (void)hipHostFree(ring_);
  for (hipEvent_t e : tev) (void)hipEventDestroy(e);
  for (hipEvent_t e : lev) (void)hipEventDestroy(e);
  for (hipEvent_t e : cev) (void)hipEventDestroy(e);
  for (hipEvent_t e : pev) (void)hipEventDestroy(e);
  if (cstream) (void)hipStreamDestroy(cstream);
  for (DevBuf* b : {&d_descs, &d_meta, &d_status, &d_fmask, &d_blk, &d_fixed, &d_raw, &d_out,
                    &d_total, &d_arena, &d_xa, &d_xp, &d_xb, &d_xs, &d_gran, &d_fail, &d_grp, &d_agran, &d_region, &d_astamps, &d_aspill, &d_relay,
                    &d_evg, &d_aggpeers, &d_pre, &d_seg, &d_segcnt, &d_psout, &d_pdb, &d_pick, &d_contrib_buf, &d_wide, &d_vsc,
                    &d_ob, &d_ob_heap, &d_ob_map, &d_tcache, &d_tcw})
    if (b->p) (void)hipFree(b->p);
  if (h_pinned) (void)hipHostFree(h_pinned);
  if (h_tcw) (void)hipHostFree(h_tcw);
  if (ev0) (void)hipEventDestroy(ev0);
  if (ev1) (void)hipEventDestroy(ev1);
}

int Engine::ensure(DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return KSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  size_t want = std::max<size_t>(bytes + bytes / 2, 256);
  HIPCHK(hipMalloc(&b.p, want));
  b.bytes = want;
  return KSG_OK;
}

int Engine::ensure_scratch(size_t desc_bytes, int pods, bool eval, int32_t arena_words) {
  const size_t cap = (size_t)c->view.cap;
  const size_t nb = cap / kBlock + 1;
  int rc;
  if ((rc = ensure(d_descs, desc_bytes))) return rc;
  // offsets + program sizes, PodStats and DevResult in one allocation laid out like the pinned staging
  // area (run_batch), so a single-chunk batch sends them up in one copy; d_off / d_stats / d_results are
  // views into it (re-derived here for every batch size)
  const size_t meta = ((size_t)pods * 8 + 15) & ~size_t(15);
  const size_t stats_b = (size_t)pods * sizeof(PodStats), res_b = (size_t)pods * sizeof(DevResult);
  if ((rc = ensure(d_meta, meta + stats_b + res_b + 16))) return rc;
  d_off.p = d_meta.p;
  d_off.bytes = (size_t)pods * 8;
  d_stats.p = (uint8_t*)d_meta.p + meta;
  d_stats.bytes = stats_b;
  d_results.p = (uint8_t*)d_meta.p + meta + stats_b;
  d_results.bytes = res_b;
  if ((rc = ensure(d_status, cap * 4))) return rc;
  if ((rc = ensure(d_fmask, nb * (kBlock / 64) * 8))) return rc;
  if ((rc = ensure(d_blk, nb * 4))) return rc;
  if ((rc = ensure(d_fixed, cap * 8))) return rc;
  if ((rc = ensure(d_raw, cap * 8 * kNumPlugins))) return rc;
  if (eval) {
    if ((rc = ensure(d_out, cap * 8 * kNumPlugins))) return rc;
    if ((rc = ensure(d_total, cap * 8))) return rc;
  }
  if (comm) {
    if ((rc = ensure(d_xa, (size_t)pods * XA_WORDS * 8))) return rc;
    if ((rc = ensure(d_xp, (size_t)pods * XP_WORDS * 8))) return rc;
    if ((rc = ensure(d_xb, (size_t)pods * XB_WORDS * 8))) return rc;
    if ((rc = ensure(d_xs, (size_t)pods * XS_WORDS * 8))) return rc;
    HIPCHK(hipMemsetAsync(d_xp.p, 0, (size_t)pods * XP_WORDS * 8, c->stream));
  }
  if (d_arena.bytes < (size_t)arena_words * 8 + 8) {
    const size_t old = d_arena.bytes;
    if ((rc = ensure(d_arena, (size_t)arena_words * 8 + 8))) return rc;
    if (d_arena.bytes != old) HIPCHK(hipMemsetAsync(d_arena.p, 0, d_arena.bytes, c->stream));
  }
  const size_t need = desc_bytes + (size_t)pods * (8 + sizeof(PodStats) + sizeof(DevResult) + 4) + 256;
  if (h_pinned_bytes < need) {
    if (h_pinned) (void)hipHostFree(h_pinned);
    h_pinned = nullptr;
    h_pinned_bytes = 0;
    size_t want = need * 2;
    HIPCHK(hipHostMalloc(&h_pinned, want, hipHostMallocDefault));
    h_pinned_bytes = want;
  }
  return KSG_OK;
}

BatchView Engine::bview(int pods) {
  (void)pods;
  BatchView b{};
  b.descs = (const uint8_t*)d_descs.p;
  b.desc_off = (const uint32_t*)d_off.p;
  b.stats = (PodStats*)d_stats.p;
  b.results = (DevResult*)d_results.p;
  b.status = (uint32_t*)d_status.p;
  b.fmask = (uint64_t*)d_fmask.p;
  b.blk_cnt = (uint32_t*)d_blk.p;
  b.fixed = (int64_t*)d_fixed.p;
  b.raw = (int64_t*)d_raw.p;
  b.out_scores = (int64_t*)d_out.p;
  b.out_total = (int64_t*)d_total.p;
  b.arena = (unsigned long long*)d_arena.p;
  b.ob = (ObState*)d_ob.p;
  b.ob_heap = (ObEnt*)d_ob_heap.p;
  return b;
}

// The loop's exchange granule array: fixed size (2 kLoopMaxPods pods x 256 participants), zeroed once,
// never reallocated (a sharded context's peers map it over IPC).  Sharded, it is uncached device
// memory: the peers' stores arrive over xGMI and the sweeps must not read a stale cached line.
int Engine::gran_setup() {
  if (!gran_all.empty()) return KSG_OK;
  // [2 kLoopMaxPods]: pod q's sampled-maxima exchange (k_sched_loop, DF_ROTDEV) sits at q + kLoopMaxPods
  const size_t bytes = (size_t)2 * kLoopMaxPods * 256 * kGran * 8;
  void* p = nullptr;
  if (comm) HIPCHK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
  else HIPCHK(hipMalloc(&p, bytes));
  d_gran.p = p;
  d_gran.bytes = bytes;
  HIPCHK(hipMemset(p, 0, bytes));
  HIPCHK(hipDeviceSynchronize());
  if (comm) {
    std::vector<void*> all;
    if (comm->share_buffers(p, &all)) {
      c->err = comm->err;
      return KSG_EDEVICE;
    }
    for (void* q : all) gran_all.push_back((unsigned long long*)q);
  } else {
    gran_all.push_back((unsigned long long*)p);
  }
  return KSG_OK;
}

// k_agg_loop's granule array ((kLoopMaxPods + 1) rows: the last is the node-sharded start barrier) and
// its per-pod shared regions (kAggGWords words per pod), fixed size, zeroed once.  Node-sharded, both
// are uncached device memory shared over IPC like k_sched_loop's granules: every workgroup stores its
// granules and adds its shared-key partials into every rank's copy.
int Engine::agg_setup() {
  if (!agran_all.empty()) return KSG_OK;
  const size_t gb = (size_t)(kLoopMaxPods + 1) * 256 * kAGran * 8, rb = (size_t)kLoopMaxPods * kAggGWords * 8;
  for (DevBuf* b : {&d_agran, &d_region}) {
    const size_t bytes = b == &d_agran ? gb : rb;
    if (b->p) (void)hipFree(b->p);
    void* p = nullptr;
    if (comm) HIPCHK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    else HIPCHK(hipMalloc(&p, bytes));
    b->p = p;
    b->bytes = bytes;
    HIPCHK(hipMemset(p, 0, bytes));
  }
  HIPCHK(hipDeviceSynchronize());
  if (comm) {
    std::vector<void*> ga, ra;
    if (comm->share_buffers(d_agran.p, &ga) || comm->share_buffers(d_region.p, &ra)) {
      c->err = comm->err;
      return KSG_EDEVICE;
    }
    for (void* q : ga) agran_all.push_back((unsigned long long*)q);
    for (void* q : ra) region_all.push_back((unsigned long long*)q);
    // the peer tables k_agg_loop reads (AggView::grans / regions): [0, W) granules, [W, 2W) regions
    std::vector<unsigned long long*> tab(agran_all);
    tab.insert(tab.end(), region_all.begin(), region_all.end());
    int rc;
    if ((rc = ensure(d_aggpeers, tab.size() * sizeof(void*)))) return rc;
    HIPCHK(hipMemcpy(d_aggpeers.p, tab.data(), tab.size() * sizeof(void*), hipMemcpyHostToDevice));
  } else {
    agran_all.push_back((unsigned long long*)d_agran.p);
    region_all.push_back((unsigned long long*)d_region.p);
  }
  return KSG_OK;
}

// Each loop launch (k_sched_loop or k_agg_loop) gets the next tag (every rank issues the same launches,
// so the tags agree).  After 65535 launches the arrays are zeroed again; sharded, behind an exchange, so
// that no rank publishes into a peer's array before that peer has cleared it.
int Engine::next_gran_tag(uint32_t* tag) {
  if (++gran_tag > 0xFFFFu) {
    gran_tag = 1;
    if (d_gran.p) HIPCHK(hipMemsetAsync(d_gran.p, 0, d_gran.bytes, c->stream));
    if (d_agran.p) HIPCHK(hipMemsetAsync(d_agran.p, 0, d_agran.bytes, c->stream));
    if (comm) {
      int rc;
      if ((rc = ensure(d_xb, XB_WORDS * 8))) return rc;
      if (comm->all_reduce_max((unsigned long long*)d_xb.p, 1, c->stream)) {
        c->err = comm->err;
        return KSG_EDEVICE;
      }
    }
  }
  *tag = gran_tag;
  return KSG_OK;
}

// The participants (p = rank * g + workgroup) a set names, per rank: "rank 0 wg {0,3-7}; rank 2 wg {0-7}"
static std::string participants_by_rank(const std::vector<uint8_t>& in, int world, int g) {
  std::string out;
  for (int r = 0; r < world; ++r) {
    std::string ws;
    int cnt = 0;
    for (int w = 0; w < g; ++w) {
      if (!in[(size_t)(r * g + w)]) continue;
      int e = w;  // a run of consecutive workgroups as a-b
      while (e + 1 < g && in[(size_t)(r * g + e + 1)]) ++e;
      ws += (cnt ? "," : "") + std::to_string(w) + (e > w ? "-" + std::to_string(e) : "");
      cnt += e - w + 1;
      w = e;
    }
    if (cnt) out += (out.empty() ? "rank " : "; rank ") + std::to_string(r) + " wg {" + ws + "} of " + std::to_string(g);
  }
  return out.empty() ? "none" : out;
}

// Which participants a loop give-up (record f, kFailWords) waited for: at the give-up (the sweep's
// missing-lane ballot; exact up to 64 participants) and still after the drain (the granule row `row`
// of this rank's array, read back).  Absent at the give-up but present after the drain: that loop was
// late -- not resident yet (a queue or CU it waited for); absent in both: it stopped or never ran.
static std::string give_up_detail(const uint32_t* f, const std::vector<unsigned long long>& row, int ng, int world, int g) {
  const int P = world * g;
  const unsigned long long ball = (unsigned long long)f[6] | ((unsigned long long)f[7] << 32);
  std::vector<uint8_t> at(P, 0), now(P, 0);
  for (int p = 0; p < P; ++p) {
    now[(size_t)p] = row.size() >= (size_t)P * ng && (row[(size_t)p * ng + f[2]] >> 48) != (unsigned long long)f[5];
    at[(size_t)p] = ((ball >> (p & 63)) & 1ull) && (P <= 64 || now[(size_t)p]);
  }
  // fail words 8..15: where and when the launch entered and gave up (HW_ID: pipe [7:6], HQD [26:24], ME [31:30];
  // s_memrealtime at 100 MHz, shown in us, one clock for every rank on the device)
  auto hw = [](uint32_t id, uint32_t xcc) {
    return "ME " + std::to_string(id >> 30) + " pipe " + std::to_string((id >> 6) & 3u) + " HQD " +
           std::to_string((id >> 24) & 7u) + " XCC " + std::to_string(xcc & 15u);
  };
  const unsigned long long te = (unsigned long long)f[10] | ((unsigned long long)f[11] << 32);
  const unsigned long long tg = (unsigned long long)f[12] | ((unsigned long long)f[13] << 32);
  return std::string(f[4] == 2 ? "k_agg_loop" : "k_sched_loop") + " granule row " + std::to_string(f[1]) + " slot " +
         std::to_string(f[2]) + ": missing at the give-up " + participants_by_rank(at, world, g) +
         (P > 64 ? " (sweep lanes fold 64 participants: intersected with the drain)" : "") + "; still missing after the drain " +
         participants_by_rank(now, world, g) + "; this launch entered at t=" + std::to_string(te / 100) + " us (" +
         hw(f[8], f[9]) + "), gave up at t=" + std::to_string(tg / 100) + " us (" + hw(f[14], f[15]) + ")";
}

// k_agg_loop: pod b's counts are defined exactly as pod a's (DF_AGG_SAME) -- the same program but for the fields
// the aggregation does not read: the pod-table slot, the rotation and the pod's own affinity terms (the last
// part of the program; the fold of a adds a's own terms to b's counts).  Pods stamped from one template, as
// every scheduler_perf workload's are, qualify; anything else only loses the shortcut.
// (also the resident k_agg_loop's ring pods: a against the pod posted before b to the same launch)
static bool agg_same(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
  if (a.size() != b.size() || a.size() < sizeof(PodDesc)) return false;
  PodDesc x, y;
  std::memcpy(&x, a.data(), sizeof(PodDesc));
  std::memcpy(&y, b.data(), sizeof(PodDesc));
  if (!(x.flags & DF_AGGREGATE) || !(y.flags & DF_AGGREGATE) || x.own_terms_off != y.own_terms_off) return false;
  for (PodDesc* z : {&x, &y}) {
    z->slot = 0;
    z->rot_start = 0;
    z->prev_pod = 0;
    z->n_own_terms = 0;
    z->flags &= ~DF_AGG_SAME;
  }
  if (std::memcmp(&x, &y, sizeof(PodDesc)) != 0) return false;
  const size_t end = x.own_terms_off > 0 ? std::min((size_t)x.own_terms_off, a.size()) : a.size();
  return end <= sizeof(PodDesc) ||
         std::memcmp(a.data() + sizeof(PodDesc), b.data() + sizeof(PodDesc), end - sizeof(PodDesc)) == 0;
}

static bool agg_same(const CompiledPod& a, const CompiledPod& b) { return !a.error && !b.error && agg_same(a.blob, b.blob); }

// The resident k_agg_loop's RING_TERMS doorbell (desc.h): pod b (program nb, entry ne) is pod a's but for its slot,
// rotation, DF_AGG_SAME, label-pool offset -- as RING_SAME -- and its own affinity terms' table indices and the
// term-pool offset of their words.  The loop's patch is replayed on a's bytes; true (and the patch words) only when
// the result equals b's program and entry byte for byte.
// (why: the first check that failed, for the loopStamps report -- 1 sizes, 2 the terms, 3 the program, 4 the entry's
// terms, 5 the entry)
static bool ring_terms_patch(const std::vector<uint8_t>& pa, const std::vector<uint8_t>& pb, const std::vector<uint8_t>& ea,
                             const uint8_t* eb, size_t eb_bytes, unsigned long long* patch, int* why) {
  *why = 1;
  if (pa.size() != pb.size() || pa.size() < sizeof(PodDesc) || ea.size() != eb_bytes || eb_bytes < sizeof(RingEntry))
    return false;
  *why = 2;
  const PodDesc& hb = *reinterpret_cast<const PodDesc*>(pb.data());
  const PodDesc& ha = *reinterpret_cast<const PodDesc*>(pa.data());
  const int32_t n = hb.n_own_terms;
  if (n <= 0 || n > 2 * (kPatchWords - 1) || ha.n_own_terms != n || ha.own_terms_off != hb.own_terms_off ||
      hb.own_terms_off < (int32_t)sizeof(PodDesc) || (size_t)hb.own_terms_off + (size_t)n * 4 > pb.size())
    return false;
  std::vector<uint8_t> p = pa;
  PodDesc& pd = *reinterpret_cast<PodDesc*>(p.data());
  pd.slot = hb.slot;
  pd.rot_start = hb.rot_start;
  pd.flags = (pd.flags & ~DF_AGG_SAME) | (hb.flags & DF_AGG_SAME);
  int32_t js[2 * (kPatchWords - 1)] = {};
  std::memcpy(js, pb.data() + hb.own_terms_off, (size_t)n * 4);
  std::memcpy(p.data() + hb.own_terms_off, js, (size_t)n * 4);
  *why = 3;
  if (std::memcmp(p.data(), pb.data(), p.size()) != 0) return false;
  *why = 4;
  std::vector<uint8_t> e = ea;
  RingEntry& en = *reinterpret_cast<RingEntry*>(e.data());
  const RingEntry& nb = *reinterpret_cast<const RingEntry*>(eb);
  if (en.nterms != n) return false;
  const size_t rt_at = sizeof(RingEntry) + (size_t)en.lbl_cnt * 8 + (size_t)((en.tpool_cnt + 1) & ~1) * 4;
  if (en.slot < 0 || rt_at + (size_t)n * sizeof(RingTerm) > e.size()) return false;
  const int32_t dt = nb.tpool_off - en.tpool_off;
  en.slot = nb.slot;
  en.lbl_off = nb.lbl_off;
  en.tpool_off = nb.tpool_off;
  for (int32_t k = 0; k < n; ++k) {
    RingTerm r;
    std::memcpy(&r, e.data() + rt_at + (size_t)k * sizeof(RingTerm), sizeof r);
    r.j = js[k];
    r.d.owner = en.slot;
    r.d.sel += dt;
    r.d.nssel += dt;
    r.d.ns_off += dt;
    std::memcpy(e.data() + rt_at + (size_t)k * sizeof(RingTerm), &r, sizeof r);
  }
  *why = 5;
  if (std::memcmp(e.data(), eb, eb_bytes) != 0) return false;
  *why = 0;
  patch[0] = (unsigned long long)(uint32_t)nb.tpool_off | ((unsigned long long)(uint32_t)n << 32);
  std::memset(patch + 1, 0, (kPatchWords - 1) * 8);
  std::memcpy(patch + 1, js, (size_t)n * 4);
  return true;
}

// k_agg_loop's template cache plan for the run [i, j) (TcWord per pod, desc.h): each pod's template takes a slot
// (a template already cached: a hit, its counts are loaded instead of gathered; else the least recently used
// slot but the active one), and per pod q the slots the loop folds pod q-1's placement into while deciding q:
// every slot written back before (a template's counts are written back when the pod after its last pod is of
// another template), but q's own (its counts are in LDS) and q+1's when q+1 loads them (folded after the load).
static void tc_plan(const std::vector<CompiledPod>& cp, int i, int j, uint32_t* out) {
  const int R = j - i;
  std::vector<int> ts((size_t)R, -1);
  std::vector<uint8_t> hit((size_t)R, 0);
  int rep[kAggTc];
  int64_t used[kAggTc];
  for (int s = 0; s < kAggTc; ++s) rep[s] = -1, used[s] = -1;
  for (int k = 0; k < R; ++k) {
    const CompiledPod& p = cp[(size_t)(i + k)];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(p.blob.data());
    if (p.error || !(d.flags & DF_AGGREGATE)) continue;  // gathered as before, no slot
    if (k > 0 && ts[(size_t)k - 1] >= 0 && agg_same(cp[(size_t)(i + k - 1)], p)) {
      ts[(size_t)k] = ts[(size_t)k - 1];
      used[ts[(size_t)k]] = k;
      continue;
    }
    int s = -1;
    for (int x = 0; x < kAggTc && s < 0; ++x)
      if (rep[x] >= 0 && agg_same(cp[(size_t)rep[x]], p)) s = x;
    if (s >= 0) {
      hit[(size_t)k] = 1;
    } else {
      const int act = k > 0 ? ts[(size_t)k - 1] : -1;
      int64_t best = INT64_MAX;
      for (int x = 0; x < kAggTc; ++x)
        if (x != act && used[x] < best) best = used[x], s = x;
      rep[s] = i + k;
    }
    ts[(size_t)k] = s;
    used[s] = k;
  }
  bool valid[kAggTc] = {}, elig[kAggTc] = {};  // elig: the slot holds its template's eligibility (static) already
  for (int k = 0; k < R; ++k) {
    const bool more = k + 1 < R;
    const int t0 = ts[(size_t)k], t1 = more ? ts[(size_t)k + 1] : -1;
    const bool h1 = more && t1 >= 0 && hit[(size_t)k + 1] && t1 != t0;
    if (more && t1 >= 0 && !hit[(size_t)k + 1] && t1 != t0) valid[t1] = elig[t1] = false;  // evicted: q+1 gathers into it
    uint32_t f = 0;
    if (k > 0)
      for (int s = 0; s < kAggTc; ++s)
        if (valid[s] && s != t0 && !(h1 && s == t1)) f |= 1u << s;
    bool ew = false;  // this write-back stores the eligibility too
    if (more && t0 >= 0 && t1 != t0) {  // written back while pod k is decided
      ew = !elig[t0];
      valid[t0] = elig[t0] = true;
    }
    out[k] = (t0 >= 0 ? (uint32_t)(t0 + 1) : 0u) | (hit[(size_t)k] ? 16u : 0u) | (ew ? 32u : 0u) | (f << 8);
  }
}

// In-process groups (localGroup, one device): this rank's persistent loop joins the group's single dispatch
// (Comm::group_launch).  The leader stages every rank's launch arguments into its own d_grp, in
// stream order, and launches world * nwg workgroups; block r * nwg + w runs rank r's workgroup w.  Rank r's
// timing events bracket the group's dispatch on the leader's stream (rank 0's ride its dispatch packet).
int Engine::group_launch(GroupReq* req, bool agg, int nwg, int unit) {
  const int W = c->cfg.world;
  void* grp = d_grp.p;  // (the leader's: only rank 0's callback runs)
  auto leader = [&](hipStream_t ls, const std::vector<void*>& reqs) -> int {
    if (!grp || (int)reqs.size() != W) return KSG_EDEVICE;
    auto rq = [&](int r) -> const GroupReq& { return *static_cast<const GroupReq*>(reqs[(size_t)r]); };
    for (int r = 0; r < W; ++r)
      if ((agg ? launch_put_group_arg(rq(r).aa, (AggGroupArg*)grp + r, ls)
               : launch_put_group_arg(rq(r).la, (LoopGroupArg*)grp + r, ls)) != hipSuccess)
        return KSG_EDEVICE;
    for (int r = 1; r < W; ++r)
      if (rq(r).t0 && hipEventRecord(rq(r).t0, ls) != hipSuccess) return KSG_EDEVICE;
    const hipError_t e = agg ? launch_agg_loop_group((const AggGroupArg*)grp, W, nwg, ls, rq(0).t0, rq(0).t1)
                             : launch_sched_loop_group((const LoopGroupArg*)grp, W, nwg, ls, rq(0).t0, rq(0).t1, unit);
    if (e != hipSuccess) return KSG_EDEVICE;
    for (int r = 1; r < W; ++r)
      if (rq(r).t1 && hipEventRecord(rq(r).t1, ls) != hipSuccess) return KSG_EDEVICE;
    return KSG_OK;
  };
  if (comm->group_launch(req, c->stream, leader) != KSG_OK) {
    c->err = comm->err;
    return KSG_EDEVICE;
  }
  return KSG_OK;
}

// RunFilterPluginsWithNominatedPods (framework.go:1211-1294) filters a node with the pods nominated to it of equal or
// higher priority added (addGENominatedPods: corev1.PodPriority >= the pod's, another uid), which this library does
// not run: a call in which some pod would see such a nomination on a snapshot node is refused before anything runs.
int Engine::check_nominations(const std::vector<const PodSpec*>& pods) {
  if (nominated.empty()) return KSG_OK;
  c->order();  // (the snapshot's index, current)
  for (const PodSpec* p : pods)
    for (const auto& kv : nominated)
      if (kv.first != p->uid && kv.second.second >= p->priority && c->index_of(kv.second.first) >= 0) {
        c->err = "pod " + p->ns + "/" + p->name + ": pod uid " + kv.first + " (priority " + std::to_string(kv.second.second) +
                 ") is nominated to node " + kv.second.first +
                 "; filtering with nominated pods (RunFilterPluginsWithNominatedPods) runs outside the device path";
        return KSG_ENOTSUP;
      }
  return KSG_OK;
}

int Engine::run_batch_api(const std::vector<const PodSpec*>& pods, const std::vector<int32_t>& handles, bool assume,
                          ksg_result* results, ksg_eval_out* eval) {
  fault_first_ = -1;
  htrace("batch", (long)pods.size());
  const int rc = run_batch(pods, handles, assume, results, eval);
  htrace("ret", rc < 0 ? -rc : rc);
  htrace_flush(comm ? c->cfg.rank : 0);
  if (fault_first_ >= 0) ++loop_give_ups_;
  if (!comm || !c->cfg.nccl_id.empty() || eval) return rc;
  // In-process groups (one device): every rank learns every rank's outcome before anyone retries.  A loop
  // give-up re-runs the chunk over the all-reduce path only when every rank gave up at the same pod (each
  // rank's loop gives up on the same missing participants; a late rank's once it runs alone); a rank that
  // finished the chunk while another gave up would otherwise pair different pods' exchanges.
  const int64_t mine = rc == KSG_OK ? -1 : (rc == KSG_EDEVICE && fault_first_ >= 0 ? fault_first_ : -2);
  std::vector<int64_t> all;
  if (comm->agree(mine, &all) != KSG_OK) {
    c->err = comm->err;
    return KSG_EDEVICE;
  }
  bool same = true;
  for (int64_t v : all) same = same && v == all[0];
  if (same && all[0] == -1) return rc;  // every rank scheduled the batch
  const int f = (int)all[0];
  if (!same || f < 0 || f >= (int)pods.size()) {
    std::string o;
    for (size_t r = 0; r < all.size(); ++r)
      o += (r ? ", rank " : "rank ") + std::to_string(r) + ": " +
           (all[r] == -1 ? std::string("scheduled") : all[r] == -2 ? std::string("error") : "gave up at pod " + std::to_string(all[r]));
    if (rc == KSG_OK) c->err.clear();
    c->err = (c->err.empty() ? std::string() : c->err + "; ") + "in-process group out of step (" + o +
             "): no retry; rebuild the group";
    return rc == KSG_OK ? KSG_EDEVICE : rc;
  }
  const std::string why = c->err;
  const std::vector<const PodSpec*> rest(pods.begin() + f, pods.end());
  const std::vector<int32_t> rh(handles.begin() + f, handles.end());
  force_allreduce_ = true;
  fault_first_ = -1;
  const int r2 = run_batch(rest, rh, assume, results + f, nullptr);
  force_allreduce_ = false;
  if (r2 == KSG_OK) {
    ++loop_retries_;
    c->err = "recovered: " + why + "; re-run over the all-reduce path";
  }
  return r2;
}

int Engine::run_batch(const std::vector<const PodSpec*>& pods, const std::vector<int32_t>& handles, bool assume,
                      ksg_result* results, ksg_eval_out* eval) {
  const int n = (int)pods.size();
  if (n == 0) return KSG_OK;
  if (eval && n != 1) return KSG_EINVAL;
  struct NomReset {
    bool* f;
    ~NomReset() { *f = false; }
  } nom_reset{&nom_batch_};
  for (int i = 0; i < n && !nom_batch_; ++i) nom_batch_ = !pods[i]->nominated_node.empty();
  c->order();
  if (c->order().empty()) {  // ErrNoNodesAvailable (schedule_one.go:569-571)
    for (int i = 0; i < n; ++i) results[i] = ksg_result{KSG_CODE_ERROR, -1, 0, 0, 0};
    return KSG_OK;
  }
  using clk = std::chrono::steady_clock;
  const auto T0 = clk::now();
  // ---- the chunk plan (needs the exchange mode of a sharded context)
  const int W = comm ? c->cfg.world : 1;
  // (in-process ranks -- localGroup, one device -- launch every rank's loop in one dispatch: group_launch below)
  const bool rccl = !c->cfg.nccl_id.empty();
  const bool dx = comm && !force_allreduce_ && (c->cfg.dev_exchange == 1 || (c->cfg.dev_exchange < 0 && rccl));
  // Host/device pipeline: the batch runs as chunks.  While the device schedules chunk k the host
  // compiles and stages chunk k+1, then mirrors the finished chunks' assumes into the cache.  Only
  // chunk 0's compile and the last chunk's bookkeeping are exposed, so chunk 0 is short (32 pods,
  // pipelineFirstChunk; 64 measured 0.04-0.06 us per pod slower at C2),
  // each next chunk at most 5x the previous (its compile, ~1 us per pod, hides under the previous
  // chunk's device time, ~6 us per pod), and the tail shrinks geometrically (60 % of what is left)
  // down to a last chunk of <= 32 pods.
  std::vector<int> bnd;
  const int kFirstChunk = c->cfg.first_chunk;
  if ((!comm || dx) && !eval && n >= 256)
    for (int r = n, prev = 0; r > 32;) {
      int take = prev == 0 ? kFirstChunk : std::min((r * 3 + 4) / 5, 5 * prev);
      take = std::min(take, r);
      bnd.push_back(n - r + take);
      r -= take;
      prev = take;
    }
  if (bnd.empty() || bnd.back() != n) bnd.push_back(n);
  auto chunk_end = [&](int i) {  // end of the chunk holding pod i
    return *std::upper_bound(bnd.begin(), bnd.end(), i);
  };
  // Compiling a chunk after chunk 0 is launched needs every pod-table slot reserved and uploaded
  // before the first launch: a later full upload would overwrite the pod_node entries the device
  // assumes wrote.  A reservation adds the pod's (anti-)affinity terms to the key tables other pods'
  // compiles read (existing-pod keys: InterPodAffinity then keeps histograms for keys no placed pod
  // has yet -- all-zero counts, the same filter outcome and a zero normalised score, as the
  // sequential compile already gives for the earlier pods of a batch that end up unplaced).
  // Batches with extended-resource pods (a compile path that can add a column) compile everything
  // before the first launch.
  bool pipe = bnd.size() > 1;
  for (int i = 0; i < n && pipe; ++i) pipe = calc_scalar_free(*pods[i]);
  const auto Tp = clk::now();
  std::vector<int32_t> pre_slot;
  struct HeadroomReset {
    Cluster* c;
    ~HeadroomReset() { c->pt_headroom = 0; }
  } headroom_reset{c};
  if (pipe && assume) {
    // A batch none of whose pods can read the pod table (the superset test pods_needed uses below: no
    // existing pod's terms, no own spread constraints or affinity terms) leaves each slot to its pod's
    // compile, which overlaps the device; the device's pod_node column only keeps room for them.
    // (and no PodTopologySpread system default can apply: no selecting object in the cache)
    bool local = c->exanti_keys.empty() && c->score_keys_req.empty() && c->score_keys_pref.empty() &&
                 (c->cfg.pts_defaults.empty() ||
                  (c->services.empty() && c->owners[0].empty() && c->owners[1].empty() && c->owners[2].empty()));
    for (int i = 0; i < n && local; ++i)
      local = pods[i]->spreads.empty() && !pods[i]->has_pod_affinity && !pods[i]->has_pod_anti;
    if (local) {
      c->pt_headroom = n;
    } else {
      pre_slot.resize(n);
      const auto Tr = clk::now();
      for (int i = 0; i < n; ++i) pre_slot[i] = c->pod_table_put(*pods[i], -1);
      reserve_us_ = std::chrono::duration<double, std::micro>(clk::now() - Tr).count();
    }
  }
  const auto Tv0 = clk::now();
  std::vector<CompiledPod> cp(n);
  int compiled = 0;
  // OpportunisticBatching: every pod of the call is one scheduling cycle, which reads the clock when it starts
  // (batch.go:202 time.Now(); here at the pod's compile, which precedes its device cycle by at most a chunk)
  const bool ob_on = ob_acting();
  const int64_t ob_clock0 = ob_clock_;
  const int64_t ob_cycle0 = ob_cycle_;
  const int32_t ob_prev0 = ob_prev_sig_;
  // compile pods [compiled, b) against the cache (PreFilter / PreScore on the host)
  std::vector<int64_t> ns_before((size_t)n, 0);  // Scheduler.nextStartNodeIndex before each pod's compile
  auto compile_upto = [&](int b) -> int {
    for (int i = compiled; i < b; ++i) {
      ns_before[(size_t)i] = c->next_start;
      next_slot_ = pre_slot.empty() ? -1 : pre_slot[i];
      const int rc = compile(*pods[i], CYCLE, -1, assume, eval != nullptr, &cp[i]);
      next_slot_ = -1;
      if (rc) return rc;
      if (cp[i].prefilter_error) cp[i].error = true;  // PreFilter Error: status Error, no launch
      if (ob_on) ob_sequence(cp[i], *pods[i], ob_now());
      if (!cp[i].prefilter_reject && !cp[i].prefilter_error && !rotdev()) {
        // nextStartNodeIndex = (old + processed) % len(allNodes) (schedule_one.go:686-687)
        const int64_t N = (int64_t)c->order().size();
        c->next_start = (c->next_start + cp[i].num_all) % N;
      }
      compiled = i + 1;
    }
    return KSG_OK;
  };
  int rc;
  const auto Tv1 = clk::now();
  {
    const int64_t start = c->next_start;
    if ((rc = compile_upto(pipe ? bnd[0] : n))) {  // nothing launched: the batch fails as a whole
      c->next_start = start;
      ob_cycle_ = ob_cycle0;
      ob_clock_ = ob_clock0;
      ob_prev_sig_ = ob_prev0;
      if (!pre_slot.empty())
        for (int32_t sl : pre_slot) c->pod_table_drop(sl);
      else
        for (int j = 0; j < compiled; ++j) c->pod_table_drop(cp[j].slot);
      return rc;
    }
  }
  const auto T1 = clk::now();
  {
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    c0_us_[0] = us(T0, Tp);
    c0_us_[1] = us(Tv0, Tv1);
    c0_us_[2] = us(Tv1, T1);
  }
  bool pods_needed = eval != nullptr;
  for (int i = 0; i < compiled && !pods_needed; ++i)
    pods_needed = (reinterpret_cast<const PodDesc*>(cp[i].blob.data())->flags & DF_AGGREGATE) != 0;
  // Later chunks are compiled after the first launch, so the table goes up now if any of their pods
  // may read it: a superset of compile_topology's DF_AGGREGATE test (own spread constraints or
  // affinity terms, or existing pods' terms that InterPodAffinity filters / scores every pod with;
  // the batch's own pods' terms are already in the key tables, reserved above).  A node-local stream
  // then skips re-uploading a pod table that grows with every batch.
  if (!pods_needed && compiled < n) {
    const bool existing_terms = !c->exanti_keys.empty() || !c->score_keys_req.empty() || !c->score_keys_pref.empty();
    for (int i = compiled; i < n && !pods_needed; ++i)
      pods_needed = existing_terms || !pods[i]->spreads.empty() || pods[i]->has_pod_affinity || pods[i]->has_pod_anti;
  }
  {  // host ports the batch's assumes can add to one node (the device row must hold them): the distinct
     // (ip, protocol, port) entries -- HostPortInfo.Add is a set insert, so a port many pods share takes one
     // slot (a batch of HostPortConflict pods needs one, not one per pod)
    std::unordered_set<std::string> distinct;
    auto add = [&](const HostPort& hp) {
      if (hp.port > 0) distinct.insert(hp.ip + '\x1f' + hp.proto + '\x1f' + std::to_string(hp.port));
    };
    for (int i = 0; i < n; ++i) {
      for (auto& k : pods[i]->containers)
        for (auto& hp : k.ports) add(hp);
      for (auto& k : pods[i]->init_containers)
        if (k.sidecar)
          for (auto& hp : k.ports) add(hp);
    }
    c->reserve_ports((int32_t)distinct.size());
  }
  const auto Tm = clk::now();
  htrace("mirror");
  if ((rc = c->ensure_mirror(pods_needed))) return rc;
  if (ob_acting() && (rc = ob_sync(c->stream))) return rc;
  mirror_us_ = std::chrono::duration<double, std::micro>(clk::now() - Tm).count();
  // ---- staging: [offsets n | program sizes n | PodStats n | DevResult n | give-up flags n | programs]
  // in pinned memory; each chunk's programs, offsets and stats go up in their own H2D copies
  size_t desc_bytes = 0;
  int32_t arena_words = 0;
  for (int i = 0; i < compiled; ++i) {
    desc_bytes += cp[i].blob.size();
    arena_words = std::max(arena_words, cp[i].arena_words);
  }
  if (compiled < n)  // room for the chunks still to be compiled (re-sized after a sync if they outgrow it)
    desc_bytes = std::max(desc_bytes * 2 * (size_t)n / (size_t)compiled, (size_t)n * 1024);
  htrace("scratch");
  if ((rc = ensure_scratch(desc_bytes, n, eval != nullptr, arena_words))) return rc;
  htrace("scratched");
  const size_t meta = ((size_t)n * 8 + 15) & ~size_t(15);
  const size_t meta_all = meta + (((size_t)n * (sizeof(PodStats) + sizeof(DevResult) + 4) + 15) & ~size_t(15));
  uint8_t* hp = nullptr;
  uint32_t* h_offs = nullptr;
  PodStats* hs = nullptr;
  DevResult* hr = nullptr;
  uint32_t* hfail = nullptr;
  uint8_t* hdesc = nullptr;
  size_t desc_cap = 0, o = 0;
  auto map_pinned = [&]() {
    hp = (uint8_t*)h_pinned;
    h_offs = (uint32_t*)hp;
    hs = (PodStats*)(hp + meta);
    hr = (DevResult*)(hs + n);
    hfail = (uint32_t*)(hr + n);
    hdesc = hp + meta_all;
    desc_cap = std::min(h_pinned_bytes - meta_all, d_descs.bytes);
  };
  map_pinned();
  hipStream_t s = c->stream;
  const MirrorView& m = c->view;
  // device-resident nextStartNodeIndex: each launched pod's k_sample_find reads the previous
  // launched pod's rotation; the first reads the host's value
  const bool rot_dev = rotdev();
  int last_launched = -1;
  // programs, offsets, stats of pods [a, b) into pinned memory, then their H2D copies
  // chunks after the first go up on the copy stream while the device runs the chunk before them;
  // the compute stream waits for them before the chunk's first launch
  // (not for in-process rank groups: the group's leader waits for each rank's compute stream before the
  // group's loop dispatch, so the staging stays on it)
  const bool copy_stream = pipe && (!comm || rccl);
  if (copy_stream && !cstream) {
    HIPCHK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
  }
  while (pev.size() < 2 * bnd.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    pev.push_back(e);
  }
  int staged_chunks = 0;
  auto stage = [&](int a, int b) -> int {
    const bool async = copy_stream && a > 0;
    hipStream_t st_ = async ? cstream : s;
    const size_t o0 = o;
    for (int i = a; i < b; ++i) {
      h_offs[i] = (uint32_t)o;
      h_offs[n + i] = (uint32_t)cp[i].blob.size();  // program sizes follow the offsets (k_sched_loop's prefetch)
      std::memcpy(hdesc + o, cp[i].blob.data(), cp[i].blob.size());
      PodStats& st = hs[i];
      std::memset(&st, 0, sizeof(PodStats));
      for (int q = 0; q < kNumPlugins; ++q) {
        st.max_raw[q] = enc_i64(INT64_MIN);
        st.min_raw[q] = enc_i64(INT64_MAX);
      }
      if (i > 0 && agg_same(cp[i - 1], cp[i])) reinterpret_cast<PodDesc*>(hdesc + o)->flags |= DF_AGG_SAME;
      if (rot_dev && !cp[i].error) {
        reinterpret_cast<PodDesc*>(hdesc + o)->prev_pod = last_launched;
        if (last_launched < 0) st.rot_in = (uint32_t)c->next_start;
        last_launched = i;
      }
      o += cp[i].blob.size();
    }
    htrace("h2d", (long)(o - o0));
    if (b > a) {
      HIPCHK(hipMemcpyAsync((uint8_t*)d_descs.p + o0, hdesc + o0, o - o0, hipMemcpyHostToDevice, st_));
      htrace("c1");
      if (a == 0 && b == n) {  // the whole batch: offsets, sizes and stats are one contiguous range
        HIPCHK(hipMemcpyAsync(d_meta.p, hp, meta + (size_t)n * sizeof(PodStats), hipMemcpyHostToDevice, st_));
      } else {
        HIPCHK(hipMemcpyAsync((uint32_t*)d_off.p + a, h_offs + a, (size_t)(b - a) * 4, hipMemcpyHostToDevice, st_));
        htrace("c2");
        HIPCHK(hipMemcpyAsync((uint32_t*)d_off.p + n + a, h_offs + n + a, (size_t)(b - a) * 4, hipMemcpyHostToDevice,
                              st_));
        htrace("c3");
        HIPCHK(hipMemcpyAsync((PodStats*)d_stats.p + a, hs + a, (size_t)(b - a) * sizeof(PodStats),
                              hipMemcpyHostToDevice, st_));
        htrace("c4");
      }
    }
    if (async) {
      HIPCHK(hipEventRecord(pev[2 * (size_t)staged_chunks], cstream));
      HIPCHK(hipStreamWaitEvent(s, pev[2 * (size_t)staged_chunks], 0));
    }
    ++staged_chunks;
    return KSG_OK;
  };
  if ((rc = stage(0, compiled))) return rc;
  if (eval) {
    HIPCHK(hipMemsetAsync(d_out.p, 0, (size_t)m.cap * 8 * kNumPlugins, s));
    HIPCHK(hipMemsetAsync(d_total.p, 0, (size_t)m.cap * 8, s));
  }
  BatchView bv = bview(n);
  const int stride = c->cfg.timing_stride;
  const size_t npairs = stride > 0 ? (size_t)((n + stride - 1) / stride) : 0;
  while (tev.size() < 2 * npairs) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    tev.push_back(e);
  }
  HIPCHK(hipEventRecord(ev0, s));
  int launches = 0, timed = 0;
  double bytes = 0;
  // persistent-loop geometry: G resident workgroups per rank, each <= kLoopMaxBlk node blocks of
  // the rank's shard (k_sched_loop).  Sharded, every rank uses the same G (from the largest shard):
  // the exchange has world * G participants.
  const int NB = (m.n + kBlock - 1) / kBlock;
  int32_t sblk0 = 0, snblk = NB;
  if (comm) shard_range(m.n, &sblk0, &snblk);
  const int NBs = (NB + W - 1) / W;
  // one resident workgroup per CU; in-process ranks share one device
  const int cus = cu_count > 0 ? cu_count : 256;
  const int max_wg = std::min(256 / W, comm && c->cfg.nccl_id.empty() ? cus / W : cus);
  int G = c->cfg.loop_wg > 0 ? c->cfg.loop_wg : 128;
  G = std::min(std::max(G, (NBs + kLoopMaxBlk - 1) / kLoopMaxBlk), std::min(std::max(NBs, 1), max_wg));
  // a single-pod call (the per-pod API) runs faster on the launch path: the loop's launch, granule
  // zeroing and LDS load of every node core cost more than two per-node launches (scripts/single_pod_probe.py)
  const bool loop_worth = comm || n > 1;
  // k_sched_loop's unit: 128-node workgroups (two evaluation waves: each role on a SIMD of its own, the
  // selection wave's phase 2 no longer shares one with phase 1) when they fit -- at most
  // kLoopMaxBlk units per workgroup, at most 256 participants -- else 256-node workgroups
  int GS = G, unit = 256;
  if (c->cfg.loop_unit != 256) {
    const int NU = 2 * NBs;  // 128-node units of the largest shard
    int g2 = c->cfg.loop_wg > 0 ? c->cfg.loop_wg : 128;
    g2 = std::min(std::max(g2, (NU + kLoopMaxBlk - 1) / kLoopMaxBlk), std::min(std::max(NU, 1), max_wg));
    if ((int64_t)g2 * kLoopMaxBlk >= NU && (int64_t)g2 * W <= 256) {
      GS = g2;
      unit = 128;
    }
  }
  // residency: a loop's workgroups spin on each other, so its whole grid -- every in-process rank's
  // grid, as those share this device -- must fit in what the CUs hold at once (loop_occ); a grid that
  // does not is never launched, instead of spinning until the give-up
  const int64_t dev_ranks = comm && !rccl ? W : 1;
  const bool use_loop = loop_worth && (!comm || dx) && !eval && c->cfg.persistent_loop && NB > 0 && GS >= 1 &&
                        (int64_t)GS * kLoopMaxBlk * unit >= (int64_t)NBs * kBlock &&
                        (int64_t)GS * dev_ranks <= (int64_t)cus * loop_occ[unit == 128 ? 0 : 1] &&
                        (int64_t)c->taint_max_per_node < ((int64_t)1 << 24) - 1;
  // k_agg_loop: the same geometry (node-sharded: over the device exchange, world * G participants);
  // every workgroup's LDS lists must hold its nodes' pods and terms plus everything this batch can add
  // (each pod, and its own terms, at most once).  Every rank decides alike: the check covers every
  // rank's workgroups (each rank holds the whole cluster).
  bool use_agg = loop_worth && (!comm || dx) && !eval && c->cfg.persistent_loop && c->cfg.agg_loop && NB > 0 && G >= 1 &&
                 G * W <= std::min(cus, 256) && (int64_t)G * kLoopMaxBlk >= NBs &&
                 (int64_t)G * dev_ranks <= (int64_t)cus * loop_occ[W > 1 ? 3 : 2] &&
                 (int64_t)c->taint_max_per_node < ((int64_t)1 << 24) - 1;
  int64_t spill_p = 0, spill_t = 0;  // k_agg_loop: HBM list entries per workgroup (AggView::spill)
  if (use_agg) {
    bool any = false;
    int64_t own = 0;
    for (int i = 0; i < compiled; ++i) any = any || agg_loop_ok(cp[i]);
    if (!pre_slot.empty())  // pods compiled later: their own terms are reserved already
      for (int32_t sl : pre_slot) own += (int64_t)c->pt_terms[(size_t)sl].size();
    else
      for (int i = 0; i < compiled; ++i) own += cp[i].own_terms;
    use_agg = any && c->pt_node.size() < ((size_t)1 << 23) && c->tt.size() < ((size_t)1 << 23);
    if (use_agg) {
      // participant p = r * G + w owns blocks [b0_r + nb_r * w / G, b0_r + nb_r * (w + 1) / G) (shard_range)
      std::vector<int32_t> wg_of((size_t)NB), np((size_t)G * W, 0), nt((size_t)G * W, 0);
      for (int r = 0; r < W; ++r) {
        const int64_t b0 = (int64_t)NB * r / W, nb = (int64_t)NB * (r + 1) / W - b0;
        for (int w = 0; w < G; ++w)
          for (int64_t k = b0 + nb * w / G; k < b0 + nb * (w + 1) / G; ++k) wg_of[(size_t)k] = r * G + w;
      }
      for (int32_t nd : c->pt_node)
        if (nd >= 0 && nd < m.n) np[(size_t)wg_of[(size_t)(nd / kBlock)]]++;
      for (const DTerm& tm : c->tt) {
        const int32_t nd = tm.kind >= 0 && tm.owner >= 0 ? c->pt_node[(size_t)tm.owner] : -1;
        if (nd >= 0 && nd < m.n) nt[(size_t)wg_of[(size_t)(nd / kBlock)]]++;
      }
      // entries past the LDS lists go to the workgroup's HBM spill rows (nodes that gathered many pods,
      // e.g. required pod affinity piling pods onto the nodes of the pods they follow)
      auto up64 = [](int64_t v) { return v <= 0 ? (int64_t)0 : (v + 63) / 64 * 64; };
      spill_p = up64(*std::max_element(np.begin(), np.end()) + (int64_t)n - kAggPods);
      spill_t = up64(*std::max_element(nt.begin(), nt.end()) + own - kAggTerms);
      use_agg = spill_p <= kAggSpillMax && spill_t <= kAggSpillMax;
    }
  }
  struct LoopRun { int first, count; double bytes; bool agg, timed; };
  std::vector<LoopRun> runs;
  // in-process ranks share one device: after a mid-batch drain (buffers regrown) the next loop launch
  // waits at the gate again, so no rank's allocation is pending while a peer's loop spins on it
  bool regate = false;
  std::vector<uint8_t> agg_pod((size_t)n, 0);  // scheduled by k_agg_loop (settle: node-sharded replicas)
  const int shard_lo = sblk0 * kBlock, shard_hi = (sblk0 + snblk) * kBlock;
  // loopTimingStride k: every k-th loop launch carries HIP events on its dispatch packet (0: none)
  auto loop_timed = [&](size_t r) { return c->cfg.loop_timing_stride > 0 && r % (size_t)c->cfg.loop_timing_stride == 0; };
  if (use_agg && (rc = agg_setup())) return rc;
  if (use_agg && (rc = ensure(d_aspill, (size_t)G * (size_t)(spill_p + spill_t) * 4 + 4))) return rc;
  if (use_loop || use_agg) {
    if (use_loop && (rc = gran_setup())) return rc;
    if ((rc = ensure(d_fail, kFailBytes))) return rc;
    HIPCHK(hipMemsetAsync(d_fail.p, 0, kFailBytes, s));
    // in-process groups: the leader's array of every rank's launch arguments (group_launch)
    if (comm && comm->in_process() && (rc = ensure(d_grp, (size_t)W * std::max(sizeof(LoopGroupArg), sizeof(AggGroupArg)))))
      return rc;
    if (c->cfg.loop_stamps) {
      const size_t sb = (size_t)n * 8 * 8 + 64 * 8 + (size_t)n * std::max(G, GS) * 8 * 8;
      if ((rc = ensure(d_stamps, sb))) return rc;
      HIPCHK(hipMemsetAsync(d_stamps.p, 0, sb, s));
#ifdef KSG_DIAG
      HIPCHK(set_diag((unsigned long long*)d_stamps.p + (size_t)n * 8));
#endif
    }
  }
  struct Chunk { int a, b; };
  std::vector<Chunk> chunks;
  while (cev.size() < bnd.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    cev.push_back(e);
  }
  auto close_chunk = [&](int upto) -> int {
    const int a = chunks.empty() ? 0 : chunks.back().b;
    hipStream_t ds = s;
    if (copy_stream) {  // results come back on the copy stream, off the compute stream's path
      HIPCHK(hipEventRecord(pev[2 * chunks.size() + 1], s));
      HIPCHK(hipStreamWaitEvent(cstream, pev[2 * chunks.size() + 1], 0));
      ds = cstream;
    }
    htrace("close", upto);
    HIPCHK(hipMemcpyAsync(hr + a, (DevResult*)d_results.p + a, (size_t)(upto - a) * sizeof(DevResult),
                          hipMemcpyDeviceToHost, ds));
    if (use_loop || use_agg) HIPCHK(hipMemcpyAsync(hfail + chunks.size(), d_fail.p, 4, hipMemcpyDeviceToHost, ds));
    HIPCHK(hipEventRecord(cev[chunks.size()], ds));
    chunks.push_back({a, upto});
    return KSG_OK;
  };
  // results + host shadow of the device-side assumes for pods [a, b)
  double settle_us = 0;  // loopStamps: host time spent mirroring results into the cache
  auto settle = [&](int a, int b) -> int {
    const auto Ts = clk::now();
    struct Acc {
      double* t; clk::time_point s;
      ~Acc() { *t += std::chrono::duration<double, std::micro>(clk::now() - s).count(); }
    } acc_{&settle_us, Ts};
    for (int i = a; i < b; ++i) {
      ksg_result& r = results[i];
      if (cp[i].error) {
        r = ksg_result{KSG_CODE_ERROR, -1, 0, 0, 0};
        c->pod_table_drop(cp[i].slot);
        continue;
      }
      const DevResult& d = hr[i];
      r.status = d.status;
      r.node_index = d.node;
      r.feasible_nodes = d.feasible;
      r.evaluated_nodes = d.feasible > 0 ? cp[i].num_all : (cp[i].prefilter_reject ? 0 : cp[i].num_all);
      if (rot_dev) {
        if (!cp[i].prefilter_reject) r.evaluated_nodes = d.evaluated;
        if (!cp[i].error) c->next_start = d.rot_next;  // the last launched pod's wins
      }
      r.total_score = d.feasible > 1 ? d.total : 0;
      const uint32_t early = reinterpret_cast<const PodDesc*>(cp[i].blob.data())->flags & DF_EARLY;
      if (d.hinted && early) {  // the hinted (k_ob_hint) or nominated (k_nominated) node alone was evaluated
                                // (other paths leave the word unset)
        r.evaluated_nodes = 1;
        if (d.hinted == 1u) ++ob_hinted_;
      }
      if (cp[i].prefilter_reject) { r.status = KSG_CODE_UNSCHEDULABLE; r.node_index = -1; r.feasible_nodes = 0; }
      if (assume && r.status == KSG_CODE_SUCCESS && r.node_index >= 0) {
        // (a per-context count, as the oracle's assumeSeq: victims name assumed pods by this uid)
        std::string uid = pods[i]->uid + "#a" + std::to_string(++assume_seq_);
        // a node-sharded k_agg_loop applies the AssumePod to the mirror on the node's own rank only (the
        // other ranks record the result and the pod table entry): theirs go up with the next node updates
        const bool foreign = agg_pod[(size_t)i] && comm &&
                             (r.node_index < shard_lo || r.node_index >= shard_hi);
        int rc2 = c->add_pod(*pods[i], uid, /*device_done=*/!foreign, cp[i].slot, &c->order()[r.node_index], &cp[i].res);
        if (rc2) return rc2;
        assumed[handles.empty() ? -1 : handles[i]] = uid;
        nominated.erase(pods[i]->uid);  // an assumed pod's nomination ends (schedule_one.go:1131-1134)
      } else {
        c->pod_table_drop(cp[i].slot);  // not placed: the reserved pod-table slot never went live
      }
    }
    return KSG_OK;
  };
  // A persistent loop gave up (a workgroup never reached an exchange): pods [first, n) are not
  // scheduled -- their results say Error, their pod-table slots are released, nextStartNodeIndex is
  // rewound to before them -- and the device mirror, which may hold some of their assumes, is
  // rebuilt from the cache shadow at the next cycle.  The context stays usable.
  auto loop_fault = [&](int first, const std::string& why) -> int {
    (void)hipStreamSynchronize(s);
    if (cstream) (void)hipStreamSynchronize(cstream);
    for (int j = first; j < n; ++j) {
      results[j] = ksg_result{KSG_CODE_ERROR, -1, 0, 0, 0};
      c->pod_table_drop(j < compiled ? cp[j].slot : (pre_slot.empty() ? -1 : pre_slot[j]));
    }
    if (first < n && !rot_dev) c->next_start = ns_before[(size_t)first];
    c->layout_dirty = true;
    c->mirror_suspect = true;  // not a gather re-layout: unchanged nodes' device columns are suspect too
    c->pods_dirty = true;
    ob_invalidate();
    c->err = why + ": pods " + std::to_string(first) + ".." + std::to_string(n - 1) +
             " of the batch were not scheduled (status Error); the device mirror is rebuilt from the cache";
    fault_first_ = first;
    return KSG_EDEVICE;
  };
  auto fault_detail = [&]() -> std::string {
    uint32_t f[kFailWords] = {};
    (void)hipMemcpyAsync(f, d_fail.p, kFailBytes, hipMemcpyDeviceToHost, s);  // not the null stream (§6)
    (void)hipStreamSynchronize(s);
    if (f[1] >= 0xfffffff0u)  // k_agg_loop's own checks (list capacity): the first failure is kept
      return "persistent loop stopped: workgroup " + std::to_string(f[2]) + " failed check " + std::to_string(0xffffffffu - f[1]) +
             " (1: its pod / term lists exceed their capacity at launch, 2: an append overflowed)";
    const bool agg = f[4] == 2;
    const int g = agg ? G : GS, ng = agg ? kAGran : kGran;
    std::vector<unsigned long long> row((size_t)W * g * ng);
    const DevBuf& gb = agg ? d_agran : d_gran;
    if (gb.p && ((size_t)f[1] + 1) * row.size() * 8 <= gb.bytes)
      (void)hipMemcpyAsync(row.data(), (const unsigned long long*)gb.p + (size_t)f[1] * row.size(), row.size() * 8,
                           hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    return "persistent loop gave up (an exchange granule never arrived) on rank " + std::to_string(comm ? c->cfg.rank : 0) +
           ": " + give_up_detail(f, row, ng, W, g);
  };
  int settled = 0;  // chunks whose results are mirrored into the cache
  auto settle_closed = [&]() -> int {  // after a stream sync: every closed chunk
    for (; settled < (int)chunks.size(); ++settled) {
      if ((use_loop || use_agg) && hfail[settled]) return loop_fault(chunks[settled].a, fault_detail());
      const int r2 = settle(chunks[settled].a, chunks[settled].b);
      if (r2) return r2;
    }
    return KSG_OK;
  };
  // compile + stage the chunk starting at pod i while the device runs the chunks before it
  auto next_chunk = [&](int i) -> int {
    const int b = chunk_end(i);
    htrace("compile", i);
    c->defer_relayout = true;  // the earlier chunks' assumes are not in the shadow yet
    int r2 = compile_upto(b);
    c->defer_relayout = false;
    htrace("compiled", b);
    auto drain = [&]() -> int {  // close chunk k, wait for both streams
      if ((chunks.empty() || chunks.back().b < i) && close_chunk(i)) return KSG_EDEVICE;
      HIPCHK(hipStreamSynchronize(s));
      if (cstream) HIPCHK(hipStreamSynchronize(cstream));
      return KSG_OK;
    };
    if (r2) {  // the pods before i are scheduled: finish their bookkeeping, release the rest's slots
      if (drain()) return KSG_EDEVICE;
      const int r3 = settle_closed();
      if (r3) return r3;
      // pods [i, compiled) took their slots in compile (node-local batches: pre_slot empty) or up front;
      // pods past them only up front
      for (int j = i; j < compiled; ++j) c->pod_table_drop(pre_slot.empty() ? cp[j].slot : pre_slot[j]);
      for (int j = compiled; j < (int)pre_slot.size(); ++j) c->pod_table_drop(pre_slot[j]);
      if (!rot_dev) c->next_start = ns_before[(size_t)i];  // pods [i, b) were compiled, never launched
      return r2;
    }
    size_t need = 0;
    int32_t aw = 0;
    for (int j = i; j < b; ++j) {
      need += cp[j].blob.size();
      aw = std::max(aw, cp[j].arena_words);
    }
    // (a stale pod table matters only to a batch with pods that read it: pods_needed)
    if (c->layout_dirty || (c->pods_dirty && pods_needed) || o + need > desc_cap || aw > arena_words) {
      // the mirror must be re-laid out or the buffers grown: drain the device and mirror what it
      // assumed first (the same state a batch boundary here would give)
      htrace("drain", i);
      if ((r2 = drain())) return r2;
      if (c->cfg.loop_stamps)
        std::fprintf(stderr, "[host] pipeline drained before pod %d (%s)\n", i,
                     c->layout_dirty || (c->pods_dirty && pods_needed) ? "mirror re-layout" : "staging grown");
      if ((r2 = settle_closed())) return r2;
      if (comm && comm->launch_gate()) {  // every rank drained before any rank allocates
        c->err = comm->err;
        return KSG_EDEVICE;
      }
      regate = true;
      if ((r2 = c->ensure_mirror())) return r2;
      arena_words = std::max(arena_words, aw);
      o = 0;
      if ((r2 = ensure_scratch(std::max(need, desc_bytes), n, false, arena_words))) return r2;
      map_pinned();
      bv = bview(n);
    }
    htrace("stage", i);
    r2 = stage(i, b);
    htrace("staged", i);
    return r2;
  };
  for (int i = 0; i < n && (!comm || dx);) {
    if (i > 0 && std::binary_search(bnd.begin(), bnd.end(), i) && (chunks.empty() || chunks.back().b < i)) {
      if (i >= compiled && (rc = next_chunk(i))) return rc;  // its H2D does not wait for chunk k
      if ((chunks.empty() || chunks.back().b < i) && (rc = close_chunk(i))) return rc;
    }
    if (cp[i].error) {
      ++i;
      continue;
    }
    if (use_loop && loop_ok(cp[i])) {  // a run of node-local pods: one k_sched_loop launch
      int j = i;
      double rb = 0;
      const int cut = chunk_end(i);
      while (j < n && j < cut && j - i < kLoopMaxPods && loop_ok(cp[j]))
        rb += algo_bytes(*reinterpret_cast<const PodDesc*>(cp[j++].blob.data())) *
              (comm && m.n > 0 ? std::min(1.0, (double)snblk * kBlock / (double)m.n) : 1.0);
      while (lev.size() < 2 * (runs.size() + 1)) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        lev.push_back(e);
      }
      LoopView lv{};
      lv.first_pod = i;
      lv.npods = j - i;
      lv.nwg = GS;
      lv.blk0 = sblk0;
      lv.nblk = snblk;
      lv.world = W;
      lv.rank = comm ? c->cfg.rank : 0;
      if ((rc = next_gran_tag(&lv.tag))) return rc;
      for (int r = 0; r < W; ++r) lv.gran[r] = gran_all[r];
      lv.fail = (uint32_t*)d_fail.p;
      lv.stamps = c->cfg.loop_stamps ? (unsigned long long*)d_stamps.p + (size_t)i * 8 : nullptr;
      lv.desc_bytes = (const uint32_t*)d_off.p + n;
      lv.give_up_at = c->cfg.debug_give_up_at;
      lv.wave_map = c->cfg.loop_wave_map;
      lv.wstamps = c->cfg.loop_stamps ? (unsigned long long*)d_stamps.p + (size_t)n * 8 + 64 + (size_t)i * GS * 8 : nullptr;
      // in-process ranks: every rank is past its allocations before any rank's first loop starts
      if ((runs.empty() || regate) && comm) htrace("gate", i);
      if ((runs.empty() || regate) && comm && comm->launch_gate()) {
        c->err = comm->err;
        return KSG_EDEVICE;
      }
      regate = false;
      const bool tl = loop_timed(runs.size());
      htrace("loop", i);
      hipEvent_t t0 = tl ? lev[2 * runs.size()] : nullptr, t1 = tl ? lev[2 * runs.size() + 1] : nullptr;
      if (comm && comm->in_process()) {
        GroupReq req{};
        req.la = LoopGroupArg{m, bv, lv};
        req.t0 = t0;
        req.t1 = t1;
        if ((rc = group_launch(&req, false, GS, unit))) return rc;
      } else {
        HIPCHK(launch_sched_loop(m, bv, lv, s, t0, t1, unit));
      }
      runs.push_back({i, j - i, rb, false, tl});
      launches += j - i;
      i = j;
      continue;
    }
    if (use_agg && agg_loop_ok(cp[i])) {  // a run of pod-table pods: one k_agg_loop launch
      int j = i;
      double rb = 0;
      int32_t gw = 1;
      const int cut = chunk_end(i);
      bool ptss = false;
      while (j < n && j < cut && j - i < kLoopMaxPods && agg_loop_ok(cp[j]) && !loop_ok(cp[j])) {
        const PodDesc& hd = *reinterpret_cast<const PodDesc*>(cp[j].blob.data());
        ptss = ptss || ((hd.score_mask >> P_PTS) & 1u) || hd.n_ptss > 0;
        rb += algo_bytes(hd) + agg_bytes(hd);
        gw = std::max(gw, hd.agg_gwords);
        ++j;
      }
      while (lev.size() < 2 * (runs.size() + 1)) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        lev.push_back(e);
      }
      gw = (gw + 15) & ~15;  // whole 128-byte lines per pod's row: no line holds two pods' sums
      const size_t rbytes = (size_t)(j - i) * (size_t)gw * 8;  // <= kLoopMaxPods * kAggGWords words
      HIPCHK(hipMemsetAsync(d_region.p, 0, rbytes, s));  // (sharded: the loop's start barrier orders the peers' adds)
      AggView av{};
      av.first_pod = i;
      av.npods = j - i;
      av.nwg = G;
      av.blk0 = sblk0;
      av.nblk = snblk;
      av.world = W;
      av.rank = comm ? c->cfg.rank : 0;
      if (comm) {
        av.grans = (unsigned long long* const*)d_aggpeers.p;
        av.regions = (unsigned long long* const*)d_aggpeers.p + W;
      }
      if ((rc = next_gran_tag(&av.tag))) return rc;
      av.gwords = gw;
      av.ptss = ptss ? 1 : 0;
      av.spill = (uint32_t*)d_aspill.p;
      av.spill_pods = (int32_t)spill_p;
      av.spill_terms = (int32_t)spill_t;
      av.debug = c->cfg.agg_debug;
      av.give_up_at = c->cfg.debug_give_up_at;
      av.gran = (unsigned long long*)d_agran.p;
      av.region = (unsigned long long*)d_region.p;
      av.fail = (uint32_t*)d_fail.p;
      av.desc_bytes = (const uint32_t*)d_off.p + n;
      // the template cache (aggLoopDebug bits 0 / 2: no folds / no same-template shortcut; bit 5: no cache)
      if (!comm && !ptss && !(c->cfg.agg_debug & (1 | 4 | 32))) {
        if (h_tcw_n < (size_t)n) {
          if (h_tcw) (void)hipHostFree(h_tcw);
          h_tcw = nullptr;
          h_tcw_n = 0;
          HIPCHK(hipHostMalloc((void**)&h_tcw, (size_t)n * 2 * 4, hipHostMallocDefault));
          h_tcw_n = (size_t)n * 2;
        }
        if ((rc = ensure(d_tcw, (size_t)n * 4 + 64))) return rc;
        if ((rc = ensure(d_tcache, (size_t)G * kAggTc * kTcWords * 8))) return rc;
        tc_plan(cp, i, j, h_tcw + i);
        HIPCHK(hipMemcpyAsync((uint32_t*)d_tcw.p + i, h_tcw + i, (size_t)(j - i) * 4, hipMemcpyHostToDevice, s));
        av.tcw = (const uint32_t*)d_tcw.p;
        av.tcache = (unsigned long long*)d_tcache.p;
      }
      if (c->cfg.loop_stamps) {
        const size_t sb = ((size_t)n * kAggStamps + (size_t)n * G * 4) * 8;
        if ((rc = ensure(d_astamps, sb))) return rc;
        if (runs.empty() || !runs.back().agg) HIPCHK(hipMemsetAsync(d_astamps.p, 0, sb, s));
      }
      av.stamps = c->cfg.loop_stamps ? (unsigned long long*)d_astamps.p + (size_t)i * kAggStamps : nullptr;
      av.wstamps = c->cfg.loop_stamps ? (unsigned long long*)d_astamps.p + (size_t)n * kAggStamps + (size_t)i * G * 4
                                      : nullptr;
      // in-process ranks: every rank is past its allocations before any rank's first loop starts
      if ((runs.empty() || regate) && comm && comm->launch_gate()) {
        c->err = comm->err;
        return KSG_EDEVICE;
      }
      regate = false;
      const bool tl = loop_timed(runs.size());
      hipEvent_t t0 = tl ? lev[2 * runs.size()] : nullptr, t1 = tl ? lev[2 * runs.size() + 1] : nullptr;
      if (comm && comm->in_process()) {
        GroupReq req{};
        req.aa = AggGroupArg{m, bv, av};
        req.t0 = t0;
        req.t1 = t1;
        if ((rc = group_launch(&req, true, G, 0))) return rc;
      } else {
        HIPCHK(launch_agg_loop(m, bv, av, s, t0, t1));
      }
      runs.push_back({i, j - i, rb, true, tl});
      std::fill(agg_pod.begin() + i, agg_pod.begin() + j, (uint8_t)1);
      launches += j - i;
      i = j;
      continue;
    }
    if (comm) {  // sharded, not loop-eligible: the per-pod RCCL exchange path
      if ((rc = run_sharded(cp, bv, i, i + 1, &launches, &bytes, &timed))) return rc;
      ++i;
      continue;
    }
    const PodDesc& hd = *reinterpret_cast<const PodDesc*>(cp[i].blob.data());
    const bool lds = cp[i].blob.size() <= (size_t)kBlobLds;
    if (hd.flags & DF_AGGREGATE) HIPCHK(launch_aggregate(m, bv, i, hd, s));
    if (hd.flags & DF_NOMINATED) HIPCHK(launch_nominated(m, bv, i, s));  // evaluateNominatedNode (counts ready)
    if (hd.flags & DF_OB) HIPCHK(launch_ob_hint(m, bv, i, s));  // GetNodeHint (its counts are ready)
    const bool t = stride > 0 && i % stride == 0;
    if (t) {
      HIPCHK(launch_filter_score(m, bv, i, s, tev[2 * (size_t)timed], tev[2 * (size_t)timed + 1], 0, -1, lds));
      timed++;
    } else {
      HIPCHK(launch_filter_score(m, bv, i, s, nullptr, nullptr, 0, -1, lds));
    }
    if (hd.flags & DF_ROTDEV) HIPCHK(launch_sample(m, bv, i, (hd.flags & DF_SAMPLE) != 0, s));
    if (hd.score_mask & (1u << P_PTS)) HIPCHK(launch_pts_score(m, bv, i, s));
    HIPCHK(launch_select(m, bv, i, s, lds));
    if (hd.flags & DF_OB) HIPCHK(launch_ob_store(bv, i, s));  // StoreScheduleResults
    bytes += algo_bytes(hd);
    launches++;
    ++i;
  }
  if (comm && !dx)  // sharded without the device exchange: every pod through the RCCL path
    if ((rc = run_sharded(cp, bv, 0, n, &launches, &bytes, &timed))) return rc;
  HIPCHK(hipEventRecord(ev1, s));
  const auto T2 = clk::now();
  if ((rc = close_chunk(n))) return rc;
  std::vector<uint32_t> st;
  std::vector<int64_t> outs, tot;
  std::vector<unsigned long long> gath;
  if (eval && comm) {
    // node-sharded: gather every rank's range of the per-node vectors (collective: every rank's call
    // carries the same evaluation request, as it carries the same pods)
    const size_t words = (size_t)(2 + kNumPlugins) * (size_t)m.n;
    if ((rc = ensure(d_evg, words * 8 + 8))) return rc;
    HIPCHK(hipMemsetAsync(d_evg.p, 0, words * 8, s));
    const int lo = shard_blk0 * kBlock, hi = std::min(m.n, (shard_blk0 + shard_nblk) * kBlock);
    HIPCHK(launch_eval_pack(bv, m.n, m.cap, lo, hi, (unsigned long long*)d_evg.p, s));
    if (comm->all_reduce_max((unsigned long long*)d_evg.p, words, s)) {
      c->err = comm->err;
      return KSG_EDEVICE;
    }
    gath.resize(words);
    HIPCHK(hipMemcpyAsync(gath.data(), d_evg.p, words * 8, hipMemcpyDeviceToHost, s));
  }
  if (eval) {
    st.resize(m.n);
    outs.resize((size_t)m.cap * kNumPlugins);
    tot.resize(m.n);
    if (!comm) {
      HIPCHK(hipMemcpyAsync(st.data(), d_status.p, (size_t)m.n * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(outs.data(), d_out.p, outs.size() * 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(tot.data(), d_total.p, (size_t)m.n * 8, hipMemcpyDeviceToHost, s));
    }
  }
  std::string chunk_log;  // loopStamps: per chunk, the host's wait for its results and its settle (us)
  if (chunks.size() > 1)  // pipelined: settle each chunk as soon as its results have landed
    for (size_t k = (size_t)settled; k < chunks.size(); ++k) {
      const auto Tw = clk::now();
      const double s0 = settle_us;
      htrace("wait", (long)k);
      HIPCHK(hipEventSynchronize(cev[k]));
      htrace("waited", (long)k);
      const double wt = std::chrono::duration<double, std::micro>(clk::now() - Tw).count();
      if ((use_loop || use_agg) && hfail[k]) return loop_fault(chunks[k].a, fault_detail());
      if ((rc = settle(chunks[k].a, chunks[k].b))) return rc;
      if (c->cfg.loop_stamps) {
        char buf[96];
        std::snprintf(buf, sizeof buf, " [%d pods: wait %.1f settle %.1f]", chunks[k].b - chunks[k].a, wt, settle_us - s0);
        chunk_log += buf;
      }
    }
  HIPCHK(hipStreamSynchronize(s));
  if (copy_stream) HIPCHK(hipStreamSynchronize(cstream));
  const auto T3 = clk::now();
  if (comm && comm->batch_end()) {
    c->err = comm->err;
    return KSG_EDEVICE;
  }
  if (!runs.empty()) {
    uint32_t fail = 0;
    HIPCHK(hipMemcpyAsync(&fail, d_fail.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (fail) return loop_fault(n, fault_detail());
  }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, ev0, ev1);
  last_kernel_ms = launches ? ms / (2.0 * launches) : 0;
  if (timed) {
    double sum = 0;
    for (int k = 0; k < timed; ++k) {
      float x = 0;
      HIPCHK(hipEventElapsedTime(&x, tev[2 * (size_t)k], tev[2 * (size_t)k + 1]));
      sum += x;
    }
    last_kernel_ms = sum / timed;
  }
  last_bytes = launches ? bytes / launches : 0;
  last_launches = launches;
  last_kernel = 0;
  if (!runs.empty()) {  // a loop dominates: per-pod time inside k_sched_loop / k_agg_loop and bytes per pod
    double lms[2] = {0, 0}, lb[2] = {0, 0};
    int lp[2] = {0, 0}, tp[2] = {0, 0};
    for (size_t r = 0; r < runs.size(); ++r) {
      const int k = runs[r].agg ? 1 : 0;
      if (runs[r].timed) {
        float x = 0;
        HIPCHK(hipEventElapsedTime(&x, lev[2 * r], lev[2 * r + 1]));
        lms[k] += x;
        tp[k] += runs[r].count;
      }
      lb[k] += runs[r].bytes;
      lp[k] += runs[r].count;
    }
    const int k = lp[1] > lp[0] ? 1 : 0;
    if (lp[k] * 2 >= launches) {
      last_kernel = 1 + k;
      last_kernel_ms = tp[k] ? lms[k] / tp[k] : 0.0;  // per pod over the timed launches
      last_bytes = lb[k] / lp[k];
      last_launches = lp[k];  // the pods that loop kernel ran
    }
    if (c->cfg.loop_stamps) {  // mean per-phase time (us) of the looped pods, workgroup 0's view
      std::vector<LoopRun> sruns, aruns;
      for (auto& r : runs) (r.agg ? aruns : sruns).push_back(r);
      {  // k_agg_loop (workgroup 0, wave 0): phase 1, A, phase 2 + B publish, B + commit, wait for the
         // next pod's gathering; then (folded pods) Z, chosen node + totals, fold + minima; gap
        std::vector<unsigned long long> st((size_t)n * kAggStamps);
        if (!aruns.empty())
          HIPCHK(hipMemcpy(st.data(), d_astamps.p, st.size() * 8, hipMemcpyDeviceToHost));
        double acc[10] = {0}, ns_prep = 0;
        int cnt = 0, cspec = 0, cns = 0;
        for (auto& r : aruns)
          for (int q = r.first; q + 1 < r.first + r.count; ++q) {
            const unsigned long long* t = &st[(size_t)q * kAggStamps];
            const unsigned long long nx = st[(size_t)(q + 1) * kAggStamps];
            bool okq = nx != 0;
            for (int k : {0, 1, 2, 3, 4, 5, 8}) okq = okq && t[k] != 0;
            if (!okq) continue;
            for (int k = 1; k <= 5; ++k) acc[k] += (double)(t[k] - t[k - 1]) / 100.0;
            if (t[6] && t[7]) {
              acc[6] += (double)(t[6] - t[5]) / 100.0;
              acc[7] += (double)(t[7] - t[6]) / 100.0;
              acc[8] += (double)(t[8] - t[7]) / 100.0;
              cspec++;
            } else {
              ns_prep += (double)(t[8] - t[5]) / 100.0;
              cns++;
            }
            acc[9] += (double)(nx - t[8]) / 100.0;
            cnt++;
          }
        {  // per-workgroup skew: spread of phase-1 start, A publish, B publish; who is last
          std::vector<unsigned long long> ws((size_t)n * G * 4);
          if (!aruns.empty())
            HIPCHK(hipMemcpy(ws.data(), (unsigned long long*)d_astamps.p + (size_t)n * kAggStamps, ws.size() * 8,
                             hipMemcpyDeviceToHost));
          double sk[4] = {0}, ph1max = 0, ph1min = 0, lastA_hop = 0;
          int sc = 0;
          for (auto& r : aruns)
            for (int q = r.first; q < r.first + r.count; ++q) {
              unsigned long long mn[4], mx[4];
              bool okq = true;
              for (int k = 0; k < 4; ++k) { mn[k] = ~0ull; mx[k] = 0; }
              double p1mx = 0, p1mn = 1e30;
              for (int g = 0; g < G; ++g)
                for (int k = 0; k < 4; ++k) {
                  const unsigned long long v = ws[((size_t)q * G + g) * 4 + k];
                  okq = okq && v != 0;
                  mn[k] = std::min(mn[k], v);
                  mx[k] = std::max(mx[k], v);
                }
              if (!okq) continue;
              for (int g = 0; g < G; ++g) {
                const double p1 = (double)(ws[((size_t)q * G + g) * 4 + 1] - ws[((size_t)q * G + g) * 4]) / 100.0;
                p1mx = std::max(p1mx, p1);
                p1mn = std::min(p1mn, p1);
              }
              for (int k = 0; k < 4; ++k) sk[k] += (double)(mx[k] - mn[k]) / 100.0;
              ph1max += p1mx;
              ph1min += p1mn;
              lastA_hop += (double)(mn[2] - mx[1]) / 100.0;  // last A publish -> first B publish
              sc++;
            }
          if (sc)
            std::fprintf(stderr, "[k_agg_loop skew over workgroups, us] phase-1 start %.3f  A publish %.3f  B publish %.3f  "
                         "commit end %.3f | phase 1 max %.3f min %.3f | last A -> first B %.3f\n", sk[0] / sc, sk[1] / sc,
                         sk[2] / sc, sk[3] / sc, ph1max / sc, ph1min / sc, lastA_hop / sc);
        }
        {  // wave 0 inside "phase2+B publish": my half, wave 1's half, B publish, BN publish
          double p2[4] = {0}, ns_half = 0;
          int c2 = 0, cns2 = 0;
          for (auto& r : aruns)
            for (int q = r.first; q < r.first + r.count; ++q) {
              const unsigned long long* t = &st[(size_t)q * kAggStamps];
              if (!t[2] || !t[10] || !t[11] || !t[12] || !t[3]) continue;
              if (!t[6]) {  // no gathering beside this phase 2 (the next pod is gathered after the barrier)
                ns_half += (double)(t[10] - t[2]) / 100.0;
                cns2++;
              }
              p2[0] += (double)(t[10] - t[2]) / 100.0;
              p2[1] += (double)(t[11] - t[10]) / 100.0;
              p2[2] += (double)(t[12] - t[11]) / 100.0;
              p2[3] += (double)(t[3] - t[12]) / 100.0;
              c2++;
            }
          if (c2)
            std::fprintf(stderr, "[k_agg_loop phase 2, us] my half %.3f (without a gathering beside it: %.3f, %d pods)  "
                         "wait wave 1 %.3f  B publish %.3f  eligibility + BN publish %.3f\n", p2[0] / c2,
                         cns2 ? ns_half / cns2 : 0.0, cns2, p2[1] / c2, p2[2] / c2, p2[3] / c2);
        }
        {  // the gathering waves' template-cache work (workgroup 0, wave 2): from phase 1's end to the write-back
           // / fold done (13), the load done (14), the window's end (15)
          double wa[3] = {0};
          int wc = 0;
          for (auto& r : aruns)
            for (int q = r.first; q < r.first + r.count; ++q) {
              const unsigned long long* t = &st[(size_t)q * kAggStamps];
              if (!t[1] || !t[13] || !t[14] || !t[15]) continue;
              wa[0] += (double)(t[13] - t[1]) / 100.0;
              wa[1] += (double)(t[14] - t[13]) / 100.0;
              wa[2] += (double)(t[15] - t[14]) / 100.0;
              wc++;
            }
          if (wc)
            std::fprintf(stderr, "[k_agg_loop template cache, %d pods, us] write-back + fold %.3f  load %.3f  rest %.3f\n",
                         wc, wa[0] / wc, wa[1] / wc, wa[2] / wc);
        }
        if (cnt)
          std::fprintf(stderr, "[k_agg_loop stamps, %d pods, us] phase1 %.3f  A %.3f  phase2+B publish %.3f  "
                       "B+commit %.3f  wait gather %.3f | folded (%d): Z %.3f  node+totals %.3f  fold+minima %.3f | "
                       "unfolded (%d): counts %.3f | gap %.3f\n", cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt,
                       acc[4] / cnt, acc[5] / cnt, cspec, cspec ? acc[6] / cspec : 0.0, cspec ? acc[7] / cspec : 0.0,
                       cspec ? acc[8] / cspec : 0.0, cns, cns ? ns_prep / cns : 0.0, acc[9] / cnt);
      }
      std::vector<unsigned long long> st((size_t)n * 8);
      HIPCHK(hipMemcpy(st.data(), d_stamps.p, st.size() * 8, hipMemcpyDeviceToHost));
      double acc[9] = {0};
      int cnt = 0;
      for (auto& r : sruns)
        for (int q = r.first; q < r.first + r.count; ++q) {
          const unsigned long long* t = &st[(size_t)q * 8];
          const unsigned long long nxt = q + 1 < r.first + r.count ? st[(size_t)(q + 1) * 8] : 0;
          if (!t[0] || !t[6] || !nxt) continue;
          for (int k = 1; k <= 6; ++k) acc[k] += (double)(t[k] - t[k - 1]) / 100.0;
          acc[7] += (double)(nxt - t[6]) / 100.0;
          acc[8] += t[7] ? (double)(t[7] - t[0]) / 100.0 : 0.0;
          cnt++;
        }
#ifdef KSG_DIAG
      {
        unsigned long long dg[20];
        HIPCHK(hipMemcpy(dg, (unsigned long long*)d_stamps.p + (size_t)n * 8, sizeof dg, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[fast path of the last pod, us] load_fast %.3f | load_core %.3f taints %.3f filters %.3f "
                     "nascore %.3f fit %.3f balanced %.3f | loop body total %.3f reduce %.3f\n", (dg[17] - dg[16]) / 100.0,
                     (dg[9] - dg[8]) / 100.0, (dg[10] - dg[9]) / 100.0, (dg[11] - dg[10]) / 100.0,
                     (dg[12] - dg[11]) / 100.0, (dg[13] - dg[12]) / 100.0, (dg[14] - dg[13]) / 100.0,
                     (dg[18] - dg[17]) / 100.0, (dg[19] - dg[18]) / 100.0);
        std::fprintf(stderr, "[eval_node steps of the last pod, us] load_core %.3f filters %.3f pre-score %.3f fit %.3f "
                     "balanced %.3f image %.3f rest %.3f\n", (dg[1] - dg[0]) / 100.0, (dg[2] - dg[1]) / 100.0,
                     (dg[3] - dg[2]) / 100.0, (dg[4] - dg[3]) / 100.0, (dg[5] - dg[4]) / 100.0,
                     (dg[6] - dg[5]) / 100.0, (dg[7] - dg[6]) / 100.0);
      }
#endif
      {  // per-workgroup publish skew: max - min over workgroups of the A and B publish times
        std::vector<unsigned long long> ws((size_t)n * GS * 8);
        HIPCHK(hipMemcpy(ws.data(), (unsigned long long*)d_stamps.p + (size_t)n * 8 + 64, ws.size() * 8,
                         hipMemcpyDeviceToHost));
        double ska = 0, skb = 0, ab = 0;
        int sc = 0;
        for (auto& r : sruns)
          for (int q = r.first; q + 1 < r.first + r.count; ++q) {
            unsigned long long amin = ~0ull, amax = 0, bmin = ~0ull, bmax = 0, an = ~0ull;
            for (int g = 0; g < GS; ++g) {
              const unsigned long long a = ws[((size_t)q * GS + g) * 8], bb = ws[((size_t)q * GS + g) * 8 + 1];
              const unsigned long long a2 = ws[((size_t)(q + 1) * GS + g) * 8];
              amin = std::min(amin, a); amax = std::max(amax, a);
              bmin = std::min(bmin, bb); bmax = std::max(bmax, bb);
              an = std::min(an, a2);
            }
            if (!amin || !bmin || !an) continue;
            ska += (amax - amin) / 100.0;
            skb += (bmax - bmin) / 100.0;
            ab += (an - bmax) / 100.0;
            sc++;
          }
        {  // mean lateness of each workgroup's A publish behind the earliest; and of the workgroup
           // that owned the previous pod's chosen node
          std::vector<double> late(GS, 0.0);
          double wl = 0;
          int wn = 0, cntq = 0;
          for (auto& r : sruns)
            for (int q = r.first + 1; q < r.first + r.count; ++q) {
              unsigned long long amin = ~0ull;
              for (int g = 0; g < GS; ++g) amin = std::min(amin, ws[((size_t)q * GS + g) * 8]);
              if (!amin) continue;
              unsigned long long amax = 0;
              int gl = -1;
              for (int g = 0; g < GS; ++g) {
                const unsigned long long a = ws[((size_t)q * GS + g) * 8];
                late[g] += (a - amin) / 100.0;
                if (a > amax) { amax = a; gl = g; }
              }
              (void)gl;
              cntq++;
            }
          double own = 0, ownlate = 0, ownx = 0, seg[5] = {0}, oth[4] = {0};
          int segn = 0;
          int on = 0;
          for (auto& r : sruns)
            for (int q = r.first; q + 1 < r.first + r.count; ++q)
              for (int g = 0; g < GS; ++g) {
                const unsigned long long c0 = ws[((size_t)q * GS + g) * 8 + 2], c1 = ws[((size_t)q * GS + g) * 8 + 3];
                if (!c0 || !c1) continue;
                unsigned long long amin = ~0ull;
                for (int h = 0; h < GS; ++h) amin = std::min(amin, ws[((size_t)(q + 1) * GS + h) * 8]);
                const unsigned long long an = ws[((size_t)(q + 1) * GS + g) * 8];
                // against the earliest A(q+1) publish: the owner's pod start, its phase 1 (of q+1) end, its
                // helper's granules ready, its B sweep done -- and the same for the other workgroups
                const unsigned long long st = ws[((size_t)q * GS + g) * 8 + 7], p1 = ws[((size_t)q * GS + g) * 8 + 6];
                const unsigned long long hr = ws[((size_t)q * GS + g) * 8 + 5], bs = ws[((size_t)q * GS + g) * 8 + 4];
                if (st && p1 && hr && bs) {
                  seg[0] += ((double)st - (double)amin) / 100.0; seg[1] += ((double)p1 - (double)amin) / 100.0;
                  seg[2] += ((double)hr - (double)amin) / 100.0; seg[3] += ((double)bs - (double)amin) / 100.0;
                  double o[4] = {0, 0, 0, 0};
                  int on2 = 0;
                  for (int h = 0; h < GS; ++h) {
                    if (h == g) continue;
                    const unsigned long long* x = &ws[((size_t)q * GS + h) * 8];
                    if (!x[7] || !x[6] || !x[5] || !x[4]) continue;
                    o[0] += ((double)x[7] - (double)amin) / 100.0; o[1] += ((double)x[6] - (double)amin) / 100.0;
                    o[2] += ((double)x[5] - (double)amin) / 100.0; o[3] += ((double)x[4] - (double)amin) / 100.0;
                    on2++;
                  }
                  if (on2) for (int k = 0; k < 4; ++k) oth[k] += o[k] / on2;
                  segn++;
                }
                own += (c1 - c0) / 100.0;
                ownx += ((double)an - (double)c1) / 100.0;
                ownlate += ((double)an - (double)amin) / 100.0;
                on++;
              }
          if (segn)
            std::fprintf(stderr, "[k_sched_loop vs the earliest next-A publish, us] owner: pod start %.3f  phase-1 end %.3f  "
                         "helper ready %.3f  B swept %.3f | others: %.3f %.3f %.3f %.3f\n", seg[0] / segn, seg[1] / segn,
                         seg[2] / segn, seg[3] / segn, oth[0] / segn, oth[1] / segn, oth[2] / segn, oth[3] / segn);
          if (on)
            std::fprintf(stderr, "[k_sched_loop owner, us] commit+fixup %.3f  fixup end -> next A publish %.3f  "
                         "owner's next A lateness %.3f (%d pods)\n", own / on, ownx / on, ownlate / on, on);
          std::string o;
          for (int g = 0; g < GS; ++g) o += " " + std::to_string((int)(1000 * late[g] / std::max(cntq, 1)));
          std::fprintf(stderr, "[k_sched_loop A lateness per workgroup, ns]%s\n", o.c_str());
          (void)wl; (void)wn;
        }
        if (sc)
          std::fprintf(stderr, "[k_sched_loop skew over workgroups, us] A publish %.3f  B publish %.3f  "
                       "last B -> first next A %.3f  (A last->B first %.3f)\n", ska / sc, skb / sc, ab / sc, 0.0);
      }
      if (cnt)
        std::fprintf(stderr,
                     "[k_sched_loop stamps, %d pods, us] exchangeA %.3f phase2 %.3f publishB+preeval+stage %.3f "
                     "waitB %.3f wait-phase1(next pod) %.3f commit+fixup %.3f gap %.3f | phase1 end %.3f\n",
                     cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt, acc[4] / cnt, acc[5] / cnt, acc[6] / cnt,
                     acc[7] / cnt, acc[8] / cnt);
    }
  }

  // ---- results + host shadow of the device-side assumes
  if (chunks.size() <= 1 && settled == 0)
    if ((rc = settle(0, n))) return rc;
  if (c->cfg.loop_stamps) {
    const auto T4 = clk::now();
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::fprintf(stderr, "[host chunks]%s  settle total %.1f us\n", chunk_log.c_str(), settle_us);
    std::fprintf(stderr, "[host, us per pod] compile %.3f  stage+launch %.3f  wait %.3f  results+assume %.3f | "
                 "batch: API entry -> run %.1f us, chunk-0 compile %.1f us (slot reservation %.1f us), mirror + pod "
                 "table before the first launch %.1f us, settle after the wait %.1f us\n",
                 us(T0, T1) / n, us(T1, T2) / n, us(T2, T3) / n, us(T3, T4) / n,
                 api_t0_.time_since_epoch().count() ? us(api_t0_, T0) : 0.0, us(T0, T1), reserve_us_, mirror_us_,
                 us(T3, T4));
    reserve_us_ = 0;
    std::fprintf(stderr, "[chunk 0, us] plan + scalar check %.1f  program vectors %.1f  compile %.1f\n", c0_us_[0],
                 c0_us_[1], c0_us_[2]);
    std::fprintf(stderr, "[compile sections, us per pod] node-affinity %.3f  taints+ports %.3f  resources+images %.3f  "
                 "topology %.3f (spread %.3f  affinity %.3f  placement+tables %.3f)  masks+assume %.3f\n", cprof_[0] / n,
                 cprof_[1] / n, cprof_[2] / n, cprof_[3] / n, cprof_[5] / n, cprof_[6] / n, cprof_[7] / n, cprof_[4] / n);
    for (double& v : cprof_) v = 0;
  }
  if (eval && comm) {  // unpack the gathered vectors
    const size_t n = (size_t)m.n;
    for (size_t i = 0; i < n; ++i) {
      st[i] = (uint32_t)gath[i];
      for (int q = 0; q < kNumPlugins; ++q) outs[(size_t)q * m.cap + i] = (int64_t)gath[(1 + q) * n + i];
      tot[i] = (int64_t)gath[(1 + kNumPlugins) * n + i];
    }
  }
  const bool hinted0 =
      eval && hr[0].hinted && (reinterpret_cast<const PodDesc*>(cp[0].blob.data())->flags & (DF_OB | DF_EARLY));
  // placed on the OpportunisticBatching hint (k_ob_hint) or on its nominated node (k_nominated), which alone went
  // through the filters (schedule_one.go:586-598, 657-669): no other node has a status, no node a score
  if (hinted0) {
    std::fill(st.begin(), st.end(), 0u);
    std::fill(outs.begin(), outs.end(), 0);
    std::fill(tot.begin(), tot.end(), 0);
  }
  if (eval) {
    const int32_t N = m.n;
    eval->prefilter_code = cp[0].prefilter_reject ? cp[0].prefilter_code : 0;
    eval->prefilter_plugin = cp[0].prefilter_reject ? cp[0].prefilter_plugin : 255;
    uint32_t smask = cp[0].score_mask;
    if (!(hr[0].ipa_any & 8u)) smask &= ~(1u << P_IPA);  // InterPodAffinity PreScore Skip (scoring.go:207-209)
    eval->score_plugin_mask = (hr[0].feasible > 1 && !cp[0].prefilter_reject && !hinted0) ? smask : 0;
    for (int32_t i = 0; i < N; ++i) {
      const uint32_t w = st[i];
      if (eval->node_code) eval->node_code[i] = (uint8_t)status_code(w);
      if (eval->node_plugin)  // feasible nodes and PreFilterResult exclusions carry no plugin
        eval->node_plugin[i] = (status_code(w) == 0 || status_plugin(w) == 15u) ? 255 : (uint8_t)status_plugin(w);
      if (eval->node_reasons) eval->node_reasons[i] = status_reasons(w);
      const bool scored = hr[0].feasible > 1 && status_code(w) == 0;
      if (eval->total_scores) eval->total_scores[i] = scored ? tot[i] : 0;
      for (int q = 0; q < kNumPlugins; ++q) {  // the device wrote NormalizeScore's output; the weights are
        const int64_t v = scored ? outs[(size_t)q * m.cap + i] : 0;  // applied here (framework.go:1434-1446)
        if (eval->normalized_scores) eval->normalized_scores[(size_t)q * N + i] = v;
        if (eval->plugin_scores) eval->plugin_scores[(size_t)q * N + i] = v * c->cfg.weight[q];
      }
    }
  }
  return KSG_OK;
}

// This rank's contiguous block range of the snapshot order.
void Engine::shard_range(int32_t n, int32_t* blk0, int32_t* nblk) const {
  const int64_t NB = ((int64_t)n + kBlock - 1) / kBlock;
  const int W = c->cfg.world, r = c->cfg.rank;
  const int64_t b0 = NB * r / W, b1 = NB * (r + 1) / W;
  *blk0 = (int32_t)b0;
  *nblk = (int32_t)(b1 - b0);
}

// Node-sharded cycles: per pod, the replicated pod-table aggregation, this rank's node blocks,
// then the stream-ordered exchanges (comm.hpp) between the kernels -- 2 all-reduces per pod
// (3 when PodTopologySpread scores) and still no host round trip inside the batch.
int Engine::run_sharded(const std::vector<CompiledPod>& cp, const BatchView& bv, int first, int last, int* launches,
                        double* bytes, int* timed_out) {
  hipStream_t s = c->stream;
  const MirrorView& m = c->view;
  ShardView sv{};
  sv.world = c->cfg.world;
  sv.rank = c->cfg.rank;
  shard_range(m.n, &sv.blk0, &sv.nblk);
  shard_blk0 = sv.blk0;
  shard_nblk = sv.nblk;
  sv.xa = (unsigned long long*)d_xa.p;
  sv.xp = (unsigned long long*)d_xp.p;
  sv.xb = (unsigned long long*)d_xb.p;
  sv.xs = (unsigned long long*)d_xs.p;
  const double frac = m.n > 0 ? std::min(1.0, (double)sv.nblk * kBlock / (double)m.n) : 0.0;
  const int stride = c->cfg.timing_stride;
  int& timed = *timed_out;
  auto xchg = [&](unsigned long long* p, size_t count) -> int {
    if (comm->all_reduce_max(p, count, s)) {
      c->err = comm->err;
      return KSG_EDEVICE;
    }
    return KSG_OK;
  };
  for (int i = first; i < last; ++i) {
    if (cp[i].error) continue;
    const PodDesc& hd = *reinterpret_cast<const PodDesc*>(cp[i].blob.data());
    if (hd.flags & DF_AGGREGATE) HIPCHK(launch_aggregate(m, bv, i, hd, s));  // replicated pod table
    if (stride > 0 && i % stride == 0 && sv.nblk > 0) {
      HIPCHK(launch_filter_score(m, bv, i, s, tev[2 * (size_t)timed], tev[2 * (size_t)timed + 1], sv.blk0, sv.nblk,
                                 cp[i].blob.size() <= (size_t)kBlobLds));
      timed++;
    } else {
      HIPCHK(launch_filter_score(m, bv, i, s, nullptr, nullptr, sv.blk0, sv.nblk, cp[i].blob.size() <= (size_t)kBlobLds));
    }
    int rc = KSG_OK;
    if (hd.flags & DF_ROTDEV) {  // percentageOfNodesToScore: the cut needs every rank's counts first
      const bool cut = (hd.flags & DF_SAMPLE) != 0;
      HIPCHK(launch_sample_shard_a(m, bv, sv, i, s));
      if (cut && (rc = xchg(sv.xs + (size_t)i * XS_WORDS, XS_WORDS))) return rc;
      HIPCHK(launch_sample_shard_b(m, bv, sv, i, cut, s));
    }
    HIPCHK(launch_xpack_a(bv, sv, i, s));
    const bool pts = (hd.score_mask & (1u << P_PTS)) != 0;
    if (comm->group_begin()) return KSG_EDEVICE;
    rc = xchg(sv.xa + (size_t)i * XA_WORDS, XA_WORDS);
    if (!rc && pts) {  // ScheduleAnyway domain presence (arena words) is OR-ed across shards
      const PtsCons* cs = reinterpret_cast<const PtsCons*>(cp[i].blob.data() + hd.ptss_off);
      for (int32_t k = 0; k < hd.n_ptss && !rc; ++k)
        if (!cs[k].hostname && cs[k].nvals > 0) rc = xchg(bv.arena + cs[k].pres_base, (size_t)cs[k].nvals);
    }
    if (comm->group_end() || rc) return rc ? rc : KSG_EDEVICE;
    if (pts) {
      HIPCHK(launch_unpack_pts(bv, sv, i, s));
      HIPCHK(launch_pts_score(m, bv, i, s, sv.blk0, sv.nblk));
      HIPCHK(launch_xpack_p(bv, sv, i, s));
      if ((rc = xchg(sv.xp + (size_t)i * XP_WORDS, XP_WORDS))) return rc;
    }
    HIPCHK(launch_select_shard(m, bv, sv, i, s));
    if ((rc = xchg(sv.xb + (size_t)i * XB_WORDS, XB_WORDS))) return rc;
    HIPCHK(launch_commit(m, bv, sv, i, s));
    *bytes += algo_bytes(hd) * frac;
    (*launches)++;
  }
  return KSG_OK;
}

int Engine::run_plugin(const PodSpec& p, Mode mode, int plugin, const uint8_t* nodes, int32_t* code, uint8_t* codes,
                       uint32_t* reasons, int64_t* raw, int64_t* norm) {
  const int32_t N = (int32_t)c->order().size();
  *code = KSG_CODE_SUCCESS;
  for (int32_t i = 0; i < N; ++i) {
    if (codes) codes[i] = 0;
    if (reasons) reasons[i] = 0;
    if (raw) raw[i] = 0;
    if (norm) norm[i] = 0;
  }
  CompiledPod cp;
  int rc = compile(p, mode, plugin, false, true, &cp, nodes);
  if (rc) return rc;
  const PodDesc& D = *reinterpret_cast<const PodDesc*>(cp.blob.data());
  if (mode == FILTER_ONE) {
    // the plugin's own PreFilter first (framework.go:934-995): a rejection every node gets, or Skip
    if (cp.prefilter_reject) {
      *code = cp.prefilter_code;
      for (int32_t i = 0; i < N; ++i) {
        if (codes) codes[i] = (uint8_t)cp.prefilter_code;
        if (reasons) reasons[i] = KSG_R_PREFILTER;
      }
      return KSG_OK;
    }
    if (!(D.filter_mask & (1u << plugin))) { *code = KSG_CODE_SKIP; return KSG_OK; }
  } else {
    if (cp.error) { *code = KSG_CODE_ERROR; return KSG_OK; }
    if (!(D.score_mask & (1u << plugin))) { *code = KSG_CODE_SKIP; return KSG_OK; }
  }
  if (N == 0) {  // nothing to launch; only InterPodAffinity's Skip depends on counts (none here)
    if (plugin == P_IPA) *code = (mode == FILTER_ONE && cp.ipa_own_req) ? KSG_CODE_SUCCESS : KSG_CODE_SKIP;
    return KSG_OK;
  }
  if ((rc = c->ensure_mirror())) return rc;
  if ((rc = ensure_scratch(cp.blob.size(), 1, true, cp.arena_words))) return rc;
  uint8_t* hp = (uint8_t*)h_pinned;
  std::memcpy(hp, cp.blob.data(), cp.blob.size());
  uint32_t off0 = 0;
  PodStats* hs = (PodStats*)(hp + ((cp.blob.size() + 15) & ~size_t(15)));
  std::memset(hs, 0, sizeof(PodStats));
  for (int q = 0; q < kNumPlugins; ++q) {
    hs->max_raw[q] = enc_i64(INT64_MIN);
    hs->min_raw[q] = enc_i64(INT64_MAX);
  }
  hipStream_t s = c->stream;
  const MirrorView& m = c->view;
  HIPCHK(hipMemcpyAsync(d_descs.p, hp, cp.blob.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_off.p, &off0, 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_stats.p, hs, sizeof(PodStats), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(d_out.p, 0, (size_t)m.cap * 8 * kNumPlugins, s));
  const BatchView bv = bview(1);
  if (D.flags & DF_AGGREGATE) HIPCHK(launch_aggregate(m, bv, 0, D, s));
  const bool lds = cp.blob.size() <= (size_t)kBlobLds;
  HIPCHK(launch_filter_score(m, bv, 0, s, nullptr, nullptr, 0, -1, lds));
  if (mode == SCORE_ONE) {
    if (D.score_mask & (1u << P_PTS)) HIPCHK(launch_pts_score(m, bv, 0, s));
    HIPCHK(launch_select(m, bv, 0, s, lds));
  } else if (D.arena_words) {
    HIPCHK(hipMemsetAsync(d_arena.p, 0, (size_t)D.arena_words * 8, s));  // k_select did not run
  }
  PodStats hstat;
  HIPCHK(hipMemcpyAsync(&hstat, d_stats.p, sizeof(PodStats), hipMemcpyDeviceToHost, s));
  std::vector<uint32_t> st(N);
  std::vector<int64_t> rv(N), nv(N);
  if (mode == FILTER_ONE) {
    HIPCHK(hipMemcpyAsync(st.data(), d_status.p, (size_t)N * 4, hipMemcpyDeviceToHost, s));
  } else {
    HIPCHK(hipMemcpyAsync(rv.data(), (int64_t*)d_raw.p + (size_t)plugin * m.cap, (size_t)N * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(nv.data(), (int64_t*)d_out.p + (size_t)plugin * m.cap, (size_t)N * 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (plugin == P_IPA) {
    // InterPodAffinity's Skip decisions depend on device counts: PreFilter skips when no existing
    // anti-affinity term matched and the pod has no required terms (filtering.go:315-317);
    // PreScore skips when no term contributed (scoring.go:207-209)
    const bool skip = mode == FILTER_ONE ? (!cp.ipa_own_req && !(hstat.ipa_any & 4u)) : !(hstat.ipa_any & 8u);
    if (skip) {
      *code = KSG_CODE_SKIP;
      return KSG_OK;
    }
  }
  for (int32_t i = 0; i < N; ++i) {
    if (mode == FILTER_ONE) {
      if (codes) codes[i] = (uint8_t)status_code(st[i]);
      if (reasons) reasons[i] = status_reasons(st[i]);
    } else if (!nodes || nodes[i]) {
      if (raw) raw[i] = (plugin == P_PTS && rv[i] == -1) ? 0 : rv[i];  // ignored node (scoring.go:203-205)
      if (norm) norm[i] = nv[i];
    }
  }
  return KSG_OK;
}

// ===================================================================================================
// The resident single-pod loop.  kube-scheduler's scheduling goroutine calls
// SchedulePod once per pod (schedule_one.go:67-192), so ksg_schedule_one is the hot entry point of a
// real deployment.  A launch per call costs the loop's start (granule setup, LDS load of every node
// core) and the HIP API's per-copy overheads; instead one k_sched_loop launch stays resident and the
// host hands it each pod through a pinned ring (desc.h PodRing): the program and a doorbell go down,
// the DevResult comes back, with no HIP call on the path.  The launch ends on the host's stop (any
// other device user, or a mirror change it cannot see), after kLoopMaxPods pods (its granule indices),
// or by itself after kResidentIdleMs without a pod -- the host relaunches once it has been idle for
// half that, so a loop never outlives its process.
// ===================================================================================================
constexpr int kResidentIdleMs = 40;
// k_agg_loop's resident launch: own affinity terms its pods may append to the lists (spill-row budget)
constexpr int kRingTermBudget = 4096;

int Engine::resident_stop() {
  if (c->cfg.loop_stamps && res_prof_[4] > 0) {  // where a single-pod call's time went (us per call)
    const double n = res_prof_[4];
    std::fprintf(stderr, "[resident loop, %d calls, us per call] compile %.2f  post %.2f  device (post -> result seen) %.2f  "
                 "settle %.2f\n", (int)n, res_prof_[0] / n, res_prof_[1] / n, res_prof_[2] / n, res_prof_[3] / n);
    for (double& v : res_prof_) v = 0;
    std::fprintf(stderr, "[k_agg_loop ring posts] same %ld  own terms patched %ld  staged: sizes %ld, terms %ld, program %ld, "
                 "entry terms %ld, entry %ld, first %ld, no entry %ld, program size %ld, entry size %ld\n", res_posts_[0],
                 res_posts_[1], res_posts_[3], res_posts_[4], res_posts_[5], res_posts_[6], res_posts_[7], res_posts_[8],
                 res_posts_[9], res_posts_[10], res_posts_[11]);
    for (long& v : res_posts_) v = 0;
  }
  if (!res_running_) return KSG_OK;
  __atomic_store_n(&ring_->ctl, kCtlStop, __ATOMIC_RELEASE);
  __atomic_store_n(&ring_->ll[0], (unsigned long long)kRingStop, __ATOMIC_RELEASE);
  res_running_ = false;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->cfg.loop_stamps && res_kind_ == 1 && res_q_ > 1 && d_stamps.p) {
    // k_sched_loop ring pods, workgroup 0 (diagnostic build): doorbell seen (7) -> exchange A start (0: relay,
    // staging, phase 1, A publish) -> A swept (1) -> phase 2 (2) -> B published (3) -> B swept (4) -> barrier (5)
    // -> commit + result posted + barrier (6) -> the next pod's doorbell seen (host settle, compile, post, poll)
    std::vector<unsigned long long> st((size_t)res_q_ * 8);
    HIPCHK(hipMemcpy(st.data(), d_stamps.p, st.size() * 8, hipMemcpyDeviceToHost));
    static const int ks[] = {7, 0, 1, 2, 3, 4, 5, 6};
    double a[8] = {0};
    int cnt = 0;
    for (int q = 0; q + 1 < res_q_; ++q) {
      const unsigned long long* t = &st[(size_t)q * 8];
      const unsigned long long nx = st[(size_t)(q + 1) * 8 + 7];
      bool ok = nx != 0;
      for (int k : ks) ok = ok && t[k] != 0;
      if (!ok) continue;
      for (int k = 0; k < 7; ++k) a[k] += (double)(t[ks[k + 1]] - t[ks[k]]) / 100.0;
      a[7] += (double)(nx - t[6]) / 100.0;
      cnt++;
    }
    if (cnt)
      std::fprintf(stderr, "[k_sched_loop ring stamps, %d pods, us] doorbell -> A start %.2f  A %.2f  phase2 %.2f  "
                   "publishB %.2f  B %.2f  barrier %.2f  commit+post %.2f | next doorbell %.2f\n", cnt, a[0] / cnt,
                   a[1] / cnt, a[2] / cnt, a[3] / cnt, a[4] / cnt, a[5] / cnt, a[6] / cnt, a[7] / cnt);
  }
  if (c->cfg.loop_stamps && res_kind_ == 2 && res_q_ > 0 && d_astamps.p) {
    // k_agg_loop ring pods, workgroup 0's view (us): ring wait -> staged -> counts gathered (+ Z) -> totals ->
    // minima | phase 1 | A | phase 2 | B publish | B sweep + commit | end of pod
    std::vector<unsigned long long> st((size_t)res_q_ * kAggStamps);
    HIPCHK(hipMemcpy(st.data(), d_astamps.p, st.size() * 8, hipMemcpyDeviceToHost));
    // gathered pods: 9 13 14 15 0 ...; folded pods (DF_AGG_SAME): 9 13 0 ...
    static const int sg[] = {9, 13, 14, 15, 0, 1, 2, 10, 12, 4, 8}, sf[] = {9, 13, 0, 1, 2, 10, 12, 4, 8};
    double ag[10] = {0}, af[8] = {0};
    int cg = 0, cf = 0;
    for (int q = 0; q < res_q_; ++q) {
      const unsigned long long* t = &st[(size_t)q * kAggStamps];
      bool okg = true, okf = !t[14];
      for (int k : sg) okg = okg && t[k] != 0;
      for (int k : sf) okf = okf && t[k] != 0;
      if (okg) {
        for (int k = 0; k < 10; ++k) ag[k] += (double)(t[sg[k + 1]] - t[sg[k]]) / 100.0;
        cg++;
      } else if (okf) {
        for (int k = 0; k < 8; ++k) af[k] += (double)(t[sf[k + 1]] - t[sf[k]]) / 100.0;
        cf++;
      }
    }
    if (cg)
      std::fprintf(stderr, "[k_agg_loop ring stamps, %d gathered pods, us] staging %.2f  gather+Z %.2f  totals %.2f  "
                   "minima %.2f | phase1 %.2f  A %.2f  phase2 %.2f  publishB %.2f  B+commit %.2f  end %.2f\n", cg,
                   ag[0] / cg, ag[1] / cg, ag[2] / cg, ag[3] / cg, ag[4] / cg, ag[5] / cg, ag[6] / cg, ag[7] / cg,
                   ag[8] / cg, ag[9] / cg);
    if (cf)
      std::fprintf(stderr, "[k_agg_loop ring stamps, %d folded pods, us] staging %.2f  fold+minima %.2f | phase1 %.2f  "
                   "A %.2f  phase2 %.2f  publishB %.2f  B+commit %.2f  end %.2f\n", cf, af[0] / cf, af[1] / cf,
                   af[2] / cf, af[3] / cf, af[4] / cf, af[5] / cf, af[6] / cf, af[7] / cf);
  }
  return KSG_OK;
}

int Engine::schedule_resident(const PodSpec& p, int32_t handle, ksg_result* res, bool* handled) {
  using clk = std::chrono::steady_clock;
  *handled = false;
  if (comm || !c->cfg.resident_loop || !c->cfg.persistent_loop) return KSG_OK;
  const int32_t N = (int32_t)c->order().size();
  if (N == 0) return KSG_OK;
  // the loops' geometry (run_batch's, unsharded): k_sched_loop's GS workgroups of `unit` nodes, and
  // k_agg_loop's G workgroups of 256-node blocks
  const int NB = (N + kBlock - 1) / kBlock;
  const int cus = cu_count > 0 ? cu_count : 256;
  int GS = c->cfg.loop_wg > 0 ? c->cfg.loop_wg : 128, unit = 256;
  GS = std::min(std::max(GS, (NB + kLoopMaxBlk - 1) / kLoopMaxBlk), std::min(std::max(NB, 1), cus));
  if (c->cfg.loop_unit != 256) {
    const int NU = 2 * NB;
    int g2 = c->cfg.loop_wg > 0 ? c->cfg.loop_wg : 128;
    g2 = std::min(std::max(g2, (NU + kLoopMaxBlk - 1) / kLoopMaxBlk), std::min(std::max(NU, 1), cus));
    if ((int64_t)g2 * kLoopMaxBlk >= NU && g2 <= 256) {
      GS = g2;
      unit = 128;
    }
  }
  const bool taint_ok = (int64_t)c->taint_max_per_node < ((int64_t)1 << 24) - 1;
  const bool sched_geo = taint_ok && (int64_t)GS * kLoopMaxBlk * unit >= (int64_t)NB * kBlock &&
                         (int64_t)GS <= (int64_t)cus * loop_occ[unit == 128 ? 0 : 1];  // residency (run_batch)
  int G = c->cfg.loop_wg > 0 ? c->cfg.loop_wg : 128;
  G = std::min(std::max(G, (NB + kLoopMaxBlk - 1) / kLoopMaxBlk), std::min(std::max(NB, 1), std::min(cus, 256)));
  const bool agg_geo = taint_ok && c->cfg.agg_loop && (int64_t)G * kLoopMaxBlk >= NB &&
                       (int64_t)G <= (int64_t)cus * loop_occ[2] && c->pt_node.size() < ((size_t)1 << 23) &&
                       c->tt.size() < ((size_t)1 << 23);
  if (!sched_geo && !agg_geo) return KSG_OK;
  // PreFilter / PreScore on the host, as run_batch's compile_upto
  const auto T0 = clk::now();
  CompiledPod cp;
  int rc = compile(p, CYCLE, -1, true, false, &cp);
  if (rc) {
    *handled = true;
    return rc;
  }
  if (cp.prefilter_error) cp.error = true;
  // which resident loop takes the pod: node-local pods k_sched_loop (or a running k_agg_loop, which takes
  // them too), PodTopologySpread / InterPodAffinity pods k_agg_loop with their pod-table entry
  alignas(16) static thread_local uint8_t entry[kRingEntryBytes];
  size_t entry_bytes = 0;
  int kind = 0;
  if (!cp.error && !cp.prefilter_reject && cp.blob.size() % 16 == 0) {
    const bool sched_ok = sched_geo && loop_ok(cp);
    const bool agg_ok = agg_geo && agg_loop_ok(cp) && cp.own_terms <= 4 * kAggMaxTerms;
    if (agg_ok && (!sched_ok || (res_running_ && res_kind_ == 2))) kind = 2;
    else if (sched_ok) kind = 1;
  }
  if (!cp.error && !cp.prefilter_reject && kind == 0) {
    c->pod_table_drop(cp.slot);  // not a resident-loop pod: the launch path compiles it again
    return KSG_OK;
  }
  *handled = true;
  // a scheduling cycle of an unsigned pod (signed ones take run_batch's path), counted once the pod can no
  // longer fall back to the launch path (whose run_batch counts it itself)
  auto ob_count = [&]() {
    if (!ob_acting()) return;
    ++ob_cycle_;
    ob_prev_sig_ = -1;
  };
  if (cp.error || cp.prefilter_reject) {  // decided on the host (run_batch's settle gives the same)
    ob_count();
    c->pod_table_drop(cp.slot);
    *res = ksg_result{};
    res->status = cp.error ? KSG_CODE_ERROR : KSG_CODE_UNSCHEDULABLE;
    res->node_index = -1;
    return KSG_OK;
  }
  const int64_t ns_before = c->next_start;
  const bool rot_dev = rotdev();  // the program's rot_start is c->next_start; the loop returns the next one
  if (!rot_dev) c->next_start = (c->next_start + cp.num_all) % (int64_t)N;  // schedule_one.go:686-687
  auto fail = [&](int code) {
    c->pod_table_drop(cp.slot);
    c->next_start = ns_before;
    return code;
  };
  {  // host ports this pod's assume can add to one node
    int32_t extra = 0;
    for (auto& k : p.containers)
      for (auto& hp : k.ports) extra += hp.port > 0;
    for (auto& k : p.init_containers)
      if (k.sidecar)
        for (auto& hp : k.ports) extra += hp.port > 0;
    c->reserve_ports(extra);
  }
  hipStream_t s = c->stream;
  if (kind == 2) {
    // the pod's pod-table entry, which the loop writes into the device table when it commits the pod:
    // it must fit the ring and the device arrays as the last upload sized them, else the table goes up
    // again before a new launch
    entry_bytes = cp.slot >= 0 ? c->ring_entry(cp.slot, entry, kRingEntryBytes) : 0;
    if (cp.slot >= 0 && entry_bytes == 0) {
      if ((rc = resident_stop())) return fail(rc);
      if ((rc = c->ensure_mirror(true))) return fail(rc);
      entry_bytes = c->ring_entry(cp.slot, entry, kRingEntryBytes);
      if (entry_bytes == 0) {  // larger than the ring's entry area: the launch path takes it
        c->pod_table_drop(cp.slot);
        c->next_start = ns_before;
        *handled = false;
        return KSG_OK;
      }
    }
  }
  bool reposted = false;
relaunch:
  // the running launch sees the mirror as it is, or it stops (so does a launch of the other kind)
  if (res_running_ && (c->mirror_pending() || res_q_ >= kLoopMaxPods || res_kind_ != kind ||
                       (kind == 1 && (GS != res_gs_ || unit != res_unit_)) || (kind == 2 && G != res_gs_) ||
                       (kind == 2 && res_terms_ + cp.own_terms > kRingTermBudget) ||
                       clk::now() - res_last_ > std::chrono::milliseconds(kResidentIdleMs / 2)))
    if ((rc = resident_stop())) return fail(rc);
  if (!res_running_) {
    if ((rc = c->ensure_mirror(kind == 2))) return fail(rc);
    if (kind == 2 && cp.slot >= 0) {  // (the upload may have moved the label pool: the entry again)
      entry_bytes = c->ring_entry(cp.slot, entry, kRingEntryBytes);
      if (entry_bytes == 0) {
        c->err = "resident loop: the pod-table entry does not fit after the upload";
        return fail(KSG_EDEVICE);
      }
    }
    if (!ring_) {
      void* hp = nullptr;
      if (hipHostMalloc(&hp, sizeof(PodRing), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        c->err = "resident loop: hipHostMalloc of the pod ring failed";
        return fail(KSG_EDEVICE);
      }
      ring_ = (PodRing*)hp;
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
        c->err = "resident loop: the pod ring has no device address";
        return fail(KSG_EDEVICE);
      }
      ring_dev_ = (PodRing*)dp;
    }
    std::memset((void*)ring_, 0, offsetof(PodRing, blob));
    if ((rc = ensure(d_fail, kFailBytes))) return fail(rc);
    if ((rc = ensure_scratch(256, kLoopMaxPods, false, 0))) return fail(rc);
    HIPCHK(hipMemsetAsync(d_fail.p, 0, kFailBytes, s));
    HIPCHK(hipMemsetAsync(d_stats.p, 0, d_stats.bytes, s));  // PodStats::ipa_any = 0 for every pod
    if (kind == 1) {
      if ((rc = gran_setup())) return fail(rc);
      LoopView lv{};
      lv.first_pod = 0;
      lv.npods = kLoopMaxPods;
      lv.nwg = GS;
      lv.blk0 = 0;
      lv.nblk = NB;
      lv.world = 1;
      lv.rank = 0;
      if ((rc = next_gran_tag(&lv.tag))) return fail(rc);
      lv.gran[0] = gran_all[0];
      lv.fail = (uint32_t*)d_fail.p;
      lv.give_up_at = -1;
      lv.wave_map = c->cfg.loop_wave_map;
      lv.ring = ring_dev_;
      lv.ring_idle = (unsigned long long)kResidentIdleMs * 100000ull;  // s_memrealtime: 100 MHz
      lv.ring_ahead = c->cfg.resident_ahead ? 1 : 0;
      if (c->cfg.loop_stamps) {  // per-pod phase stamps (the resident instance writes them in the diagnostic build)
        if ((rc = ensure(d_stamps, (size_t)kLoopMaxPods * 8 * 8))) return fail(rc);
        HIPCHK(hipMemsetAsync(d_stamps.p, 0, (size_t)kLoopMaxPods * 8 * 8, s));
        lv.stamps = (unsigned long long*)d_stamps.p;
      }
      if (c->cfg.ring_relay_min > 0 && GS >= c->cfg.ring_relay_min) {  // as k_agg_loop's below (one buffer)
        if ((rc = ensure(d_relay, (size_t)kRelayWords * 8))) return fail(rc);
        HIPCHK(hipMemsetAsync(d_relay.p, 0, (size_t)kRelayWords * 8, s));
        lv.relay = (unsigned long long*)d_relay.p;
      }
      HIPCHK(launch_sched_loop(c->view, bview(kLoopMaxPods), lv, s, nullptr, nullptr, unit));
      res_gs_ = GS;
      res_unit_ = unit;
    } else {
      if ((rc = agg_setup())) return fail(rc);
      // every workgroup's pod / term lists: its nodes' pods and terms now, plus what the launch can append
      // (kLoopMaxPods pods and kRingTermBudget terms), past kAggRingPods / kAggRingTerms in its HBM spill rows
      std::vector<int32_t> np((size_t)G, 0), nt((size_t)G, 0);
      auto wg_of = [&](int32_t nd) { return (int)((int64_t)(nd / kBlock) * G / NB); };
      auto owner = [&](int32_t nd) {  // the workgroup whose block range [NB w / G, NB (w + 1) / G) holds nd
        int w = wg_of(nd);
        while (w > 0 && (int64_t)NB * w / G > nd / kBlock) --w;
        while (w + 1 < G && (int64_t)NB * (w + 1) / G <= nd / kBlock) ++w;
        return w;
      };
      for (int32_t nd : c->pt_node)
        if (nd >= 0 && nd < c->view.n) np[(size_t)owner(nd)]++;
      for (const DTerm& tm : c->tt) {
        const int32_t nd = tm.kind >= 0 && tm.owner >= 0 ? c->pt_node[(size_t)tm.owner] : -1;
        if (nd >= 0 && nd < c->view.n) nt[(size_t)owner(nd)]++;
      }
      auto up64 = [](int64_t v) { return v <= 0 ? (int64_t)0 : (v + 63) / 64 * 64; };
      const int64_t spill_p = up64(*std::max_element(np.begin(), np.end()) + (int64_t)kLoopMaxPods - kAggRingPods);
      const int64_t spill_t = up64(*std::max_element(nt.begin(), nt.end()) + (int64_t)kRingTermBudget - kAggRingTerms);
      if (spill_p > kAggSpillMax || spill_t > kAggSpillMax) {  // no resident launch: the launch path
        c->pod_table_drop(cp.slot);
        c->next_start = ns_before;
        *handled = false;
        return KSG_OK;
      }
      if ((rc = ensure(d_aspill, (size_t)G * (size_t)(spill_p + spill_t) * 4 + 4))) return fail(rc);
      HIPCHK(hipMemsetAsync(d_region.p, 0, (size_t)kLoopMaxPods * kAggGWords * 8, s));
      AggView av{};
      av.first_pod = 0;
      av.npods = kLoopMaxPods;
      av.nwg = G;
      av.blk0 = 0;
      av.nblk = NB;
      av.world = 1;
      av.rank = 0;
      if ((rc = next_gran_tag(&av.tag))) return fail(rc);
      av.gwords = kAggGWords;
      av.ptss = 1;
      av.spill = (uint32_t*)d_aspill.p;
      av.spill_pods = (int32_t)spill_p;
      av.spill_terms = (int32_t)spill_t;
      av.debug = c->cfg.agg_debug | (c->cfg.resident_ahead ? 0 : 128);  // 128: no phase 1 ahead of the doorbell
      av.give_up_at = -1;
      av.gran = (unsigned long long*)d_agran.p;
      av.region = (unsigned long long*)d_region.p;
      av.fail = (uint32_t*)d_fail.p;
      av.ring = ring_dev_;
      av.ring_idle = (unsigned long long)kResidentIdleMs * 100000ull;
      if (c->cfg.ring_relay_min > 0 && G >= c->cfg.ring_relay_min) {  // stale tags would pass for new ones: zeroed
        if ((rc = ensure(d_relay, (size_t)kRelayWords * 8))) return fail(rc);
        HIPCHK(hipMemsetAsync(d_relay.p, 0, (size_t)kRelayWords * 8, s));
        av.relay = (unsigned long long*)d_relay.p;
      }
      if (c->cfg.loop_stamps) {  // workgroup 0's phase stamps per ring pod (resident_stop prints them)
        const size_t sb = (size_t)kLoopMaxPods * kAggStamps * 8;
        if ((rc = ensure(d_astamps, sb))) return fail(rc);
        HIPCHK(hipMemsetAsync(d_astamps.p, 0, sb, s));
        av.stamps = (unsigned long long*)d_astamps.p;
      }
      HIPCHK(launch_agg_loop(c->view, bview(kLoopMaxPods), av, s, nullptr, nullptr));
      res_gs_ = G;
      res_terms_ = 0;
    }
    res_running_ = true;
    res_kind_ = kind;
    res_q_ = 0;
  }
  // post the pod (and its pod-table entry), wait for its result
  if (!reposted) ob_count();
  const auto T1 = clk::now();
  const int q = res_q_;
  const uint32_t bytes = (uint32_t)cp.blob.size();
  if (kind == 1) {
    // the previous call's program but for the slot and the rotation: the loop copies it in LDS (RING_SAME)
    bool same = q > 0 && res_prev_blob_.size() == cp.blob.size() && !(c->cfg.agg_debug & 8);
    const PodDesc& hd = *reinterpret_cast<const PodDesc*>(cp.blob.data());
    if (same) {
      PodDesc& pd = *reinterpret_cast<PodDesc*>(res_prev_blob_.data());
      const PodDesc keep = pd;
      pd.slot = hd.slot;
      pd.rot_start = hd.rot_start;
      same = std::memcmp(res_prev_blob_.data(), cp.blob.data(), bytes) == 0;
      pd = keep;
    }
    same = same && hd.slot >= -1 && hd.slot < (1 << 23) - 1 && hd.rot_start >= 0 && hd.rot_start < (1 << 25);
    unsigned long long ctl = (unsigned long long)(uint32_t)(q + 1);
    if (same) {
      ctl |= (1ull << 11) | ((unsigned long long)(hd.slot + 1) << 12) | ((unsigned long long)hd.rot_start << 35);
    } else {
      std::memcpy(ring_->blob[q % kRingSlots], cp.blob.data(), bytes);
      ctl |= (unsigned long long)bytes << 12;
    }
    __atomic_store_n(&ring_->ctl, ctl, __ATOMIC_RELEASE);
    res_prev_blob_ = cp.blob;
  } else {
    res_terms_ += cp.own_terms;
    // the same template as the pod before it in this launch: the loop folds that pod's placement into
    // the counts it holds instead of gathering them again (k_agg_loop's batch shortcut, DF_AGG_SAME)
    const bool aggsame = q > 0 && agg_same(res_prev_blob_, cp.blob);
    PodDesc& hd = *reinterpret_cast<PodDesc*>(cp.blob.data());
    hd.flags = aggsame ? (hd.flags | DF_AGG_SAME) : (hd.flags & ~DF_AGG_SAME);  // (a repost after a relaunch: q 0)
    // the previous pod's program and entry but for the slot, the rotation and the label-pool offset: the
    // loop copies them in LDS (PodRing::ll, RING_SAME) instead of reading both over PCIe
    bool same = q > 0 && res_prev_blob_.size() == cp.blob.size() && res_prev_entry_.size() == entry_bytes;
    uint32_t lbl_off = 0;
    if (same) {
      PodDesc& pd = *reinterpret_cast<PodDesc*>(res_prev_blob_.data());
      const PodDesc keep = pd;
      pd.slot = hd.slot;
      pd.rot_start = hd.rot_start;
      pd.flags = (pd.flags & ~DF_AGG_SAME) | (hd.flags & DF_AGG_SAME);  // the one flag the loop patches
      same = std::memcmp(res_prev_blob_.data(), cp.blob.data(), bytes) == 0;
      pd = keep;
    }
    if (same && entry_bytes) {
      RingEntry& pe = *reinterpret_cast<RingEntry*>(res_prev_entry_.data());
      const RingEntry& ne = *reinterpret_cast<const RingEntry*>(entry);
      const RingEntry keep = pe;
      lbl_off = ne.lbl_off;
      pe.slot = ne.slot;
      pe.lbl_off = ne.lbl_off;
      if (pe.tpool_cnt == 0 && ne.tpool_cnt == 0) pe.tpool_off = ne.tpool_off;  // unread without terms
      same = std::memcmp(res_prev_entry_.data(), entry, entry_bytes) == 0;
      pe = keep;
    }
    // else, a pod of the same template with own affinity terms: the same but for the terms' table indices and the
    // term-pool offset of their words (RING_TERMS) -- the patch is replayed here on the previous bytes, and taken
    // only when that reproduces this pod's program and entry exactly
    bool terms = false;
    unsigned long long patch[kPatchWords] = {};
    int why = q == 0 ? 6 : !entry_bytes ? 7 : res_prev_blob_.size() != cp.blob.size() ? 8 : 9;
    if (!same && q > 0 && entry_bytes && res_prev_blob_.size() == cp.blob.size() && res_prev_entry_.size() == entry_bytes)
      terms = ring_terms_patch(res_prev_blob_, cp.blob, res_prev_entry_, entry, entry_bytes, patch, &why);
    res_posts_[same ? 0 : terms ? 1 : 2 + why]++;
    if (terms) {
      same = true;
      lbl_off = reinterpret_cast<const RingEntry*>(entry)->lbl_off;
    }
    if (c->cfg.agg_debug & 8) same = terms = false;  // diagnostic: every pod staged over PCIe
    uint32_t dw[kRingLL];
    if (same) {
      if (terms) std::memcpy(ring_->patch[q % kRingSlots], patch, sizeof patch);
      dw[0] = RING_SAME | (terms ? RING_TERMS : 0u) | (aggsame ? RING_AGG_SAME : 0u);
      dw[1] = (uint32_t)hd.slot;
      dw[2] = (uint32_t)hd.rot_start;
      dw[3] = lbl_off;
    } else {
      std::memcpy(ring_->blob[q % kRingSlots], cp.blob.data(), bytes);
      if (entry_bytes) std::memcpy(ring_->entry[q % kRingSlots], entry, entry_bytes);
      dw[0] = aggsame ? RING_AGG_SAME : 0u;
      dw[1] = bytes;
      dw[2] = (uint32_t)entry_bytes;
      dw[3] = 0;
    }
    for (int k = kRingLL - 1; k >= 0; --k)
      __atomic_store_n(&ring_->ll[k], (unsigned long long)(uint32_t)(q + 1) | ((unsigned long long)dw[k] << 32),
                       __ATOMIC_RELEASE);
    res_prev_blob_ = cp.blob;
    res_prev_entry_.assign(entry, entry + entry_bytes);
  }
  RingResult& rr = ring_->res[q % kRingSlots];
  const auto tw = clk::now();
  const auto T2 = tw;
  for (uint64_t spins = 1; __atomic_load_n(&rr.seq, __ATOMIC_ACQUIRE) != (uint32_t)(q + 1); ++spins) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
    if ((spins & 0xfffu) == 0 && clk::now() - tw > std::chrono::seconds(5)) {  // never: fail loudly, not hang
      __atomic_store_n(&ring_->ctl, kCtlStop, __ATOMIC_RELEASE);
      __atomic_store_n(&ring_->ll[0], (unsigned long long)kRingStop, __ATOMIC_RELEASE);
      // the loop leaves at its next poll (or at its exchanges' own give-up): drained before anything else
      // uses the stream; it may still have committed the pod into the device mirror, which is therefore
      // rebuilt from the cache, where the pod never arrives
      (void)hipStreamSynchronize(s);
      res_running_ = false;
      c->layout_dirty = true;
      c->mirror_suspect = true;
      c->pods_dirty = true;
      c->err = "resident loop: no result for the posted pod after 5 s; the device mirror is rebuilt from the cache";
      return fail(KSG_EDEVICE);
    }
    if ((spins & 0xfffu) == 0 && hipStreamQuery(s) != hipErrorNotReady) {  // the launch ended without it
      res_running_ = false;
      (void)hipStreamSynchronize(s);
      if (__atomic_load_n(&rr.seq, __ATOMIC_ACQUIRE) == (uint32_t)(q + 1)) break;  // it landed after all
      uint32_t f[kFailWords] = {};
      (void)hipMemcpyAsync(f, d_fail.p, kFailBytes, hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      if (!f[0] && __atomic_load_n(&ring_->exited, __ATOMIC_ACQUIRE) == 1u && !reposted) {
        // the loop left on its idle timer before this pod was posted (a host thread held up past the
        // window, e.g. by the cgroup quota): no workgroup took the pod -- one that had would have waited
        // for the others' exchanges and given up (f[0]) -- so a new launch takes it
        reposted = true;
        goto relaunch;
      }
      const int ng = res_kind_ == 2 ? kAGran : kGran;
      const DevBuf& gb = res_kind_ == 2 ? d_agran : d_gran;
      std::vector<unsigned long long> row((size_t)res_gs_ * ng);
      if (f[0] && ((size_t)f[1] + 1) * row.size() * 8 <= gb.bytes)
        (void)hipMemcpyAsync(row.data(), (const unsigned long long*)gb.p + (size_t)f[1] * row.size(), row.size() * 8,
                             hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      c->layout_dirty = true;
      c->mirror_suspect = true;
      c->pods_dirty = true;
      c->err = std::string("resident loop ended without the pod's result") +
               (f[0] ? " (" + (f[1] >= 0xfffffff0u ? "a list check failed" : "an exchange granule never arrived: " +
                                                                                 give_up_detail(f, row, ng, 1, res_gs_)) + ")"
                     : std::string()) +
               "; the device mirror is rebuilt from the cache";
      return fail(KSG_EDEVICE);
    }
  }
  const DevResult d = rr.r;
  res_q_ = q + 1;
  res_last_ = clk::now();
  const auto T3 = res_last_;
  // the result and the host shadow of the device-side assume (run_batch's settle)
  *res = ksg_result{};
  res->status = d.status;
  res->node_index = d.node;
  res->feasible_nodes = d.feasible;
  res->evaluated_nodes = cp.num_all;
  if (rot_dev) {  // processedNodes and nextStartNodeIndex from the loop (schedule_one.go:686-687)
    res->evaluated_nodes = d.evaluated;
    c->next_start = d.rot_next;
  }
  res->total_score = d.feasible > 1 ? d.total : 0;
  if (res->status == KSG_CODE_SUCCESS && res->node_index >= 0) {
    std::string uid = p.uid + "#a" + std::to_string(++assume_seq_);  // (as run_batch: the oracle's naming)
    if ((rc = c->add_pod(p, uid, /*device_done=*/true, cp.slot, &c->order()[(size_t)res->node_index], &cp.res)))
      return rc;
    assumed[handle] = uid;
    nominated.erase(p.uid);  // (schedule_one.go:1131-1134)
  } else {
    c->pod_table_drop(cp.slot);
  }
  last_kernel = kind == 2 ? 2 : 1;
  if (c->cfg.loop_stamps) {
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    res_prof_[0] += us(T0, T1);
    res_prof_[1] += us(T1, T2);
    res_prof_[2] += us(T2, T3);
    res_prof_[3] += us(T3, clk::now());
    res_prof_[4] += 1;
  }
  return KSG_OK;
}

}  // namespace ksg
