// oracle.cpp -- PARITY ORACLE: CPU restatement of kube-scheduler's per-pod node
// evaluation (test infrastructure; never shipped, never the thing measured as GPU).
//
// Follows, step by step and in the reference's own data structures' semantics:
//   Scheduler.schedulePod            pkg/scheduler/schedule_one.go:564-618
//   findNodesThatFitPod              schedule_one.go:622-712
//   findNodesThatPassFilters         schedule_one.go:771-854   (parallelism=1 order)
//   numFeasibleNodesToFind           schedule_one.go:858-884
//   prioritizeNodes                  schedule_one.go:937-1048
//   nodeScoreHeap + container/heap   schedule_one.go:1050-1098 (Go stdlib heap, literal)
//   RunPreFilter/Filter/PreScore/ScorePlugins  framework/runtime/framework.go:934-1458
//   plugins: nodeunschedulable, nodename, tainttoleration, nodeaffinity, nodeports,
//            noderesources (fit, least/most/RTCR, balanced), podtopologyspread,
//            interpodaffinity, imagelocality           (framework/plugins/*)
//   cache/snapshot: NodeInfo.update (framework/types.go:445-468), nodeTree
//            (backend/cache/node_tree.go), image states (cache.go:712-759)
// Parity is pinned by the reference's own unit-test vectors (tests/golden/).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "ksg_oracle.h"
#include "oracle_model.hpp"

using namespace oracle;

namespace {

// ---------------------------------------------------------------------------
// Go math.Log (src/math/log.go, FreeBSD e_log.c algorithm), restated bit-for-bit
// ---------------------------------------------------------------------------
double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
               L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
               L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || std::isinf(x)) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < 0.70710678118654752440084436210484903928483593768847) {  // Sqrt2/2
    f1 *= 2;
    ki--;
  }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// ---------------------------------------------------------------------------
// container/heap (Go stdlib) with nodeScoreHeap.Less (schedule_one.go:1082-1085)
// ---------------------------------------------------------------------------
struct HeapEnt { int64_t total; int64_t randomizer; int32_t idx; };
static bool heap_less(const std::vector<HeapEnt>& h, int i, int j) {
  return h[i].total > h[j].total || (h[i].total == h[j].total && h[i].randomizer > h[j].randomizer);
}
static void heap_down(std::vector<HeapEnt>& h, int i0, int n) {
  int i = i0;
  while (true) {
    int j1 = 2 * i + 1;
    if (j1 >= n || j1 < 0) break;
    int j = j1;
    int j2 = j1 + 1;
    if (j2 < n && heap_less(h, j2, j1)) j = j2;
    if (!heap_less(h, j, i)) break;
    std::swap(h[i], h[j]);
    i = j;
  }
}
static int heap_pop_index(std::vector<HeapEnt> h) {  // heap.Init then heap.Pop
  int n = (int)h.size();
  for (int i = n / 2 - 1; i >= 0; i--) heap_down(h, i, n);
  // Pop: swap(0, n-1), down(0, n-1), return h[n-1] == the root after Init
  return h[0].idx;
}

// ---------------------------------------------------------------------------
// configuration
// ---------------------------------------------------------------------------
static const char* kPluginNames[KSG_NUM_PLUGINS] = {
    "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
    "NodeResourcesFit", "PodTopologySpread", "InterPodAffinity", "NodeResourcesBalancedAllocation",
    "ImageLocality"};
static int plugin_id(const std::string& n) {
  for (int i = 0; i < KSG_NUM_PLUGINS; ++i)
    if (n == kPluginNames[i]) return i;
  if (n == "BalancedAllocation") return KSG_PLUGIN_BALANCED_ALLOCATION;
  return -1;
}

struct Config {
  int pct = 100;
  int threads = 1;  // CPU-baseline mode: Filter / Score over nodes on this many threads (Parallelizer.Until)
  // CPU-baseline mode: how long an idle worker spins before parking.  Longer spins avoid futex wake-ups
  // between a cycle's parallel passes on an idle machine (C4, 8 threads, this container: 227 -> 328 pods/s at
  // 1 ms), but on the GPU box's 16-CPU cgroup quota the spinning workers are throttled instead (C3, 16
  // threads: 1595 pods/s at 50 µs, 1202 at 1 ms; profiles/r04k_cpu_pool_c3.txt)
  int spin_us = 50;
  bool par_weights = false;  // CPU-baseline mode: NormalizeScore / weights on the pool too (framework.go:1409-1452)
  bool taintCompareOps = false;  // featureGates.TaintTolerationComparisonOperators
  bool enabled[KSG_NUM_PLUGINS];
  int64_t weight[KSG_NUM_PLUGINS];
  int fitStrategy = 0;  // 0 LeastAllocated 1 MostAllocated 2 RequestedToCapacityRatio
  std::vector<std::pair<std::string, int64_t>> fitResources{{"cpu", 1}, {"memory", 1}};
  std::vector<std::pair<int64_t, int64_t>> rtcrShape;  // (utilization, score*10)
  std::set<std::string> ignoredResources, ignoredResourceGroups;
  std::vector<std::pair<std::string, int64_t>> balancedResources{{"cpu", 1}, {"memory", 1}};
  int32_t hardPodAffinityWeight = 1;
  bool ignorePreferredTermsOfExistingPods = false;
  bool hasAddedRequired = false;
  std::vector<ParsedNodeSelectorTerm> addedRequired;
  bool hasAddedPreferred = false;
  PreferredTerms addedPreferred;
  // PodTopologySpreadArgs: DefaultingType System (v1 default, defaults.go:225-229) -> the plugin's
  // systemDefaultConstraints (podtopologyspread/plugin.go:46-57,124-127); List -> DefaultConstraints
  bool ptsSystemDefaulted = true;
  std::vector<TopologySpreadConstraint> ptsDefaults;
  bool obGate = true;  // featureGates.OpportunisticBatching (Beta, on: pkg/features/kube_features.go:1674-1676)
  Config() {
    // default_plugins.go:35-50
    const int64_t w[KSG_NUM_PLUGINS] = {0, 0, 3, 2, 0, 1, 2, 2, 1, 1};
    for (int i = 0; i < KSG_NUM_PLUGINS; ++i) { enabled[i] = true; weight[i] = w[i]; }
    TopologySpreadConstraint h, z;
    h.topologyKey = "kubernetes.io/hostname";
    h.whenUnsatisfiable = "ScheduleAnyway";
    h.maxSkew = 3;
    z.topologyKey = "topology.kubernetes.io/zone";
    z.whenUnsatisfiable = "ScheduleAnyway";
    z.maxSkew = 5;
    ptsDefaults = {h, z};
  }
};

static std::vector<std::pair<std::string, int64_t>> decode_res_specs(const mj::Value* v) {
  std::vector<std::pair<std::string, int64_t>> out;
  if (v && v->is_arr())
    for (auto& r : v->arr) {
      int64_t w = r.i64("weight", 0);
      if (w == 0) w = 1;  // defaults.go:218-221
      out.push_back({r.str("name"), w});
    }
  return out;
}

static bool decode_config(const mj::Value& v, Config* c, std::string* err) {
  if (!v.is_obj()) return true;
  if (v.has("percentageOfNodesToScore")) c->pct = (int)v.i64("percentageOfNodesToScore");
  if (v.has("cpuThreads")) c->threads = std::max(1, (int)v.i64("cpuThreads"));
  if (v.has("cpuSpinUs")) c->spin_us = std::max(0, (int)v.i64("cpuSpinUs"));
  if (v.has("cpuParallelWeights")) c->par_weights = v.boolean("cpuParallelWeights");
  if (auto fg = v.has("featureGates")) {
    c->taintCompareOps = fg->boolean("TaintTolerationComparisonOperators");
    c->obGate = fg->boolean("OpportunisticBatching", true);
  }
  if (auto w = v.has("scoreWeights"))
    for (auto& kv : w->obj) {
      int id = plugin_id(kv.first);
      if (id < 0) { *err = "unknown plugin " + kv.first; return false; }
      c->weight[id] = std::strtoll(kv.second.s.c_str(), nullptr, 10);
    }
  if (auto d = v.has("disabledPlugins"))
    for (auto& x : d->arr) {
      int id = plugin_id(x.s);
      if (id < 0) { *err = "unknown plugin " + x.s; return false; }
      c->enabled[id] = false;
    }
  if (auto f = v.has("nodeResourcesFit")) {
    if (auto ss = f->has("scoringStrategy")) {
      std::string t = ss->str("type", "LeastAllocated");
      if (t == "LeastAllocated") c->fitStrategy = 0;
      else if (t == "MostAllocated") c->fitStrategy = 1;
      else if (t == "RequestedToCapacityRatio") c->fitStrategy = 2;
      else { *err = "bad scoring strategy"; return false; }
      if (ss->has("resources")) c->fitResources = decode_res_specs(ss->get("resources"));
      if (auto r = ss->has("requestedToCapacityRatio"))
        if (auto sh = r->has("shape"))
          for (auto& p : sh->arr)  // score scaled by MaxNodeScore/MaxCustomPriorityScore (=10)
            c->rtcrShape.push_back({p.i64("utilization"), p.i64("score") * 10});
    }
    if (auto ir = f->has("ignoredResources"))
      for (auto& x : ir->arr) c->ignoredResources.insert(x.s);
    if (auto ig = f->has("ignoredResourceGroups"))
      for (auto& x : ig->arr) c->ignoredResourceGroups.insert(x.s);
  }
  if (auto b = v.has("balancedAllocation"))
    if (b->has("resources")) c->balancedResources = decode_res_specs(b->get("resources"));
  if (auto ipa = v.has("interPodAffinity")) {
    if (ipa->has("hardPodAffinityWeight")) c->hardPodAffinityWeight = (int32_t)ipa->i64("hardPodAffinityWeight");
    c->ignorePreferredTermsOfExistingPods = ipa->boolean("ignorePreferredTermsOfExistingPods");
  }
  if (auto pa = v.has("podTopologySpread")) {  // validation_pluginargs.go:102-174
    std::string dt = pa->str("defaultingType", "System");
    if (dt != "System" && dt != "List") { *err = "defaultingType: Unsupported value"; return false; }
    std::vector<TopologySpreadConstraint> list;
    if (auto dc = pa->has("defaultConstraints"))
      for (auto& x : dc->arr) {
        TopologySpreadConstraint t = decode_tsc(x);
        Requirement probe;
        if (t.maxSkew <= 0 || t.topologyKey.empty() || !new_requirement(t.topologyKey, Op::Exists, {}, &probe) ||
            (t.whenUnsatisfiable != "DoNotSchedule" && t.whenUnsatisfiable != "ScheduleAnyway") ||
            t.labelSelector.present) {
          *err = "invalid default constraint";
          return false;
        }
        for (auto& o : list)
          if (o.topologyKey == t.topologyKey && o.whenUnsatisfiable == t.whenUnsatisfiable) {
            *err = "duplicate default constraint";
            return false;
          }
        list.push_back(t);
      }
    if (dt == "System" && !list.empty()) { *err = "System defaulting with defaultConstraints"; return false; }
    c->ptsSystemDefaulted = dt == "System";
    if (!c->ptsSystemDefaulted) c->ptsDefaults = list;
  }
  if (auto na = v.has("nodeAffinity"))
    if (auto aa = na->has("addedAffinity")) {
      if (auto rq = aa->has("requiredDuringSchedulingIgnoredDuringExecution")) {
        std::vector<NodeSelectorTerm> terms;
        if (auto ts = rq->has("nodeSelectorTerms"))
          for (auto& t : ts->arr) {
            NodeSelectorTerm nt;
            for (auto& e : t.has("matchExpressions") ? t.get("matchExpressions")->arr : std::vector<mj::Value>{}) {
              std::vector<std::string> vals;
              if (auto vs = e.has("values")) for (auto& x : vs->arr) vals.push_back(x.s);
              nt.matchExpressions.push_back({e.str("key"), e.str("operator"), vals});
            }
            for (auto& e : t.has("matchFields") ? t.get("matchFields")->arr : std::vector<mj::Value>{}) {
              std::vector<std::string> vals;
              if (auto vs = e.has("values")) for (auto& x : vs->arr) vals.push_back(x.s);
              nt.matchFields.push_back({e.str("key"), e.str("operator"), vals});
            }
            terms.push_back(nt);
          }
        if (!new_node_selector(terms, &c->addedRequired)) { *err = "bad addedAffinity"; return false; }
        c->hasAddedRequired = true;
      }
      if (auto pf = aa->has("preferredDuringSchedulingIgnoredDuringExecution")) {
        std::vector<PreferredSchedulingTerm> terms;
        for (auto& t : pf->arr) {
          PreferredSchedulingTerm p;
          p.weight = (int32_t)t.i64("weight");
          if (auto pr = t.has("preference")) {
            for (auto& e : pr->has("matchExpressions") ? pr->get("matchExpressions")->arr : std::vector<mj::Value>{}) {
              std::vector<std::string> vals;
              if (auto vs = e.has("values")) for (auto& x : vs->arr) vals.push_back(x.s);
              p.preference.matchExpressions.push_back({e.str("key"), e.str("operator"), vals});
            }
          }
          terms.push_back(p);
        }
        if (!terms.empty()) {
          if (!new_preferred_terms(terms, &c->addedPreferred)) { *err = "bad addedAffinity"; return false; }
          c->hasAddedPreferred = true;
        }
      }
    }
  return true;
}

// apis/config/validation/validation_pluginargs.go:81-97,176-239,295-340
static bool validate_config(const Config& c, std::string* err) {
  for (auto& r : c.fitResources)
    if (r.second <= 0 || r.second > 100) { *err = "resource weight of " + r.first + " not in valid range (0, 100]"; return false; }
  std::set<std::string> seen;
  for (auto& r : c.balancedResources) {
    if (!seen.insert(r.first).second) { *err = "duplicate balanced resource " + r.first; return false; }
    if (r.second != 1) { *err = "balanced resource weight must be 1"; return false; }
  }
  if (c.hardPodAffinityWeight < 0 || c.hardPodAffinityWeight > 100) { *err = "hardPodAffinityWeight not in [0,100]"; return false; }
  if (c.fitStrategy == 2) {
    if (c.rtcrShape.empty()) { *err = "requestedToCapacityRatio shape required"; return false; }
    for (size_t i = 0; i < c.rtcrShape.size(); ++i) {
      if (i && c.rtcrShape[i - 1].first >= c.rtcrShape[i].first) { *err = "shape not sorted"; return false; }
      if (c.rtcrShape[i].first < 0 || c.rtcrShape[i].first > 100) { *err = "utilization out of range"; return false; }
      if (c.rtcrShape[i].second < 0 || c.rtcrShape[i].second > 100) { *err = "score out of range"; return false; }
    }
  }
  for (int p = 0; p < KSG_NUM_PLUGINS; ++p)
    if (c.weight[p] < 0) { *err = "negative plugin weight"; return false; }
  return true;
}

// ---------------------------------------------------------------------------
// cache / snapshot state
// ---------------------------------------------------------------------------
struct ImageState { int64_t size = 0; std::set<std::string> nodes; };
using HostPorts = std::map<std::string, std::set<std::pair<std::string, int32_t>>>;  // ip -> {(proto, port)}

struct NodeInfoO {  // framework.NodeInfo (framework/types.go:172-220)
  int pos = -1;  // index in the snapshot list (set by rebuild_list; the result's node index)
  bool hasNode = false;  // Node() != nil; false: a ghost (cache.go:442-446, 666-689)
  Node node;
  std::vector<PodInfo*> pods;
  std::vector<PodInfo*> podsWithAffinity, podsWithRequiredAntiAffinity;
  Resource requested, nonzero, allocatable;
  HostPorts usedPorts;
};

struct HostPortWant { std::string ip, proto; int32_t port; };
// util.GetHostPorts (scheduler/util/utils.go:241-272)
static std::vector<HostPortWant> get_host_ports(const Pod& p) {
  std::vector<HostPortWant> out;
  auto take = [&](const Container& c) {
    for (auto& cp : c.ports)
      if (cp.hostPort > 0) out.push_back({cp.hostIP, cp.protocol, cp.hostPort});
  };
  for (auto& c : p.initContainers)
    if (c.restartAlways) take(c);
  for (auto& c : p.containers) take(c);
  return out;
}
static void sanitize(std::string& ip, std::string& proto) {  // HostPortInfo.sanitize (types.go:634-641)
  if (ip.empty()) ip = "0.0.0.0";
  if (proto.empty()) proto = "TCP";
}
static bool check_conflict(const HostPorts& h, std::string ip, std::string proto, int32_t port) {  // :603-631
  if (port <= 0) return false;
  sanitize(ip, proto);
  auto pp = std::make_pair(proto, port);
  if (ip == "0.0.0.0") {
    for (auto& kv : h)
      if (kv.second.count(pp)) return true;
    return false;
  }
  for (const std::string& key : {std::string("0.0.0.0"), ip}) {
    auto it = h.find(key);
    if (it != h.end() && it->second.count(pp)) return true;
  }
  return false;
}

static Resource node_allocatable(const Node& n) {  // NewResource(node.Status.Allocatable), types.go:1263-1291
  Resource r;
  for (auto& kv : n.allocatable) {
    if (kv.first == "cpu") r.milliCPU += kv.second;
    else if (kv.first == "memory") r.memory += milli_to_value(kv.second);
    else if (kv.first == "pods") r.allowedPods += milli_to_value(kv.second);
    else if (kv.first == "ephemeral-storage") r.ephemeral += milli_to_value(kv.second);
    else if (is_scalar_resource_name(kv.first)) r.scalar[kv.first] += milli_to_value(kv.second);
  }
  return r;
}

static void node_update(NodeInfoO& ni, PodInfo* pi, int64_t sign) {  // NodeInfo.update, types.go:445-468
  const PodResource& pr = pi->calc;
  ni.requested.milliCPU += sign * pr.res.milliCPU;
  ni.requested.memory += sign * pr.res.memory;
  ni.requested.ephemeral += sign * pr.res.ephemeral;
  for (auto& kv : pr.res.scalar) ni.requested.scalar[kv.first] += sign * kv.second;
  ni.nonzero.milliCPU += sign * pr.non0CPU;
  ni.nonzero.memory += sign * pr.non0Mem;
  for (auto hp : get_host_ports(pi->pod)) {  // updateUsedPorts :503-511
    if (hp.port <= 0) continue;
    sanitize(hp.ip, hp.proto);
    if (sign > 0) ni.usedPorts[hp.ip].insert({hp.proto, hp.port});
    else {
      auto it = ni.usedPorts.find(hp.ip);
      if (it != ni.usedPorts.end()) {
        it->second.erase({hp.proto, hp.port});
        if (it->second.empty()) ni.usedPorts.erase(it);
      }
    }
  }
}
static void node_add_pod(NodeInfoO& ni, PodInfo* pi) {  // AddPodInfo :367-376
  ni.pods.push_back(pi);
  if (pi->withAffinity()) ni.podsWithAffinity.push_back(pi);
  if (pi->withRequiredAnti()) ni.podsWithRequiredAntiAffinity.push_back(pi);
  node_update(ni, pi, 1);
}
static void remove_from_slice(std::vector<PodInfo*>& s, const std::string& uid) {  // :397-420
  for (size_t i = 0; i < s.size(); ++i)
    if (s[i]->pod.uid == uid) {
      s[i] = s.back();
      s.pop_back();
      return;
    }
}
static bool node_remove_pod(NodeInfoO& ni, const std::string& uid) {  // RemovePod :423-441
  PodInfo* found = nullptr;
  for (auto* p : ni.pods)
    if (p->pod.uid == uid) found = p;
  if (!found) return false;
  if (found->withAffinity()) remove_from_slice(ni.podsWithAffinity, uid);
  if (found->withRequiredAnti()) remove_from_slice(ni.podsWithRequiredAntiAffinity, uid);
  remove_from_slice(ni.pods, uid);
  node_update(ni, found, -1);
  return true;
}

// ---------------------------------------------------------------------------
// status helpers
// ---------------------------------------------------------------------------
struct Status {
  int code = KSG_CODE_SUCCESS;
  uint32_t reasons = 0;
  int plugin = KSG_PLUGIN_NONE;
  bool ok() const { return code == KSG_CODE_SUCCESS; }
};
static Status mk(int code, uint32_t r) { Status s; s.code = code; s.reasons = r; return s; }

}  // namespace

// ---------------------------------------------------------------------------
// the oracle context
// ---------------------------------------------------------------------------
// Worker pool for the CPU-baseline mode: the reference runs the per-node Filter and Score loops
// through Parallelizer.Until (framework/parallelize/parallelism.go:28-76): pieces cut into chunks of
// chunkSizeFor(n, 16) = min(sqrt(n), n/16 + 1) that workqueue.ParallelizeUntil's workers claim one at a
// time.  Go starts those goroutines on runtime threads that stay alive and spin briefly for work, so
// the workers here are persistent threads that spin on a generation counter for up to kSpinUs before
// parking on a condition variable.  until(n, fn) calls fn(chunk, lo, hi) for every chunk; the caller
// claims chunks too and returns once every chunk is done, so a worker that is still asleep delays
// nothing.  A chunk ticket is {job generation | job's chunk count | next chunk} in one word, so a claim
// (a compare-and-swap of the whole word) succeeds only for a chunk of the job still posted.
class Pool {
 public:
  Pool(int n, int spin_us) : n_(n), spin_us_(spin_us) {
    for (int k = 1; k < n; ++k) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    stop_.store(true);
    {
      std::lock_guard<std::mutex> g(m_);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  static int chunk_size(int n, int par) {  // parallelism.go:36-45
    int cs = (int)std::sqrt((double)n);
    const int r = n / par + 1;
    if (cs > r) cs = r;
    else if (cs < 1) cs = 1;
    return cs;
  }
  int chunks(int pieces) const { return pieces <= 0 ? 0 : (pieces + chunk_size(pieces, n_) - 1) / chunk_size(pieces, n_); }
  void until(int pieces, const std::function<void(int, int, int)>& fn) {
    if (pieces <= 0) return;
    const int cs = chunk_size(pieces, n_), nc = (pieces + cs - 1) / cs;  // nc < 2^16 for any int pieces
    fn_.store(&fn, std::memory_order_relaxed);
    pieces_.store(pieces, std::memory_order_relaxed);
    csize_.store(cs, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    const uint64_t g = gen_.load() + 1;
    ticket_.store((g << 32) | ((uint64_t)nc << 16), std::memory_order_release);  // claimable from here
    gen_.store(g);  // seq_cst: pairs with a parking worker's sleepers_ increment (no lost wakeup)
    if (sleepers_.load() > 0) {
      { std::lock_guard<std::mutex> l(m_); }
      cv_.notify_all();
    }
    work(g);
    while (done_.load(std::memory_order_acquire) < nc) cpu_relax();
  }

 private:
  static void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  // claim and run chunks of job `g` until none is left (or the job is not g any more)
  void work(uint64_t g) {
    uint64_t t = ticket_.load(std::memory_order_acquire);
    for (;;) {
      if ((t >> 32) != (g & 0xffffffffull)) return;
      const int c = (int)(t & 0xffffu), nc = (int)((t >> 16) & 0xffffu);
      if (c >= nc) return;
      if (!ticket_.compare_exchange_weak(t, t + 1, std::memory_order_acq_rel)) continue;
      const int cs = csize_.load(std::memory_order_relaxed), lo = c * cs;
      (*fn_.load(std::memory_order_relaxed))(c, lo, std::min(pieces_.load(std::memory_order_relaxed), lo + cs));
      done_.fetch_add(1, std::memory_order_release);
      t = ticket_.load(std::memory_order_acquire);
    }
  }
  void loop() {
    uint64_t seen = 0;  // gen_ at construction: a job posted before this thread runs is not missed
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int spins = 0; gen_.load(std::memory_order_acquire) == seen; ++spins) {
        cpu_relax();
        if ((spins & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
          std::unique_lock<std::mutex> l(m_);
          sleepers_.fetch_add(1);
          cv_.wait(l, [&] { return gen_.load() != seen; });
          sleepers_.fetch_sub(1);
        }
      }
      seen = gen_.load();
      if (stop_.load()) return;
      work(seen);
    }
  }
  int n_, spin_us_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0}, ticket_{0};
  std::atomic<int> sleepers_{0}, done_{0}, pieces_{0}, csize_{1};
  std::atomic<bool> stop_{false};
  std::atomic<const std::function<void(int, int, int)>*> fn_{nullptr};
};

static inline double nowus() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
// framework.SortedScoredNodes (framework/interface.go:158-162): what schedulePod hands
// StoreScheduleResults -- sortedNodeScores, the nodeScoreHeap after heap.Init and the winner's Pop
// (schedule_one.go:1050-1098); or, for TestBatchBasic (runtime/batch_test.go:165-185), a plain list.
struct SortedScoredNodes {
  bool isList = false;
  std::vector<HeapEnt> heap;       // heap order; HeapEnt::idx indexes names
  std::vector<std::string> names;  // node names (list: in pop order)
  size_t head = 0;
  int Len() const { return isList ? (int)(names.size() - head) : (int)heap.size(); }
  std::string Pop() {  // sortedNodeScores.Pop: heap.Pop (swap(0, n-1), down(0, n-1), drop the last)
    if (isList) return names[head++];
    const int n = (int)heap.size() - 1;
    std::swap(heap[0], heap[n]);
    heap_down(heap, 0, n);
    const HeapEnt e = heap[n];
    heap.pop_back();
    return names[e.idx];
  }
};

// OpportunisticBatching (framework/runtime/batch.go:31-242): the state a signed pod's cycle leaves for the
// next pod of the same signature.
struct OpportunisticBatch {
  struct State { std::string signature; std::unique_ptr<SortedScoredNodes> sortedNodes; int64_t creationNs = 0; };
  std::unique_ptr<State> state;
  int64_t lastCycleCount = 0;  // lastCycle (batch.go:51-55)
  std::string lastChosenNode;
  bool lastSucceeded = false;
  int64_t batchedPods = 0;
  bool genericWorkloadEnabled = false;
  static constexpr int64_t kMaxBatchAgeNs = 500LL * 1000 * 1000;  // maxBatchAge (:57)

  bool stateEmpty() const {  // :230-232
    return !state || !state->sortedNodes || state->sortedNodes->Len() == 0;
  }
  // batchStateCompatible (:167-226); lastChosenRejected(name) runs RunFilterPlugins on the node: -1 when
  // the node is not in the snapshot (BatchFlushNodeMissing), 1 when the pod is rejected there
  template <typename RejectFn>
  bool compatible(const std::string* signature, const std::string& nominated, int64_t cycleCount, int64_t now,
                  RejectFn lastChosenRejected) const {
    if (stateEmpty()) return false;
    if (cycleCount != lastCycleCount + 1)
      if (!genericWorkloadEnabled || cycleCount != lastCycleCount) return false;  // BatchFlushPodSkipped
    if (!lastSucceeded) return false;                                             // BatchFlushPodFailed
    if (!nominated.empty()) return false;                                         // BatchFlushPodNominated
    if (!signature || *signature != state->signature) return false;               // BatchFlushPodIncompatible
    if (now > state->creationNs + kMaxBatchAgeNs) return false;                   // BatchFlushExpired
    return lastChosenRejected(lastChosenNode) == 1;  // else BatchFlushNodeMissing / BatchFlushNodeNotFull
  }
  template <typename RejectFn>
  std::string GetNodeHint(const std::string* signature, const std::string& nominated, int64_t cycleCount, int64_t now,
                          RejectFn lastChosenRejected) {  // :65-95
    if (!compatible(signature, nominated, cycleCount, now, lastChosenRejected)) return "";
    return state->sortedNodes->Pop();
  }
  // StoreScheduleResults (:98-158); otherNodes may be null (schedulePod's one-feasible-node path)
  void StoreScheduleResults(const std::string* signature, const std::string& hinted, const std::string& chosen,
                            std::unique_ptr<SortedScoredNodes> otherNodes, int64_t cycleCount, int64_t now) {
    lastCycleCount = cycleCount;
    lastChosenNode = chosen;
    lastSucceeded = true;
    if (hinted == chosen) {
      batchedPods++;
      return;
    }
    if (signature && otherNodes && otherNodes->Len() > 0) {
      state.reset(new State{*signature, std::move(otherNodes), now});
    } else {
      state.reset();
    }
  }
};

struct ksgo_ctx {
  Config cfg;
  double prof[10] = {};  // ksgo_debug_profile: microseconds per cycle section (CPU-baseline breakdown)
  std::unique_ptr<Pool> pool;  // cfg.threads > 1
  std::vector<NodeInfoO*> filt_buf;  // CPU-baseline filter pass: per-chunk feasible runs, reused per cycle
  std::vector<int> filt_lo, filt_cnt, filt_fail;
  std::string err;
  std::map<std::string, Namespace> namespaces;
  // Service / ReplicationController / ReplicaSet / StatefulSet listers (podtopologyspread/plugin.go:145-150)
  std::map<std::string, std::map<std::string, SelectorObject>> services;  // namespace -> name
  std::map<std::tuple<std::string, std::string, std::string>, SelectorObject> owners;  // (kind, ns, name)
  std::map<std::string, std::unique_ptr<NodeInfoO>> nodes;
  // nodeTree (backend/cache/node_tree.go)
  std::vector<std::string> zones;
  std::map<std::string, std::vector<std::string>> tree;
  std::map<std::string, ImageState> imageStates;  // cache.imageStates
  std::map<std::string, std::unique_ptr<PodInfo>> pods;  // bound/assumed pods by uid
  std::vector<NodeInfoO*> list;  // snapshot nodeInfoList order
  std::set<std::string> snapMap;  // snapshot.nodeInfoMap's names
  std::vector<std::string> changed;  // nodes given a Node object since the last snapshot
  int numNodes = 0;                  // nodeTree.numNodes
  int64_t nextStartNodeIndex = 0;
  uint64_t assumeSeq = 0;
  std::map<int32_t, std::unique_ptr<Pod>> queue;  // compiled pods
  int32_t nextHandle = 1;
  std::map<int32_t, std::string> assumedUid;  // handle -> assumed pod uid
  OpportunisticBatch batch;  // frameworkImpl.batch (framework/runtime/framework.go:1620-1626)
  int64_t cycleCount = 0;    // SchedulingQueue.SchedulingCycle(): one per scheduling cycle of this context
  int64_t clockNs = 0;       // ksgo_set_clock: time.Now() of the next cycles (0: the wall clock)
  // the scheduling queue's nominator (backend/queue/nominator.go:60-150; ksgo_add_nominated_pod): uid -> (node,
  // priority).  Boundary, as the product (include/ksg.h): RunFilterPluginsWithNominatedPods is not restated; a
  // call in which a pod would see another pod's nomination of equal or higher priority is refused
  std::map<std::string, std::pair<std::string, int32_t>> nominated;
  int64_t clockStep = 0;     // ksgo_debug_clock_step: the fixed clock advances by this per cycle (per read)
  int64_t now() {
    if (clockNs) {
      const int64_t v = clockNs;
      clockNs += clockStep;
      return v;
    }
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  // UpdateSnapshot (backend/cache/cache.go:190-296), its list part.  A NodeInfo object stays alive
  // while its name is in snapMap (the snapshot owns copies upstream; here the list points at the
  // cache's objects, so a removed node's object lives until the snapshot drops it).
  void rebuild_list() {
    bool updateAll = false;
    for (auto& nm : changed) {  // the generation walk (:223-261): a node new to the map
      auto it = nodes.find(nm);
      if (it != nodes.end() && it->second->hasNode && snapMap.insert(nm).second) updateAll = true;
    }
    changed.clear();
    if ((int)snapMap.size() > numNodes) {  // removeDeletedNodesFromSnapshot (:270-273, 361-372)
      for (auto it = snapMap.begin(); it != snapMap.end();) {
        auto n = nodes.find(*it);
        if (n == nodes.end() || !n->second->hasNode) {
          if (n != nodes.end() && n->second->pods.empty()) nodes.erase(n);  // removeNodeInfoFromList
          it = snapMap.erase(it);
        } else {
          ++it;
        }
      }
      updateAll = true;
    }
    if (!updateAll) return;
    // updateNodeInfoSnapshotList(updateAll) (:318-345) over nodeTree.list (node_tree.go:119-143)
    list.clear();
    size_t maxLen = 0;
    for (auto& z : zones) maxLen = std::max(maxLen, tree[z].size());
    for (size_t idx = 0; idx < maxLen; ++idx)
      for (auto& z : zones) {
        auto& na = tree[z];
        if (idx < na.size()) list.push_back(nodes[na[idx]].get());
      }
    for (size_t i = 0; i < list.size(); ++i) list[i]->pos = (int)i;
  }
  // a node object with neither Node nor pods leaves the cache (cache.go:493-494, 685-686) unless
  // the snapshot still lists it
  void maybe_drop(const std::string& name) {
    auto it = nodes.find(name);
    if (it != nodes.end() && !it->second->hasNode && it->second->pods.empty() && !snapMap.count(name)) nodes.erase(it);
  }
  const Labels* ns_labels(const std::string& ns) const {  // GetNamespaceLabelsSnapshot (ipa plugin.go:150-159)
    auto it = namespaces.find(ns);
    return it == namespaces.end() ? nullptr : &it->second.labels;
  }
  ImageState* image_state(const std::string& name) {
    auto it = imageStates.find(name);
    return it == imageStates.end() ? nullptr : &it->second;
  }
};

namespace {

static thread_local std::string g_create_error;

// ===========================================================================
// per-cycle evaluation
// ===========================================================================
// Go's maps are hash maps: the PreFilter / PreScore aggregation counts (merged sequentially after the parallel
// passes, as the reference merges its per-node maps) are hash maps here too.  No result depends on their
// iteration order (lookups, integer sums, minima); the preemption restatement seeds criticalPaths from
// tpMatch in key order, over a sorted copy.
struct PairHash {
  size_t operator()(const std::pair<std::string, std::string>& p) const {
    return std::hash<std::string>()(p.first) * 1000003u ^ std::hash<std::string>()(p.second);
  }
};
using PairCounts = std::unordered_map<std::pair<std::string, std::string>, int64_t, PairHash>;
using StrCounts = std::unordered_map<std::string, int64_t>;

struct Cycle {
  ksgo_ctx* c;
  const Pod* pod;
  PodInfo pinfo;
  bool pinfoOk = true;
  bool skipFilter[KSG_NUM_PLUGINS] = {};
  bool skipScore[KSG_NUM_PLUGINS] = {};
  // Fit prefilter state
  Resource podReq;
  // NodePorts
  std::vector<HostPortWant> wantPorts;
  // NodeAffinity
  RequiredNodeAffinity reqNA;
  PreferredTerms prefNA;
  bool hasPrefNA = false;
  // TaintToleration
  std::vector<Toleration> tolPrefer;
  // Fit / Balanced PreScore
  std::vector<int64_t> fitPodReqs, balPodReqs;
  // PTS
  struct TSC { int32_t maxSkew; std::string key; Selector sel; int32_t minDomains; bool affHonor, taintHonor; };
  std::vector<TSC> ptsF;
  std::vector<StrCounts> tpMatch;  // TpValueToMatchNum
  std::vector<int64_t> critMin;
  std::vector<TSC> ptsS;
  std::set<std::string> ignored;
  std::vector<StrCounts> tpCounts;  // TopologyValueToPodCounts (entries exist)
  std::vector<double> tpWeight;
  // IPA
  PairCounts existingAnti, affCounts, antiCounts;
  std::map<std::string, StrCounts> topoScore;
  std::vector<AffinityTerm> ipaReqAff, ipaReqAnti;
  std::vector<WeightedAffinityTerm> ipaPrefAff, ipaPrefAnti;
  const Labels* nsLabels = nullptr;
};

static std::vector<int> prefilter_order() {  // defaults.go PreFilter list
  return {KSG_PLUGIN_NODE_AFFINITY, KSG_PLUGIN_NODE_PORTS, KSG_PLUGIN_NODE_RESOURCES_FIT,
          KSG_PLUGIN_POD_TOPOLOGY_SPREAD, KSG_PLUGIN_INTER_POD_AFFINITY};
}
static const int kFilterOrder[] = {KSG_PLUGIN_NODE_UNSCHEDULABLE, KSG_PLUGIN_NODE_NAME, KSG_PLUGIN_TAINT_TOLERATION,
                                   KSG_PLUGIN_NODE_AFFINITY,      KSG_PLUGIN_NODE_PORTS, KSG_PLUGIN_NODE_RESOURCES_FIT,
                                   KSG_PLUGIN_POD_TOPOLOGY_SPREAD, KSG_PLUGIN_INTER_POD_AFFINITY};
static const int kPreScoreOrder[] = {KSG_PLUGIN_TAINT_TOLERATION, KSG_PLUGIN_NODE_AFFINITY, KSG_PLUGIN_NODE_RESOURCES_FIT,
                                     KSG_PLUGIN_POD_TOPOLOGY_SPREAD, KSG_PLUGIN_INTER_POD_AFFINITY,
                                     KSG_PLUGIN_BALANCED_ALLOCATION};
static const int kScoreOrder[] = {KSG_PLUGIN_TAINT_TOLERATION, KSG_PLUGIN_NODE_AFFINITY, KSG_PLUGIN_NODE_RESOURCES_FIT,
                                  KSG_PLUGIN_POD_TOPOLOGY_SPREAD, KSG_PLUGIN_INTER_POD_AFFINITY,
                                  KSG_PLUGIN_BALANCED_ALLOCATION, KSG_PLUGIN_IMAGE_LOCALITY};

// ---- PodTopologySpread helpers (podtopologyspread/common.go) -------------------------
static bool node_labels_match_spread(const Labels& nl, const std::vector<Cycle::TSC>& cs) {  // :73-80
  for (auto& c : cs)
    if (!nl.count(c.key)) return false;
  return true;
}
static bool match_inclusion(const Cycle& cy, const Cycle::TSC& c, const Node& n) {  // :43-57
  if (c.affHonor && !cy.reqNA.match(n)) return false;
  if (c.taintHonor && find_untolerated_noschedule(n.taints, cy.pod->tolerations)) return false;
  return true;
}
// CPU-baseline mode: a PreFilter / PreScore aggregation over every node of the snapshot runs through
// Parallelizer.Until as the reference's does (podtopologyspread/filtering.go:292, scoring.go:190,
// interpodaffinity/filtering.go:231,275, scoring.go:209): body(node, chunk-local state) per node on the
// pool's chunks, then merge(chunk state) in chunk order.  Every merge here is a sum of counts, so the result
// is the sequential loop's.  Without a pool, the sequential loop over one local state.
template <class M, class Body, class Merge>
static void over_all_nodes(ksgo_ctx* c, Body&& body, Merge&& merge) {
  const int n = (int)c->list.size();
  if (!c->pool || n < 2) {
    M acc{};
    for (auto* ni : c->list) body(ni, acc);
    merge(acc);
    return;
  }
  std::vector<M> part((size_t)c->pool->chunks(n));
  c->pool->until(n, [&](int k, int lo, int hi) {
    for (int i = lo; i < hi; ++i) body(c->list[(size_t)i], part[(size_t)k]);
  });
  for (const M& m : part) merge(m);
}
static int64_t count_pods_match(const std::vector<PodInfo*>& pods, const Selector& sel, const std::string& ns) {  // :145-160
  if (sel.empty()) return 0;
  int64_t n = 0;
  for (auto* p : pods) {
    if (p->pod.terminating || p->pod.ns != ns) continue;
    if (selector_matches(sel, p->pod.labels)) ++n;
  }
  return n;
}
// helper.DefaultSelector (plugins/helper/spread.go:37-95)
static Selector default_selector(const ksgo_ctx* c, const Pod& pod) {
  Labels labelSet;
  auto sit = c->services.find(pod.ns);  // GetPodServices (:98-119)
  if (sit != c->services.end())
    for (auto& kv : sit->second) {
      const SelectorObject& svc = kv.second;
      if (!svc.hasMap) continue;  // nil selector matches nothing
      bool m = true;              // labels.Set(selector).AsSelectorPreValidated().Matches
      for (auto& r : svc.map) {
        auto it = pod.labels.find(r.first);
        if (it == pod.labels.end() || it->second != r.second) m = false;
      }
      if (m)
        for (auto& r : svc.map) labelSet[r.first] = r.second;  // labels.Merge
    }
  auto as_selector = [](const Labels& set) {  // labels.SelectorFromValidatedSet (selector.go:976-987)
    Selector s;
    for (auto& kv : set) s.reqs.push_back({kv.first, Op::Equals, {kv.second}});
    return s;
  };
  Selector selector = as_selector(labelSet);
  if (!pod.hasController) return selector;
  std::string group, version;  // schema.ParseGroupVersion (runtime/schema/group_version.go:211-227)
  const std::string& gv = pod.ownerAPIVersion;
  if (!(gv.empty() || gv == "/")) {
    size_t n = std::count(gv.begin(), gv.end(), '/');
    if (n == 0) version = gv;
    else if (n == 1) { group = gv.substr(0, gv.find('/')); version = gv.substr(gv.find('/') + 1); }
    else return selector;
  }
  auto find = [&](const char* kind) -> const SelectorObject* {
    auto it = c->owners.find({kind, pod.ns, pod.ownerName});
    return it == c->owners.end() ? nullptr : &it->second;
  };
  if (group.empty() && version == "v1" && pod.ownerKind == "ReplicationController") {
    if (const SelectorObject* rc = find("ReplicationController")) {
      for (auto& kv : rc->map) labelSet[kv.first] = kv.second;
      selector = as_selector(labelSet);
    }
  } else if (group == "apps" && version == "v1" && (pod.ownerKind == "ReplicaSet" || pod.ownerKind == "StatefulSet")) {
    if (const SelectorObject* o = find(pod.ownerKind.c_str())) {
      Selector other;
      // LabelSelectorAsSelector; Requirements() of labels.Nothing() is (nil, false)
      if (label_selector_as_selector(o->sel, &other) && !other.nothing)
        for (auto& r : other.reqs) selector.reqs.push_back(r);
    }
  }
  return selector;
}

// filterTopologySpreadConstraints (common.go:87-128)
static bool filter_tsc(const std::vector<TopologySpreadConstraint>& tsc, const Pod& pod, const std::string& action,
                       std::vector<Cycle::TSC>* out) {
  out->clear();
  for (auto& c : tsc) {
    if (c.whenUnsatisfiable != action) continue;
    Selector sel;
    if (!label_selector_as_selector(c.labelSelector, &sel)) return false;
    if (!c.matchLabelKeys.empty()) {  // MatchLabelKeysInPodTopologySpread (on by default)
      std::vector<std::pair<std::string, std::string>> ml;
      for (auto& k : c.matchLabelKeys) {
        auto it = pod.labels.find(k);
        if (it != pod.labels.end()) ml.push_back({k, it->second});
      }
      if (!ml.empty() && !sel.nothing) {  // mergeLabelSetWithSelector :130-143
        Selector merged;
        std::map<std::string, std::string> set(ml.begin(), ml.end());
        for (auto& kv : set) merged.reqs.push_back({kv.first, Op::Equals, {kv.second}});
        for (auto& r : sel.reqs) merged.reqs.push_back(r);
        sel = merged;
      }
    }
    Cycle::TSC t;
    t.maxSkew = c.maxSkew;
    t.key = c.topologyKey;
    t.sel = sel;
    t.minDomains = c.hasMinDomains ? c.minDomains : 1;
    t.affHonor = c.nodeAffinityPolicy.empty() ? true : c.nodeAffinityPolicy == "Honor";
    t.taintHonor = c.nodeTaintsPolicy.empty() ? false : c.nodeTaintsPolicy == "Honor";
    out->push_back(t);
  }
  return true;
}
// getConstraints (filtering.go:220-235) / initPreScoreState's choice (scoring.go:66-80): the pod's own
// constraints, else buildDefaultConstraints (common.go:59-75)
static bool get_constraints(const ksgo_ctx* c, const Pod& pod, const std::string& action, std::vector<Cycle::TSC>* out) {
  if (!pod.tsc.empty()) return filter_tsc(pod.tsc, pod, action, out);
  if (!filter_tsc(c->cfg.ptsDefaults, pod, action, out) || out->empty()) return true;
  Selector sel = default_selector(c, pod);
  if (sel.empty()) {
    out->clear();
    return true;
  }
  for (auto& t : *out) t.sel = sel;
  return true;
}

// ---- IPA helpers --------------------------------------------------------------------
static bool pod_matches_all_terms(const std::vector<AffinityTerm>& terms, const Pod& p) {  // filtering.go:188-200
  if (terms.empty()) return false;
  for (auto& t : terms)
    if (!t.matches(p, nullptr)) return false;
  return true;
}
// mergeAffinityTermNamespacesIfNotEmpty (interpodaffinity/plugin.go:134-147): the term's
// namespace set gains the namespaces the selector lists; the selector itself is kept
// (the assignment to NamespaceSelector in the reference hits a copy).
static void merge_ns(ksgo_ctx* c, AffinityTerm& at) {
  if (at.nsSelector.empty()) return;
  for (auto& kv : c->namespaces)
    if (selector_matches(at.nsSelector, kv.second.labels)) at.namespaces.insert(kv.first);
}

// ===========================================================================
// PreFilter (framework.go:934-995)
// ===========================================================================
static Status run_prefilter_plugin(Cycle& cy, int p, bool* skip, std::vector<std::string>* nodeNames,
                                   bool* restricts) {
  ksgo_ctx* c = cy.c;
  const Pod& pod = *cy.pod;
  *skip = false;
  *restricts = false;
  switch (p) {
    case KSG_PLUGIN_NODE_AFFINITY: {  // node_affinity.go:148-198
      bool noNA = !pod.hasRequiredNA;
      if (noNA && !c->cfg.hasAddedRequired && !pod.hasNodeSelector) { *skip = true; return Status{}; }
      cy.reqNA = get_required_node_affinity(pod);
      if (noNA || pod.requiredNA.empty()) return Status{};
      std::set<std::string> names;
      bool namesNil = true;
      for (auto& t : pod.requiredNA) {
        bool termNil = true;
        std::set<std::string> termNames;
        for (auto& r : t.matchFields)
          if (r.key == "metadata.name" && r.op == "In") {
            std::set<std::string> s(r.values.begin(), r.values.end());
            if (termNil) { termNames = s; termNil = false; }
            else {
              std::set<std::string> x;
              for (auto& n : termNames)
                if (s.count(n)) x.insert(n);
              termNames = x;
            }
          }
        if (termNil) return Status{};  // all nodes eligible
        namesNil = false;
        names.insert(termNames.begin(), termNames.end());
      }
      if (!namesNil && names.empty()) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_PREFILTER);
      if (!names.empty()) { *restricts = true; nodeNames->assign(names.begin(), names.end()); }
      return Status{};
    }
    case KSG_PLUGIN_NODE_PORTS:  // node_ports.go:73-82
      cy.wantPorts = get_host_ports(pod);
      if (cy.wantPorts.empty()) *skip = true;
      return Status{};
    case KSG_PLUGIN_NODE_RESOURCES_FIT: {  // fit.go:317-335 computePodResourceRequest
      ResList reqs = pod_requests(pod, nullptr, false);  // "pod hasn't scheduled yet": no status resources
      Resource r;  // SetMaxResource (types.go:1325-1344)
      for (auto& kv : reqs) {
        if (kv.first == "memory") r.memory = std::max(r.memory, milli_to_value(kv.second));
        else if (kv.first == "cpu") r.milliCPU = std::max(r.milliCPU, kv.second);
        else if (kv.first == "ephemeral-storage") r.ephemeral = std::max(r.ephemeral, milli_to_value(kv.second));
        else if (is_scalar_resource_name(kv.first)) r.scalar[kv.first] = std::max(r.scalar[kv.first], milli_to_value(kv.second));
      }
      cy.podReq = r;
      return Status{};
    }
    case KSG_PLUGIN_POD_TOPOLOGY_SPREAD: {  // filtering.go:139-149, 237-311
      if (!get_constraints(c, pod, "DoNotSchedule", &cy.ptsF)) return mk(KSG_CODE_ERROR, 0);
      if (cy.ptsF.empty()) { *skip = true; return Status{}; }
      size_t nc = cy.ptsF.size();
      cy.tpMatch.assign(nc, {});
      for (size_t i = 0; i < nc; ++i)  // make(map, sizeHeuristic(len(allNodes), c)) (filtering.go:252-254,361-366)
        if (cy.ptsF[i].key == "kubernetes.io/hostname") cy.tpMatch[i].reserve(c->list.size());
      using TpMatch = std::vector<StrCounts>;
      over_all_nodes<TpMatch>(c, [&](NodeInfoO* ni, TpMatch& tm) {  // processNode (filtering.go:255-300)
        const Node& n = ni->node;
        if (!node_labels_match_spread(n.labels, cy.ptsF)) return;
        tm.resize(nc);
        for (size_t i = 0; i < nc; ++i) {
          auto& con = cy.ptsF[i];
          if (!match_inclusion(cy, con, n)) continue;
          const std::string& v = n.labels.at(con.key);
          tm[i][v] += count_pods_match(ni->pods, con.sel, pod.ns);
        }
      }, [&](const TpMatch& tm) {
        for (size_t i = 0; i < tm.size(); ++i)
          for (auto& kv : tm[i]) cy.tpMatch[i][kv.first] += kv.second;
      });
      cy.critMin.assign(nc, INT32_MAX);
      for (size_t i = 0; i < nc; ++i)
        for (auto& kv : cy.tpMatch[i]) cy.critMin[i] = std::min(cy.critMin[i], kv.second);
      return Status{};
    }
    case KSG_PLUGIN_INTER_POD_AFFINITY: {  // interpodaffinity/filtering.go:286-321
      PodInfo pi;
      if (!new_pod_info(pod, &pi)) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_PREFILTER);
      cy.ipaReqAff = pi.reqAff;
      cy.ipaReqAnti = pi.reqAnti;
      for (auto& t : cy.ipaReqAff) merge_ns(c, t);
      for (auto& t : cy.ipaReqAnti) merge_ns(c, t);
      cy.nsLabels = c->ns_labels(pod.ns);
      using TopoCounts = PairCounts;
      cy.existingAnti.clear();
      over_all_nodes<TopoCounts>(c, [&](NodeInfoO* ni, TopoCounts& ea) {  // getExistingAntiAffinityCounts :216-240
        for (auto* ep : ni->podsWithRequiredAntiAffinity)
          for (auto& t : ep->reqAnti)
            if (t.matches(pod, cy.nsLabels)) {
              auto it = ni->node.labels.find(t.topologyKey);
              if (it != ni->node.labels.end()) ea[{t.topologyKey, it->second}] += 1;
            }
      }, [&](const TopoCounts& ea) {
        for (auto& kv : ea) cy.existingAnti[kv.first] += kv.second;
      });
      cy.affCounts.clear();
      cy.antiCounts.clear();
      if (!cy.ipaReqAff.empty() || !cy.ipaReqAnti.empty()) {  // :246-283
        using Two = std::pair<TopoCounts, TopoCounts>;
        over_all_nodes<Two>(c, [&](NodeInfoO* ni, Two& ac) {
          for (auto* ep : ni->pods) {
            if (pod_matches_all_terms(cy.ipaReqAff, ep->pod))
              for (auto& t : cy.ipaReqAff) {
                auto it = ni->node.labels.find(t.topologyKey);
                if (it != ni->node.labels.end()) ac.first[{t.topologyKey, it->second}] += 1;
              }
            for (auto& t : cy.ipaReqAnti)
              if (t.matches(ep->pod, nullptr)) {
                auto it = ni->node.labels.find(t.topologyKey);
                if (it != ni->node.labels.end()) ac.second[{t.topologyKey, it->second}] += 1;
              }
          }
        }, [&](const Two& ac) {
          for (auto& kv : ac.first) cy.affCounts[kv.first] += kv.second;
          for (auto& kv : ac.second) cy.antiCounts[kv.first] += kv.second;
        });
      }
      if (cy.existingAnti.empty() && cy.ipaReqAff.empty() && cy.ipaReqAnti.empty()) *skip = true;
      return Status{};
    }
  }
  return Status{};
}

// ===========================================================================
// Filter plugins
// ===========================================================================
static Status run_filter(Cycle& cy, int p, NodeInfoO* ni) {
  const Pod& pod = *cy.pod;
  const Node& node = ni->node;
  switch (p) {
    case KSG_PLUGIN_NODE_UNSCHEDULABLE: {  // node_unschedulable.go:125-143
      if (!node.unschedulable) return Status{};
      Taint t{"node.kubernetes.io/unschedulable", "", "NoSchedule"};
      if (!tolerations_tolerate(pod.tolerations, t)) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_UNSCHEDULABLE);
      return Status{};
    }
    case KSG_PLUGIN_NODE_NAME:  // node_name.go:67-83
      if (!pod.nodeName.empty() && pod.nodeName != node.name)
        return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_NODE_NAME);
      return Status{};
    case KSG_PLUGIN_TAINT_TOLERATION:  // taint_toleration.go:102-116
      if (find_untolerated_noschedule(node.taints, pod.tolerations))
        return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_TAINT);
      return Status{};
    case KSG_PLUGIN_NODE_AFFINITY: {  // node_affinity.go:207-228
      if (cy.c->cfg.hasAddedRequired) {
        bool m = false;
        for (auto& t : cy.c->cfg.addedRequired)
          if (t.match(node)) { m = true; break; }
        if (!m) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_NODE_AFFINITY_ENFORCED);
      }
      if (!cy.reqNA.match(node)) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_NODE_AFFINITY_POD);
      return Status{};
    }
    case KSG_PLUGIN_NODE_PORTS:  // node_ports.go:150-176
      for (auto& w : cy.wantPorts)
        if (check_conflict(ni->usedPorts, w.ip, w.proto, w.port)) return mk(KSG_CODE_UNSCHEDULABLE, KSG_R_NODE_PORTS);
      return Status{};
    case KSG_PLUGIN_NODE_RESOURCES_FIT: {  // fit.go:593-734
      const Resource& r = cy.podReq;
      uint32_t reasons = 0;
      bool unresolvable = false;
      if ((int64_t)ni->pods.size() + 1 > ni->allocatable.allowedPods) reasons |= KSG_R_TOO_MANY_PODS;
      bool anyScalar = false;
      for (auto& kv : r.scalar) anyScalar = true, (void)kv;
      if (!(r.milliCPU == 0 && r.memory == 0 && r.ephemeral == 0 && !anyScalar)) {
        if (r.milliCPU > 0 && r.milliCPU > ni->allocatable.milliCPU - ni->requested.milliCPU) {
          reasons |= KSG_R_INSUFFICIENT_CPU;
          if (r.milliCPU > ni->allocatable.milliCPU) unresolvable = true;
        }
        if (r.memory > 0 && r.memory > ni->allocatable.memory - ni->requested.memory) {
          reasons |= KSG_R_INSUFFICIENT_MEMORY;
          if (r.memory > ni->allocatable.memory) unresolvable = true;
        }
        if (r.ephemeral > 0 && r.ephemeral > ni->allocatable.ephemeral - ni->requested.ephemeral) {
          reasons |= KSG_R_INSUFFICIENT_EPHEMERAL;
          if (r.ephemeral > ni->allocatable.ephemeral) unresolvable = true;
        }
        for (auto& kv : r.scalar) {
          if (kv.second == 0) continue;
          bool extended = kv.first.find('/') != std::string::npos && kv.first.find("kubernetes.io/") == std::string::npos;
          if (extended) {
            std::string prefix = kv.first.substr(0, kv.first.find('/'));
            if (cy.c->cfg.ignoredResources.count(kv.first) || cy.c->cfg.ignoredResourceGroups.count(prefix)) continue;
          }
          int64_t alloc = ni->allocatable.scalar.count(kv.first) ? ni->allocatable.scalar.at(kv.first) : 0;
          int64_t used = ni->requested.scalar.count(kv.first) ? ni->requested.scalar.at(kv.first) : 0;
          if (kv.second > alloc - used) {
            reasons |= KSG_R_INSUFFICIENT_SCALAR;
            if (kv.second > alloc) unresolvable = true;
          }
        }
      }
      if (reasons) return mk(unresolvable ? KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE : KSG_CODE_UNSCHEDULABLE, reasons);
      return Status{};
    }
    case KSG_PLUGIN_POD_TOPOLOGY_SPREAD: {  // filtering.go:314-359
      if (cy.ptsF.empty()) return Status{};
      for (size_t i = 0; i < cy.ptsF.size(); ++i) {
        auto& con = cy.ptsF[i];
        auto it = node.labels.find(con.key);
        if (it == node.labels.end()) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_PTS_MISSING_LABEL);
        int64_t minMatch = cy.critMin[i];
        if ((int64_t)cy.tpMatch[i].size() < con.minDomains) minMatch = 0;
        int64_t self = selector_matches(con.sel, pod.labels) ? 1 : 0;
        auto mt = cy.tpMatch[i].find(it->second);
        int64_t matchNum = mt == cy.tpMatch[i].end() ? 0 : mt->second;
        if (matchNum + self - minMatch > con.maxSkew) return mk(KSG_CODE_UNSCHEDULABLE, KSG_R_PTS_SKEW);
      }
      return Status{};
    }
    case KSG_PLUGIN_INTER_POD_AFFINITY: {  // interpodaffinity/filtering.go:364-444
      // satisfyPodAffinity :394-420
      bool podsExist = true;
      for (auto& t : cy.ipaReqAff) {
        auto it = node.labels.find(t.topologyKey);
        if (it == node.labels.end()) return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_IPA_AFFINITY);
        auto ct = cy.affCounts.find({t.topologyKey, it->second});
        if (ct == cy.affCounts.end() || ct->second <= 0) podsExist = false;
      }
      if (!podsExist) {
        if (!(cy.affCounts.empty() && pod_matches_all_terms(cy.ipaReqAff, pod)))
          return mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_IPA_AFFINITY);
      }
      // satisfyPodAntiAffinity :379-391
      if (!cy.antiCounts.empty())
        for (auto& t : cy.ipaReqAnti) {
          auto it = node.labels.find(t.topologyKey);
          if (it == node.labels.end()) continue;
          auto ct = cy.antiCounts.find({t.topologyKey, it->second});
          if (ct != cy.antiCounts.end() && ct->second > 0) return mk(KSG_CODE_UNSCHEDULABLE, KSG_R_IPA_ANTI_AFFINITY);
        }
      // satisfyExistingPodsAntiAffinity :364-376
      if (!cy.existingAnti.empty())
        for (auto& kv : node.labels) {
          auto ct = cy.existingAnti.find({kv.first, kv.second});
          if (ct != cy.existingAnti.end() && ct->second > 0) return mk(KSG_CODE_UNSCHEDULABLE, KSG_R_IPA_EXISTING_ANTI);
        }
      return Status{};
    }
  }
  return Status{};
}

// ===========================================================================
// Score plugins
// ===========================================================================
// resource_allocation.go:236-259 calculatePodResourceRequest
static int64_t pod_resource_request(const Pod& pod, const std::string& name, bool useRequested) {
  ResList nonMissing;
  if (!useRequested) { nonMissing["cpu"] = 100; nonMissing["memory"] = 200LL * 1024 * 1024 * 1000; }
  ResList reqs = pod_requests(pod, useRequested ? nullptr : &nonMissing, true);  // UseStatusResources
  auto it = reqs.find(name);
  int64_t m = it == reqs.end() ? 0 : it->second;
  return name == "cpu" ? m : milli_to_value(m);
}

// resource_allocation.go:167-232
static void node_alloc_request(const NodeInfoO* ni, const std::vector<std::pair<std::string, int64_t>>& res,
                               const std::vector<int64_t>& podReqs, bool useRequested,
                               std::vector<int64_t>* requested, std::vector<int64_t>* allocated,
                               std::vector<int64_t>* allocatable) {
  size_t n = res.size();
  requested->assign(n, 0);
  allocated->assign(n, 0);
  allocatable->assign(n, 0);
  const Resource& rq = useRequested ? ni->requested : ni->nonzero;
  for (size_t i = 0; i < n; ++i) {
    const std::string& name = res[i].first;
    if (podReqs[i] == 0 && is_scalar_resource_name(name)) continue;
    int64_t a = 0, al = 0;
    if (name == "cpu") { a = ni->allocatable.milliCPU; al = rq.milliCPU; }
    else if (name == "memory") { a = ni->allocatable.memory; al = rq.memory; }
    else if (name == "ephemeral-storage") { a = ni->allocatable.ephemeral; al = ni->requested.ephemeral; }
    else {
      auto it = ni->allocatable.scalar.find(name);
      if (it != ni->allocatable.scalar.end()) {
        a = it->second;
        auto jt = ni->requested.scalar.find(name);
        al = jt == ni->requested.scalar.end() ? 0 : jt->second;
      }
    }
    if (a == 0) continue;
    (*allocatable)[i] = a;
    (*allocated)[i] = al;
    (*requested)[i] = al + podReqs[i];
  }
}

static int64_t fit_score(const Config& cfg, const std::vector<int64_t>& requested, const std::vector<int64_t>& allocatable) {
  int64_t nodeScore = 0, weightSum = 0;
  const auto& res = cfg.fitResources;
  if (cfg.fitStrategy == 0) {  // least_allocated.go:30-61
    for (size_t i = 0; i < requested.size(); ++i) {
      if (allocatable[i] == 0) continue;
      int64_t w = res[i].second;
      int64_t s = requested[i] > allocatable[i] ? 0 : ((allocatable[i] - requested[i]) * 100) / allocatable[i];
      nodeScore += s * w;
      weightSum += w;
    }
    return weightSum == 0 ? 0 : nodeScore / weightSum;
  }
  if (cfg.fitStrategy == 1) {  // most_allocated.go:30-65
    for (size_t i = 0; i < requested.size(); ++i) {
      if (allocatable[i] == 0) continue;
      int64_t w = res[i].second;
      int64_t rq = requested[i] > allocatable[i] ? allocatable[i] : requested[i];
      nodeScore += (rq * 100) / allocatable[i] * w;
      weightSum += w;
    }
    return weightSum == 0 ? 0 : nodeScore / weightSum;
  }
  // requested_to_capacity_ratio.go:30-58 + helper/shape_score.go:39-51
  auto shape = [&](int64_t p) -> int64_t {
    const auto& s = cfg.rtcrShape;
    for (size_t i = 0; i < s.size(); ++i)
      if (p <= s[i].first) {
        if (i == 0) return s[0].second;
        return s[i - 1].second + (s[i].second - s[i - 1].second) * (p - s[i - 1].first) / (s[i].first - s[i - 1].first);
      }
    return s.back().second;
  };
  for (size_t i = 0; i < requested.size(); ++i) {
    if (allocatable[i] == 0) continue;
    int64_t w = res[i].second;
    int64_t rs = (requested[i] > allocatable[i]) ? shape(100) : shape(requested[i] * 100 / allocatable[i]);
    if (rs > 0) { nodeScore += rs * w; weightSum += w; }
  }
  if (weightSum == 0) return 0;
  return (int64_t)std::round((double)nodeScore / (double)weightSum);
}

static int64_t balanced_resource_score(const std::vector<int64_t>& req, const std::vector<int64_t>& alloc) {  // :220-254
  std::vector<double> fr;
  double total = 0;
  for (size_t i = 0; i < req.size(); ++i) {
    if (alloc[i] == 0) continue;
    double f = (double)req[i] / (double)alloc[i];
    if (f > 1) f = 1;
    total += f;
    fr.push_back(f);
  }
  double std_ = 0.0;
  if (fr.size() == 2) {
    std_ = std::fabs((fr[0] - fr[1]) / 2);
  } else if (fr.size() > 2) {
    double mean = total / (double)fr.size();
    double sum = 0;
    for (double f : fr) {
      double d = f - mean;
      double sq = d * d;
      sum = sum + sq;
    }
    std_ = std::sqrt(sum / (double)fr.size());
  }
  double one_minus = 1 - std_;
  double scaled = one_minus * 100.0;
  return (int64_t)scaled;
}


// ---- RunPreScorePlugins body for one plugin (framework.go:1300-1333) -------------
static Status prescore_plugin(Cycle& cy, int p, const std::vector<NodeInfoO*>& nodes) {
  ksgo_ctx* c = cy.c;
  const Pod& pod = *cy.pod;
  switch (p) {
    case KSG_PLUGIN_TAINT_TOLERATION:  // taint_toleration.go:140-147
      cy.tolPrefer.clear();
      for (auto& t : pod.tolerations)
        if (t.effect.empty() || t.effect == "PreferNoSchedule") cy.tolPrefer.push_back(t);
      break;
    case KSG_PLUGIN_NODE_AFFINITY: {  // node_affinity.go:242-256
      cy.hasPrefNA = false;
      if (pod.hasPreferredNA) {
        if (!new_preferred_terms(pod.preferredNA, &cy.prefNA)) return mk(KSG_CODE_ERROR, 0);
        cy.hasPrefNA = true;
      }
      if (!cy.hasPrefNA && !c->cfg.hasAddedPreferred) return mk(KSG_CODE_SKIP, 0);
      break;
    }
    case KSG_PLUGIN_NODE_RESOURCES_FIT:  // fit.go:136-153
      cy.fitPodReqs.clear();
      for (auto& r : c->cfg.fitResources) cy.fitPodReqs.push_back(pod_resource_request(pod, r.first, false));
      break;
    case KSG_PLUGIN_BALANCED_ALLOCATION: {  // balanced_allocation.go:78-100
      cy.balPodReqs.clear();
      bool best = true;
      for (auto& r : c->cfg.balancedResources) {
        cy.balPodReqs.push_back(pod_resource_request(pod, r.first, true));
        if (cy.balPodReqs.back() != 0) best = false;
      }
      if (best) return mk(KSG_CODE_SKIP, 0);
      break;
    }
    case KSG_PLUGIN_POD_TOPOLOGY_SPREAD: {  // scoring.go:118-194
      if (c->list.empty()) { return mk(KSG_CODE_SKIP, 0); }
      bool requireAll = !pod.tsc.empty() || !c->cfg.ptsSystemDefaulted;  // scoring.go:141-144
      if (!get_constraints(c, pod, "ScheduleAnyway", &cy.ptsS)) return mk(KSG_CODE_ERROR, 0);
      if (cy.ptsS.empty()) { return mk(KSG_CODE_SKIP, 0); }
      size_t nc = cy.ptsS.size();
      cy.ignored.clear();
      cy.tpCounts.assign(nc, {});
      std::vector<int64_t> topoSize(nc, 0);
      for (auto* ni : nodes) {  // initPreScoreState :61-115
        if (requireAll && !node_labels_match_spread(ni->node.labels, cy.ptsS)) {
          cy.ignored.insert(ni->node.name);
          continue;
        }
        for (size_t i = 0; i < nc; ++i) {
          if (cy.ptsS[i].key == "kubernetes.io/hostname") continue;
          auto it = ni->node.labels.find(cy.ptsS[i].key);
          std::string v = it == ni->node.labels.end() ? "" : it->second;
          if (!cy.tpCounts[i].count(v)) { cy.tpCounts[i][v] = 0; topoSize[i]++; }
        }
      }
      cy.tpWeight.assign(nc, 0);
      for (size_t i = 0; i < nc; ++i) {
        int64_t sz = topoSize[i];
        if (cy.ptsS[i].key == "kubernetes.io/hostname") sz = (int64_t)nodes.size() - (int64_t)cy.ignored.size();
        cy.tpWeight[i] = go_log((double)(sz + 2));
      }
      cy.reqNA = get_required_node_affinity(pod);
      using TpCounts = std::vector<StrCounts>;
      over_all_nodes<TpCounts>(c, [&](NodeInfoO* ni, TpCounts& tc) {  // processAllNode :155-189
        if (requireAll && !node_labels_match_spread(ni->node.labels, cy.ptsS)) return;
        tc.resize(nc);
        for (size_t i = 0; i < nc; ++i) {
          auto& con = cy.ptsS[i];
          if (!match_inclusion(cy, con, ni->node)) continue;
          auto it = ni->node.labels.find(con.key);
          std::string v = it == ni->node.labels.end() ? "" : it->second;
          if (!cy.tpCounts[i].count(v)) continue;  // (the entries initPreScoreState made; read-only here)
          tc[i][v] += count_pods_match(ni->pods, con.sel, pod.ns);
        }
      }, [&](const TpCounts& tc) {
        for (size_t i = 0; i < tc.size(); ++i)
          for (auto& kv : tc[i]) cy.tpCounts[i][kv.first] += kv.second;
      });
      break;
    }
    case KSG_PLUGIN_INTER_POD_AFFINITY: {  // interpodaffinity/scoring.go:128-221
      bool hasPrefA = pod.hasPodAffinity && !pod.affPref.empty();
      bool hasPrefAnti = pod.hasPodAntiAffinity && !pod.antiPref.empty();
      bool hasConstraints = hasPrefA || hasPrefAnti;
      if (c->cfg.ignorePreferredTermsOfExistingPods && !hasConstraints) { return mk(KSG_CODE_SKIP, 0); }
      PodInfo pi;
      if (!new_pod_info(pod, &pi)) return mk(KSG_CODE_ERROR, 0);
      cy.ipaPrefAff = pi.prefAff;
      cy.ipaPrefAnti = pi.prefAnti;
      for (auto& t : cy.ipaPrefAff) merge_ns(c, t.term);
      for (auto& t : cy.ipaPrefAnti) merge_ns(c, t.term);
      const Labels* nsl = c->ns_labels(pod.ns);
      cy.topoScore.clear();
      bool any = false;
      using TopoScoreAcc = std::pair<bool, std::map<std::string, StrCounts>>;  // {some node scored, sums}
      auto processTerm = [&](TopoScoreAcc& m, const AffinityTerm& t, int32_t weight, const Pod& target,
                             const Labels* nl, const Node& node, int32_t mult) {
        if (t.matches(target, nl)) {
          auto it = node.labels.find(t.topologyKey);
          if (it != node.labels.end()) {
            m.second[t.topologyKey][it->second] += (int64_t)(weight * mult);
            m.first = true;  // the node's topoScore is non-empty (scoring.go:192-195)
          }
        }
      };
      // (each chunk adds its nodes' scores straight into its accumulator: a per-node map, merged, sums the same)
      over_all_nodes<TopoScoreAcc>(c, [&](NodeInfoO* ni, TopoScoreAcc& acc) {  // processNode (scoring.go:166-199)
        if (!hasConstraints && ni->podsWithAffinity.empty()) return;
        const auto& podsToProcess = hasConstraints ? ni->pods : ni->podsWithAffinity;
        for (auto* ep : podsToProcess) {  // processExistingPod :81-125
          const Node& node = ni->node;
          if (node.labels.empty()) continue;
          for (auto& t : cy.ipaPrefAff) processTerm(acc, t.term, t.weight, ep->pod, nullptr, node, 1);
          for (auto& t : cy.ipaPrefAnti) processTerm(acc, t.term, t.weight, ep->pod, nullptr, node, -1);
          if (c->cfg.hardPodAffinityWeight > 0)
            for (auto& t : ep->reqAff) processTerm(acc, t, c->cfg.hardPodAffinityWeight, pod, nsl, node, 1);
          for (auto& t : ep->prefAff) processTerm(acc, t.term, t.weight, pod, nsl, node, 1);
          for (auto& t : ep->prefAnti) processTerm(acc, t.term, t.weight, pod, nsl, node, -1);
        }
      }, [&](const TopoScoreAcc& acc) {
        any = any || acc.first;
        for (auto& kv : acc.second)
          for (auto& vv : kv.second) cy.topoScore[kv.first][vv.first] += vv.second;
      });
      if (!any) return mk(KSG_CODE_SKIP, 0);
      break;
    }
  }
  return Status{};
}

// ---- ScorePlugin.Score for one node ---------------------------------------------------
static int64_t score_node(Cycle& cy, int p, NodeInfoO* ni, int* code) {
  ksgo_ctx* c = cy.c;
  const Pod& pod = *cy.pod;
  const Node& node = ni->node;
  int64_t s = 0;
  *code = KSG_CODE_SUCCESS;
    switch (p) {
      case KSG_PLUGIN_TAINT_TOLERATION:  // taint_toleration.go:163-196
        for (auto& t : node.taints)
          if (t.effect == "PreferNoSchedule" && !tolerations_tolerate(cy.tolPrefer, t)) s++;
        break;
      case KSG_PLUGIN_NODE_AFFINITY:  // node_affinity.go:261-286
        if (c->cfg.hasAddedPreferred) s += preferred_score(c->cfg.addedPreferred, node);
        if (cy.hasPrefNA) s += preferred_score(cy.prefNA, node);
        break;
      case KSG_PLUGIN_NODE_RESOURCES_FIT: {  // fit.go:737-755, resource_allocation.go:138-165
        if (c->cfg.fitResources.empty()) { *code = KSG_CODE_ERROR; return 0; }  // :149-151
        std::vector<int64_t> rq, al, ac;
        node_alloc_request(ni, c->cfg.fitResources, cy.fitPodReqs, false, &rq, &al, &ac);
        s = fit_score(c->cfg, rq, ac);
        break;
      }
      case KSG_PLUGIN_BALANCED_ALLOCATION: {  // balanced_allocation.go:146-218
        if (c->cfg.balancedResources.empty()) { *code = KSG_CODE_ERROR; return 0; }
        std::vector<int64_t> rq, al, ac;
        node_alloc_request(ni, c->cfg.balancedResources, cy.balPodReqs, true, &rq, &al, &ac);
        int64_t with = balanced_resource_score(rq, ac);
        int64_t without = balanced_resource_score(al, ac);
        s = 100 / 2 + (100 / 2 + with - without) / 2;
        break;
      }
      case KSG_PLUGIN_IMAGE_LOCALITY: {  // image_locality.go:70-152
        int64_t total = (int64_t)c->list.size();
        int64_t sum = 0;
        auto scaled = [&](const std::string& img) {
          std::string nm = normalized_image_name(img);
          bool onNode = false;
          for (auto& im : node.images)
            for (auto& n : im.names)
              if (n == nm) onNode = true;
          if (!onNode) return;
          ImageState* st = c->image_state(nm);
          double spread = (double)(int64_t)st->nodes.size() / (double)total;
          sum += (int64_t)((double)st->size * spread);
        };
        for (auto& ctr : pod.initContainers) scaled(ctr.image);
        for (auto& ctr : pod.containers) scaled(ctr.image);
        int64_t imageCount = (int64_t)pod.initContainers.size() + (int64_t)pod.containers.size();
        for (auto& v : pod.imageVolumes) { scaled(v); imageCount++; }
        const int64_t mb = 1024 * 1024, minT = 23 * mb, maxT = 1000 * mb * imageCount;
        if (sum < minT) sum = minT;
        else if (sum > maxT) sum = maxT;
        s = 100 * (sum - minT) / (maxT - minT);
        break;
      }
      case KSG_PLUGIN_POD_TOPOLOGY_SPREAD: {  // scoring.go:199-226
        if (cy.ignored.count(node.name)) { s = 0; break; }
        double score = 0;
        for (size_t k = 0; k < cy.ptsS.size(); ++k) {
          auto& con = cy.ptsS[k];
          auto it = node.labels.find(con.key);
          if (it == node.labels.end()) continue;
          int64_t cnt;
          if (con.key == "kubernetes.io/hostname") cnt = count_pods_match(ni->pods, con.sel, pod.ns);
          else cnt = cy.tpCounts[k].at(it->second);
          double prod = (double)cnt * cy.tpWeight[k];
          double term = prod + (double)(con.maxSkew - 1);
          score += term;
        }
        s = (int64_t)std::round(score);
        break;
      }
      case KSG_PLUGIN_INTER_POD_AFFINITY:  // scoring.go:240-255
        for (auto& kv : cy.topoScore) {
          auto it = node.labels.find(kv.first);
          if (it == node.labels.end()) continue;
          auto vt = kv.second.find(it->second);
          if (vt != kv.second.end()) s += vt->second;
        }
        break;
    }
  return s;
}

// ---- ScoreExtensions.NormalizeScore -------------------------------------------------
static void normalize_scores(Cycle& cy, int p, std::vector<int64_t>& sc, const std::vector<NodeInfoO*>& nodes) {
  const int F = (int)nodes.size();

    if (p == KSG_PLUGIN_TAINT_TOLERATION || p == KSG_PLUGIN_NODE_AFFINITY) {  // helper/normalize_score.go:27-55
      bool reverse = p == KSG_PLUGIN_TAINT_TOLERATION;
      int64_t maxCount = 0;
      for (auto v : sc) maxCount = std::max(maxCount, v);
      if (maxCount == 0) {
        if (reverse)
          for (auto& v : sc) v = 100;
      } else {
        for (auto& v : sc) {
          int64_t x = 100 * v / maxCount;
          v = reverse ? 100 - x : x;
        }
      }
    } else if (p == KSG_PLUGIN_POD_TOPOLOGY_SPREAD) {  // scoring.go:229-268
      int64_t mn = INT64_MAX, mx = 0;
      std::vector<bool> ign(F);
      for (int i = 0; i < F; ++i) {
        ign[i] = cy.ignored.count(nodes[i]->node.name) > 0;
        if (ign[i]) { sc[i] = -1; continue; }
        mn = std::min(mn, sc[i]);
        mx = std::max(mx, sc[i]);
      }
      for (int i = 0; i < F; ++i) {
        if (sc[i] == -1) { sc[i] = 0; continue; }
        if (mx == 0) { sc[i] = 100; continue; }
        sc[i] = 100 * (mx + mn - sc[i]) / mx;
      }
    } else if (p == KSG_PLUGIN_INTER_POD_AFFINITY) {  // scoring.go:258-290
      if (!cy.topoScore.empty()) {
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        for (auto v : sc) { mx = std::max(mx, v); mn = std::min(mn, v); }
        int64_t diff = mx - mn;
        for (auto& v : sc) {
          double f = 0;
          if (diff > 0) f = 100.0 * ((double)(v - mn) / (double)diff);
          v = (int64_t)f;
        }
      }
    }
  
}

}  // namespace

// ===========================================================================
// schedulePod (schedule_one.go:564-618)
// ===========================================================================
// frameworkImpl.SignPod (framework/runtime/framework.go:884-924) over the profile's plugins, every one of
// which implements SignPlugin (computeBatchablePlugins, :832-876): the fragments keyed by signer name, or
// nil (false) as soon as one plugin refuses.  The volume plugins, DynamicResources and NodeDeclaredFeatures
// are always in the profile here; a pod that needs a declared feature never reaches a cycle.
static bool sign_pod(const ksgo_ctx* c, const Pod& p, std::string* sig) {
  const Config& k = c->cfg;
  const Pod::SignFragments& f = p.sign;
  std::string o = "sched=" + f.schedulerName;  // SchedulerNameSignerName
  if (k.enabled[KSG_PLUGIN_NODE_RESOURCES_FIT] || k.enabled[KSG_PLUGIN_BALANCED_ALLOCATION]) {
    // Fit.SignPod / BalancedAllocation.SignPod (fit.go:174-195, balanced_allocation.go:121-142):
    // computePodResourceRequest -- the preFilterState Resource as Fit's PreFilter builds it
    Resource r;
    int64_t pods = 0;
    bool scalar = false;
    for (auto& kv : pod_requests(p, nullptr, false)) {
      if (kv.first == "memory") r.memory = std::max(r.memory, milli_to_value(kv.second));
      else if (kv.first == "cpu") r.milliCPU = std::max(r.milliCPU, kv.second);
      else if (kv.first == "ephemeral-storage") r.ephemeral = std::max(r.ephemeral, milli_to_value(kv.second));
      else if (kv.first == "pods") pods = std::max(pods, milli_to_value(kv.second));
      else if (is_scalar_resource_name(kv.first)) {
        scalar = true;
        r.scalar[kv.first] = std::max(r.scalar[kv.first], milli_to_value(kv.second));
      }
    }
    o += "|res=" + std::to_string(r.milliCPU) + "," + std::to_string(r.memory) + "," + std::to_string(r.ephemeral) +
         "," + std::to_string(pods) + (scalar ? ",{" : ",null");
    if (scalar) {
      for (auto& kv : r.scalar) o += kv.first + "=" + std::to_string(kv.second) + ";";
      o += "}";
    }
  }
  if (k.enabled[KSG_PLUGIN_TAINT_TOLERATION] || k.enabled[KSG_PLUGIN_NODE_UNSCHEDULABLE])
    o += "|tol=" + f.tolerations;  // TolerationsSignerName (taint_toleration.go:61-65, node_unschedulable.go:118-122)
  if (k.enabled[KSG_PLUGIN_INTER_POD_AFFINITY]) {  // interpodaffinity/plugin.go:62-78
    if (p.hasPodAffinity || p.hasPodAntiAffinity) return false;
    if (!k.ignorePreferredTermsOfExistingPods) o += "|lbl=" + f.labels;
  }
  if (k.enabled[KSG_PLUGIN_NODE_PORTS]) o += "|ports=" + f.hostPorts;  // node_ports.go:66-70
  if (k.enabled[KSG_PLUGIN_POD_TOPOLOGY_SPREAD]) {                  // podtopologyspread/plugin.go:92-102
    if (!p.tsc.empty()) return false;
    if (k.ptsSystemDefaulted || !k.ptsDefaults.empty()) return false;  // pl.defaultConstraints non-empty
  }
  if (k.enabled[KSG_PLUGIN_NODE_AFFINITY]) o += "|na=" + f.nodeAffinity + "|nsel=" + f.nodeSelector;  // :78-88
  if (k.enabled[KSG_PLUGIN_NODE_NAME]) o += "|nn=" + p.nodeName;          // node_name.go:60-64
  if (k.enabled[KSG_PLUGIN_IMAGE_LOCALITY]) o += "|img=" + f.images;     // image_locality.go:55-67
  o += "|vol=" + f.volumes;  // VolumeRestrictions / NodeVolumeLimits / VolumeBinding / VolumeZone
  if (f.hasClaims) return false;  // DynamicResources (dynamicresources.go:236-241)
  o += "|feat=";  // NodeDeclaredFeatures: no required feature
  *sig = std::move(o);
  return true;
}

static int run_cycle(ksgo_ctx* c, const Pod& pod, ksg_result* res, ksg_eval_out* ev, bool cycle) {
  const double R0 = nowus();
  c->rebuild_list();
  c->prof[9] += nowus() - R0;
  g_taint_compare_ops = c->cfg.taintCompareOps;
  const int N = (int)c->list.size();
  // OpportunisticBatching's inputs: the cycle count, the pod's signature (SignPod, computed when the pod is
  // queued upstream; the same value here), the clock
  const int64_t cycleCount = cycle ? ++c->cycleCount : c->cycleCount;
  std::string sigv;
  const bool ob = cycle && c->cfg.obGate;
  const std::string* sig = ob && sign_pod(c, pod, &sigv) ? &sigv : nullptr;
  const int64_t now = ob ? c->now() : 0;
  res->status = KSG_CODE_SUCCESS;
  res->node_index = -1;
  res->evaluated_nodes = 0;
  res->feasible_nodes = 0;
  res->total_score = 0;
  if (ev) {
    ev->prefilter_code = 0;
    ev->prefilter_plugin = KSG_PLUGIN_NONE;
    ev->score_plugin_mask = 0;
    for (int i = 0; i < N; ++i) {
      if (ev->node_code) ev->node_code[i] = 0;
      if (ev->node_plugin) ev->node_plugin[i] = KSG_PLUGIN_NONE;
      if (ev->node_reasons) ev->node_reasons[i] = 0;
      if (ev->total_scores) ev->total_scores[i] = 0;
    }
    if (ev->plugin_scores)
      for (int i = 0; i < N * KSG_NUM_PLUGINS; ++i) ev->plugin_scores[i] = 0;
    if (ev->normalized_scores)
      for (int i = 0; i < N * KSG_NUM_PLUGINS; ++i) ev->normalized_scores[i] = 0;
  }
  auto idx_of = [](const NodeInfoO* ni) { return ni->pos; };
  if (N == 0) { res->status = KSG_CODE_ERROR; return KSG_OK; }  // ErrNoNodesAvailable
  double T0 = nowus();
  Cycle cy;
  cy.c = c;
  cy.pod = &pod;
  cy.reqNA = get_required_node_affinity(pod);  // PTS computes its own copy (filtering.go:257)
  // ---- RunPreFilterPlugins (framework.go:934-995)
  Status returnStatus;
  bool resultAll = true;
  std::set<std::string> resultNames;
  for (int p : prefilter_order()) {
    if (!c->cfg.enabled[p]) { cy.skipFilter[p] = true; continue; }
    bool skip = false, restricts = false;
    std::vector<std::string> names;
    Status s = run_prefilter_plugin(cy, p, &skip, &names, &restricts);
    if (skip) { cy.skipFilter[p] = true; continue; }
    if (!s.ok()) {
      s.plugin = p;
      if (s.code == KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE) { returnStatus = s; break; }
      if (s.code == KSG_CODE_UNSCHEDULABLE) { returnStatus = s; continue; }
      res->status = KSG_CODE_ERROR;
      if (ev) { ev->prefilter_code = KSG_CODE_ERROR; ev->prefilter_plugin = p; }
      return KSG_OK;
    }
    if (restricts) {  // PreFilterResult.Merge
      std::set<std::string> ns(names.begin(), names.end());
      if (resultAll) { resultNames = ns; resultAll = false; }
      else {
        std::set<std::string> x;
        for (auto& n : resultNames)
          if (ns.count(n)) x.insert(n);
        resultNames = x;
      }
      if (resultNames.empty()) { returnStatus = mk(KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, KSG_R_PREFILTER); returnStatus.plugin = p; break; }
    }
  }
  for (int p = 0; p < KSG_NUM_PLUGINS; ++p)
    if (!c->cfg.enabled[p]) cy.skipFilter[p] = true;
  if (!returnStatus.ok()) {  // schedule_one.go:635-648: every node gets the PreFilter status
    res->status = KSG_CODE_UNSCHEDULABLE;  // FitError
    res->evaluated_nodes = 0;
    if (ev) {
      ev->prefilter_code = returnStatus.code;
      ev->prefilter_plugin = returnStatus.plugin;
      for (int i = 0; i < N; ++i) {
        if (ev->node_code) ev->node_code[i] = (uint8_t)returnStatus.code;
        if (ev->node_plugin) ev->node_plugin[i] = (uint8_t)returnStatus.plugin;
        if (ev->node_reasons) ev->node_reasons[i] = returnStatus.reasons | KSG_R_PREFILTER;
      }
    }
    return KSG_OK;
  }

  double T1 = nowus(); c->prof[0] += T1 - T0;
  // ---- nodes to evaluate (schedule_one.go:671-682; map order -> snapshot order)
  std::vector<NodeInfoO*> nodes;
  if (resultAll) nodes = c->list;
  else {
    for (auto* ni : c->list)
      if (resultNames.count(ni->node.name)) nodes.push_back(ni);
    if (ev)
      for (int i = 0; i < N; ++i)
        if (!resultNames.count(c->list[i]->node.name)) {
          if (ev->node_code) ev->node_code[i] = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
          if (ev->node_reasons) ev->node_reasons[i] = KSG_R_PREFILTER;
        }
  }

  // ---- findNodesThatPassFilters (schedule_one.go:771-854), sequential order
  bool hasScore = false;
  for (int p : kScoreOrder)
    if (c->cfg.enabled[p]) hasScore = true;
  int numAll = (int)nodes.size();
  int64_t numToFind;
  {  // numFeasibleNodesToFind :858-884
    if (numAll < 100) numToFind = numAll;
    else {
      int64_t pct = c->cfg.pct;
      if (pct == 0) { pct = 50 - numAll / 125; if (pct < 5) pct = 5; }
      numToFind = (int64_t)numAll * pct / 100;
      if (numToFind < 100) numToFind = 100;
    }
    if (!hasScore) numToFind = 1;
  }
  std::vector<NodeInfoO*> feasible;
  int failed = 0;
  int visited = numAll;  // rotated positions [0, visited) went through the filters (the rest: cut off)
  auto filter_node = [&](NodeInfoO* ni) {
    Status st;
    for (int p : kFilterOrder) {
      if (cy.skipFilter[p]) continue;
      st = run_filter(cy, p, ni);
      if (!st.ok()) { st.plugin = p; break; }
    }
    return st;
  };
  auto record_failed = [&](NodeInfoO* ni, const Status& st) {
    if (ev) {
      int idx = idx_of(ni);
      if (ev->node_code) ev->node_code[idx] = (uint8_t)st.code;
      if (ev->node_plugin) ev->node_plugin[idx] = (uint8_t)st.plugin;
      if (ev->node_reasons) ev->node_reasons[idx] = st.reasons;
    }
  };
  // ---- GetNodeHint (schedule_one.go:650-655, batch.go:65-95), then evaluateNominatedNode (:657-669,714-745) with
  // the pod's status.nominatedNodeName, else the hint: that node alone through findNodesThatPassFilters;
  // feasible -> it is the result (nextStartNodeIndex stays), else its status joins NodeToStatus and the full
  // pass follows.  A name not in the snapshot: GetNodeInPlacement and Get fail, the error is logged
  // (HandleErrorWithContext) and the full pass follows.
  std::string hint;
  int hintFailed = -1;  // a nominated / hinted node that failed its filters (its status is in NodeToStatus)
  if (ob)
    hint = c->batch.GetNodeHint(sig, pod.nominatedNodeName, cycleCount, now, [&](const std::string& nm) {
      NodeInfoO* ni = c->snapMap.count(nm) ? c->nodes[nm].get() : nullptr;  // nodeInfos.Get
      if (!ni) return -1;
      return filter_node(ni).ok() ? 0 : 1;  // RunFilterPlugins: IsRejected
    });
  const std::string& nnn = !pod.nominatedNodeName.empty() ? pod.nominatedNodeName : hint;
  if (!nnn.empty() && c->snapMap.count(nnn)) {
    NodeInfoO* hn = c->nodes[nnn].get();
    Status st = filter_node(hn);
    if (st.ok()) {  // schedulePod's one-feasible-node path (:586-598)
      if (ob) c->batch.StoreScheduleResults(sig, hint, nnn, nullptr, cycleCount, now);
      res->node_index = idx_of(hn);
      res->feasible_nodes = 1;
      res->evaluated_nodes = 1;
      return KSG_OK;
    }
    record_failed(hn, st);
    hintFailed = idx_of(hn);
  }
  if (c->pool && numToFind >= numAll) {
    // CPU-baseline mode: Parallelizer.Until's chunks of the rotated order (schedule_one.go:840), then
    // the per-chunk feasible lists concatenated in chunk order -- the sequential loop's result
    // exactly (with every node to be found there is no early stop to race on)
    // (one buffer for every chunk, as the reference's feasibleNodes slice: chunk k writes its feasible
    // nodes from its own first index on, so no allocation happens inside the parallel pass)
    const int T = c->pool->chunks(numAll);
    c->filt_buf.resize((size_t)numAll);
    c->filt_lo.assign((size_t)T, 0);
    c->filt_cnt.assign((size_t)T, 0);
    c->filt_fail.assign((size_t)T, 0);
    NodeInfoO** buf = c->filt_buf.data();
    c->pool->until(numAll, [&](int k, int a, int b) {
      int cnt = 0, nf = 0;
      for (int i = a; i < b; ++i) {
        NodeInfoO* ni = nodes[(c->nextStartNodeIndex + i) % numAll];
        Status st = filter_node(ni);
        if (st.ok()) buf[a + cnt++] = ni;
        else { ++nf; record_failed(ni, st); }
      }
      c->filt_lo[(size_t)k] = a;
      c->filt_cnt[(size_t)k] = cnt;
      c->filt_fail[(size_t)k] = nf;
    });
    feasible.reserve((size_t)numAll);
    for (int k = 0; k < T; ++k) {
      feasible.insert(feasible.end(), buf + c->filt_lo[(size_t)k], buf + c->filt_lo[(size_t)k] + c->filt_cnt[(size_t)k]);
      failed += c->filt_fail[(size_t)k];
    }
  } else {
    for (int i = 0; i < numAll; ++i) {
      NodeInfoO* ni = nodes[(c->nextStartNodeIndex + i) % numAll];
      Status st = filter_node(ni);
      if (st.ok()) {
        if ((int64_t)feasible.size() + 1 > numToFind) {  // cancel: enough feasible nodes
          visited = i;
          break;
        }
        feasible.push_back(ni);
      } else {
        ++failed;
        record_failed(ni, st);
      }
    }
  }
  double T2 = nowus(); c->prof[1] += T2 - T1;
  if (hintFailed >= 0) {  // NodeToStatus is keyed by node: the nominated / hinted node counts once -- again only if
                          // the full pass reached it (it fails there too: same state, same filters)
    bool again = false;
    for (int i = 0; i < visited && !again; ++i) again = idx_of(nodes[(c->nextStartNodeIndex + i) % numAll]) == hintFailed;
    if (!again) ++failed;
  }
  int processed = (int)feasible.size() + failed;
  int diagLen = failed;  // NodeToStatus.Len(): explicit per-node statuses only
  c->nextStartNodeIndex = (c->nextStartNodeIndex + processed) % N;  // :686-687
  if (feasible.empty()) {  // FitError (schedule_one.go:579-585)
    res->status = KSG_CODE_UNSCHEDULABLE;
    res->feasible_nodes = 0;
    res->evaluated_nodes = diagLen;
    return KSG_OK;
  }
  res->feasible_nodes = (int)feasible.size();
  if (feasible.size() == 1) {  // :588-598
    res->node_index = idx_of(feasible[0]);
    res->evaluated_nodes = 1 + diagLen;
    if (ob) c->batch.StoreScheduleResults(sig, hint, feasible[0]->node.name, nullptr, cycleCount, now);
    return KSG_OK;
  }
  res->evaluated_nodes = (int)feasible.size() + diagLen;

  // ---- prioritizeNodes (:937-1048)
  const int F = (int)feasible.size();
  std::vector<int64_t> totals(F, 0);
  if (!hasScore) {
    for (int i = 0; i < F; ++i) totals[i] = 1;
  } else {
    // RunPreScorePlugins (framework.go:1300-1333)
    for (int p : kPreScoreOrder) {
      if (!c->cfg.enabled[p]) { cy.skipScore[p] = true; continue; }
      Status st = prescore_plugin(cy, p, feasible);
      if (st.code == KSG_CODE_SKIP) { cy.skipScore[p] = true; continue; }
      if (!st.ok()) { res->status = KSG_CODE_ERROR; return KSG_OK; }
    }
    c->prof[2] += nowus() - T2; T2 = nowus();
    // RunScorePlugins (framework.go:1351-1458)
    std::vector<int> active;
    for (int p : kScoreOrder)
      if (c->cfg.enabled[p] && !cy.skipScore[p]) active.push_back(p);
    std::vector<std::vector<int64_t>> scores(active.size(), std::vector<int64_t>(F, 0));
    if (c->pool) {  // CPU-baseline mode: one Parallelizer.Until pass over the nodes, every plugin's
                    // Score per node (framework.go:1378-1402), then NormalizeScore per plugin
      std::atomic<bool> bad{false};
      c->pool->until(F, [&](int, int lo, int hi) {
        for (int i = lo; i < hi; ++i)
          for (size_t a = 0; a < active.size(); ++a) {
            int code;
            scores[a][i] = score_node(cy, active[a], feasible[i], &code);
            if (code != KSG_CODE_SUCCESS) bad = true;
          }
      });
      if (bad) { res->status = KSG_CODE_ERROR; return KSG_OK; }
    }
    for (size_t a = 0; a < active.size(); ++a) {
      int p = active[a];
      if (!c->pool) {
        for (int i = 0; i < F; ++i) {
          int code;
          scores[a][i] = score_node(cy, p, feasible[i], &code);
          if (code != KSG_CODE_SUCCESS) { res->status = KSG_CODE_ERROR; return KSG_OK; }
        }
      }
      if (!c->pool || !c->cfg.par_weights) normalize_scores(cy, p, scores[a], feasible);
    }
    if (c->pool && c->cfg.par_weights)  // NormalizeScore per plugin in parallel (framework.go:1409-1423)
      c->pool->until((int)active.size(), [&](int, int lo, int hi) {
        for (int a = lo; a < hi; ++a) normalize_scores(cy, active[a], scores[a], feasible);
      });
    c->prof[3] += nowus() - T2; T2 = nowus();
    // weights + totals (framework.go:1428-1452; in parallel over the nodes in CPU-baseline mode)
    const bool pw = c->pool && c->cfg.par_weights;
    if (pw) {
      std::atomic<bool> bad{false};
      c->pool->until(F, [&](int, int lo, int hi) {
        for (int i = lo; i < hi; ++i)
          for (size_t a = 0; a < active.size(); ++a) {
            const int64_t s = scores[a][i];
            if (s > 100 || s < 0) bad = true;
            totals[i] += s * c->cfg.weight[active[a]];
          }
      });
      if (bad) { res->status = KSG_CODE_ERROR; return KSG_OK; }
    }
    for (size_t a = 0; a < active.size(); ++a) {
      if (pw && !ev) break;  // done above (ev: the per-plugin record below, totals already summed)
      int p = active[a];
      if (ev) ev->score_plugin_mask |= 1u << p;
      for (int i = 0; i < F; ++i) {
        int64_t s = scores[a][i];
        if (s > 100 || s < 0) { res->status = KSG_CODE_ERROR; return KSG_OK; }
        int64_t w = s * c->cfg.weight[p];
        if (!pw) totals[i] += w;
        if (ev && ev->plugin_scores) ev->plugin_scores[(size_t)p * N + idx_of(feasible[i])] = w;
        if (ev && ev->normalized_scores) ev->normalized_scores[(size_t)p * N + idx_of(feasible[i])] = s;
      }
    }
  }
  if (ev && ev->total_scores)
    for (int i = 0; i < F; ++i) ev->total_scores[idx_of(feasible[i])] = totals[i];
  c->prof[4] += nowus() - T2; T2 = nowus();
  // ---- host selection: heap.Init + heap.Pop (schedule_one.go:605-606,1054-1063)
  std::vector<HeapEnt> h(F);
  for (int i = 0; i < F; ++i) h[i] = {totals[i], 0, i};
  int win = heap_pop_index(h);
  res->node_index = idx_of(feasible[win]);
  res->total_score = totals[win];
  if (ob) {  // newSortedNodeScores + Pop, then StoreScheduleResults with the rest (:605-611)
    auto rest = std::make_unique<SortedScoredNodes>();
    rest->heap = std::move(h);
    for (auto* ni : feasible) rest->names.push_back(ni->node.name);
    for (int i = F / 2 - 1; i >= 0; i--) heap_down(rest->heap, i, F);  // heap.Init
    const std::string top = rest->Pop();
    if (top != feasible[win]->node.name) { c->err = "oracle: heap root differs from the pop"; return KSG_EINVAL; }
    c->batch.StoreScheduleResults(sig, hint, top, std::move(rest), cycleCount, now);
  }
  c->prof[5] += nowus() - T2;
  return KSG_OK;
}

// ===========================================================================
// C API
// ===========================================================================
extern "C" {

ksgo_ctx* ksgo_create(const char* json, size_t len) {
  auto* c = new ksgo_ctx();
  try {
    if (json && len) {
      mj::Value v = mj::parse(json, len);
      std::string err;
      if (!decode_config(v, &c->cfg, &err) || !validate_config(c->cfg, &err)) {
        g_create_error = err;
        delete c;
        return nullptr;
      }
    }
  } catch (std::exception& e) {
    g_create_error = e.what();
    delete c;
    return nullptr;
  }
  if (c->cfg.threads > 1) c->pool.reset(new Pool(c->cfg.threads, c->cfg.spin_us));
  return c;
}
const char* ksgo_create_error(void) { return g_create_error.c_str(); }
void ksgo_destroy(ksgo_ctx* c) { delete c; }
const char* ksgo_last_error(const ksgo_ctx* c) { return c->err.c_str(); }

int ksgo_upsert_object(ksgo_ctx* c, const char* json, size_t len) {
  SelectorObject o;
  try {
    mj::Value v = mj::parse(json, len);
    if (!decode_selector_object(v, &o, &c->err)) return KSG_EINVAL;
  } catch (std::exception& e) {
    c->err = e.what();
    return KSG_EINVAL;
  }
  if (o.kind == "Service") c->services[o.ns][o.name] = o;
  else c->owners[{o.kind, o.ns, o.name}] = o;
  return KSG_OK;
}
int ksgo_remove_object(ksgo_ctx* c, const char* kind, const char* ns, const char* name) {
  std::string k = kind, n = (ns && *ns) ? ns : "default", nm = name;
  if (k == "Service") {
    auto it = c->services.find(n);
    if (it == c->services.end() || !it->second.erase(nm)) return KSG_ENOTFOUND;
    return KSG_OK;
  }
  if (k != "ReplicationController" && k != "ReplicaSet" && k != "StatefulSet") return KSG_EINVAL;
  return c->owners.erase({k, n, nm}) ? KSG_OK : KSG_ENOTFOUND;
}

int ksgo_upsert_namespace(ksgo_ctx* c, const char* json, size_t len) {
  try {
    Namespace ns;
    if (!decode_namespace(mj::parse(json, len), &ns, &c->err)) return KSG_EINVAL;
    c->namespaces[ns.name] = ns;
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}

static void add_node_images(ksgo_ctx* c, const Node& n) {  // cache.go:712-735
  for (auto& im : n.images)
    for (auto& name : im.names) {
      auto it = c->imageStates.find(name);
      if (it == c->imageStates.end()) {
        ImageState st;
        st.size = im.sizeBytes;
        st.nodes.insert(n.name);
        c->imageStates[name] = st;
      } else {
        it->second.nodes.insert(n.name);
      }
    }
}
static void remove_node_images(ksgo_ctx* c, const Node& n) {  // cache.go:740-759
  for (auto& im : n.images)
    for (auto& name : im.names) {
      auto it = c->imageStates.find(name);
      if (it != c->imageStates.end()) {
        it->second.nodes.erase(n.name);
        if (it->second.nodes.empty()) c->imageStates.erase(it);
      }
    }
}
static void tree_add(ksgo_ctx* c, const Node& n) {  // node_tree.go:52-70
  std::string z = get_zone_key(n);
  auto it = c->tree.find(z);
  if (it == c->tree.end()) { c->zones.push_back(z); c->tree[z] = {n.name}; }
  else {
    for (auto& nm : it->second)
      if (nm == n.name) return;
    it->second.push_back(n.name);
  }
  c->numNodes++;
}
static void tree_remove(ksgo_ctx* c, const Node& n) {  // node_tree.go:73-98
  std::string z = get_zone_key(n);
  auto it = c->tree.find(z);
  if (it == c->tree.end()) return;
  auto& na = it->second;
  for (size_t i = 0; i < na.size(); ++i)
    if (na[i] == n.name) {
      na.erase(na.begin() + i);
      if (na.empty()) {
        c->tree.erase(it);
        c->zones.erase(std::find(c->zones.begin(), c->zones.end(), z));
      }
      c->numNodes--;
      return;
    }
}

// Cache.AddNode (cache.go:630-646).  An AddNode for a node the cache holds with its Node object is
// taken as UpdateNode (as the product does): upstream would append the name to a second zone list
// when the zone changed, which the informer never asks for.
int ksgo_update_node(ksgo_ctx* c, const char* json, size_t len);
int ksgo_add_node(ksgo_ctx* c, const char* json, size_t len) {
  try {
    Node n;
    if (!decode_node(mj::parse(json, len), &n, &c->err)) return KSG_EINVAL;
    auto it = c->nodes.find(n.name);
    NodeInfoO* ni;
    if (it == c->nodes.end()) {
      auto up = std::make_unique<NodeInfoO>();
      ni = up.get();
      c->nodes[n.name] = std::move(up);
    } else if (it->second->hasNode) {
      return ksgo_update_node(c, json, len);
    } else {
      ni = it->second.get();  // a ghost: removeNodeImageStates(nil) is a no-op
    }
    tree_add(c, n);
    add_node_images(c, n);
    ni->node = n;
    ni->hasNode = true;
    ni->allocatable = node_allocatable(n);
    c->changed.push_back(n.name);
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}

int ksgo_update_node(ksgo_ctx* c, const char* json, size_t len) {  // cache.go:648-664
  try {
    Node n;
    if (!decode_node(mj::parse(json, len), &n, &c->err)) return KSG_EINVAL;
    auto it = c->nodes.find(n.name);
    if (it == c->nodes.end() || !it->second->hasNode) return ksgo_add_node(c, json, len);
    NodeInfoO* ni = it->second.get();
    remove_node_images(c, ni->node);
    if (get_zone_key(ni->node) != get_zone_key(n)) { tree_remove(c, ni->node); tree_add(c, n); }  // node_tree.go:102-115
    add_node_images(c, n);
    ni->node = n;
    ni->allocatable = node_allocatable(n);
    c->changed.push_back(n.name);
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}

int ksgo_remove_node(ksgo_ctx* c, const char* name) {  // cache.go:672-695
  auto it = c->nodes.find(name);
  if (it == c->nodes.end() || !it->second->hasNode) { c->err = "node not found"; return KSG_ENOTFOUND; }
  NodeInfoO* ni = it->second.get();
  tree_remove(c, ni->node);
  remove_node_images(c, ni->node);
  ni->hasNode = false;  // n.info.RemoveNode(); the pods stay until their delete events
  c->maybe_drop(name);
  return KSG_OK;
}

int ksgo_add_pod(ksgo_ctx* c, const char* json, size_t len) {  // cache.go:437-466 addPod
  try {
    Pod p;
    if (!decode_pod(mj::parse(json, len), &p, &c->err)) return KSG_EINVAL;
    if (p.nodeName.empty()) { c->err = "pod is not bound"; return KSG_EINVAL; }
    if (c->pods.count(p.uid)) { c->err = "pod exists"; return KSG_EEXIST; }
    auto it = c->nodes.find(p.nodeName);
    if (it == c->nodes.end())  // a ghost NodeInfo (cache.go:442-446)
      it = c->nodes.emplace(p.nodeName, std::make_unique<NodeInfoO>()).first;
    auto pi = std::make_unique<PodInfo>();
    new_pod_info(p, pi.get());
    node_add_pod(*it->second, pi.get());
    c->pods[p.uid] = std::move(pi);
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}

int ksgo_remove_pod(ksgo_ctx* c, const char* uid) {  // cache.go:480-513 removePod
  auto it = c->pods.find(uid);
  if (it == c->pods.end()) return KSG_ENOTFOUND;
  const std::string node = it->second->pod.nodeName;
  auto nt = c->nodes.find(node);
  if (nt != c->nodes.end()) node_remove_pod(*nt->second, uid);
  c->pods.erase(it);
  c->maybe_drop(node);
  return KSG_OK;
}

int ksgo_num_nodes(const ksgo_ctx* c) {
  const_cast<ksgo_ctx*>(c)->rebuild_list();
  return (int)c->list.size();
}

int ksgo_node_name(const ksgo_ctx* c, int32_t index, char* buf, size_t cap) {
  const_cast<ksgo_ctx*>(c)->rebuild_list();
  if (index < 0 || index >= (int32_t)c->list.size()) return KSG_ENOTFOUND;
  const std::string& n = c->list[index]->node.name;
  if (buf && cap) {
    size_t k = std::min(cap - 1, n.size());
    std::memcpy(buf, n.data(), k);
    buf[k] = 0;
  }
  return (int)n.size();
}

int ksgo_pod_compile(ksgo_ctx* c, const char* json, size_t len, int32_t* handle) {
  try {
    mj::Value v = mj::parse(json, len);
    auto p = std::make_unique<Pod>();
    if (!decode_pod(v, p.get(), &c->err)) return KSG_EINVAL;
    // the contract's plugin set: volume plugins / DynamicResources would not Skip their PreFilter for
    // these pods (volume_binding.go:350-358, nodevolumelimits/csi.go:239-249, volume_restrictions.go:
    // 168-197, dynamicresources.go:446-479), so the pod is declined as the product declines it
    if (auto sp = v.has("spec")) {
      if (auto vols = sp->has("volumes"))
        for (auto& vol : vols->arr)
          for (const char* k : {"persistentVolumeClaim", "ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "cinder",
                                "azureDisk", "azureFile", "vsphereVolume", "portworxVolume", "rbd", "iscsi"})
            if (vol.has(k)) { c->err = std::string("volume needs ") + k + " plugins"; return KSG_ENOTSUP; }
      if (auto rc = sp->has("resourceClaims"))
        if (rc->is_arr() && !rc->arr.empty()) { c->err = "resourceClaims"; return KSG_ENOTSUP; }
    }
    if (p->needsNodeFeatures) {  // NodeDeclaredFeatures' PreFilter would not Skip (nodedeclaredfeatures.go:86-104)
      c->err = "the pod needs a declared node feature (NodeDeclaredFeatures)";
      return KSG_ENOTSUP;
    }
    int32_t h = c->nextHandle++;
    c->queue[h] = std::move(p);
    *handle = h;
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}

int ksgo_set_clock(ksgo_ctx* c, int64_t now_ns) {
  c->clockNs = now_ns;
  return KSG_OK;
}
int ksgo_debug_clock_step(ksgo_ctx* c, int64_t step_ns) {
  if (!c || step_ns < 0) return KSG_EINVAL;
  c->clockStep = step_ns;
  return KSG_OK;
}

// TestBatchBasic (framework/runtime/batch_test.go:187-436), one case: the first pod's GetNodeHint and (if it
// was scheduled) StoreScheduleResults at cycle 1, then the second pod's GetNodeHint at cycle 2 (3 when a pod of
// another profile came between, 1 for the same PodGroup cycle) against the lister holding the first chosen
// node, whose filter rejects the second pod iff both pod ids start with 'b' (BatchTestPlugin.Filter), and its
// StoreScheduleResults.  in: {"firstPodID", "firstSig", "firstPodScheduledSuccessfully", "firstChosenNode",
// "firstOtherNodes": [..] | null, "sameCycle", "skipPod", "secondPodID", "secondPodNominatedNodeName",
// "secondSig", "secondChosenNode", "secondOtherNodes": [..] | null, "genericWorkloadEnabled"}; out: {"hint",
// "empty", "signature", "sortedNodes": [..]}.
int ksgo_debug_batch_basic(const char* json, size_t len, char* out, size_t cap) {
  try {
    mj::Value v = mj::parse(json, len);
    OpportunisticBatch b;
    b.genericWorkloadEnabled = v.boolean("genericWorkloadEnabled");
    auto list = [&](const char* k) -> std::unique_ptr<SortedScoredNodes> {
      const mj::Value* a = v.has(k);
      if (!a) return nullptr;
      auto s = std::make_unique<SortedScoredNodes>();
      s->isList = true;
      for (auto& x : a->arr) s->names.push_back(x.s);
      return s;
    };
    const std::string fs = v.str("firstSig"), ss = v.str("secondSig");
    auto never = [](const std::string&) { return -1; };
    std::string hint = b.GetNodeHint(&fs, "", 1, 0, never);
    if (!hint.empty()) { std::snprintf(out, cap, "{\"error\":\"first pod got a hint\"}"); return KSG_EINVAL; }
    if (v.boolean("firstPodScheduledSuccessfully"))
      b.StoreScheduleResults(&fs, hint, v.str("firstChosenNode"), list("firstOtherNodes"), 1, 0);
    const int64_t cycle = v.boolean("skipPod") ? 3 : v.boolean("sameCycle") ? 1 : 2;
    const std::string first = v.str("firstChosenNode");
    const bool blocking = v.str("firstPodID").rfind("b", 0) == 0 && v.str("secondPodID").rfind("b", 0) == 0;
    hint = b.GetNodeHint(&ss, v.str("secondPodNominatedNodeName"), cycle, 0, [&](const std::string& nm) {
      if (nm != first) return -1;  // the lister holds only the first chosen node
      return blocking ? 1 : 0;
    });
    b.StoreScheduleResults(&ss, hint, v.str("secondChosenNode"), list("secondOtherNodes"), cycle, 0);
    std::string o = "{\"hint\":\"" + hint + "\",\"empty\":" + (b.stateEmpty() ? "true" : "false");
    if (!b.stateEmpty()) {
      o += ",\"signature\":\"" + b.state->signature + "\",\"sortedNodes\":[";
      SortedScoredNodes& sn = *b.state->sortedNodes;
      for (size_t i = sn.head; i < sn.names.size(); ++i) o += (i > sn.head ? ",\"" : "\"") + sn.names[i] + "\"";
      o += "]";
    }
    o += "}";
    if (o.size() + 1 > cap) return KSG_ENOMEM;
    std::memcpy(out, o.c_str(), o.size() + 1);
    return KSG_OK;
  } catch (std::exception& e) {
    std::snprintf(out, cap, "{\"error\":\"%s\"}", e.what());
    return KSG_EINVAL;
  }
}

int ksgo_pod_release(ksgo_ctx* c, int32_t handle) {
  return c->queue.erase(handle) ? KSG_OK : KSG_ENOTFOUND;
}

// addGENominatedPods' condition (framework.go:1265-1294): another uid nominated to a snapshot node with priority >= the
// pod's -- refused (the boundary above)
static int check_nominations(ksgo_ctx* c, const Pod& p) {
  if (c->nominated.empty()) return KSG_OK;
  c->rebuild_list();
  for (const auto& kv : c->nominated)
    if (kv.first != p.uid && kv.second.second >= p.priority && c->snapMap.count(kv.second.first)) {
      c->err = "another pod of equal or higher priority is nominated to node " + kv.second.first;
      return KSG_ENOTSUP;
    }
  return KSG_OK;
}

int ksgo_add_nominated_pod(ksgo_ctx* c, const char* json, size_t len) {  // nominator.go:60-103 (ModeNoop)
  try {
    Pod p;
    if (!decode_pod(mj::parse(json, len), &p, &c->err)) return KSG_EINVAL;
    if (p.uid.empty()) { c->err = "metadata.uid is empty"; return KSG_EINVAL; }
    c->nominated.erase(p.uid);
    if (!p.nominatedNodeName.empty()) c->nominated[p.uid] = {p.nominatedNodeName, p.priority};
    return KSG_OK;
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
}
int ksgo_delete_nominated_pod(ksgo_ctx* c, const char* uid) {  // nominator.go:138-150
  c->nominated.erase(uid);
  return KSG_OK;
}

int ksgo_schedule_one(ksgo_ctx* c, int32_t handle, uint32_t flags, ksg_result* result, ksg_eval_out* ev) {
  auto it = c->queue.find(handle);
  if (it == c->queue.end()) return KSG_ENOTFOUND;
  if (const int rn = check_nominations(c, *it->second)) return rn;
  double A0 = nowus();
  int rc = run_cycle(c, *it->second, result, ev, true);
  double A1 = nowus(); c->prof[6] += A1 - A0; c->prof[8] += 1;
  if (rc != KSG_OK) return rc;
  if ((flags & KSG_FLAG_ASSUME) && result->status == KSG_CODE_SUCCESS && result->node_index >= 0) {
    // Scheduler.assume (schedule_one.go:1102-1137) -> Cache.AssumePod (cache.go:397)
    Pod p = *it->second;
    p.nodeName = c->list[result->node_index]->node.name;
    p.uid = p.uid + "#a" + std::to_string(++c->assumeSeq);  // unique per assume
    auto pi = std::make_unique<PodInfo>();
    new_pod_info(p, pi.get());
    node_add_pod(*c->nodes[p.nodeName], pi.get());
    c->assumedUid[handle] = p.uid;
    c->pods[p.uid] = std::move(pi);
    c->nominated.erase(it->second->uid);  // DeleteNominatedPodIfExists (schedule_one.go:1131-1134)
  }
  c->prof[7] += nowus() - A1;
  return KSG_OK;
}
// CPU-baseline breakdown (bench.py): totals since the last call, in microseconds -- [0] PreFilter,
// [1] Filter pass, [2] PreScore, [3] Score pass + NormalizeScore, [4] weights, [5] selectHost,
// [6] whole cycle, [7] assume, [8] cycles, [9] snapshot update (inside [6]); then reset
int ksgo_debug_profile(ksgo_ctx* c, double* out, int n) {
  for (int k = 0; k < n && k < 10; ++k) out[k] = c->prof[k];
  for (double& v : c->prof) v = 0;
  return KSG_OK;
}

int ksgo_schedule_batch(ksgo_ctx* c, const int32_t* handles, int32_t n, uint32_t flags, ksg_result* results) {
  for (int32_t i = 0; i < n; ++i) {  // (refused as a whole, before any pod: the product's contract)
    auto it = c->queue.find(handles[i]);
    if (it == c->queue.end()) return KSG_ENOTFOUND;
    if (const int rn = check_nominations(c, *it->second)) return rn;
  }
  for (int32_t i = 0; i < n; ++i) {
    int rc = ksgo_schedule_one(c, handles[i], flags, &results[i], nullptr);
    if (rc != KSG_OK) return rc;
  }
  return KSG_OK;
}

int ksgo_forget(ksgo_ctx* c, int32_t handle) {  // Cache.ForgetPod (cache.go:412-434)
  auto it = c->assumedUid.find(handle);
  if (it == c->assumedUid.end()) return KSG_ENOTFOUND;
  int rc = ksgo_remove_pod(c, it->second.c_str());
  c->assumedUid.erase(it);
  return rc;
}


// ---- plugin-granular entry points (FilterPlugin / ScorePlugin contracts) --------------
static Cycle* new_cycle(ksgo_ctx* c, const Pod& pod) {
  c->rebuild_list();
  g_taint_compare_ops = c->cfg.taintCompareOps;
  Cycle* cy = new Cycle();
  cy->c = c;
  cy->pod = &pod;
  cy->reqNA = get_required_node_affinity(pod);
  return cy;
}

int ksgo_run_filter_plugin(ksgo_ctx* c, int32_t handle, int32_t plugin, int32_t* prefilter_code, uint8_t* codes,
                           uint32_t* reasons) {
  auto it = c->queue.find(handle);
  if (it == c->queue.end()) return KSG_ENOTFOUND;
  if (plugin < 0 || plugin > KSG_PLUGIN_INTER_POD_AFFINITY) return KSG_EINVAL;
  std::unique_ptr<Cycle> cy(new_cycle(c, *it->second));
  const int N = (int)c->list.size();
  *prefilter_code = KSG_CODE_SUCCESS;
  for (int i = 0; i < N; ++i) { codes[i] = 0; reasons[i] = 0; }
  bool hasPre = false;
  for (int p : prefilter_order()) hasPre |= p == plugin;
  if (hasPre) {
    bool skip = false, restricts = false;
    std::vector<std::string> names;
    Status s = run_prefilter_plugin(*cy, plugin, &skip, &names, &restricts);
    if (skip) { *prefilter_code = KSG_CODE_SKIP; return KSG_OK; }
    if (!s.ok()) {
      *prefilter_code = s.code;
      for (int i = 0; i < N; ++i) { codes[i] = (uint8_t)s.code; reasons[i] = s.reasons | KSG_R_PREFILTER; }
      return KSG_OK;
    }
  }
  for (int i = 0; i < N; ++i) {
    Status st = run_filter(*cy, plugin, c->list[i]);
    codes[i] = (uint8_t)st.code;
    reasons[i] = st.reasons;
  }
  return KSG_OK;
}

int ksgo_run_score_plugin(ksgo_ctx* c, int32_t handle, int32_t plugin, const uint8_t* nodes, int32_t* status_code,
                          int64_t* raw, int64_t* normalized) {
  auto it = c->queue.find(handle);
  if (it == c->queue.end()) return KSG_ENOTFOUND;
  bool isScore = false;
  for (int p : kScoreOrder) isScore |= p == plugin;
  if (!isScore) return KSG_EINVAL;
  std::unique_ptr<Cycle> cy(new_cycle(c, *it->second));
  const int N = (int)c->list.size();
  for (int i = 0; i < N; ++i) { raw[i] = 0; normalized[i] = 0; }
  *status_code = KSG_CODE_SUCCESS;
  // the node list prioritizeNodes would pass (feasible nodes in snapshot order)
  std::vector<NodeInfoO*> list;
  std::vector<int> idx;
  for (int i = 0; i < N; ++i)
    if (!nodes || nodes[i]) { list.push_back(c->list[i]); idx.push_back(i); }
  bool hasPre = false;
  for (int p : kPreScoreOrder) hasPre |= p == plugin;
  if (hasPre) {
    Status st = prescore_plugin(*cy, plugin, list);
    if (!st.ok()) { *status_code = st.code; return KSG_OK; }
  }
  std::vector<int64_t> sc(list.size());
  for (size_t i = 0; i < list.size(); ++i) {
    int code;
    sc[i] = score_node(*cy, plugin, list[i], &code);
    raw[idx[i]] = sc[i];
    if (code != KSG_CODE_SUCCESS) *status_code = code;
  }
  if (*status_code != KSG_CODE_SUCCESS) return KSG_OK;
  normalize_scores(*cy, plugin, sc, list);
  for (size_t i = 0; i < list.size(); ++i) normalized[idx[i]] = sc[i];
  return KSG_OK;
}

// ---- DefaultPreemption PostFilter (plugins/defaultpreemption/default_preemption.go,
// framework/preemption/preemption.go) -------------------------------------------------------
// PreFilter once, as the failed cycle ran it (framework.go:934-995); the cycle's state is cloned per
// node for the dry run (preemption.go:420-424).
static bool preempt_prefilter(ksgo_ctx* c, Cycle& cy) {
  for (int p : prefilter_order()) {
    if (!c->cfg.enabled[p]) { cy.skipFilter[p] = true; continue; }
    bool skip = false, restricts = false;
    std::vector<std::string> names;
    Status s = run_prefilter_plugin(cy, p, &skip, &names, &restricts);
    if (skip) { cy.skipFilter[p] = true; continue; }
    if (!s.ok()) return false;
  }
  for (int p = 0; p < KSG_NUM_PLUGINS; ++p)
    if (!c->cfg.enabled[p]) cy.skipFilter[p] = true;
  return true;
}
static Status preempt_filter_node(Cycle& cy, NodeInfoO* ni) {  // RunFilterPluginsWithNominatedPods (no nominated pods)
  Status st;
  for (int p : kFilterOrder) {
    if (cy.skipFilter[p]) continue;
    st = run_filter(cy, p, ni);
    if (!st.ok()) { st.plugin = p; break; }
  }
  return st;
}
// criticalPaths (podtopologyspread/filtering.go:84-136), the two smallest (value, count) of a constraint
struct CritPaths { std::string v[2]; int64_t n[2] = {INT32_MAX, INT32_MAX}; };
static void crit_update(CritPaths& p, const std::string& tv, int64_t num) {  // :108-136
  int i = -1;
  if (tv == p.v[0]) i = 0;
  else if (tv == p.v[1]) i = 1;
  if (i >= 0) {
    p.n[i] = num;
    if (p.n[0] > p.n[1]) { std::swap(p.v[0], p.v[1]); std::swap(p.n[0], p.n[1]); }
  } else if (num < p.n[0]) {
    p.v[1] = p.v[0]; p.n[1] = p.n[0];
    p.v[0] = tv; p.n[0] = num;
  } else if (num < p.n[1]) {
    p.v[1] = tv; p.n[1] = num;
  }
}
static void pair_update(PairCounts& m, const Node& n, const std::string& tk, int64_t v) {  // filtering.go:111-120
  auto it = n.labels.find(tk);
  if (it == n.labels.end()) return;
  auto& x = m[{tk, it->second}];
  x += v;
  if (x == 0) m.erase({tk, it->second});
}
// the PreFilter extensions' AddPod / RemovePod (PodTopologySpread filtering.go:157-212,
// InterPodAffinity filtering.go:75-85,329-346) on a cloned state
static void preempt_update(Cycle& cy, std::vector<CritPaths>& crit, const PodInfo* pi, const Node& node, int64_t d) {
  const Pod& pod = *cy.pod;
  if (!cy.skipFilter[KSG_PLUGIN_POD_TOPOLOGY_SPREAD] && pi->pod.ns == pod.ns &&
      node_labels_match_spread(node.labels, cy.ptsF)) {
    for (size_t i = 0; i < cy.ptsF.size(); ++i) {
      auto& con = cy.ptsF[i];
      if (!selector_matches(con.sel, pi->pod.labels)) continue;
      if (!match_inclusion(cy, con, node)) continue;
      const std::string& v = node.labels.at(con.key);
      int64_t& x = cy.tpMatch[i][v];
      x += d;
      crit_update(crit[i], v, x);
      cy.critMin[i] = crit[i].n[0];
    }
  }
  if (!cy.skipFilter[KSG_PLUGIN_INTER_POD_AFFINITY]) {
    for (auto& t : pi->reqAnti)
      if (t.matches(pod, cy.nsLabels)) pair_update(cy.existingAnti, node, t.topologyKey, d);
    if (pod_matches_all_terms(cy.ipaReqAff, pi->pod))
      for (auto& t : cy.ipaReqAff) pair_update(cy.affCounts, node, t.topologyKey, d);
    for (auto& t : cy.ipaReqAnti)
      if (t.matches(pi->pod, nullptr)) pair_update(cy.antiCounts, node, t.topologyKey, d);
  }
}

struct OPdb { std::string ns; Selector sel; bool ok = false; int32_t allowed = 0; std::set<std::string> disrupted; };
struct OVictims { std::vector<PodInfo*> pods; int64_t viol = 0; };

// SelectVictimsOnNode (default_preemption.go:252-354); returns the status code (0: victims found)
static int select_victims(ksgo_ctx* c, const Cycle& cy0, const std::vector<CritPaths>& crit0, const Pod& pod,
                          NodeInfoO* orig, const std::vector<OPdb>& pdbs, int64_t now, OVictims* out) {
  NodeInfoO ni = *orig;  // nodeInfo.Snapshot()
  Cycle cy = cy0;        // state.Clone()
  std::vector<CritPaths> crit = crit0;
  auto start = [&](const PodInfo* p) { return p->pod.hasStartTime ? p->pod.startTimeNs : now; };
  auto more_important = [&](const PodInfo* a, const PodInfo* b) {  // util.MoreImportantPod
    if (a->pod.priority != b->pod.priority) return a->pod.priority > b->pod.priority;
    return start(a) < start(b);
  };
  std::vector<PodInfo*> pot;
  for (auto* pi : ni.pods)
    if (pi->pod.priority < pod.priority) pot.push_back(pi);  // isPreemptionAllowed
  for (auto* pi : pot) {
    node_remove_pod(ni, pi->pod.uid);
    preempt_update(cy, crit, pi, ni.node, -1);
  }
  if (pot.empty()) return KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;  // "No preemption victims found"
  Status st = preempt_filter_node(cy, &ni);
  if (!st.ok()) return st.code;
  // sort.Slice: an insertion sort (stable) up to 12 elements; equal keys keep NodeInfo.Pods order
  std::stable_sort(pot.begin(), pot.end(), more_important);
  // filterPodsWithPDBViolation (:406-452)
  std::vector<int32_t> allowed;
  for (auto& b : pdbs) allowed.push_back(b.allowed);
  std::vector<PodInfo*> violating, nonViolating;
  for (auto* pi : pot) {
    bool v = false;
    if (!pi->pod.labels.empty())
      for (size_t i = 0; i < pdbs.size(); ++i) {
        const OPdb& b = pdbs[i];
        if (b.ns != pi->pod.ns || !b.ok || !selector_matches(b.sel, pi->pod.labels)) continue;
        if (b.disrupted.count(pi->pod.name)) continue;
        if (--allowed[i] < 0) v = true;
      }
    (v ? violating : nonViolating).push_back(pi);
  }
  std::vector<PodInfo*> victims;
  int64_t numViol = 0;
  auto reprieve = [&](PodInfo* pi) {  // :316-330
    node_add_pod(ni, pi);
    preempt_update(cy, crit, pi, ni.node, +1);
    bool fits = preempt_filter_node(cy, &ni).ok();
    if (!fits) {
      node_remove_pod(ni, pi->pod.uid);
      preempt_update(cy, crit, pi, ni.node, -1);
      victims.push_back(pi);
    }
    return fits;
  };
  for (auto* pi : violating)
    if (!reprieve(pi)) ++numViol;
  for (auto* pi : nonViolating) reprieve(pi);
  if (!violating.empty() && !nonViolating.empty()) std::stable_sort(victims.begin(), victims.end(), more_important);
  if (victims.empty()) return KSG_CODE_ERROR;  // "expected at least one victim pod on node"
  out->pods = victims;
  out->viol = numViol;
  return KSG_CODE_SUCCESS;
}

static void ojson_str(std::string& o, const std::string& s) {
  o += '"';
  for (char ch : s) {
    if (ch == '"' || ch == '\\') { o += '\\'; o += ch; }
    else o += ch;
  }
  o += '"';
}

int ksgo_preempt(ksgo_ctx* c, int32_t handle, const char* args_json, size_t args_len, ksg_preempt_result* res,
                 char* detail, size_t detail_cap, size_t* detail_len) {
  auto it = c->queue.find(handle);
  if (it == c->queue.end()) return KSG_ENOTFOUND;
  const Pod& pod = *it->second;
  if (const int rn = check_nominations(c, pod)) return rn;  // (SelectVictimsOnNode filters with them too)
  *res = ksg_preempt_result{};
  res->status = KSG_CODE_UNSCHEDULABLE;
  res->node_index = -1;
  int64_t offsetIn = 0, now = 0;
  int64_t pct = 10, absn = 100;
  bool allNodes = false, list = false;
  std::vector<OPdb> pdbs;
  try {
    mj::Value a = (args_json && args_len) ? mj::parse(args_json, args_len) : mj::Value{};
    offsetIn = a.i64("offset", 0);
    // GetPodStartTime's time.Now() for pods without status.startTime (preemption/util.go): the call's
    // "now", or the wall clock read once per call (the product's default too)
    now = a.has("now") ? a.i64("now", 0)
                       : (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                             std::chrono::system_clock::now().time_since_epoch()).count();
    pct = a.i64("minCandidateNodesPercentage", 10);
    absn = a.i64("minCandidateNodesAbsolute", 100);
    if (const mj::Value* b = a.has("allNodes")) allNodes = b->kind == mj::Value::Bool && b->b;
    if (const mj::Value* b = a.has("listCandidates")) list = b->kind == mj::Value::Bool && b->b;
    if (const mj::Value* ps = a.has("pdbs"))
      for (auto& v : ps->arr) {
        OPdb b;
        if (const mj::Value* md = v.has("metadata")) b.ns = md->str("namespace", "default");
        if (b.ns.empty()) b.ns = "default";
        LabelSelectorSpec ls;
        if (const mj::Value* sp = v.has("spec")) ls = decode_label_selector(sp->has("selector"));
        // LabelSelectorAsSelector: an error, nil (Nothing) or empty (Empty()) selector matches nothing
        b.ok = label_selector_as_selector(ls, &b.sel) && ls.present && !(ls.matchLabels.empty() && ls.matchExpressions.empty());
        if (const mj::Value* st = v.has("status")) {
          b.allowed = (int32_t)st->i64("disruptionsAllowed", 0);
          if (const mj::Value* dp = st->has("disruptedPods"))
            for (auto& kv : dp->obj) b.disrupted.insert(kv.first);
        }
        pdbs.push_back(std::move(b));
      }
  } catch (std::exception& e) { c->err = e.what(); return KSG_EINVAL; }
  if (pct < 0 || pct > 100 || absn < 0 || (pct == 0 && absn == 0)) { c->err = "bad DefaultPreemptionArgs"; return KSG_EINVAL; }
  std::string msg, dj;
  auto finish = [&]() {
    if (detail_len) *detail_len = dj.size();
    if (detail) {
      if (dj.size() + 1 > detail_cap) return KSG_ENOMEM;
      std::memcpy(detail, dj.c_str(), dj.size() + 1);
    }
    return KSG_OK;
  };
  // 1) PodEligibleToPreemptOthers (default_preemption.go:364-388)
  if (pod.preemptionPolicy == "Never") {
    res->reason = KSG_PREEMPT_NOT_ELIGIBLE;
    dj = "{\"message\":\"not eligible due to preemptionPolicy=Never.\",\"candidates\":[]}";
    return finish();
  }
  // the failed cycle's Diagnosis.NodeToStatus
  c->rebuild_list();
  const int N = (int)c->list.size();
  std::vector<uint8_t> code(std::max(N, 1));
  ksg_eval_out ev{};
  ev.node_code = code.data();
  ksg_result cr;
  int rc = run_cycle(c, pod, &cr, &ev, false);  // the failed cycle's statuses again: not a new cycle
  if (rc) return rc;
  if (!pod.nominatedNodeName.empty()) {
    NodeInfoO* nn = nullptr;
    for (auto* ni : c->list)
      if (ni->node.name == pod.nominatedNodeName) nn = ni;
    if (nn && code[nn->pos] != KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE)
      for (auto* pi : nn->pods)
        if (pi->pod.priority < pod.priority && pi->pod.terminatingByPreemption) {
          res->reason = KSG_PREEMPT_NOT_ELIGIBLE;
          dj = "{\"message\":\"not eligible due to a terminating pod on the nominated node.\",\"candidates\":[]}";
          return finish();
        }
  }
  // 2) findCandidates (preemption.go:174-196): NodesForStatusCode(Unschedulable), snapshot order
  std::vector<NodeInfoO*> pot;
  for (auto* ni : c->list)
    if (allNodes || code[ni->pos] == KSG_CODE_UNSCHEDULABLE) pot.push_back(ni);
  const int64_t P = (int64_t)pot.size();
  res->num_potential = (int32_t)P;
  Cycle cy;
  cy.c = c;
  cy.pod = &pod;
  cy.reqNA = get_required_node_affinity(pod);
  std::vector<CritPaths> crit;
  std::vector<std::pair<NodeInfoO*, OVictims>> nv, vl;
  int64_t offset = 0, ncand = 0;
  if (P > 0 && preempt_prefilter(c, cy)) {
    for (auto& m : cy.tpMatch) {  // initial criticalPaths over the domains (in key order)
      CritPaths p;
      const std::map<std::string, int64_t> sorted(m.begin(), m.end());
      for (auto& kv : sorted) crit_update(p, kv.first, kv.second);
      crit.push_back(p);
    }
    offset = ((offsetIn % P) + P) % P;
    ncand = P * pct / 100;  // calculateNumCandidates (default_preemption.go:219-228)
    if (ncand < absn) ncand = absn;
    if (ncand > P) ncand = P;
    // DryRunPreemption (preemption.go:404-457), Parallelizer with parallelism 1
    for (int64_t i = 0; i < P; ++i) {
      NodeInfoO* ni = pot[(offset + i) % P];
      OVictims v;
      if (select_victims(c, cy, crit, pod, ni, pdbs, now, &v) != KSG_CODE_SUCCESS) continue;
      auto& l = v.viol == 0 ? nv : vl;
      if ((int64_t)l.size() < ncand) l.push_back({ni, v});  // candidateList.add drops past capacity
      if (!nv.empty() && (int64_t)(nv.size() + vl.size()) >= ncand) break;
    }
  }
  std::vector<std::pair<NodeInfoO*, OVictims>> cands = nv;
  cands.insert(cands.end(), vl.begin(), vl.end());
  res->num_candidates = (int32_t)cands.size();
  // 4) SelectCandidate -> pickOneNodeForPreemption (preemption.go:262-397)
  int best = -1;
  if (cands.size() == 1) best = 0;
  else if (!cands.empty()) {
    auto startOf = [&](const PodInfo* p) { return p->pod.hasStartTime ? p->pod.startTimeNs : now; };
    std::vector<std::function<int64_t(int)>> fs = {
        [&](int k) { return -cands[k].second.viol; },
        [&](int k) { return -(int64_t)cands[k].second.pods[0]->pod.priority; },
        [&](int k) {
          int64_t s = 0;
          for (auto* p : cands[k].second.pods) s += (int64_t)p->pod.priority + (int64_t)INT32_MAX + 1;
          return -s;
        },
        [&](int k) { return -(int64_t)cands[k].second.pods.size(); },
        [&](int k) {  // util.GetEarliestPodStartTime
          auto& ps = cands[k].second.pods;
          int64_t t = startOf(ps[0]);
          int32_t mp = ps[0]->pod.priority;
          for (auto* p : ps) {
            if (p->pod.priority == mp) { if (startOf(p) < t) t = startOf(p); }
            else if (p->pod.priority > mp) { mp = p->pod.priority; t = startOf(p); }
          }
          return t;
        }};
    std::vector<int> all;
    for (size_t k = 0; k < cands.size(); ++k) all.push_back((int)k);
    for (auto& f : fs) {
      std::vector<int> sel;
      int64_t mx = INT64_MIN;
      for (int k : all) {
        int64_t s = f(k);
        if (s > mx) { mx = s; sel.clear(); }
        if (s == mx) sel.push_back(k);
      }
      all = sel;
      if (all.size() == 1) break;
    }
    best = all[0];
  }
  if (best >= 0) {
    res->status = KSG_CODE_SUCCESS;
    res->reason = KSG_PREEMPT_OK;
    res->node_index = cands[best].first->pos;
    res->num_victims = (int32_t)cands[best].second.pods.size();
    res->num_pdb_violations = cands[best].second.viol;
  } else {
    res->reason = KSG_PREEMPT_NO_CANDIDATES;
    msg = "0/" + std::to_string(N) + " nodes are available: preemption is not helpful for scheduling.";
  }
  dj = "{\"offset\":" + std::to_string(offset) + ",\"numCandidates\":" + std::to_string(ncand) +
       ",\"potential\":" + std::to_string(P) + ",\"message\":";
  ojson_str(dj, msg);
  dj += ",\"candidates\":[";
  auto vlist = [&](const OVictims& v) {
    std::string o = "[";
    for (size_t q = 0; q < v.pods.size(); ++q) {
      if (q) o += ",";
      ojson_str(o, v.pods[q]->pod.uid);
    }
    return o + "]";
  };
  for (size_t k = 0; list && k < cands.size(); ++k) {
    if (k) dj += ",";
    dj += "{\"node\":";
    ojson_str(dj, cands[k].first->node.name);
    dj += ",\"numPDBViolations\":" + std::to_string(cands[k].second.viol) + ",\"victims\":" + vlist(cands[k].second) + "}";
  }
  dj += "],\"selected\":";
  if (best >= 0) ojson_str(dj, cands[best].first->node.name);
  else dj += "null";
  dj += ",\"victims\":" + (best >= 0 ? vlist(cands[best].second) : std::string("[]")) + "}";
  return finish();
}

double ksgo_go_log(double x) { return go_log(x); }

// CalculateResource (framework/types.go:1035-1076) and Fit's computePodResourceRequest (fit.go:317-325)
// of one pod: out[0..4] MilliCPU, Memory, EphemeralStorage, Non0CPU, Non0Mem; out[5..7] the Fit request
int ksgo_debug_pod_resources(const char* json, size_t len, int64_t* out, int32_t cap) {
  if (!json || !out || cap < 8) return KSG_EINVAL;
  std::string err;
  Pod p;
  try {
    if (!decode_pod(mj::parse(json, len), &p, &err)) return KSG_EINVAL;
  } catch (const std::exception&) {
    return KSG_EINVAL;
  }
  const PodResource r = calculate_resource(p);
  int64_t fit[3] = {0, 0, 0};
  for (auto& kv : pod_requests(p, nullptr, false)) {
    if (kv.first == "cpu") fit[0] = kv.second;
    else if (kv.first == "memory") fit[1] = milli_to_value(kv.second);
    else if (kv.first == "ephemeral-storage") fit[2] = milli_to_value(kv.second);
  }
  const int64_t o[8] = {r.res.milliCPU, r.res.memory, r.res.ephemeral, r.non0CPU, r.non0Mem, fit[0], fit[1], fit[2]};
  for (int k = 0; k < 8; ++k) out[k] = o[k];
  return 8;
}

// SignPod of one pod under one profile (sign_pod above), as ksg_debug_pod_signature: 1 signed (text in out),
// 0 nil, KSG_EINVAL on bad input.
int ksgo_debug_pod_signature(const char* cfg, size_t cfg_len, const char* json, size_t len, char* out, size_t cap,
                             size_t* out_len) {
  if (!json || !out || !out_len) return KSG_EINVAL;
  std::unique_ptr<ksgo_ctx, void (*)(ksgo_ctx*)> c(ksgo_create(cfg, cfg_len), ksgo_destroy);
  if (!c) return KSG_EINVAL;
  std::string err, sig;
  Pod p;
  try {
    if (!decode_pod(mj::parse(json, len), &p, &err)) return KSG_EINVAL;
  } catch (const std::exception&) {
    return KSG_EINVAL;
  }
  if (!sign_pod(c.get(), p, &sig)) {
    *out_len = 0;
    if (cap) out[0] = 0;
    return 0;
  }
  if (sig.size() + 1 > cap) return KSG_EINVAL;
  std::memcpy(out, sig.c_str(), sig.size() + 1);
  *out_len = sig.size();
  return 1;
}

int32_t ksgo_heap_root(const int64_t* scores, int32_t n) {
  if (n <= 0) return -1;
  std::vector<HeapEnt> h(n);
  for (int32_t i = 0; i < n; ++i) h[i] = {scores[i], 0, i};
  return heap_pop_index(h);
}

}  // extern "C"
