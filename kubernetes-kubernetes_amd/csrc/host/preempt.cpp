// preempt.cpp -- DefaultPreemption's PostFilter.
//
// Evaluator.Preempt (framework/preemption/preemption.go:103-170) for one pod that failed its cycle:
//   PodEligibleToPreemptOthers (default_preemption.go:364-388) on the host;
//   the cycle's Filter statuses (the FitError diagnosis) from k_filter_score on the device;
//   SelectVictimsOnNode (default_preemption.go:252-354) for every node findCandidates would pass to
//   DryRunPreemption (preemption.go:174-196, 404-457) -- k_preempt, one thread per node;
//   the candidate cut of DryRunPreemption with sequential Parallelizer semantics (parallelism 1, the
//   reference's own deterministic test mode) and SelectCandidate / pickOneNodeForPreemption
//   (preemption.go:262-397) in k_preempt_pick on the device; with listCandidates the host re-derives
//   both over the per-node results and fails the call if they disagree.
// Actuation (deleting victims, patching nominatedNodeName, executor.go) is the caller's: the result
// names the node and the victims.
//
// Determinism contract (each documented in ksg.h): the random offset is the caller's; pods without
// status.startTime get the caller's clock (GetPodStartTime's time.Now(), utils.go:52-58); victims of
// equal priority and start time keep NodeInfo.Pods order (sort.Slice is an insertion sort, hence
// stable, up to 12 elements); candidates tie-break in candidate-list order (the reference iterates a
// Go map there, preemption.go:316-319).
#include <algorithm>
#include <chrono>
#include <cstring>

#include "host.hpp"

namespace ksg {

hipError_t launch_aggregate(const MirrorView& m, const BatchView& b, int pod, const PodDesc& d, hipStream_t s);
hipError_t launch_filter_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, hipEvent_t t0,
                               hipEvent_t t1, int blk0, int nblk, bool lds);
hipError_t launch_preempt(const MirrorView& m, const BatchView& b, int pod, const PNode* pn, const PVictim* pv,
                          uint8_t* vout, POut* out, int all_nodes, const PreemptIn& in, hipStream_t s);
hipError_t launch_preempt_seg(const MirrorView& m, const BatchView& b, int pod, const PreemptView& pv, hipStream_t s);
hipError_t launch_pts_minima(const BatchView& b, int pod, int ncons, long long* mm, hipStream_t s);
hipError_t launch_aff_totals(const BatchView& b, int pod, int nterms, long long* out, hipStream_t s);
hipError_t launch_preempt_terms(const MirrorView& m, const BatchView& b, int pod, int32_t* contrib, hipStream_t s);
hipError_t launch_preempt_pick(const PSegOut* out, int n, int64_t offset, int64_t pct, int64_t absn, int32_t* pot,
                               PickOut* res, hipStream_t s);

#define PCHK(x)                                                         \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      c->err = std::string("HIP: ") + hipGetErrorString(e_) + " @" #x;  \
      return KSG_EDEVICE;                                               \
    }                                                                   \
  } while (0)

namespace {

enum : int { P_PORTS = KSG_PLUGIN_NODE_PORTS, P_PTS = KSG_PLUGIN_POD_TOPOLOGY_SPREAD, P_IPA = KSG_PLUGIN_INTER_POD_AFFINITY };

struct Pdb {  // policy/v1 PodDisruptionBudget, the fields filterPodsWithPDBViolation reads
  std::string ns;
  bool sel_ok = false;  // a non-nil, non-empty selector that LabelSelectorAsSelector accepts
  LabelSel sel;
  int32_t allowed = 0;
  std::set<std::string> disrupted;  // status.disruptedPods names
};

bool valid_lsel(const LabelSel& s) {  // metav1.LabelSelectorAsSelector errors (helpers.go:36-71)
  for (auto& kv : s.match)
    if (!valid_label_key(kv.first) || !valid_label_value(kv.second)) return false;
  for (auto& e : s.exprs) {
    if (!valid_label_key(e.key)) return false;
    if (e.op == "In" || e.op == "NotIn") {
      if (e.values.empty()) return false;
      for (auto& v : e.values)
        if (!valid_label_value(v)) return false;
    } else if (e.op == "Exists" || e.op == "DoesNotExist") {
      if (!e.values.empty()) return false;
    } else {
      return false;
    }
  }
  return true;
}

// labels.Selector.Matches over a pod-table slot's interned label set
bool lsel_match_slot(const Cluster& c, const LabelSel& s, int32_t slot) {
  const unsigned long long* lb = c.pt_pool.data() + c.pt_lbl_off[slot];
  const uint32_t n = c.pt_lbl_cnt[slot];
  auto value_of = [&](const std::string& key, int32_t* vid) {  // false: the pod has no such key
    const int32_t k = c.label_keys.find(key);
    if (k < 0) return false;
    for (uint32_t q = 0; q < n; ++q)
      if ((int32_t)(lb[q] >> 32) == k) {
        *vid = (int32_t)(uint32_t)lb[q];
        return true;
      }
    return false;
  };
  auto is = [&](const std::string& key, int32_t vid, const std::string& v) {
    return c.keys[c.label_keys.find(key)].values.find(v) == vid;
  };
  for (auto& kv : s.match) {
    int32_t v;
    if (!value_of(kv.first, &v) || !is(kv.first, v, kv.second)) return false;
  }
  for (auto& e : s.exprs) {
    int32_t v;
    const bool has = value_of(e.key, &v);
    bool in = false;
    if (has)
      for (auto& x : e.values) in |= is(e.key, v, x);
    if (e.op == "In" && !(has && in)) return false;
    if (e.op == "NotIn" && has && in) return false;
    if (e.op == "Exists" && !has) return false;
    if (e.op == "DoesNotExist" && has) return false;
  }
  return true;
}

LabelSel decode_lsel(const JDoc& d, const JVal* v) {
  LabelSel s;
  if (!v) return s;
  s.present = true;
  d.each(d.get(*v, "matchLabels"), [&](const JVal& kv) { s.match.push_back({kv.key, kv.s}); });
  std::sort(s.match.begin(), s.match.end());
  d.each(d.get(*v, "matchExpressions"), [&](const JVal& e) {
    Expr x;
    x.key = d.str(e, "key");
    x.op = d.str(e, "operator");
    d.each(d.get(e, "values"), [&](const JVal& y) { x.values.push_back(y.s); });
    s.exprs.push_back(std::move(x));
  });
  return s;
}

struct Victim {
  const std::string* uid;
  const BoundPod* bp;
  int64_t start;
  bool viol = false;
};

// util.MoreImportantPod (scheduler/util/utils.go:89-96) with GetPodStartTime's clock supplied
bool more_important(const Victim& a, const Victim& b) {
  if (a.bp->priority != b.bp->priority) return a.bp->priority > b.bp->priority;
  return a.start < b.start;
}

void json_str(std::string& o, const std::string& s) {
  o.push_back('"');
  for (char ch : s) {
    if (ch == '"' || ch == '\\') {
      o.push_back('\\');
      o.push_back(ch);
    } else if ((unsigned char)ch < 0x20) {
      char b[8];
      std::snprintf(b, sizeof b, "\\u%04x", (unsigned)(unsigned char)ch);
      o += b;
    } else {
      o.push_back(ch);
    }
  }
  o.push_back('"');
}

}  // namespace

// One node's importance-ordered segment (k_preempt_seg).  The order is util.MoreImportantPod's with the
// pods that have no status.startTime last among their priority: GetPodStartTime gives them the call's
// clock, later than every start time the cache holds when now > Cluster::max_start_ns (the condition
// Engine::preempt checks before using the segments).  Equal keys keep NodeInfo.Pods order.
void Engine::seg_build(int32_t i, NodeRec& r) {
  auto& v = seg_pods[i];
  v.clear();
  for (const std::string& uid : r.pods) v.push_back(&c->pods.at(uid));
  std::stable_sort(v.begin(), v.end(), [](const BoundPod* a, const BoundPod* b) {
    if (a->priority != b->priority) return a->priority > b->priority;
    const int64_t ta = a->has_start ? a->start_ns : INT64_MAX, tb = b->has_start ? b->start_ns : INT64_MAX;
    return ta < tb;
  });
  const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)kSegCap);
  uint8_t fl = v.size() > (size_t)kSegCap ? 1u : 0u;
  PRec* out = h_seg.data() + (size_t)i * kSegCap;
  for (int32_t q = 0; q < n; ++q) {
    const BoundPod& bp = *v[q];
    PRec x{};
    x.cpu = bp.res.cpu;
    x.mem = bp.res.mem;
    x.eph = bp.res.eph;
    x.start = bp.has_start ? bp.start_ns : INT64_MAX;
    x.prio = bp.priority;
    x.slot = bp.slot;
    x.port[0] = x.port[1] = 0xffffffffu;
    for (size_t k = 0; k < bp.port_ids.size() && k < 2; ++k) x.port[k] = bp.port_ids[k];
    if (bp.port_ids.size() > 2) {
      x.flags |= PR_MANY_PORTS;
      fl |= 2u;
    }
    if (!bp.res.scalar.empty()) x.flags |= PR_SCALAR;
    out[q] = x;
  }
  h_segcnt[i] = n;
  seg_overflow += (fl & 1u) - (seg_flags[i] & 1u);
  seg_many_ports += ((fl >> 1) & 1u) - ((seg_flags[i] >> 1) & 1u);
  seg_flags[i] = fl;
  r.pre_dirty = false;
}

// Brings the device segments up to the cache: every node after a re-layout (node order changed),
// otherwise only the nodes whose pods changed since the last call (Cluster::pre_dirty_nodes).
int Engine::seg_refresh() {
  const std::vector<std::string>& order = c->order();
  const int32_t N = (int32_t)order.size();
  hipStream_t s = c->stream;
  int rc;
  if (seg_epoch != c->layout_epoch() || seg_n != N) {
    h_seg.assign((size_t)N * kSegCap, PRec{});
    h_segcnt.assign((size_t)N, 0);
    seg_pods.assign((size_t)N, {});
    seg_flags.assign((size_t)N, 0);
    seg_overflow = seg_many_ports = 0;
    for (int32_t i = 0; i < N; ++i) seg_build(i, *c->node(order[i]));
    if ((rc = ensure(d_seg, sizeof(PRec) * (size_t)std::max(N, 1) * kSegCap))) return rc;
    if ((rc = ensure(d_segcnt, 4 * (size_t)std::max(N, 1)))) return rc;
    PCHK(hipMemcpyAsync(d_seg.p, h_seg.data(), sizeof(PRec) * h_seg.size(), hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_segcnt.p, h_segcnt.data(), 4 * h_segcnt.size(), hipMemcpyHostToDevice, s));
    PCHK(hipStreamSynchronize(s));  // pageable sources
    seg_epoch = c->layout_epoch();
    seg_n = N;
    c->pre_dirty_nodes.clear();
    return KSG_OK;
  }
  bool any = false;
  for (const std::string& name : c->pre_dirty_nodes) {
    NodeRec* r = c->node(name);
    if (!r || !r->real || !r->pre_dirty) continue;
    const int32_t i = c->index_of(name);
    if (i < 0) continue;
    seg_build(i, *r);
    PRec* dseg = (PRec*)d_seg.p + (size_t)i * kSegCap;
    if (h_segcnt[i])
      PCHK(hipMemcpyAsync(dseg, h_seg.data() + (size_t)i * kSegCap, sizeof(PRec) * (size_t)h_segcnt[i],
                          hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync((int32_t*)d_segcnt.p + i, &h_segcnt[i], 4, hipMemcpyHostToDevice, s));
    any = true;
  }
  c->pre_dirty_nodes.clear();
  if (any) PCHK(hipStreamSynchronize(s));  // pageable sources
  return KSG_OK;
}

int Engine::preempt(const PodSpec& p, const char* args_json, size_t args_len, ksg_preempt_result* res,
                    std::string* detail) {
  *res = ksg_preempt_result{};
  res->status = KSG_CODE_UNSCHEDULABLE;
  res->node_index = -1;
  // ---- DefaultPreemptionArgs + the call's inputs (validation_pluginargs.go:113-125)
  int64_t offset_in = 0, now = 0;
  int32_t pct = 10, absn = 100;
  bool all_nodes = false, staged = false, list = false, force_wide = false;
  std::vector<Pdb> pdbs;
  try {
    JDoc d(args_json && args_len ? args_json : "{}", args_json && args_len ? args_len : 2);
    const JVal& r = d.root();
    offset_in = d.num(r, "offset", 0);
    // GetPodStartTime's clock for pods without status.startTime (utils.go:52-58: time.Now()); absent,
    // the wall clock, as upstream -- so the device-resident segments serve the call (seg below)
    now = d.get(r, "now") ? d.num(r, "now", 0)
                          : (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::system_clock::now().time_since_epoch()).count();
    pct = (int32_t)d.num(r, "minCandidateNodesPercentage", 10);
    absn = (int32_t)d.num(r, "minCandidateNodesAbsolute", 100);
    all_nodes = d.boolean(r, "allNodes");
    staged = d.boolean(r, "debugHostStaged");  // diagnostic: force the host-staged victim records
    force_wide = d.boolean(r, "debugWideDryRun");  // diagnostic: the workspace-resident dry run at any size
    list = d.boolean(r, "listCandidates");      // detail lists every DryRunPreemption candidate
    d.each(d.get(r, "pdbs"), [&](const JVal& v) {
      Pdb b;
      if (const JVal* md = d.get(v, "metadata")) b.ns = d.str(*md, "namespace", "default");
      if (b.ns.empty()) b.ns = "default";
      if (const JVal* sp = d.get(v, "spec")) b.sel = decode_lsel(d, d.get(*sp, "selector"));
      // LabelSelectorAsSelector: nil -> Nothing, empty -> Everything (Empty()); both match nothing here
      b.sel_ok = b.sel.present && !(b.sel.match.empty() && b.sel.exprs.empty()) && valid_lsel(b.sel);
      if (const JVal* st = d.get(v, "status")) {
        b.allowed = (int32_t)d.num(*st, "disruptionsAllowed", 0);
        d.each(d.get(*st, "disruptedPods"), [&](const JVal& kv) { b.disrupted.insert(kv.key); });
      }
      pdbs.push_back(std::move(b));
    });
  } catch (std::exception& e) {
    c->err = std::string("preemption args: ") + e.what();
    return KSG_EINVAL;
  }
  if (pct < 0 || pct > 100 || absn < 0 || (pct == 0 && absn == 0)) {
    c->err = "preemption args: minCandidateNodesPercentage must be in [0, 100], minCandidateNodesAbsolute >= 0, "
             "not both 0";
    return KSG_EINVAL;
  }
  // ---- 1) PodEligibleToPreemptOthers, the PreemptionPolicy half (default_preemption.go:365-367)
  if (p.preempt_never) {
    res->reason = KSG_PREEMPT_NOT_ELIGIBLE;
    if (detail) *detail = "{\"message\":\"not eligible due to preemptionPolicy=Never.\",\"candidates\":[]}";
    return KSG_OK;
  }
  const std::vector<std::string>& order = c->order();
  const int32_t N = (int32_t)order.size();
  CompiledPod cp;
  int rc = compile(p, CYCLE, -1, false, true, &cp);
  if (rc) return rc;
  // the failed cycle's statuses again, not a new cycle: OpportunisticBatching's state stays as it is
  reinterpret_cast<PodDesc*>(cp.blob.data())->flags &= ~DF_OB;
  const PodDesc& D = *reinterpret_cast<const PodDesc*>(cp.blob.data());

  const bool pts_on = (D.filter_mask >> P_PTS & 1u) && D.n_ptsf > 0;
  const bool ports_on = (D.filter_mask >> P_PORTS) & 1u;
  int32_t nom_ix = p.nominated_node.empty() ? -1 : c->index_of(p.nominated_node);
  if (N > 0 && (rc = c->ensure_mirror())) return rc;
  // The device-resident segments serve every pod whose victims' order the cache already knows (no pod
  // sorted by the call's clock, see seg_build) and that the device groups itself: at most kMaxPdb budgets.
  // The rest take the host-staged records (the same per-node core, k_preempt).
  bool seg = N > 0 && !staged && pdbs.size() <= (size_t)kMaxPdb && (c->nostart_pods == 0 || now > c->max_start_ns);
  const bool ipa_on = (D.filter_mask >> P_IPA) & 1u;
  if (seg && (rc = seg_refresh())) return rc;
  seg = seg && seg_overflow == 0 && (!ports_on || seg_many_ports == 0);

  struct NodeOut { uint32_t st; int32_t nvictims, nviolating; uint32_t flags; };
  std::vector<NodeOut> po((size_t)std::max(N, 1));
  uint32_t nom_status = 0;
  // staged path: the potential victims of every node, in reprieve order
  std::vector<PNode> pn;
  std::vector<PVictim> pv;
  std::vector<Victim> all;  // parallel to pv
  std::vector<uint8_t> vo;
  // segment path: per-node victim masks (listCandidates), the device's cut and pick
  std::vector<PSegOut> so;
  PickOut pick{};

  uint8_t* hp = (uint8_t*)h_pinned;
  hipStream_t s = c->stream;
  const MirrorView& m = c->view;
  BatchView bv{};
  auto stage_pod = [&]() -> int {  // the preemptor's program + stats, then the cycle's statuses
    if ((rc = ensure_scratch(cp.blob.size(), 1, true, cp.arena_words))) return rc;
    hp = (uint8_t*)h_pinned;
    std::memcpy(hp, cp.blob.data(), cp.blob.size());
    uint32_t off0 = 0;
    PodStats* hs = (PodStats*)(hp + ((cp.blob.size() + 15) & ~size_t(15)));
    std::memset(hs, 0, sizeof(PodStats));
    for (int q = 0; q < kNumPlugins; ++q) {
      hs->max_raw[q] = enc_i64(INT64_MIN);
      hs->min_raw[q] = enc_i64(INT64_MAX);
    }
    PCHK(hipMemcpyAsync(d_descs.p, hp, cp.blob.size(), hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_off.p, &off0, 4, hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_stats.p, hs, sizeof(PodStats), hipMemcpyHostToDevice, s));
    bv = bview(1);
    if (D.flags & DF_AGGREGATE) PCHK(launch_aggregate(m, bv, 0, D, s));
    PCHK(launch_filter_score(m, bv, 0, s, nullptr, nullptr, 0, -1, cp.blob.size() <= (size_t)kBlobLds));
    return KSG_OK;
  };
  // what both kernels read about the victims beyond Requested (PreemptIn): the cycle's DoNotSchedule minima,
  // the self-matching affinity totals, the existing anti-affinity terms per victim slot, and the victims'
  // requests of the preemptor's extended resources; d_pdb's head holds the minima and totals
  PreemptIn pin{};
  const size_t mm_words = 3 * (size_t)D.n_ptsf + (size_t)D.n_raff;
  auto topo_prelude = [&]() -> int {
    // d_pdb's head: k_pts_minima's [3 n_ptsf], then k_aff_totals' [n_raff] (mm_words)
    if ((rc = ensure(d_pdb, 8 * mm_words + 64))) return rc;
    long long* d_mm = (long long*)d_pdb.p;
    if (pts_on) PCHK(launch_pts_minima(bv, 0, D.n_ptsf, d_mm, s));
    // a preemptor matching its own required affinity terms: the cycle's per-term totals (PreemptTopo::any)
    const bool aff_tot = ipa_on && (D.ipa_flags & IPA_SELF_ALL) && D.n_raff > 0;
    if (aff_tot) PCHK(launch_aff_totals(bv, 0, D.n_raff, d_mm + 3 * D.n_ptsf, s));
    // existing pods' required anti-affinity terms matching the preemptor, per slot and key
    const bool terms = ipa_on && D.n_exkeys > 0 && m.n_terms > 0;
    if (terms) {
      const size_t cb = sizeof(int32_t) * (size_t)D.n_exkeys * (size_t)std::max(m.pods_hw, 1);
      if ((rc = ensure(d_contrib_buf, cb + 64))) return rc;
      PCHK(hipMemsetAsync(d_contrib_buf.p, 0, cb, s));
      PCHK(launch_preempt_terms(m, bv, 0, (int32_t*)d_contrib_buf.p, s));
    }
    // more DoNotSchedule constraints, affinity terms or existing-anti keys than the registers hold: the
    // dry run keeps its per-node counts in a workspace (PreemptWide)
    const int32_t wc = pts_on ? D.n_ptsf : 0;
    const int32_t wg = ipa_on ? std::max(D.n_raff, std::max(D.n_ranti, D.n_exkeys)) : 0;
    if (force_wide || wc > kPreemptCons || wg > kPreemptCons) {
      const size_t wb = 8 * (size_t)std::max(5 * wc + 10 * wg, 1) * (size_t)std::max(std::max(N, m.n), 1);
      if ((rc = ensure(d_wide, wb + 64))) return rc;
      pin.wide = (long long*)d_wide.p;
      pin.wide_c = wc;
      pin.wide_g = wg;
    }
    pin.ex_stride = D.n_exkeys;
    pin.pts_check = pts_on ? 1 : 0;
    pin.ipa_check = ipa_on ? 1 : 0;
    pin.pts_mm = d_mm;
    pin.aff_tot = aff_tot ? d_mm + 3 * D.n_ptsf : nullptr;
    pin.ex_contrib = terms ? (const int32_t*)d_contrib_buf.p : nullptr;
    if (D.n_scalar > 0 && N > 0) {
      // each pod's request of the preemptor's extended resources, by pod-table slot (only pods that request
      // extended resources have non-zero rows), and the kernels' per-node scratch of the node's Requested
      const int ns = D.n_scalar;
      const ScalarReq* sr = reinterpret_cast<const ScalarReq*>(cp.blob.data() + D.scalar_off);
      std::vector<int64_t> vsc((size_t)std::max(m.pods_hw, 1) * ns, 0);
      for (auto& kv : c->pods) {
        const BoundPod& bp = kv.second;
        if (bp.res.scalar.empty() || bp.slot < 0 || bp.slot >= m.pods_hw) continue;
        for (int k = 0; k < ns; ++k)
          for (auto& sv : bp.res.scalar)
            if (sv.first == c->scalar_ix.strs[sr[k].slot]) vsc[(size_t)bp.slot * ns + k] += sv.second;
      }
      const size_t vb = vsc.size() * 8, sb = (size_t)N * ns * 8;
      if ((rc = ensure(d_vsc, vb + sb + 64))) return rc;
      PCHK(hipMemcpyAsync(d_vsc.p, vsc.data(), vb, hipMemcpyHostToDevice, s));
      PCHK(hipStreamSynchronize(s));  // pageable source
      pin.vsc = (const int64_t*)d_vsc.p;
      pin.sreq = (int64_t*)((uint8_t*)d_vsc.p + ((vb + 63) & ~(size_t)63));
    }
    return KSG_OK;
  };
  auto finish_device = [&]() -> int {
    if (D.arena_words) PCHK(hipMemsetAsync(d_arena.p, 0, (size_t)D.arena_words * 8, s));  // k_select did not run
    if (nom_ix >= 0) PCHK(hipMemcpyAsync(&nom_status, bv.status + nom_ix, 4, hipMemcpyDeviceToHost, s));
    PCHK(hipStreamSynchronize(s));
    return KSG_OK;
  };

  if (seg) {
    // ---- PodDisruptionBudgets as selector programs over the pod table's labels
    std::vector<int32_t> pool;
    std::vector<PdbDev> pd(pdbs.size());
    bool any_dis = false;
    for (size_t k = 0; k < pdbs.size(); ++k) {
      int32_t off = 0;
      const bool ok = pdbs[k].sel_ok && c->compile_lsel(pdbs[k].sel, nullptr, &pool, &off);
      pd[k] = PdbDev{c->ns_id(pdbs[k].ns), off, pdbs[k].allowed, ok ? 1 : 0};
      any_dis |= !pdbs[k].disrupted.empty();
    }
    std::vector<uint8_t> dis;
    if (any_dis) {  // DisruptedPods names -> pod-table slots (rare: a budget mid-eviction)
      dis.assign(c->pt_node.size(), 0);
      for (auto& kv : c->pods)
        for (size_t k = 0; k < pdbs.size(); ++k)
          if (pdbs[k].disrupted.count(kv.second.name)) dis[kv.second.slot] |= (uint8_t)(1u << k);
    }
    if ((rc = stage_pod())) return rc;
    const size_t mm_b = (8 * mm_words + 63) & ~(size_t)63;  // the prelude's minima and totals, then the budgets
    const size_t pd_b = sizeof(PdbDev) * pd.size(), pool_b = 4 * pool.size(), dis_b = dis.size();
    if ((rc = ensure(d_pdb, mm_b + pd_b + pool_b + dis_b + 64))) return rc;
    if ((rc = topo_prelude())) return rc;
    if ((rc = ensure(d_psout, sizeof(PSegOut) * (size_t)N))) return rc;
    uint8_t* dp = (uint8_t*)d_pdb.p + mm_b;
    if (pd_b) PCHK(hipMemcpyAsync(dp, pd.data(), pd_b, hipMemcpyHostToDevice, s));
    if (pool_b) PCHK(hipMemcpyAsync(dp + pd_b, pool.data(), pool_b, hipMemcpyHostToDevice, s));
    if (dis_b) PCHK(hipMemcpyAsync(dp + pd_b + pool_b, dis.data(), dis_b, hipMemcpyHostToDevice, s));
    PreemptView v{};
    v.seg = (const PRec*)d_seg.p;
    v.cnt = (const int32_t*)d_segcnt.p;
    v.pdb = (const PdbDev*)dp;
    v.pdb_pool = (const int32_t*)(dp + pd_b);
    v.disrupted = dis_b ? dp + pd_b + pool_b : nullptr;
    v.out = (PSegOut*)d_psout.p;
    v.npdb = (int32_t)pd.size();
    v.prio = p.priority;
    v.all_nodes = all_nodes ? 1 : 0;
    v.now = now;
    v.in = pin;
    PCHK(launch_preempt_seg(m, bv, 0, v, s));
    if ((rc = ensure(d_pick, sizeof(PickOut) + 4 * (size_t)N + 64))) return rc;
    PickOut* d_po = (PickOut*)d_pick.p;
    PCHK(launch_preempt_pick((const PSegOut*)d_psout.p, N, offset_in, pct, absn, (int32_t*)(d_po + 1), d_po, s));
    PCHK(hipMemcpyAsync(&pick, d_po, sizeof(PickOut), hipMemcpyDeviceToHost, s));
    if (list) {  // the whole per-node result, for the candidate listing (and a host check of the pick)
      so.resize((size_t)N);
      PCHK(hipMemcpyAsync(so.data(), d_psout.p, sizeof(PSegOut) * (size_t)N, hipMemcpyDeviceToHost, s));
    }
    if ((rc = finish_device())) return rc;
    if (pick.unsupported) {  // the register dry run met more entries than it holds: a host sizing bug
      c->err = "preemption: internal error (dry-run store smaller than the preemptor's constraints)";
      return KSG_EDEVICE;
    }
    for (int32_t i = 0; list && i < N; ++i) po[i] = NodeOut{so[i].st, so[i].nvictims, so[i].nviolating, so[i].flags};
  } else {
    // ---- host-staged records: the potential victims of every node, in reprieve order
    pn.assign((size_t)std::max(N, 1), PNode{});
    const uint32_t* conflict = reinterpret_cast<const uint32_t*>(cp.blob.data() + D.port_conflict_off);
    auto conflicts = [&](uint32_t pid) {
      return ports_on && (int32_t)(pid >> 5) < D.n_port_words && ((conflict[pid >> 5] >> (pid & 31u)) & 1u);
    };
    std::vector<Victim> vs;
    for (int32_t i = 0; i < N; ++i) {
      NodeRec* r = c->node(order[i]);
      PNode& nd = pn[i];
      nd = PNode{(int32_t)pv.size(), 0, 0u, 0};
      vs.clear();
      for (const std::string& uid : r->pods) {  // isPreemptionAllowed (:396-399): lower priority
        const BoundPod& bp = c->pods.at(uid);
        if (bp.priority < p.priority) vs.push_back(Victim{&uid, &bp, bp.has_start ? bp.start_ns : now, false});
      }
      if (vs.empty()) continue;
      std::stable_sort(vs.begin(), vs.end(), more_important);  // sort.Slice (:309-311), see header
      // filterPodsWithPDBViolation (:406-452) over the sorted list
      std::vector<int32_t> allowed(pdbs.size());
      for (size_t k = 0; k < pdbs.size(); ++k) allowed[k] = pdbs[k].allowed;
      for (Victim& v : vs) {
        if (c->pt_lbl_cnt[v.bp->slot] == 0) continue;  // a pod with no labels matches no PDB
        const std::string& vns = c->ns_ix.strs[c->pt_ns[v.bp->slot]];
        for (size_t k = 0; k < pdbs.size(); ++k) {
          const Pdb& b = pdbs[k];
          if (b.ns != vns || !b.sel_ok || !lsel_match_slot(*c, b.sel, v.bp->slot)) continue;
          if (b.disrupted.count(v.bp->name)) continue;
          if (--allowed[k] < 0) v.viol = true;
        }
      }
      std::stable_partition(vs.begin(), vs.end(), [](const Victim& v) { return v.viol; });
      std::set<uint32_t> vports;
      for (const Victim& v : vs) {
        PVictim x{};
        x.cpu = v.bp->res.cpu;
        x.mem = v.bp->res.mem;
        x.eph = v.bp->res.eph;
        x.slot = v.bp->slot;
        for (uint32_t pid : v.bp->port_ids) {
          vports.insert(pid);
          if (conflicts(pid)) x.flags |= PV_PORT;
        }
        if (v.viol) x.flags |= PV_VIOL;
        pv.push_back(x);
        all.push_back(v);
      }
      nd.vcnt = (int32_t)vs.size();
      // NodeInfo.RemovePod drops a victim's ports from the node's set even if another pod holds them too
      for (uint32_t pid : r->ports)
        if (!vports.count(pid) && conflicts(pid)) nd.flags |= PN_BASE_PORT;
    }
    const int32_t V = (int32_t)pv.size();
    std::vector<POut> pout((size_t)std::max(N, 1));
    vo.assign((size_t)std::max(V, 1), 0);
    if (N > 0) {
      if ((rc = stage_pod())) return rc;
      if ((rc = topo_prelude())) return rc;
      const size_t pn_b = sizeof(PNode) * (size_t)N, pv_b = sizeof(PVictim) * (size_t)std::max(V, 1);
      const size_t po_b = sizeof(POut) * (size_t)N, vo_b = (size_t)std::max(V, 1);
      if ((rc = ensure(d_pre, pn_b + pv_b + po_b + vo_b + 64))) return rc;
      uint8_t* dp = (uint8_t*)d_pre.p;
      PNode* d_pn = (PNode*)dp;
      PVictim* d_pv = (PVictim*)(dp + pn_b);
      POut* d_po = (POut*)(dp + pn_b + pv_b);
      uint8_t* d_vo = dp + pn_b + pv_b + po_b;
      PCHK(hipMemcpyAsync(d_pn, pn.data(), pn_b, hipMemcpyHostToDevice, s));
      if (V) PCHK(hipMemcpyAsync(d_pv, pv.data(), pv_b, hipMemcpyHostToDevice, s));
      PCHK(launch_preempt(m, bv, 0, d_pn, d_pv, d_vo, d_po, all_nodes ? 1 : 0, pin, s));
      PCHK(hipMemcpyAsync(pout.data(), d_po, po_b, hipMemcpyDeviceToHost, s));
      if (V) PCHK(hipMemcpyAsync(vo.data(), d_vo, vo_b, hipMemcpyDeviceToHost, s));
      if ((rc = finish_device())) return rc;
    }
    for (int32_t i = 0; i < N; ++i) po[i] = NodeOut{pout[i].st, pout[i].nvictims, pout[i].nviolating, pout[i].flags};
  }
  // ---- 1) PodEligibleToPreemptOthers, the nominated-node half (:369-386)
  if (nom_ix >= 0 && status_code(nom_status) != KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE) {
    const NodeRec* r = c->node(p.nominated_node);
    for (const std::string& uid : r->pods) {
      const BoundPod& bp = c->pods.at(uid);
      if (bp.priority < p.priority && bp.preempt_terminating) {
        res->reason = KSG_PREEMPT_NOT_ELIGIBLE;
        if (detail)
          *detail = "{\"message\":\"not eligible due to a terminating pod on the nominated node.\",\"candidates\":[]}";
        return KSG_OK;
      }
    }
  }
  // ---- 2) findCandidates: potential nodes in snapshot order, offset, numCandidates (:215-238)
  // (the segment path's k_preempt_pick did this on the device; with listCandidates the host redoes it
  // over the whole per-node result and checks that both agree)
  const bool host_cut = !seg || list;
  std::vector<int32_t> pot;
  for (int32_t i = 0; host_cut && i < N; ++i)
    if (po[i].st != PS_NOT_CHECKED) pot.push_back(i);
  int32_t P = (int32_t)pot.size();
  struct Cand { int32_t node; int64_t viol; };
  std::vector<Cand> nv, vl;
  int32_t offset = 0, ncand = 0;
  if (host_cut && P > 0) {
    offset = (int32_t)(((offset_in % P) + P) % P);
    int64_t n = (int64_t)P * pct / 100;
    if (n < absn) n = absn;
    if (n > P) n = P;
    ncand = (int32_t)n;
    // DryRunPreemption (:404-457) with sequential semantics: stop once a non-violating candidate is
    // held and both lists (each capped at numCandidates) reach numCandidates together
    bool unsup = false;  // a node the dry run reaches whose result the device could not compute (flag bit 0)
    for (int32_t j = 0; j < P; ++j) {
      const int32_t i = pot[(offset + j) % P];
      unsup |= (po[i].flags & 1u) != 0;
      if (po[i].st != 0 || po[i].nvictims == 0) continue;
      std::vector<Cand>& l = po[i].nviolating == 0 ? nv : vl;
      if ((int32_t)l.size() < ncand) l.push_back(Cand{i, po[i].nviolating});
      if (!nv.empty() && (int32_t)(nv.size() + vl.size()) >= ncand) break;
    }
    if (unsup && !seg) {
      c->err = "preemption: internal error (dry-run store smaller than the preemptor's constraints)";
      return KSG_EDEVICE;
    }
  }
  std::vector<Cand> cands = nv;
  cands.insert(cands.end(), vl.begin(), vl.end());
  int32_t ncandidates = (int32_t)cands.size();
  // each candidate's victims, importance order (reprieve order, sorted again when both PDB groups
  // contributed, :345-348)
  auto victims_of = [&](int32_t i) {
    std::vector<Victim> out;
    bool g0 = false, g1 = false;
    if (seg) {
      const PSegOut& o = list ? so[i] : pick.best_out;
      const auto& sp = seg_pods[i];
      for (int pass = 0; pass < 2; ++pass)
        for (int q = 0; q < h_segcnt[i]; ++q) {
          const bool vic = (o.vmask[q >> 6] >> (q & 63)) & 1ull, isv = (o.violmask[q >> 6] >> (q & 63)) & 1ull;
          if (!vic || isv != (pass == 0)) continue;
          out.push_back(Victim{&sp[q]->uid, sp[q], sp[q]->has_start ? sp[q]->start_ns : now, isv});
        }
    } else {
      const PNode& nd = pn[i];
      for (int32_t q = 0; q < nd.vcnt; ++q)
        if (vo[nd.voff + q]) out.push_back(all[nd.voff + q]);
    }
    for (const Victim& v : out) (v.viol ? g0 : g1) = true;
    if (g0 && g1) std::stable_sort(out.begin(), out.end(), more_important);
    return out;
  };
  // ---- 4) SelectCandidate / pickOneNodeForPreemption (:262-397)
  int32_t best = -1;  // index into cands
  if (!host_cut) {
  } else if (cands.size() == 1) {
    best = 0;
  } else if (!cands.empty()) {
    std::vector<std::vector<Victim>> cv;
    for (auto& cd : cands) cv.push_back(victims_of(cd.node));
    std::vector<int32_t> sel(cands.size());
    for (size_t k = 0; k < cands.size(); ++k) sel[k] = (int32_t)k;
    auto score = [&](int f, int32_t k) -> int64_t {
      const auto& v = cv[k];
      switch (f) {
        case 0: return -cands[k].viol;                      // minNumPDBViolating
        case 1: return -(int64_t)v[0].bp->priority;         // minHighestPriority
        case 2: {                                           // minSumPriorities
          int64_t sum = 0;
          for (auto& x : v) sum += (int64_t)x.bp->priority + (int64_t)2147483648LL;
          return -sum;
        }
        case 3: return -(int64_t)v.size();                  // minNumPods
        default: {                                          // latestStartTime: GetEarliestPodStartTime
          int64_t t = v[0].start;
          int32_t mp = v[0].bp->priority;
          for (auto& x : v) {
            if (x.bp->priority == mp) {
              if (x.start < t) t = x.start;
            } else if (x.bp->priority > mp) {
              mp = x.bp->priority;
              t = x.start;
            }
          }
          return t;
        }
      }
    };
    for (int f = 0; f < 5 && sel.size() > 1; ++f) {
      std::vector<int32_t> next;
      int64_t mx = INT64_MIN;
      for (int32_t k : sel) {
        const int64_t sc = score(f, k);
        if (sc > mx) {
          mx = sc;
          next.clear();
        }
        if (sc == mx) next.push_back(k);
      }
      sel = next;
    }
    best = sel[0];
  }
  int32_t best_node = best >= 0 ? cands[best].node : -1;
  int64_t best_viol = best >= 0 ? cands[best].viol : 0;
  if (seg) {
    if (host_cut && (pick.best != best_node || pick.potential != P || pick.ncandidates != ncandidates)) {
      c->err = "preemption: the device's candidate pick differs from the host's";
      return KSG_EDEVICE;
    }
    P = pick.potential;
    offset = pick.offset;
    ncand = pick.ncand;
    ncandidates = pick.ncandidates;
    best_node = pick.best;
    if (best_node >= 0) best_viol = pick.best_out.nviolating;
  }
  res->num_potential = P;
  res->num_candidates = ncandidates;
  std::string msg;
  if (best_node >= 0) {
    const int32_t i = best_node;
    res->status = KSG_CODE_SUCCESS;
    res->reason = KSG_PREEMPT_OK;
    res->node_index = i;
    res->num_victims = (seg && !list) ? pick.best_out.nvictims : po[i].nvictims;
    res->num_pdb_violations = best_viol;
  } else {
    res->reason = KSG_PREEMPT_NO_CANDIDATES;
    msg = "0/" + std::to_string(N) + " nodes are available: preemption is not helpful for scheduling.";
  }
  if (detail) {
    std::string& o = *detail;
    o = "{\"offset\":" + std::to_string(offset) + ",\"numCandidates\":" + std::to_string(ncand) +
        ",\"potential\":" + std::to_string(P) + ",\"message\":";
    json_str(o, msg);
    o += ",\"candidates\":[";
    for (size_t k = 0; list && k < cands.size(); ++k) {
      if (k) o += ",";
      o += "{\"node\":";
      json_str(o, order[cands[k].node]);
      o += ",\"numPDBViolations\":" + std::to_string(cands[k].viol) + ",\"victims\":[";
      auto v = victims_of(cands[k].node);
      for (size_t q = 0; q < v.size(); ++q) {
        if (q) o += ",";
        json_str(o, *v[q].uid);
      }
      o += "]}";
    }
    o += "],\"selected\":";
    if (best_node >= 0) json_str(o, order[best_node]);
    else o += "null";
    o += ",\"victims\":[";
    if (best_node >= 0) {
      auto v = victims_of(best_node);
      for (size_t q = 0; q < v.size(); ++q) {
        if (q) o += ",";
        json_str(o, *v[q].uid);
      }
    }
    o += "]}";
  }
  return KSG_OK;
}

}  // namespace ksg
