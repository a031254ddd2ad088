// preempt.cpp -- DefaultPreemption's PostFilter.
//
// Evaluator.Preempt (framework/preemption/preemption.go:103-170) for one pod that failed its cycle:
//   PodEligibleToPreemptOthers (default_preemption.go:364-388) on the host;
//   the cycle's Filter statuses (the FitError diagnosis) from k_filter_score on the device;
//   SelectVictimsOnNode (default_preemption.go:252-354) for every node findCandidates would pass to
//   DryRunPreemption (preemption.go:174-196, 404-457) -- k_preempt, one thread per node;
//   the candidate cut of DryRunPreemption with sequential Parallelizer semantics (parallelism 1, the
//   reference's own deterministic test mode) and SelectCandidate / pickOneNodeForPreemption
//   (preemption.go:262-397) on the host, over the per-node results.
// Actuation (deleting victims, patching nominatedNodeName, executor.go) is the caller's: the result
// names the node and the victims.
//
// Determinism contract (each documented in ksg.h): the random offset is the caller's; pods without
// status.startTime get the caller's clock (GetPodStartTime's time.Now(), utils.go:52-58); victims of
// equal priority and start time keep NodeInfo.Pods order (sort.Slice is an insertion sort, hence
// stable, up to 12 elements); candidates tie-break in candidate-list order (the reference iterates a
// Go map there, preemption.go:316-319).
#include <algorithm>
#include <cstring>

#include "host.hpp"

namespace ksg {

hipError_t launch_aggregate(const MirrorView& m, const BatchView& b, int pod, const PodDesc& d, hipStream_t s);
hipError_t launch_filter_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, hipEvent_t t0,
                               hipEvent_t t1, int blk0, int nblk, bool lds);
hipError_t launch_preempt(const MirrorView& m, const BatchView& b, int pod, const PNode* pn, const PVictim* pv,
                          uint8_t* vout, POut* out, int all_nodes, hipStream_t s);

#define PCHK(x)                                                         \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      c->err = std::string("HIP: ") + hipGetErrorString(e_) + " @" #x;  \
      return KSG_EDEVICE;                                               \
    }                                                                   \
  } while (0)

namespace {

enum : int { P_PORTS = KSG_PLUGIN_NODE_PORTS, P_PTS = KSG_PLUGIN_POD_TOPOLOGY_SPREAD };

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
  std::string uid;
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

int Engine::preempt(const PodSpec& p, const char* args_json, size_t args_len, ksg_preempt_result* res,
                    std::string* detail) {
  *res = ksg_preempt_result{};
  res->status = KSG_CODE_UNSCHEDULABLE;
  res->node_index = -1;
  // ---- DefaultPreemptionArgs + the call's inputs (validation_pluginargs.go:113-125)
  int64_t offset_in = 0, now = 0;
  int32_t pct = 10, absn = 100;
  bool all_nodes = false;
  std::vector<Pdb> pdbs;
  try {
    JDoc d(args_json && args_len ? args_json : "{}", args_json && args_len ? args_len : 2);
    const JVal& r = d.root();
    offset_in = d.num(r, "offset", 0);
    now = d.num(r, "now", 0);
    pct = (int32_t)d.num(r, "minCandidateNodesPercentage", 10);
    absn = (int32_t)d.num(r, "minCandidateNodesAbsolute", 100);
    all_nodes = d.boolean(r, "allNodes");
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
  const PodDesc& D = *reinterpret_cast<const PodDesc*>(cp.blob.data());
  if (D.n_scalar > kPreemptScalar) {
    c->err = "preemption: the pod requests more than 4 scalar resources";
    return KSG_ENOTSUP;
  }

  // ---- the potential victims of every node, in reprieve order
  std::vector<PNode> pn((size_t)std::max(N, 1));
  std::vector<PVictim> pv;
  std::vector<Victim> all;  // parallel to pv
  const uint32_t* conflict = reinterpret_cast<const uint32_t*>(cp.blob.data() + D.port_conflict_off);
  auto conflicts = [&](uint32_t pid) {
    return (D.filter_mask >> P_PORTS & 1u) && (int32_t)(pid >> 5) < D.n_port_words &&
           ((conflict[pid >> 5] >> (pid & 31u)) & 1u);
  };
  const int32_t pns = c->ns_id(p.ns);
  std::vector<std::pair<std::string, int32_t>> scal;  // the preemptor's scalar resources in PodDesc order
  {
    const ScalarReq* sr = reinterpret_cast<const ScalarReq*>(cp.blob.data() + D.scalar_off);
    for (int k = 0; k < D.n_scalar; ++k) scal.push_back({c->scalar_ix.strs[sr[k].slot], sr[k].slot});
  }
  const bool pts_on = (D.filter_mask >> P_PTS & 1u) && D.n_ptsf > 0;
  const bool ipa_req = !p.aff_req.empty() || !p.anti_req.empty();
  std::vector<Victim> vs;
  for (int32_t i = 0; i < N; ++i) {
    NodeRec* r = c->node(order[i]);
    PNode& nd = pn[i];
    nd = PNode{(int32_t)pv.size(), 0, 0u, 0};
    vs.clear();
    for (const std::string& uid : r->pods) {  // isPreemptionAllowed (:396-399): lower priority
      const BoundPod& bp = c->pods.at(uid);
      if (bp.priority < p.priority) vs.push_back(Victim{uid, &bp, bp.has_start ? bp.start_ns : now, false});
    }
    if (vs.empty()) continue;
    // PodTopologySpread / InterPodAffinity counts a victim could change (their RemovePod/AddPod
    // extensions) are outside what k_preempt re-evaluates: refuse rather than approximate
    for (const Victim& v : vs) {
      if (pts_on && c->pt_ns[v.bp->slot] == pns)
        for (auto& sp : p.spreads)
          if (sp.when == "DoNotSchedule" && sp.sel.present && lsel_match_slot(*c, sp.sel, v.bp->slot)) {
            c->err = "preemption: a victim changes the pod's PodTopologySpread counts (not supported on the device)";
            return KSG_ENOTSUP;
          }
      if (ipa_req || v.bp->req_anti) {
        c->err = "preemption: InterPodAffinity terms between the pod and a victim (not supported on the device)";
        return KSG_ENOTSUP;
      }
    }
    std::stable_sort(vs.begin(), vs.end(), more_important);  // sort.Slice (:309-311), see header
    // filterPodsWithPDBViolation (:406-452) over the sorted list
    std::vector<int32_t> allowed(pdbs.size());
    for (size_t k = 0; k < pdbs.size(); ++k) allowed[k] = pdbs[k].allowed;
    const std::string* vns = nullptr;
    for (Victim& v : vs) {
      if (c->pt_lbl_cnt[v.bp->slot] == 0) continue;  // a pod with no labels matches no PDB
      for (size_t k = 0; k < pdbs.size(); ++k) {
        const Pdb& b = pdbs[k];
        vns = &c->ns_ix.strs[c->pt_ns[v.bp->slot]];
        if (b.ns != *vns || !b.sel_ok || !lsel_match_slot(*c, b.sel, v.bp->slot)) continue;
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
      for (size_t k = 0; k < scal.size(); ++k)
        for (auto& sv : v.bp->res.scalar)
          if (sv.first == scal[k].first) x.sc[k] += sv.second;
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

  // ---- device: the cycle's statuses, then SelectVictimsOnNode per node
  std::vector<POut> po((size_t)std::max(N, 1));
  std::vector<uint8_t> vo((size_t)std::max(V, 1));
  uint32_t nom_status = 0;
  int32_t nom_ix = p.nominated_node.empty() ? -1 : c->index_of(p.nominated_node);
  if (N > 0) {
    if ((rc = c->ensure_mirror())) return rc;
    if ((rc = ensure_scratch(cp.blob.size(), 1, true, cp.arena_words))) return rc;
    const size_t pn_b = sizeof(PNode) * (size_t)N, pv_b = sizeof(PVictim) * (size_t)std::max(V, 1);
    const size_t po_b = sizeof(POut) * (size_t)N, vo_b = (size_t)std::max(V, 1);
    if ((rc = ensure(d_pre, pn_b + pv_b + po_b + vo_b + 64))) return rc;
    uint8_t* dp = (uint8_t*)d_pre.p;
    PNode* d_pn = (PNode*)dp;
    PVictim* d_pv = (PVictim*)(dp + pn_b);
    POut* d_po = (POut*)(dp + pn_b + pv_b);
    uint8_t* d_vo = dp + pn_b + pv_b + po_b;
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
    PCHK(hipMemcpyAsync(d_descs.p, hp, cp.blob.size(), hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_off.p, &off0, 4, hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_stats.p, hs, sizeof(PodStats), hipMemcpyHostToDevice, s));
    PCHK(hipMemcpyAsync(d_pn, pn.data(), pn_b, hipMemcpyHostToDevice, s));
    if (V) PCHK(hipMemcpyAsync(d_pv, pv.data(), pv_b, hipMemcpyHostToDevice, s));
    const BatchView bv = bview(1);
    if (D.flags & DF_AGGREGATE) PCHK(launch_aggregate(m, bv, 0, D, s));
    const bool lds = cp.blob.size() <= (size_t)kBlobLds;
    PCHK(launch_filter_score(m, bv, 0, s, nullptr, nullptr, 0, -1, lds));
    PCHK(launch_preempt(m, bv, 0, d_pn, d_pv, d_vo, d_po, all_nodes ? 1 : 0, s));
    if (D.arena_words) PCHK(hipMemsetAsync(d_arena.p, 0, (size_t)D.arena_words * 8, s));  // k_select did not run
    PCHK(hipMemcpyAsync(po.data(), d_po, po_b, hipMemcpyDeviceToHost, s));
    if (V) PCHK(hipMemcpyAsync(vo.data(), d_vo, vo_b, hipMemcpyDeviceToHost, s));
    if (nom_ix >= 0) PCHK(hipMemcpyAsync(&nom_status, bv.status + nom_ix, 4, hipMemcpyDeviceToHost, s));
    PCHK(hipStreamSynchronize(s));
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
  std::vector<int32_t> pot;
  for (int32_t i = 0; i < N; ++i)
    if (po[i].st != PS_NOT_CHECKED) pot.push_back(i);
  const int32_t P = (int32_t)pot.size();
  res->num_potential = P;
  struct Cand { int32_t node; int64_t viol; };
  std::vector<Cand> nv, vl;
  int32_t offset = 0, ncand = 0;
  if (P > 0) {
    offset = (int32_t)(((offset_in % P) + P) % P);
    int64_t n = (int64_t)P * pct / 100;
    if (n < absn) n = absn;
    if (n > P) n = P;
    ncand = (int32_t)n;
    // DryRunPreemption (:404-457) with sequential semantics: stop once a non-violating candidate is
    // held and both lists (each capped at numCandidates) reach numCandidates together
    for (int32_t j = 0; j < P; ++j) {
      const int32_t i = pot[(offset + j) % P];
      if (po[i].st != 0 || po[i].nvictims == 0) continue;
      std::vector<Cand>& l = po[i].nviolating == 0 ? nv : vl;
      if ((int32_t)l.size() < ncand) l.push_back(Cand{i, po[i].nviolating});
      if (!nv.empty() && (int32_t)(nv.size() + vl.size()) >= ncand) break;
    }
  }
  std::vector<Cand> cands = nv;
  cands.insert(cands.end(), vl.begin(), vl.end());
  res->num_candidates = (int32_t)cands.size();
  // each candidate's victims, importance order (sorted again when both groups contributed, :345-348)
  auto victims_of = [&](int32_t i) {
    std::vector<const Victim*> out;
    const PNode& nd = pn[i];
    bool g0 = false, g1 = false;
    for (int32_t q = 0; q < nd.vcnt; ++q)
      if (vo[nd.voff + q]) {
        out.push_back(&all[nd.voff + q]);
        (all[nd.voff + q].viol ? g0 : g1) = true;
      }
    if (g0 && g1)
      std::stable_sort(out.begin(), out.end(), [](const Victim* a, const Victim* b) { return more_important(*a, *b); });
    return out;
  };
  // ---- 4) SelectCandidate / pickOneNodeForPreemption (:262-397)
  int32_t best = -1;
  if (cands.size() == 1) {
    best = 0;
  } else if (!cands.empty()) {
    std::vector<std::vector<const Victim*>> cv;
    for (auto& cd : cands) cv.push_back(victims_of(cd.node));
    std::vector<int32_t> sel(cands.size());
    for (size_t k = 0; k < cands.size(); ++k) sel[k] = (int32_t)k;
    auto score = [&](int f, int32_t k) -> int64_t {
      const auto& v = cv[k];
      switch (f) {
        case 0: return -cands[k].viol;                      // minNumPDBViolating
        case 1: return -(int64_t)v[0]->bp->priority;        // minHighestPriority
        case 2: {                                           // minSumPriorities
          int64_t sum = 0;
          for (auto* x : v) sum += (int64_t)x->bp->priority + (int64_t)2147483648LL;
          return -sum;
        }
        case 3: return -(int64_t)v.size();                  // minNumPods
        default: {                                          // latestStartTime: GetEarliestPodStartTime
          int64_t t = v[0]->start;
          int32_t mp = v[0]->bp->priority;
          for (auto* x : v) {
            if (x->bp->priority == mp) {
              if (x->start < t) t = x->start;
            } else if (x->bp->priority > mp) {
              mp = x->bp->priority;
              t = x->start;
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
  std::string msg;
  if (best >= 0) {
    const int32_t i = cands[best].node;
    res->status = KSG_CODE_SUCCESS;
    res->reason = KSG_PREEMPT_OK;
    res->node_index = i;
    res->num_victims = po[i].nvictims;
    res->num_pdb_violations = cands[best].viol;
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
    for (size_t k = 0; k < cands.size(); ++k) {
      if (k) o += ",";
      o += "{\"node\":";
      json_str(o, order[cands[k].node]);
      o += ",\"numPDBViolations\":" + std::to_string(cands[k].viol) + ",\"victims\":[";
      auto v = victims_of(cands[k].node);
      for (size_t q = 0; q < v.size(); ++q) {
        if (q) o += ",";
        json_str(o, v[q]->uid);
      }
      o += "]}";
    }
    o += "],\"selected\":";
    if (best >= 0) json_str(o, order[cands[best].node]);
    else o += "null";
    o += ",\"victims\":[";
    if (best >= 0) {
      auto v = victims_of(cands[best].node);
      for (size_t q = 0; q < v.size(); ++q) {
        if (q) o += ",";
        json_str(o, v[q]->uid);
      }
    }
    o += "]}";
  }
  return KSG_OK;
}

}  // namespace ksg
