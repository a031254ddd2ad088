// podtable.cpp -- the pod table behind PodTopologySpread and InterPodAffinity on the device.
//
// The reference walks NodeInfo.Pods of every snapshot node in PreFilter/PreScore
// (podtopologyspread/filtering.go:237-311, scoring.go:118-194; interpodaffinity/filtering.go:216-283,
// scoring.go:128-221).  Here every bound or assumed pod is one slot of a flat structure-of-arrays
// table in HBM -- node index, namespace id, terminating flag, sorted label set -- and every
// affinity term an existing pod carries (framework.PodInfo's RequiredAffinityTerms etc.,
// kube-scheduler/framework/types.go:380-396, 1183-1226) is one entry of a term table.  The
// per-pod aggregation kernel (k_aggregate) streams both tables into per-domain histograms.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "host.hpp"

namespace ksg {

std::vector<unsigned long long> Cluster::label_set(const StrMap& labels) {
  std::vector<unsigned long long> out;
  out.reserve(labels.size());
  for (auto& kv : labels) {
    const int32_t k = key_id(kv.first);
    const int32_t v = keys[k].values.get(kv.second);
    out.push_back(((unsigned long long)(uint32_t)k << 32) | (uint32_t)v);
  }
  std::sort(out.begin(), out.end());
  return out;
}

// metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:36-71) with
// labels.NewRequirement validation (selector.go:185-226).  merge_labels: the matchLabelKeys
// label set PodTopologySpread prepends (common.go:96-106,130-143).
bool Cluster::compile_lsel(const LabelSel& s, const StrMap* merge_labels, std::vector<int32_t>* pool, int32_t* off,
                           bool prevalidated_match) {
  *off = (int32_t)pool->size();
  if (!s.present) {  // nil selector: labels.Nothing()
    pool->push_back(1);
    pool->push_back(0);
    return true;
  }
  struct Req { std::string key; int32_t op; std::vector<std::string> vals; };
  std::vector<Req> reqs;
  bool ok = true;
  for (auto& kv : s.match) {
    // labels.SelectorFromValidatedSet (selector.go:976-987) does not validate: DefaultSelector's merged maps
    ok = ok && (prevalidated_match || (valid_label_key(kv.first) && valid_label_value(kv.second)));
    reqs.push_back({kv.first, LS_IN, {kv.second}});
  }
  for (auto& e : s.exprs) {
    int32_t op;
    if (e.op == "In") op = LS_IN;
    else if (e.op == "NotIn") op = LS_NOTIN;
    else if (e.op == "Exists") op = LS_EXISTS;
    else if (e.op == "DoesNotExist") op = LS_DNE;
    else return false;
    ok = ok && valid_label_key(e.key);
    if (op == LS_IN || op == LS_NOTIN) ok = ok && !e.values.empty();
    else ok = ok && e.values.empty();
    for (auto& v : e.values) ok = ok && valid_label_value(v);
    reqs.push_back({e.key, op, e.values});
  }
  if (!ok) return false;
  if (merge_labels && !merge_labels->empty())
    for (auto& kv : *merge_labels) reqs.push_back({kv.first, LS_IN, {kv.second}});
  pool->push_back(0);
  pool->push_back((int32_t)reqs.size());
  for (auto& r : reqs) {
    const int32_t k = key_id(r.key);
    pool->push_back(k);
    pool->push_back(r.op);
    pool->push_back((int32_t)r.vals.size());
    for (auto& v : r.vals) pool->push_back(keys[k].values.get(v));
  }
  return true;
}

// framework.NewPodInfo + GetPod*AffinityTerms for an existing pod: a category whose terms do
// not parse is dropped as a whole (the oracle does the same, oracle_model.cpp new_pod_info).
void Cluster::pod_table_precompile(const PodSpec& p) {
  auto pre = std::make_shared<PodTablePre>();
  pre->labels = label_set(p.labels);
  auto category = [&](const std::vector<PATerm>& in, int32_t kind) {
    const size_t w0 = pre->words.size(), t0 = pre->terms.size();
    for (auto& t : in) {
      PodTablePre::Term d{};
      d.kind = kind;
      d.weight = t.weight;
      d.key = key_id(t.topo);
      int32_t so, no;
      if (!compile_lsel(t.sel, nullptr, &pre->words, &so) || !compile_lsel(t.ns_sel, nullptr, &pre->words, &no)) {
        pre->words.resize(w0);  // the whole category is dropped, as pod_table_put always did
        pre->terms.resize(t0);
        return;
      }
      d.sel = so;
      d.nssel = no;
      d.ns_off = (int32_t)pre->words.size();
      if (t.namespaces.empty() && !t.ns_sel.present) {  // newAffinityTerm defaulting (types.go:422-448)
        pre->words.push_back(ns_id(p.ns));
      } else {
        for (auto& n : t.namespaces) pre->words.push_back(ns_id(n));
      }
      d.ns_cnt = (int32_t)pre->words.size() - d.ns_off;
      pre->terms.push_back(d);
    }
  };
  if (p.has_pod_affinity) {
    category(p.aff_req, T_REQ_AFF);
    category(p.aff_pref, T_PREF_AFF);
  }
  if (p.has_pod_anti) {
    category(p.anti_req, T_REQ_ANTI);
    category(p.anti_pref, T_PREF_ANTI);
  }
  p.pt_pre = std::move(pre);
}

int32_t Cluster::pod_table_put(const PodSpec& p, int32_t node_index) {
  if (!p.pt_pre) pod_table_precompile(p);
  const PodTablePre& pre = *p.pt_pre;
  int32_t s;
  if (!pt_free.empty()) {
    s = pt_free.back();
    pt_free.pop_back();
  } else {
    s = (int32_t)pt_node.size();
    pt_node.push_back(-1);
    pt_ns.push_back(0);
    pt_flags.push_back(0);
    pt_lbl_off.push_back(0);
    pt_lbl_cnt.push_back(0);
    pt_terms.emplace_back();
  }
  pt_node[s] = node_index;
  pt_ns[s] = ns_id(p.ns);
  pt_flags[s] = p.terminating ? 1u : 0u;
  pt_lbl_off[s] = (uint32_t)pt_pool.size();
  pt_lbl_cnt[s] = (uint32_t)pre.labels.size();
  pt_pool.insert(pt_pool.end(), pre.labels.begin(), pre.labels.end());
  // the terms: their words appended to the term pool, offsets rebased
  const int32_t base = (int32_t)tt_pool.size();
  tt_pool.insert(tt_pool.end(), pre.words.begin(), pre.words.end());
  last_tpool_off = base;
  last_tpool_cnt = (int32_t)pre.words.size();
  for (const PodTablePre::Term& t : pre.terms) {
    DTerm d{};
    d.owner = s;
    d.kind = t.kind;
    d.weight = t.weight;
    d.key = t.key;
    d.sel = base + t.sel;
    d.nssel = base + t.nssel;
    d.ns_off = base + t.ns_off;
    d.ns_cnt = t.ns_cnt;
    ensure_label_slot(d.key);
    int32_t j;
    if (!tt_free.empty()) {
      j = tt_free.back();
      tt_free.pop_back();
      tt[j] = d;
    } else {
      j = (int32_t)tt.size();
      tt.push_back(d);
    }
    pt_terms[s].push_back(j);
    auto& m = t.kind == T_REQ_ANTI ? exanti_keys : t.kind == T_REQ_AFF ? score_keys_req : score_keys_pref;
    m[d.key]++;
  }
  pods_dirty = true;
  return s;
}


size_t Cluster::ring_entry(int32_t s, uint8_t* out, size_t cap) const {
  if (s < 0 || s >= (int32_t)pt_node.size()) return 0;
  const uint32_t lo = pt_lbl_off[(size_t)s], lc = pt_lbl_cnt[(size_t)s];
  const std::vector<int32_t>& js = pt_terms[(size_t)s];
  const size_t tw = ((size_t)last_tpool_cnt + 1) & ~(size_t)1;
  const size_t bytes = sizeof(RingEntry) + (size_t)lc * 8 + tw * 4 + js.size() * sizeof(RingTerm);
  if (bytes > cap || bytes % 8 != 0) return 0;
  // the device arrays must already hold every index the entry writes (as upload_pod_table sized them)
  int32_t jmax = -1;
  for (int32_t j : js) jmax = std::max(jmax, j);
  // the entry carries the words of the last pod put, which must be this slot's: every word its terms name lies in
  // them (the resident k_agg_loop writes them to the device pool, and folds the pod from them in LDS)
  const int64_t wlo = last_tpool_off, whi = (int64_t)last_tpool_off + last_tpool_cnt;
  for (int32_t j : js) {
    const DTerm& d = tt[(size_t)j];
    if (d.sel < wlo || d.sel >= whi || d.nssel < wlo || d.nssel >= whi || d.ns_off < wlo || d.ns_off + d.ns_cnt > whi)
      return 0;
  }
  const size_t ps = ((size_t)s + 1) * 4;
  if (!pt_dev_[0].p || pt_dev_[0].bytes < ps || pt_dev_[1].bytes < ps || pt_dev_[2].bytes < ps || pt_dev_[3].bytes < ps ||
      pt_dev_[4].bytes < ps || pt_dev_[5].bytes < ((size_t)lo + lc) * 8 ||
      pt_dev_[6].bytes < (size_t)(jmax + 1) * sizeof(DTerm) ||
      pt_dev_[7].bytes < ((size_t)last_tpool_off + (size_t)last_tpool_cnt) * 4)
    return 0;
  RingEntry h{};
  h.slot = s;
  h.ns = pt_ns[(size_t)s];
  h.flags = pt_flags[(size_t)s];
  h.lbl_off = lo;
  h.lbl_cnt = lc;
  h.tpool_off = last_tpool_off;
  h.tpool_cnt = last_tpool_cnt;
  h.nterms = (int32_t)js.size();
  uint8_t* o = out;
  std::memcpy(o, &h, sizeof h);
  o += sizeof h;
  std::memcpy(o, pt_pool.data() + lo, (size_t)lc * 8);
  o += (size_t)lc * 8;
  std::memset(o, 0, tw * 4);
  std::memcpy(o, tt_pool.data() + last_tpool_off, (size_t)last_tpool_cnt * 4);
  o += tw * 4;
  for (int32_t j : js) {
    RingTerm r{};
    r.j = j;
    r.d = tt[(size_t)j];
    std::memcpy(o, &r, sizeof r);
    o += sizeof r;
  }
  return bytes;
}

void Cluster::pod_table_drop(int32_t s) {
  if (s < 0 || s >= (int32_t)pt_node.size()) return;
  for (int32_t j : pt_terms[s]) {
    DTerm& d = tt[j];
    auto& m = d.kind == T_REQ_ANTI ? exanti_keys : d.kind == T_REQ_AFF ? score_keys_req : score_keys_pref;
    auto it = m.find(d.key);
    if (it != m.end() && --it->second <= 0) m.erase(it);
    d.kind = T_DEAD;
    d.owner = -1;
    tt_free.push_back(j);
  }
  pt_terms[s].clear();
  pt_node[s] = -1;
  pt_lbl_cnt[s] = 0;
  pt_free.push_back(s);
  pods_dirty = true;
}

int Cluster::grow(DevBuf& b, size_t bytes) {
  if (b.p && b.bytes >= bytes) return KSG_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  const size_t want = std::max<size_t>(4096, bytes + bytes / 2);
  if (hipMalloc(&b.p, want) != hipSuccess) {
    err = "hipMalloc failed for the pod table";
    return KSG_EDEVICE;
  }
  b.bytes = want;
  return KSG_OK;
}

// Go's math.Log (math/log.go: the FreeBSD e_log.c reduction and polynomial), evaluated without
// fused multiply-adds (objects are built with -ffp-contract=off) -- the weights
// PodTopologySpread multiplies domain counts by (scoring.go:287-299).
double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
  if (x < 0) return std::nan("");
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < M_SQRT2 / 2) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1;
  const double k = (double)ki;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

int Cluster::upload_pod_table(bool lazy) {
  // a call whose pods never read the pod table (no PodTopologySpread / InterPodAffinity work) only needs
  // pod_node to have room for the slots its assumes write: the table goes up with the next call that
  // reads it (every single-pod call of a node-local stream would otherwise re-upload the whole table)
  const bool room = pt_dev_[0].p && pt_dev_[0].bytes >= (pt_node.size() + (size_t)pt_headroom) * 4 + 4;
  if (lazy && pods_dirty && room) return KSG_OK;
  // log table covers topoSize + 2 for every topoSize <= N (scoring.go:293-299)
  const int32_t need_log = (int32_t)order_.size() + 4;
  bool log_dirty = false;
  if ((int32_t)log_tab.size() < need_log) {
    const size_t old = log_tab.size();
    log_tab.resize((size_t)need_log * 2);
    for (size_t k = old; k < log_tab.size(); ++k) log_tab[k] = go_log((double)k);
    log_dirty = true;
  }
  if (!pods_dirty && !log_dirty && room) return KSG_OK;  // (a batch's headroom may need a larger pod_node)
  // compact the label pool when most of it is garbage
  size_t live = 0;
  for (size_t s = 0; s < pt_node.size(); ++s) live += pt_lbl_cnt[s];
  if (pt_pool.size() > 4 * live + 65536) {
    std::vector<unsigned long long> np;
    np.reserve(live * 2);
    for (size_t s = 0; s < pt_node.size(); ++s) {
      const uint32_t o = pt_lbl_off[s], c = pt_lbl_cnt[s];
      pt_lbl_off[s] = (uint32_t)np.size();
      np.insert(np.end(), pt_pool.begin() + o, pt_pool.begin() + o + c);
    }
    pt_pool.swap(np);
  }
  int rc;
  const size_t P = pt_node.size(), T = tt.size();
  if ((rc = grow(pt_dev_[0], (P + (size_t)pt_headroom) * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[1], P * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[2], P * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[3], P * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[4], P * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[5], pt_pool.size() * 8 + 8))) return rc;
  if ((rc = grow(pt_dev_[6], T * sizeof(DTerm) + sizeof(DTerm)))) return rc;
  if ((rc = grow(pt_dev_[7], tt_pool.size() * 4 + 4))) return rc;
  if ((rc = grow(pt_dev_[8], log_tab.size() * 8))) return rc;
  auto up = [&](DevBuf& b, const void* src, size_t bytes) -> int {
    if (!bytes) return KSG_OK;
    if (hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
      err = "pod table upload failed";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  };
  if ((rc = up(pt_dev_[0], pt_node.data(), P * 4))) return rc;
  if ((rc = up(pt_dev_[1], pt_ns.data(), P * 4))) return rc;
  if ((rc = up(pt_dev_[2], pt_flags.data(), P * 4))) return rc;
  if ((rc = up(pt_dev_[3], pt_lbl_off.data(), P * 4))) return rc;
  if ((rc = up(pt_dev_[4], pt_lbl_cnt.data(), P * 4))) return rc;
  if ((rc = up(pt_dev_[5], pt_pool.data(), pt_pool.size() * 8))) return rc;
  if ((rc = up(pt_dev_[6], tt.data(), T * sizeof(DTerm)))) return rc;
  if ((rc = up(pt_dev_[7], tt_pool.data(), tt_pool.size() * 4))) return rc;
  if ((rc = up(pt_dev_[8], log_tab.data(), log_tab.size() * 8))) return rc;
  if (hipStreamSynchronize(stream) != hipSuccess) {  // host vectors may change right after
    err = "pod table upload failed";
    return KSG_EDEVICE;
  }
  view.pods_hw = (int32_t)P;
  view.n_terms = (int32_t)T;
  view.pod_node = (int32_t*)pt_dev_[0].p;
  view.pod_ns = (const int32_t*)pt_dev_[1].p;
  view.pod_flags = (const uint32_t*)pt_dev_[2].p;
  view.pod_lbl_off = (const uint32_t*)pt_dev_[3].p;
  view.pod_lbl_cnt = (const uint32_t*)pt_dev_[4].p;
  view.lbl_pool = (const unsigned long long*)pt_dev_[5].p;
  view.terms = (const DTerm*)pt_dev_[6].p;
  view.term_pool = (const int32_t*)pt_dev_[7].p;
  view.log_tab = (const double*)pt_dev_[8].p;
  view.log_n = (int32_t)log_tab.size();
  pods_dirty = false;
  return KSG_OK;
}

}  // namespace ksg
