// device.hpp -- device helpers shared by the node-pass kernels (kernels.hip) and the
// pod-table aggregation kernels (aggregate.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../common/desc.h"

namespace ksg {

#define KSG_R_UNSCHEDULABLE (1u << 0)
#define KSG_R_NODE_NAME (1u << 1)
#define KSG_R_TAINT (1u << 2)
#define KSG_R_NODE_AFFINITY_POD (1u << 3)
#define KSG_R_NODE_AFFINITY_ENFORCED (1u << 4)
#define KSG_R_NODE_PORTS (1u << 5)
#define KSG_R_TOO_MANY_PODS (1u << 6)
#define KSG_R_INSUFFICIENT_CPU (1u << 7)
#define KSG_R_INSUFFICIENT_MEMORY (1u << 8)
#define KSG_R_INSUFFICIENT_EPHEMERAL (1u << 9)
#define KSG_R_INSUFFICIENT_SCALAR (1u << 10)
#define KSG_R_PTS_MISSING_LABEL (1u << 11)
#define KSG_R_PTS_SKEW (1u << 12)
#define KSG_R_IPA_AFFINITY (1u << 13)
#define KSG_R_IPA_ANTI_AFFINITY (1u << 14)
#define KSG_R_IPA_EXISTING_ANTI (1u << 15)
#define KSG_R_PREFILTER (1u << 16)

enum : int { P_UNSCHED = 0, P_NODENAME = 1, P_TAINT = 2, P_NA = 3, P_PORTS = 4, P_FIT = 5, P_PTS = 6,
             P_IPA = 7, P_BAL = 8, P_IMG = 9 };
enum : uint32_t { C_OK = 0, C_ERROR = 1, C_UNSCHED = 2, C_UU = 3 };

// Domain presence: set flags[v] (0 -> 1) for every active lane with `want`, and add to *counter the
// number of flags this call set first.  A few domains shared by many nodes (zones) would make every
// lane exchange the same words: the first four distinct values of a wave are issued by one leader
// lane each, the rest (hostname-like keys, all distinct) one exchange per lane.  One counter atomic
// per wave.  Called by whole waves (inactive lanes simply do not take part).
__device__ __forceinline__ void mark_domains(unsigned long long* flags, int v, bool want, uint32_t* counter) {
  const int lane = threadIdx.x & 63;
  const bool cand = want && flags[v] == 0ull;
  unsigned long long todo = __ballot(cand);
  bool lead = false;
  for (int it = 0; it < 4 && todo; ++it) {
    const int l = __builtin_ctzll(todo);
    const int lv = __shfl(v, l, 64);
    const unsigned long long same = __ballot(cand && v == lv);
    lead |= lane == l;
    todo &= ~same;
  }
  lead |= ((todo >> lane) & 1ull) != 0;
  const bool won = lead && atomicExch(flags + v, 1ull) == 0ull;
  const unsigned long long wb = __ballot(won);
  if (wb && lane == __builtin_ctzll(wb)) atomicAdd(counter, (uint32_t)__popcll(wb));
}

// Go int64 `a / b` (truncating) without the ~60-instruction 64-bit division expansion on the
// common path: operands that fit 32 bits use the 32-bit unit; non-negative operands below 2^52
// divide in FP64 (exact inputs, correctly rounded quotient) and the truncated quotient is fixed
// up by one with the exact remainder.  Anything else takes the generic int64 division.
__device__ __forceinline__ int64_t go_div(int64_t a, int64_t b) {
  if (a >= 0 && b > 0) {
    if (((uint64_t)a | (uint64_t)b) >> 32 == 0) return (int64_t)((uint32_t)a / (uint32_t)b);
    if (a < (1ll << 52) && b < (1ll << 52)) {
      int64_t q = (int64_t)((double)a / (double)b);
      const int64_t r = a - q * b;
      if (r < 0) --q;
      else if (r >= b) ++q;
      return q;
    }
  }
  return a / b;
}

template <typename T>
__device__ __forceinline__ const T* at(const uint8_t* base, int32_t off) {
  return reinterpret_cast<const T*>(base + off);
}
__device__ __forceinline__ bool bit(const uint8_t* base, int32_t off, uint32_t id, int32_t nwords) {
  uint32_t w = id >> 5;
  if ((int32_t)w >= nwords) return false;
  return (at<uint32_t>(base, off)[w] >> (id & 31u)) & 1u;
}

// ---- selector programs ---------------------------------------------------------------------
// labels.Requirement.Matches (apimachinery/pkg/labels/selector.go:247-294) against the
// node's label columns; metadata.name field requirements (nodeaffinity.go:190-201).
__device__ bool req_match(const MirrorView& m, const uint8_t* base, const PodDesc& d, const SelReq& r, int i) {
  const size_t col = (size_t)r.slot * (size_t)m.cap + (size_t)i;
  switch (r.op) {
    case SEL_IN:
    case SEL_NOTIN: {
      int32_t v = m.labels[col];
      if (v < 0) return r.op == SEL_NOTIN;
      const int32_t* vals = at<int32_t>(base, d.vals_off) + r.vals_off;
      bool has = false;
      for (int k = 0; k < r.nvals; ++k) has |= vals[k] == v;
      return r.op == SEL_IN ? has : !has;
    }
    case SEL_EXISTS: return m.labels[col] >= 0;
    case SEL_DNE: return m.labels[col] < 0;
    case SEL_GT:
    case SEL_LT: {
      if (m.labels[col] < 0 || !m.label_num_ok[col]) return false;
      int64_t x = m.label_num[col];
      return r.op == SEL_GT ? x > r.num : x < r.num;
    }
    case SEL_NODE_EQ: return (int64_t)i == r.num;
    case SEL_NODE_NE: return (int64_t)i != r.num;
    case SEL_TRUE: return true;
    default: return false;
  }
}
__device__ bool term_match(const MirrorView& m, const uint8_t* base, const PodDesc& d, const SelTerm& t, int i) {
  if (t.parse_err) return false;
  const SelReq* reqs = at<SelReq>(base, d.req_off) + t.req_off;
  for (int k = 0; k < t.nreq; ++k)
    if (!req_match(m, base, d, reqs[k], i)) return false;
  return true;
}
__device__ bool prog_any(const MirrorView& m, const uint8_t* base, const PodDesc& d, SelProg p, int i) {
  const SelTerm* terms = at<SelTerm>(base, p.term_off);
  for (int k = 0; k < p.nterm; ++k)
    if (term_match(m, base, d, terms[k], i)) return true;
  return false;
}
__device__ int64_t prog_weight(const MirrorView& m, const uint8_t* base, const PodDesc& d, SelProg p, int i) {
  const SelTerm* terms = at<SelTerm>(base, p.term_off);
  int64_t s = 0;
  for (int k = 0; k < p.nterm; ++k)
    if (term_match(m, base, d, terms[k], i)) s += terms[k].weight;
  return s;
}


__device__ __forceinline__ int32_t node_label(const MirrorView& m, int32_t slot, int i) {
  return m.labels[(size_t)slot * (size_t)m.cap + (size_t)i];
}
// RequiredNodeAffinity.Match of the pod's own nodeSelector + required terms (nodeaffinity.go:323-333)
__device__ __forceinline__ bool required_na_match(const MirrorView& m, const uint8_t* base, const PodDesc& d, int i) {
  if ((d.flags & DF_HAS_SELECTOR) && !prog_any(m, base, d, d.na_selector, i)) return false;
  if ((d.flags & DF_HAS_REQUIRED_NA) && !prog_any(m, base, d, d.na_required, i)) return false;
  return true;
}
// FindMatchingUntoleratedTaint with DoNotScheduleTaintsFilterFunc (NoSchedule / NoExecute)
__device__ __forceinline__ bool untolerated_noschedule(const MirrorView& m, const uint8_t* base, const PodDesc& d,
                                                       int i) {
  const uint32_t lo = m.taint_off[i], hi = m.taint_off[i + 1];
  for (uint32_t q = lo; q < hi; ++q)
    if (bit(base, d.untol_ns_off, m.taint_ids[q], d.n_taint_words)) return true;
  return false;
}
// nodeLabelsMatchSpreadConstraints + matchNodeInclusionPolicies per constraint
// (podtopologyspread/common.go:43-80): bit c set if node i counts for constraint c
// need_all = false: requireAllTopologies off (system-default scoring, scoring.go:171-174), every node counts
__device__ __forceinline__ uint32_t pts_eligible(const MirrorView& m, const uint8_t* base, const PodDesc& d,
                                                 const PtsCons* cs, int32_t n, int i, bool need_all = true) {
  if (need_all)
    for (int32_t c = 0; c < n; ++c)
      if (node_label(m, cs[c].slot, i) < 0) return 0u;
  int na = -1, tn = -1;
  uint32_t bits = 0;
  for (int32_t c = 0; c < n; ++c) {
    if (cs[c].aff_honor) {
      if (na < 0) na = required_na_match(m, base, d, i) ? 1 : 0;
      if (!na) continue;
    }
    if (cs[c].taint_honor) {
      if (tn < 0) tn = untolerated_noschedule(m, base, d, i) ? 1 : 0;
      if (tn) continue;
    }
    bits |= 1u << c;
  }
  return bits;
}

// PodTopologySpread PreScore's domain of node i for ScheduleAnyway constraint c: the key's value, or
// with DF_PTS_ANYTOPO the "" domain of a node without the key (node.Labels[key] == "", scoring.go:95-106,
// 175-181); -1 otherwise
__device__ __forceinline__ int32_t pts_domain(const MirrorView& m, const PtsCons& c, int i) {
  const int32_t v = node_label(m, c.slot, i);
  return v >= 0 ? v : c.absent;
}
// a feasible node PreScore ignores (IgnoredNodes, scoring.go:82-88): some key missing, requireAllTopologies on
__device__ __forceinline__ bool pts_ignored(const MirrorView& m, const PodDesc& d, const PtsCons* cs, int i) {
  if (d.flags & DF_PTS_ANYTOPO) return false;
  bool ignored = false;
  for (int32_t c = 0; c < d.n_ptss; ++c) ignored |= node_label(m, cs[c].slot, i) < 0;
  return ignored;
}

__device__ __forceinline__ bool term_matches_pod(const int32_t* sp, const IpaTerm& t, int32_t ns,
                                                 const unsigned long long* lbl, int32_t n) {
  // AffinityTerm.Matches(pod, nil) for the incoming pod's (namespace-merged) terms (types.go:391-396)
  return (t.all_ns || id_in(sp + t.ns_off, t.ns_cnt, ns)) && lsel_match(sp + t.sel, lbl, n);
}

}  // namespace ksg
