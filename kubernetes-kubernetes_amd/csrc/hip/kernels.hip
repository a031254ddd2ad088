// kernels.hip -- per-pod node evaluation on gfx950 (CDNA4, wave64).
//
// One pod is evaluated by two launches over the snapshot's nodes (one thread per node,
// 256-thread blocks = 4 waves):
//
//   k_filter_score  : RunFilterPlugins for every node (framework/runtime/framework.go:1105-1138)
//                     in the default filter order, the raw Score of every active plugin for
//                     the feasible nodes (framework.go:1378-1402), the feasibility bitmask by
//                     wave ballots, per-block feasible counts, and per-plugin max/min of the
//                     raw scores that a NormalizeScore needs (block reduction + one atomic).
//   k_select        : NormalizeScore + weight + sum (framework.go:1409-1452) for every feasible
//                     node, the node's position in the feasible list (global prefix of the
//                     per-block counts + ballot popcounts), the packed (TotalScore, heap
//                     pre-order key) max that reproduces heap.Init+Pop (schedule_one.go:
//                     1054-1085), and -- in the last block to arrive -- the winner lookup and
//                     the device-side AssumePod (NodeInfo.update, framework/types.go:445-468).
//
// Integer arithmetic is int64 with truncating division as in Go; the two FP64 paths
// (BalancedAllocation, RequestedToCapacityRatio rounding) are compiled with
// -ffp-contract=off so no a*b+c is fused (Go/amd64 never fuses).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace ksg {

// ---- resources --------------------------------------------------------------------------------
// The node columns every default-plugin pod reads, loaded once at kernel entry (independent of the
// pod descriptor, so the loads are in flight while the descriptor's scalar loads resolve).
struct NodeCore {
  int64_t acpu, amem, aeph, rcpu, rmem, reph, nzcpu, nzmem;
  int32_t apods, npods;
  uint32_t flags, tlo, thi, ilo, ihi;  // taint and image CSR ranges
};
__device__ __forceinline__ NodeCore load_core(const MirrorView& m, int i) {
  NodeCore c;
  c.acpu = m.alloc_cpu[i];
  c.amem = m.alloc_mem[i];
  c.aeph = m.alloc_eph[i];
  c.rcpu = m.req_cpu[i];
  c.rmem = m.req_mem[i];
  c.reph = m.req_eph[i];
  c.nzcpu = m.nz_cpu[i];
  c.nzmem = m.nz_mem[i];
  c.apods = m.alloc_pods[i];
  c.npods = m.num_pods[i];
  c.flags = m.flags[i];
  c.tlo = m.taint_off[i];
  c.thi = m.taint_off[i + 1];
  c.ilo = m.img_off[i];
  c.ihi = m.img_off[i + 1];
  return c;
}

__device__ __forceinline__ void node_res(const MirrorView& m, const NodeCore& nc, const ScoreRes& r, int i,
                                         bool useRequested, int64_t* alloc, int64_t* allocated) {
  // resource_allocation.go:198-232 calculateResourceAllocatableRequest
  switch (r.kind) {
    case RES_CPU: *alloc = nc.acpu; *allocated = useRequested ? nc.rcpu : nc.nzcpu; break;
    case RES_MEM: *alloc = nc.amem; *allocated = useRequested ? nc.rmem : nc.nzmem; break;
    case RES_EPH: *alloc = nc.aeph; *allocated = nc.reph; break;
    case RES_SCALAR: {
      size_t c = (size_t)r.slot * (size_t)m.cap + (size_t)i;
      *alloc = m.scalar_alloc[c];
      *allocated = m.scalar_req[c];
      break;
    }
    default: *alloc = 0; *allocated = 0;
  }
}

__device__ int64_t rtcr_shape(const uint8_t* base, const PodDesc& d, int64_t p) {  // helper/shape_score.go:39-51
  const int64_t* s = at<int64_t>(base, d.rtcr_off);
  for (int k = 0; k < d.n_rtcr; ++k)
    if (p <= s[2 * k]) {
      if (k == 0) return s[1];
      return s[2 * k - 1] + go_div((s[2 * k + 1] - s[2 * k - 1]) * (p - s[2 * k - 2]), s[2 * k] - s[2 * k - 2]);
    }
  return s[2 * d.n_rtcr - 1];
}

// NodeResourcesFit.Score (fit.go:737-755 -> resource_allocation.go:138-193 + scorer)
__device__ int64_t fit_score(const MirrorView& m, const NodeCore& nc, const uint8_t* base, const PodDesc& d, int i) {
  const ScoreRes* res = at<ScoreRes>(base, d.fit_res_off);
  int64_t nodeScore = 0, weightSum = 0;
  for (int k = 0; k < d.n_fit_res; ++k) {
    const ScoreRes r = res[k];
    if (r.kind == RES_SKIP) continue;
    int64_t alloc, allocated;
    node_res(m, nc, r, i, false, &alloc, &allocated);
    if (alloc == 0) continue;
    int64_t requested = allocated + r.pod_req;
    int64_t s;
    if (d.fit_strategy == 0) {  // least_allocated.go:52-61
      s = requested > alloc ? 0 : go_div((alloc - requested) * 100, alloc);
    } else if (d.fit_strategy == 1) {  // most_allocated.go:55-65
      int64_t rq = requested > alloc ? alloc : requested;
      s = go_div(rq * 100, alloc);
    } else {  // requested_to_capacity_ratio.go:30-36
      s = requested > alloc ? rtcr_shape(base, d, 100) : rtcr_shape(base, d, go_div(requested * 100, alloc));
      if (s <= 0) continue;
    }
    nodeScore += s * r.weight;
    weightSum += r.weight;
  }
  if (weightSum == 0) return 0;
  if (d.fit_strategy == 2) return (int64_t)round((double)nodeScore / (double)weightSum);
  return go_div(nodeScore, weightSum);
}

// balanced_allocation.go:220-254, without private arrays (a per-lane array would live in scratch,
// and a kernel with scratch waits for the runtime's scratch grant before its first wave starts).
// Fraction f_k of resource k, or false when the node's allocatable is 0 (the reference skips it);
// recomputed in the variance pass, bit-identically.
__device__ __forceinline__ bool bal_frac(const MirrorView& m, const NodeCore& nc, const ScoreRes& r, int i, bool with,
                                         double* f) {
  if (r.kind == RES_SKIP) return false;
  int64_t alloc, al;
  node_res(m, nc, r, i, true, &alloc, &al);
  if (alloc == 0) return false;
  double x = (double)(with ? al + r.pod_req : al) / (double)alloc;
  if (x > 1) x = 1;
  *f = x;
  return true;
}

__device__ int64_t balanced_score(const MirrorView& m, const NodeCore& nc, const ScoreRes* res, int n, int i,
                                  bool with) {
  int nf = 0;
  double total = 0, f0 = 0, f1 = 0;
  for (int k = 0; k < n; ++k) {
    double f;
    if (!bal_frac(m, nc, res[k], i, with, &f)) continue;
    total = total + f;
    if (nf == 0) f0 = f;
    else if (nf == 1) f1 = f;
    ++nf;
  }
  double sd = 0.0;
  if (nf == 2) {
    sd = fabs((f0 - f1) / 2);
  } else if (nf > 2) {
    double mean = total / (double)nf;
    double sum = 0;
    for (int k = 0; k < n; ++k) {
      double f;
      if (!bal_frac(m, nc, res[k], i, with, &f)) continue;
      double dd = f - mean;
      double sq = dd * dd;
      sum = sum + sq;
    }
    sd = sqrt(sum / (double)nf);
  }
  double om = 1 - sd;
  double sc = om * 100.0;
  return (int64_t)sc;
}

__device__ int64_t balanced_alloc_score(const MirrorView& m, const NodeCore& nc, const uint8_t* base,
                                        const PodDesc& d, int i) {
  const ScoreRes* res = at<ScoreRes>(base, d.bal_res_off);
  const int64_t with = balanced_score(m, nc, res, d.n_bal_res, i, true);
  const int64_t without = balanced_score(m, nc, res, d.n_bal_res, i, false);
  return 100 / 2 + (100 / 2 + with - without) / 2;  // balanced_allocation.go:204-218
}

// image_locality.go:70-152 (per-image scaled scores precomputed per pod on the host)
__device__ __forceinline__ int64_t image_score_range(const MirrorView& m, const uint8_t* base, const PodDesc& d,
                                                     uint32_t lo, uint32_t hi) {
  const ImageTerm* terms = at<ImageTerm>(base, d.img_off);
  int64_t sum = 0;
  for (int k = 0; k < d.n_img; ++k) {
    const uint32_t want = (uint32_t)terms[k].image;
    bool on = false;
    for (uint32_t q = lo; q < hi; ++q) on |= m.img_ids[q] == want;
    if (on) sum += terms[k].scaled * terms[k].mult;
  }
  const int64_t mb = 1024 * 1024, minT = 23 * mb, maxT = 1000 * mb * d.img_count;
  if (sum < minT) sum = minT;
  else if (sum > maxT) sum = maxT;
  return go_div(100 * (sum - minT), maxT - minT);
}
__device__ int64_t image_score(const MirrorView& m, const uint8_t* base, const PodDesc& d, int i) {
  return image_score_range(m, base, d, m.img_off[i], m.img_off[i + 1]);
}

// ---- diagnostic build (make DIAG=1 -> lib/libksg_diag.so): per-step stamps inside eval_node ----------
#ifdef KSG_DIAG
__device__ unsigned long long* g_diag;  // [64] slots, workgroup 0 lane 0, last pod wins
__shared__ unsigned long long s_diag[24];  // stamps land in LDS (a global store's ack would skew the next one)
#define DIAG_STAMP(k)                                                                       \
  do {                                                                                      \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                             \
    if (blockIdx.x == 0 && threadIdx.x == 0) s_diag[k] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)
#define DIAG_FLUSH()                                                                        \
  do {                                                                                      \
    if (g_diag && blockIdx.x == 0 && threadIdx.x == 0)                                      \
      for (int k_ = 0; k_ < 24; ++k_) g_diag[k_] = s_diag[k_];                              \
  } while (0)
#else
#define DIAG_FLUSH() \
  do {               \
  } while (0)
#define DIAG_STAMP(k) \
  do {                \
  } while (0)
#endif

// ---- filters ------------------------------------------------------------------------------------
// Where PodTopologySpread / InterPodAffinity read the pod's per-domain counts.  The launch path:
// k_aggregate's arena in HBM and its PodStats reductions.  k_agg_loop: AggTopo (LDS).
struct ArenaTopo {
  const PodStats* ps;
  const unsigned long long* arena;
  __device__ __forceinline__ int64_t cnt(int32_t hist_base, int32_t, int32_t v, int) const {
    return (int64_t)arena[hist_base + v];
  }
  __device__ __forceinline__ int64_t pmin(int c) const { return ps->pts_min[c]; }
  __device__ __forceinline__ uint32_t pndom(int c) const { return ps->pts_ndom[c]; }
  __device__ __forceinline__ uint32_t any() const { return ps->ipa_any; }
};

template <typename Topo>
__device__ __forceinline__ uint32_t topo_filters(const MirrorView& m, const uint8_t* base, const PodDesc& d, int i,
                                                 const Topo& tp, int ls);
// Returns the packed Filter status of node i (0 = Success), first failing plugin in the
// RunFilterPlugins order wins.  *raw_taint gets the PreferNoSchedule count while the taint
// list is in registers.  ls: node i's slot in the caller's topology view (k_agg_loop).
template <typename Topo>
__device__ uint32_t run_filters(const MirrorView& m, const NodeCore& nc, const uint8_t* base, const PodDesc& d, int i,
                                int64_t* raw_taint, const Topo& tp, int ls) {
  const uint32_t fm = d.filter_mask;
  // NodeUnschedulable (node_unschedulable.go:125-143)
  if ((fm >> P_UNSCHED) & 1u)
    if ((nc.flags & 1u) && !(d.flags & DF_TOLERATES_UNSCHED)) return pack_status(C_UU, P_UNSCHED, KSG_R_UNSCHEDULABLE);
  // NodeName (node_name.go:67-83)
  if ((fm >> P_NODENAME) & 1u)
    if (d.node_name != -1 && d.node_name != i) return pack_status(C_UU, P_NODENAME, KSG_R_NODE_NAME);
  // TaintToleration (taint_toleration.go:102-116, 163-196)
  {
    const uint32_t lo = nc.tlo, hi = nc.thi;
    bool untol = false;
    int64_t cnt = 0;
    for (uint32_t q = lo; q < hi; ++q) {
      uint32_t id = m.taint_ids[q];
      untol |= bit(base, d.untol_ns_off, id, d.n_taint_words);
      cnt += bit(base, d.intol_pns_off, id, d.n_taint_words) ? 1 : 0;
    }
    *raw_taint = cnt;
    if (((fm >> P_TAINT) & 1u) && untol) return pack_status(C_UU, P_TAINT, KSG_R_TAINT);
  }
  // NodeAffinity (node_affinity.go:207-228)
  if ((fm >> P_NA) & 1u) {
    if ((d.flags & DF_HAS_ADDED_NA) && !prog_any(m, base, d, d.na_added, i))
      return pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_ENFORCED);
    if ((d.flags & DF_HAS_SELECTOR) && !prog_any(m, base, d, d.na_selector, i))
      return pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_POD);
    if ((d.flags & DF_HAS_REQUIRED_NA) && !prog_any(m, base, d, d.na_required, i))
      return pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_POD);
  }
  // NodePorts (node_ports.go:150-176 -> HostPortInfo.CheckConflict, precompiled per port id)
  if ((fm >> P_PORTS) & 1u) {
    const uint32_t* slots = m.ports + (size_t)i * m.port_slots;
    for (int s = 0; s < m.port_slots; ++s) {
      uint32_t pid = slots[s];
      if (pid != 0xffffffffu && bit(base, d.port_conflict_off, pid, d.n_port_words))
        return pack_status(C_UNSCHED, P_PORTS, KSG_R_NODE_PORTS);
    }
  }
  // NodeResourcesFit (fit.go:593-734 fitsRequest)
  if ((fm >> P_FIT) & 1u) {
    uint32_t reasons = 0;
    bool unresolvable = false;
    if ((int64_t)nc.npods + 1 > (int64_t)nc.apods) reasons |= KSG_R_TOO_MANY_PODS;
    if (d.fit_any) {
      const int64_t acpu = nc.acpu, amem = nc.amem, aeph = nc.aeph;
      if (d.req_cpu > 0 && d.req_cpu > acpu - nc.rcpu) {
        reasons |= KSG_R_INSUFFICIENT_CPU;
        unresolvable |= d.req_cpu > acpu;
      }
      if (d.req_mem > 0 && d.req_mem > amem - nc.rmem) {
        reasons |= KSG_R_INSUFFICIENT_MEMORY;
        unresolvable |= d.req_mem > amem;
      }
      if (d.req_eph > 0 && d.req_eph > aeph - nc.reph) {
        reasons |= KSG_R_INSUFFICIENT_EPHEMERAL;
        unresolvable |= d.req_eph > aeph;
      }
      const ScalarReq* sr = at<ScalarReq>(base, d.scalar_off);
      for (int k = 0; k < d.n_scalar; ++k) {
        size_t c = (size_t)sr[k].slot * (size_t)m.cap + (size_t)i;
        int64_t a = m.scalar_alloc[c];
        if (sr[k].qty > a - m.scalar_req[c]) {
          reasons |= KSG_R_INSUFFICIENT_SCALAR;
          unresolvable |= sr[k].qty > a;
        }
      }
    }
    if (reasons) return pack_status(unresolvable ? C_UU : C_UNSCHED, P_FIT, reasons);
  }
  return topo_filters(m, base, d, i, tp, ls);
}

// PodTopologySpread + InterPodAffinity Filter of node i (the last two in the RunFilterPlugins order)
template <typename Topo>
__device__ __forceinline__ uint32_t topo_filters(const MirrorView& m, const uint8_t* base, const PodDesc& d, int i,
                                                 const Topo& tp, int ls) {
  const uint32_t fm = d.filter_mask;
  // PodTopologySpread (podtopologyspread/filtering.go:314-359) against k_aggregate's counts
  if ((fm >> P_PTS) & 1u) {
    const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
    for (int32_t c = 0; c < d.n_ptsf; ++c) {
      const int32_t v = node_label(m, cs[c].slot, i);
      if (v < 0) return pack_status(C_UU, P_PTS, KSG_R_PTS_MISSING_LABEL);
      const int64_t minMatch = (int64_t)tp.pndom(c) < (int64_t)cs[c].min_domains ? 0 : tp.pmin(c);
      const int64_t matchNum = tp.cnt(cs[c].hist_base, cs[c].lref, v, ls);
      if (matchNum + cs[c].self_match - minMatch > (int64_t)cs[c].max_skew)
        return pack_status(C_UNSCHED, P_PTS, KSG_R_PTS_SKEW);
    }
  }
  // InterPodAffinity (interpodaffinity/filtering.go:364-444)
  if ((fm >> P_IPA) & 1u) {
    const IpaTerm* ra = at<IpaTerm>(base, d.raff_off);
    bool podsExist = true;  // satisfyPodAffinity :394-420
    for (int32_t k = 0; k < d.n_raff; ++k) {
      const int32_t v = node_label(m, ra[k].slot, i);
      if (v < 0) return pack_status(C_UU, P_IPA, KSG_R_IPA_AFFINITY);
      if (tp.cnt(ra[k].hist_base, ra[k].lref, v, ls) <= 0) podsExist = false;
    }
    const uint32_t any = tp.any();
    if (!podsExist && !((any & 1u) == 0 && (d.ipa_flags & IPA_SELF_ALL)))
      return pack_status(C_UU, P_IPA, KSG_R_IPA_AFFINITY);
    if (any & 2u) {  // satisfyPodAntiAffinity :379-391
      const IpaTerm* rn = at<IpaTerm>(base, d.ranti_off);
      for (int32_t k = 0; k < d.n_ranti; ++k) {
        const int32_t v = node_label(m, rn[k].slot, i);
        if (v >= 0 && tp.cnt(rn[k].hist_base, rn[k].lref, v, ls) > 0)
          return pack_status(C_UNSCHED, P_IPA, KSG_R_IPA_ANTI_AFFINITY);
      }
    }
    if (any & 4u) {  // satisfyExistingPodsAntiAffinity :364-376
      const KeyHist* ek = at<KeyHist>(base, d.exkeys_off);
      for (int32_t k = 0; k < d.n_exkeys; ++k) {
        const int32_t v = node_label(m, ek[k].slot, i);
        if (v >= 0 && tp.cnt(ek[k].base, ek[k].lref, v, ls) > 0)
          return pack_status(C_UNSCHED, P_IPA, KSG_R_IPA_EXISTING_ANTI);
      }
    }
  }
  return 0;
}

// ---- wave/block reductions ------------------------------------------------------------------------
// DPP scan steps (row_shr 1/2/4/8, row_bcast 15/31; disabled or out-of-row lanes contribute 0, the
// identity of an unsigned max or sum): the wave's result ends in lane 63.  All 64 lanes active.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, false);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ unsigned long long dpp_max_step(unsigned long long v) {
  const unsigned long long w = ((unsigned long long)dpp_u32<kCtrl, kRowMask>((uint32_t)(v >> 32)) << 32) |
                               dpp_u32<kCtrl, kRowMask>((uint32_t)v);
  return w > v ? w : v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  v = dpp_max_step<0x111, 0xf>(v);
  v = dpp_max_step<0x112, 0xf>(v);
  v = dpp_max_step<0x114, 0xf>(v);
  v = dpp_max_step<0x118, 0xf>(v);
  v = dpp_max_step<0x142, 0xa>(v);
  v = dpp_max_step<0x143, 0xc>(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_u32<0x111, 0xf>(v);
  v += dpp_u32<0x112, 0xf>(v);
  v += dpp_u32<0x114, 0xf>(v);
  v += dpp_u32<0x118, 0xf>(v);
  v += dpp_u32<0x142, 0xa>(v);
  v += dpp_u32<0x143, 0xc>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// =====================================================================================================
// per-node evaluation (shared by k_filter_score and the persistent k_sched_loop)
// =====================================================================================================
struct NodeEval {
  uint32_t st;      // packed Filter status (0 = feasible)
  bool pts;         // feasible and not ignored by PodTopologySpread scoring
  int64_t rt, rna, ripa;  // raw TaintToleration / NodeAffinity / InterPodAffinity scores
  int64_t fixed;    // weighted sum of the non-normalising scores (Fit, BalancedAllocation, ImageLocality)
};

// RunFilterPlugins + the raw Score of every active plugin for node i (framework.go:1105-1138,
// 1378-1402).  kStore: write the node's status word (evaluation output), the weighted sum of the
// non-normalising scores and the raw scores the normalising plugins need to the batch scratch
// (the launch path's k_select reads them back; the persistent loop keeps them in registers).
template <bool kStore>
__device__ __forceinline__ NodeEval eval_node(const MirrorView& m, const BatchView& b, const uint8_t* base, const PodDesc& d, int pod,
                              int i, bool valid) {
  const bool eval = (d.flags & DF_EVAL_OUT) != 0;
  NodeEval r{0u, false, 0, 0, 0, 0};
  uint32_t st = 0;
  int64_t raw_taint = 0;
  NodeCore nc{};
  DIAG_STAMP(0);
  if (valid) nc = load_core(m, i);
  DIAG_STAMP(1);
  if (valid) {
    if (d.flags & DF_PREFILTER_REJECT) {
      st = pack_status((uint32_t)d.prefilter_code, (uint32_t)d.prefilter_plugin & 15u, KSG_R_PREFILTER);
    } else if (d.flags & DF_SUBSET) {
      // PreFilterResult.NodeNames: nodes outside are UnschedulableAndUnresolvable (schedule_one.go:671-682)
      const int32_t* sub = at<int32_t>(base, d.subset_off);
      bool in = false;
      for (int k = 0; k < d.subset_cnt; ++k) in |= sub[k] == i;
      // (a nominated node outside the list that failed alone keeps that status: NodeToStatus holds it, the
      // absent-node status is only the default, schedule_one.go:657-682; it fails again here, never feasible)
      if constexpr (kStore)  // (the launch path: nominated pods never run in the persistent loops)
        in |= (d.flags & DF_NOMINATED) && b.stats[pod].nom_failed == (uint32_t)i + 1u;
      st = in ? 0u : pack_status(C_UU, 15u, KSG_R_PREFILTER);
    }
    if (st == 0) {
      uint32_t f = run_filters(m, nc, base, d, i, &raw_taint, ArenaTopo{b.stats + pod, b.arena}, 0);
      if (d.flags & DF_ALL_FEASIBLE)  // plugin-eval mode: the caller's node list is the feasible list
        f = ((d.flags & DF_NODE_LIST) && !bit(base, d.node_list_off, (uint32_t)i, (m.n + 31) / 32))
                ? pack_status(C_UU, 15u, 0u)
                : 0u;
      st = f;
    }
    if (kStore && eval) b.status[i] = st;
  }
  DIAG_STAMP(2);
  r.st = valid ? st : 1u;
  if (!valid || st != 0) return r;

  // raw scores of the feasible node (framework.go:1378-1402)
  int64_t fixed = 0;
  const uint32_t sm = d.score_mask;
  const size_t cap = (size_t)m.cap;
  if ((sm >> P_TAINT) & 1u) r.rt = raw_taint;
  if ((sm >> P_NA) & 1u) {
    int64_t sc = 0;
    if (d.flags & DF_HAS_ADDED_PREF) sc += prog_weight(m, base, d, d.na_added_pref, i);
    if (d.flags & DF_HAS_PREF_NA) sc += prog_weight(m, base, d, d.na_preferred, i);
    r.rna = sc;
  }
  int64_t rf = 0, rb = 0, ri = 0;
  DIAG_STAMP(3);
  if ((sm >> P_FIT) & 1u) { rf = fit_score(m, nc, base, d, i); fixed += rf * d.weight[P_FIT]; }
  DIAG_STAMP(4);
  if ((sm >> P_BAL) & 1u) { rb = balanced_alloc_score(m, nc, base, d, i); fixed += rb * d.weight[P_BAL]; }
  DIAG_STAMP(5);
  if ((sm >> P_IMG) & 1u) { ri = image_score(m, base, d, i); fixed += ri * d.weight[P_IMG]; }
  DIAG_STAMP(6);
  r.fixed = fixed;
  if (kStore) {
    b.fixed[i] = fixed;
    if ((sm >> P_TAINT) & 1u) b.raw[P_TAINT * cap + i] = r.rt;
    if ((sm >> P_NA) & 1u) b.raw[P_NA * cap + i] = r.rna;
  }
  if (kStore && eval) {
    b.raw[P_FIT * cap + i] = rf;
    b.raw[P_BAL * cap + i] = rb;
    b.raw[P_IMG * cap + i] = ri;
  }
  if ((sm >> P_IPA) & 1u) {  // InterPodAffinity.Score (interpodaffinity/scoring.go:240-255)
    const KeyHist* tk = at<KeyHist>(base, d.topokeys_off);
    int64_t sc = 0;
    for (int32_t k = 0; k < d.n_topokeys; ++k) {
      const int32_t v = node_label(m, tk[k].slot, i);
      if (v >= 0) sc += (int64_t)b.arena[tk[k].base + v];
    }
    r.ripa = sc;
    if (kStore) b.raw[P_IPA * cap + i] = sc;
  }
  // PodTopologySpread PreScore over the feasible list: ignored nodes and per-constraint domain
  // counts feed the normalising weights (podtopologyspread/scoring.go:61-115)
  if ((sm >> P_PTS) & 1u) {
    const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
    if (!pts_ignored(m, d, cs, i)) {
      r.pts = true;
      PodStats* ps = b.stats + pod;
      // a cut feasible list (DF_SAMPLE): k_sample_apply marks the kept nodes' domains instead
      for (int32_t c = 0; c < ((d.flags & DF_SAMPLE) ? 0 : d.n_ptss); ++c) {
        if (cs[c].hostname) continue;
        mark_domains(b.arena + cs[c].pres_base, pts_domain(m, cs[c], i), true, &ps->pts_distinct[c]);
      }
    }
  }
  DIAG_STAMP(7);
  return r;
}

// ---- the pod program in LDS ------------------------------------------------------------------------
// Every node thread reads the same PodDesc fields and blob arrays, often behind data-dependent
// branches; read from global memory they are re-fetched at L2 latency after every store the
// compiler cannot prove disjoint.  Programs up to kBlobLds bytes are staged in LDS once per
// workgroup (16 B per thread per step); larger ones run from global memory (kLds = false).
__device__ __forceinline__ void stage_blob(const uint8_t* g, uint32_t bytes, uint8_t* lds) {
  const uint4* src = reinterpret_cast<const uint4*>(g);
  uint4* dst = reinterpret_cast<uint4*>(lds);
  for (uint32_t o = threadIdx.x; o < bytes / 16u; o += kBlock) dst[o] = src[o];
}

// =====================================================================================================
// eval_node_fast -- the default-plugin shape, straight-line (DF_FAST, set by the host compiler)
// =====================================================================================================
// Pods whose NodeResourcesFit scores exactly cpu+memory (LeastAllocated / MostAllocated), whose
// BalancedAllocation uses cpu+memory, that request no extended resources, have no PreFilterResult
// subset and no image present in the cluster.  The pod's parameters are read from the LDS program
// once per pod into registers (PodFast); the node's filters and the two score chains are
// branch-light straight-line code the compiler can interleave.  Same arithmetic as the generic
// path (fit.go:647-734, least_allocated.go:30-61, most_allocated.go:55-65,
// balanced_allocation.go:204-254).
struct PodFast {
  uint32_t flags, fm, sm;
  int32_t node_name, n_taint_words, untol_off, intol_off, fit_any, most;
  int64_t req_cpu, req_mem, req_eph;
  int64_t fw_cpu, fw_mem, fpr_cpu, fpr_mem;  // Fit score: weights, pod requests (non-zero defaults)
  int64_t bpr_cpu, bpr_mem;                  // BalancedAllocation pod requests
  int64_t wt_fit, wt_bal;
};
__device__ __forceinline__ PodFast load_fast(const uint8_t* base, const PodDesc& d) {
  PodFast f;
  f.flags = d.flags;
  f.fm = d.filter_mask;
  f.sm = d.score_mask;
  f.node_name = d.node_name;
  f.n_taint_words = d.n_taint_words;
  f.untol_off = d.untol_ns_off;
  f.intol_off = d.intol_pns_off;
  f.fit_any = d.fit_any;
  f.most = d.fit_strategy == 1;
  f.req_cpu = d.req_cpu;
  f.req_mem = d.req_mem;
  f.req_eph = d.req_eph;
  const ScoreRes* fr = at<ScoreRes>(base, d.fit_res_off);
  const ScoreRes* br = at<ScoreRes>(base, d.bal_res_off);
  f.fw_cpu = fr[0].weight;
  f.fw_mem = fr[1].weight;
  f.fpr_cpu = fr[0].pod_req;
  f.fpr_mem = fr[1].pod_req;
  f.bpr_cpu = br[0].pod_req;
  f.bpr_mem = br[1].pod_req;
  f.wt_fit = d.weight[P_FIT];
  f.wt_bal = d.weight[P_BAL];
  return f;
}
// floor(a / b) for 0 <= a < 2^52, 0 < b < 2^52 (host-checked bounds): correctly rounded FP64
// quotient, truncated, fixed up by one with the exact remainder
__device__ __forceinline__ int64_t fdiv52(int64_t a, int64_t b) {
  int64_t q = (int64_t)((double)a / (double)b);
  const int64_t r = a - q * b;
  q -= r < 0 ? 1 : 0;
  q += r >= b ? 1 : 0;
  return q;
}
// 0 <= x < 2^52 as a double, exactly: the integer in the mantissa of 2^52, minus 2^52
__device__ __forceinline__ double u52_to_f64(int64_t x) {
  return __longlong_as_double(x | 0x4330000000000000ll) - 4503599627370496.0;
}
// floor(a / b) for 0 <= a <= 100 b, 0 < b, a < 2^52 (the Least/MostAllocated ratios and the
// weighted mean of Fit's scores): a * rcp(b) is within one of a / b, fixed up with the exact remainder
__device__ __forceinline__ int64_t qdiv100(int64_t a, int64_t b) {
  int32_t q = (int32_t)(u52_to_f64(a) * __builtin_amdgcn_rcp(u52_to_f64(b)));
  const int64_t r = a - (int64_t)q * b;
  q -= r < 0 ? 1 : 0;
  q += r >= b ? 1 : 0;
  return q;
}
// balanced_allocation.go:220-254 for the (cpu, memory) pair
__device__ __forceinline__ int64_t bal2(int64_t rc, int64_t ac, int64_t rm, int64_t am) {
  double f0 = ac != 0 ? (double)rc / (double)ac : 0.0;
  double f1 = am != 0 ? (double)rm / (double)am : 0.0;
  f0 = f0 > 1 ? 1 : f0;
  f1 = f1 > 1 ? 1 : f1;
  double sd = 0.0;
  if (ac != 0 && am != 0) sd = fabs((f0 - f1) / 2);
  const double om = 1 - sd;
  const double sc = om * 100.0;
  return (int64_t)sc;
}
// nc: node i's core columns -- loaded here (launch path) or held in registers by its owner (k_sched_loop)
// bal_wo: bal2 of the node without the pod (pod-independent: the loop keeps it per node)
// bal_with: bal2 of the node with the pod, when the caller already has it (else kNoBal)
constexpr int64_t kNoBal = INT64_MIN;
__device__ __forceinline__ NodeEval eval_core_fast(const MirrorView& m, const NodeCore& nc, int64_t bal_wo,
                                                   const PodFast& pf, const uint8_t* base, const PodDesc& d, int i,
                                                   int64_t bal_with = kNoBal) {
  NodeEval r{1u, false, 0, 0, 0, 0};
  DIAG_STAMP(9);
  bool untol = false;
  int64_t tcnt = 0;
  for (uint32_t q = nc.tlo; q < nc.thi; ++q) {
    const uint32_t id = m.taint_ids[q];
    untol |= bit(base, pf.untol_off, id, pf.n_taint_words);
    tcnt += bit(base, pf.intol_off, id, pf.n_taint_words) ? 1 : 0;
  }
  DIAG_STAMP(10);
  // Fit filter inputs (fit.go:650-699): independent of the filter order, computed up front
  const bool too_many = (int64_t)nc.npods + 1 > (int64_t)nc.apods;
  const bool ic = pf.fit_any && pf.req_cpu > 0 && pf.req_cpu > nc.acpu - nc.rcpu;
  const bool im = pf.fit_any && pf.req_mem > 0 && pf.req_mem > nc.amem - nc.rmem;
  const bool ie = pf.fit_any && pf.req_eph > 0 && pf.req_eph > nc.aeph - nc.reph;
  uint32_t st = 0;
  const uint32_t fm = pf.fm;
  if (((fm >> P_UNSCHED) & 1u) && (nc.flags & 1u) && !(pf.flags & DF_TOLERATES_UNSCHED)) {
    st = pack_status(C_UU, P_UNSCHED, KSG_R_UNSCHEDULABLE);
  } else if (((fm >> P_NODENAME) & 1u) && pf.node_name != -1 && pf.node_name != i) {
    st = pack_status(C_UU, P_NODENAME, KSG_R_NODE_NAME);
  } else if (((fm >> P_TAINT) & 1u) && untol) {
    st = pack_status(C_UU, P_TAINT, KSG_R_TAINT);
  } else {
    if ((fm >> P_NA) & 1u) {  // NodeAffinity (node_affinity.go:207-228), generic programs
      if ((pf.flags & DF_HAS_ADDED_NA) && !prog_any(m, base, d, d.na_added, i))
        st = pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_ENFORCED);
      else if ((pf.flags & DF_HAS_SELECTOR) && !prog_any(m, base, d, d.na_selector, i))
        st = pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_POD);
      else if ((pf.flags & DF_HAS_REQUIRED_NA) && !prog_any(m, base, d, d.na_required, i))
        st = pack_status(C_UU, P_NA, KSG_R_NODE_AFFINITY_POD);
    }
    if (st == 0 && ((fm >> P_PORTS) & 1u)) {  // NodePorts
      const uint32_t* slots = m.ports + (size_t)i * m.port_slots;
      for (int k = 0; k < m.port_slots; ++k) {
        const uint32_t pid = slots[k];
        if (pid != 0xffffffffu && bit(base, d.port_conflict_off, pid, d.n_port_words)) {
          st = pack_status(C_UNSCHED, P_PORTS, KSG_R_NODE_PORTS);
          break;
        }
      }
    }
    if (st == 0 && ((fm >> P_FIT) & 1u) && (too_many || ic || im || ie)) {
      const uint32_t reasons = (too_many ? KSG_R_TOO_MANY_PODS : 0u) | (ic ? KSG_R_INSUFFICIENT_CPU : 0u) |
                               (im ? KSG_R_INSUFFICIENT_MEMORY : 0u) | (ie ? KSG_R_INSUFFICIENT_EPHEMERAL : 0u);
      const bool unres = (ic && pf.req_cpu > nc.acpu) || (im && pf.req_mem > nc.amem) || (ie && pf.req_eph > nc.aeph);
      st = pack_status(unres ? C_UU : C_UNSCHED, P_FIT, reasons);
    }
  }
  r.st = st;
  DIAG_STAMP(11);
  if (st != 0) return r;
  const uint32_t sm = pf.sm;
  r.rt = ((sm >> P_TAINT) & 1u) ? tcnt : 0;
  if ((sm >> P_NA) & 1u) {
    int64_t sc = 0;
    if (pf.flags & DF_HAS_ADDED_PREF) sc += prog_weight(m, base, d, d.na_added_pref, i);
    if (pf.flags & DF_HAS_PREF_NA) sc += prog_weight(m, base, d, d.na_preferred, i);
    r.rna = sc;
  }
  int64_t fixed = 0;
  DIAG_STAMP(12);
  if ((sm >> P_FIT) & 1u) {  // resource_allocation.go:138-165 with cpu (NonZeroRequested) and memory
    const int64_t qc = nc.nzcpu + pf.fpr_cpu, qm = nc.nzmem + pf.fpr_mem;
    int64_t sc, smm;
    if (pf.most) {  // most_allocated.go:55-65
      sc = nc.acpu > 0 ? qdiv100((qc > nc.acpu ? nc.acpu : qc) * 100, nc.acpu) : 0;
      smm = nc.amem > 0 ? qdiv100((qm > nc.amem ? nc.amem : qm) * 100, nc.amem) : 0;
    } else {  // least_allocated.go:52-61
      sc = nc.acpu > 0 && qc <= nc.acpu ? qdiv100((nc.acpu - qc) * 100, nc.acpu) : 0;
      smm = nc.amem > 0 && qm <= nc.amem ? qdiv100((nc.amem - qm) * 100, nc.amem) : 0;
    }
    const int64_t ws = (nc.acpu != 0 ? pf.fw_cpu : 0) + (nc.amem != 0 ? pf.fw_mem : 0);
    const int64_t num = (nc.acpu != 0 ? sc * pf.fw_cpu : 0) + (nc.amem != 0 ? smm * pf.fw_mem : 0);
    fixed += (ws == 0 ? 0 : qdiv100(num, ws)) * pf.wt_fit;  // weights > 0: num <= 100 ws
  }
  DIAG_STAMP(13);
  if ((sm >> P_BAL) & 1u) {  // balanced_allocation.go:204-218 (Requested, useRequested=true)
    const int64_t with =
        bal_with != kNoBal ? bal_with : bal2(nc.rcpu + pf.bpr_cpu, nc.acpu, nc.rmem + pf.bpr_mem, nc.amem);
    fixed += (100 / 2 + (100 / 2 + with - bal_wo) / 2) * pf.wt_bal;
  }
  // ImageLocality: no image of the pod present anywhere (n_img == 0) scores 0 on every node
  if (((sm >> P_IMG) & 1u) && d.n_img > 0) fixed += image_score_range(m, base, d, nc.ilo, nc.ihi) * d.weight[P_IMG];
  r.fixed = fixed;
  DIAG_STAMP(14);
  return r;
}
__device__ NodeEval eval_node_fast(const MirrorView& m, const PodFast& pf, const uint8_t* base, const PodDesc& d,
                                   int i, bool valid) {
  if (!valid) return NodeEval{1u, false, 0, 0, 0, 0};
  DIAG_STAMP(8);
  const NodeCore nc = load_core(m, i);
  return eval_core_fast(m, nc, bal2(nc.rcpu, nc.acpu, nc.rmem, nc.amem), pf, base, d, i);
}

// A pod k_ob_hint placed on the stored heap's next node (OpportunisticBatching), or k_nominated on its nominated
// node, skips the full evaluation (every launch of its per-pod path returns at once; k_select still clears its
// histograms)
__device__ __forceinline__ bool ob_skip(const BatchView& b, int pod) {
  const PodDesc* d = reinterpret_cast<const PodDesc*>(b.descs + b.desc_off[pod]);
  return (d->flags & DF_EARLY) && b.stats[pod].ob_done;
}

// =====================================================================================================
// k_filter_score
// =====================================================================================================
template <bool kLds>
__global__ __launch_bounds__(kBlock) void k_filter_score(MirrorView m, BatchView b, int pod, int blk0) {
  __shared__ __align__(16) uint8_t s_blob[kLds ? kBlobLds : 16];
  if (ob_skip(b, pod)) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  if constexpr (kLds) {
    stage_blob(base, reinterpret_cast<const PodDesc*>(base)->blob_bytes, s_blob);
    __syncthreads();
    base = s_blob;
  }
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  const int blk = blk0 + (int)blockIdx.x;  // node-sharded launches cover blocks [blk0, blk0 + gridDim.x)
  const int i = blk * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const NodeEval ne = eval_node<true>(m, b, base, d, pod, i, i < m.n);
  const bool feas = ne.st == 0;
  const unsigned long long ballot = __ballot(feas);
  if (lane == 0) b.fmask[(size_t)blk * (kBlock / 64) + wave] = ballot;
  const uint32_t sm = d.score_mask;

  // per-block feasible count + per-plugin max (and IPA min) of the normalising plugins' raw scores
  __shared__ uint32_t s_cnt[kBlock / 64], s_pts[kBlock / 64];
  __shared__ unsigned long long s_max[3][kBlock / 64], s_min[kBlock / 64];
  unsigned long long mt = feas ? enc_i64(ne.rt) : 0ull;
  unsigned long long mn = feas ? enc_i64(ne.rna) : 0ull;
  unsigned long long mi = feas ? enc_i64(ne.ripa) : 0ull;
  unsigned long long ni = feas ? enc_i64(ne.ripa) : ~0ull;
  mt = wave_max_u64(mt);
  mn = wave_max_u64(mn);
  if ((sm >> P_IPA) & 1u) {
    mi = wave_max_u64(mi);
    ni = wave_min_u64(ni);
  }
  const unsigned long long pball = __ballot(ne.pts);
  if (lane == 0) {
    s_cnt[wave] = (uint32_t)__popcll(ballot);
    s_pts[wave] = (uint32_t)__popcll(pball);
    s_max[0][wave] = mt;
    s_max[1][wave] = mn;
    s_max[2][wave] = mi;
    s_min[wave] = ni;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0, pc = 0;
    unsigned long long a = 0, bb = 0, ia = 0, in = ~0ull;
    for (int w = 0; w < kBlock / 64; ++w) {
      c += s_cnt[w];
      pc += s_pts[w];
      a = s_max[0][w] > a ? s_max[0][w] : a;
      bb = s_max[1][w] > bb ? s_max[1][w] : bb;
      ia = s_max[2][w] > ia ? s_max[2][w] : ia;
      in = s_min[w] < in ? s_min[w] : in;
    }
    b.blk_cnt[blk] = c;
    if (c && !(d.flags & DF_SAMPLE)) {  // a cut feasible list: k_sample_apply reduces the kept nodes
      PodStats* ps = b.stats + pod;
      if ((sm >> P_TAINT) & 1u) atomicMax(&ps->max_raw[P_TAINT], a);
      if ((sm >> P_NA) & 1u) atomicMax(&ps->max_raw[P_NA], bb);
      if ((sm >> P_IPA) & 1u) {
        atomicMax(&ps->max_raw[P_IPA], ia);
        atomicMin(&ps->min_raw[P_IPA], in);
      }
      if (pc) atomicAdd(&ps->pts_nonignored, pc);
    }
  }
}

// =====================================================================================================
// k_select (+ the node-sharded k_select_shard / k_commit)
// =====================================================================================================
__device__ __forceinline__ uint32_t wave_prefix_count(unsigned long long ballot, int lane) {  // lanes below mine
  (void)lane;
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(ballot >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ballot, 0u));
}

// The maxima / minima the NormalizeScore passes need, gathered over the whole feasible list.
struct NormStats {
  int64_t mx_taint, mx_na, mx_pts, mn_pts, mx_ipa, mn_ipa;
  uint32_t ipa_any;
};

// NormalizeScore + weight + sum for feasible node i (framework.go:1409-1452)
__device__ int64_t node_total(const BatchView& b, const PodDesc& d, const NormStats& ns, size_t cap, int i,
                              bool eval) {
  if (d.flags & DF_NO_SCORE) return 1;  // no score plugins: TotalScore 1 (schedule_one.go:948-957)
  int64_t total = b.fixed[i];
  const uint32_t sm = d.score_mask;
  if ((sm >> P_TAINT) & 1u) {  // DefaultNormalizeScore(100, reverse=true) (helper/normalize_score.go:27-55)
    const int64_t mx = ns.mx_taint;
    const int64_t r = b.raw[P_TAINT * cap + i];
    const int64_t v = mx == 0 ? 100 : 100 - go_div(100 * r, mx);
    total += v * d.weight[P_TAINT];
    if (eval) b.out_scores[P_TAINT * cap + i] = v;
  }
  if ((sm >> P_NA) & 1u) {  // DefaultNormalizeScore(100, reverse=false)
    const int64_t mx = ns.mx_na;
    const int64_t r = b.raw[P_NA * cap + i];
    const int64_t v = mx == 0 ? 0 : go_div(100 * r, mx);
    total += v * d.weight[P_NA];
    if (eval) b.out_scores[P_NA * cap + i] = v;
  }
  if ((sm >> P_PTS) & 1u) {  // PodTopologySpread.NormalizeScore (podtopologyspread/scoring.go:229-268)
    const int64_t mx = ns.mx_pts, mn = ns.mn_pts;
    const int64_t r = b.raw[P_PTS * cap + i];
    const int64_t v = r == -1 ? 0 : (mx == 0 ? 100 : go_div(100 * (mx + mn - r), mx));
    total += v * d.weight[P_PTS];
    if (eval) b.out_scores[P_PTS * cap + i] = v;
  }
  if ((sm >> P_IPA) & 1u) {  // InterPodAffinity.NormalizeScore (interpodaffinity/scoring.go:258-290)
    const int64_t r = b.raw[P_IPA * cap + i];
    int64_t v = r;
    if (ns.ipa_any & 8u) {
      const int64_t mx = ns.mx_ipa, mn = ns.mn_ipa;
      const int64_t diff = mx - mn;
      double f = 0.0;
      if (diff > 0) f = 100.0 * ((double)(r - mn) / (double)diff);
      v = (int64_t)f;
    }
    total += v * d.weight[P_IPA];
    if (eval) b.out_scores[P_IPA * cap + i] = v;
  }
  if (eval) {  // evaluation output: each plugin's normalised, unweighted score (the host applies the weights)
    if ((sm >> P_FIT) & 1u) b.out_scores[P_FIT * cap + i] = b.raw[P_FIT * cap + i];
    if ((sm >> P_BAL) & 1u) b.out_scores[P_BAL * cap + i] = b.raw[P_BAL * cap + i];
    if ((sm >> P_IMG) & 1u) b.out_scores[P_IMG * cap + i] = b.raw[P_IMG * cap + i];
  }
  return total;
}

// Block-cooperative: the snapshot index of the g-th feasible node (0-based) counted over the
// blocks [k0, k1) of blk_cnt / fmask; -1 if g is not in that range.  All threads must call it.
__device__ int find_rank_node(const BatchView& b, int k0, int k1, uint32_t g) {
  __shared__ uint32_t s_wsum[kBlock / 64];
  __shared__ int s_node;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_node = -1;
  // each thread owns a contiguous chunk of blocks; block-wide exclusive scan of the chunk sums
  // (wave shuffles + one LDS word per wave)
  const int nb = k1 - k0;
  const int per = (nb + kBlock - 1) / kBlock;
  const int c0 = k0 + threadIdx.x * per;
  const int c1 = (c0 + per) < k1 ? (c0 + per) : k1;
  uint32_t csum = 0;
  for (int k = c0; k < c1; ++k) csum += b.blk_cnt[k];
  uint32_t incl = csum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  __syncthreads();
  uint32_t acc = incl - csum;
  for (int w = 0; w < wave; ++w) acc += s_wsum[w];
  if (g >= acc && g < acc + csum) {  // exactly one thread owns rank g
    for (int k = c0; k < c1; ++k) {
      const uint32_t c = b.blk_cnt[k];
      if (g < acc + c) {
        uint32_t need = g - acc;
        const uint64_t* fw = b.fmask + (size_t)k * (kBlock / 64);
        for (int w = 0; w < kBlock / 64; ++w) {
          const uint32_t wc = (uint32_t)__popcll(fw[w]);
          if (need < wc) {
            uint64_t x = fw[w];
            for (uint32_t q = 0; q < need; ++q) x &= x - 1ull;  // drop the lowest set bits
            s_node = k * kBlock + w * 64 + (int)__builtin_ctzll(x);
            break;
          }
          need -= wc;
        }
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  return s_node;
}

// Feasible nodes of blocks [k0, k1) with snapshot index < s (block-cooperative, thread 0's value
// is the total; other threads' values are partial).
__device__ uint32_t count_below(const BatchView& b, int k0, int k1, int s) {
  __shared__ uint32_t s_red[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sb = s / kBlock;
  uint32_t c = 0;
  for (int k = k0 + threadIdx.x; k < k1; k += kBlock) {
    if (k < sb) {
      c += b.blk_cnt[k];
    } else if (k == sb) {
      const uint64_t* fw = b.fmask + (size_t)sb * (kBlock / 64);
      int rem = s - sb * kBlock;
      for (int w = 0; w < kBlock / 64 && rem > 0; ++w) {
        const int take = rem >= 64 ? 64 : rem;
        const uint64_t msk = take == 64 ? ~0ull : ((1ull << take) - 1ull);
        c += (uint32_t)__popcll(fw[w] & msk);
        rem -= take;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) s_red[wave] = c;
  __syncthreads();
  c = 0;
  for (int w = 0; w < kBlock / 64; ++w) c += s_red[w];
  __syncthreads();
  return c;
}

// Normalise every feasible node of this block, reduce the packed (TotalScore, heap pre-order
// key) max into *best, zero this pod's share of the arena, take the arrival ticket.  Returns
// true in the last block to arrive (which may then read *best).
__device__ bool select_block(const MirrorView& m, const BatchView& b, const PodDesc& d, PodStats* ps,
                             const NormStats& ns, int blk, int nblocks, uint32_t pre, uint32_t F, uint32_t ps_before,
                             int arena_base, int arena_stride) {
  const int i = blk * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t cap = (size_t)m.cap;
  const bool eval = (d.flags & DF_EVAL_OUT) != 0;
  const unsigned long long ballot = b.fmask[(size_t)blk * (kBlock / 64) + wave];
  __shared__ uint32_t s_wcnt[kBlock / 64];
  if (lane == 0) s_wcnt[wave] = (uint32_t)__popcll(ballot);
  __syncthreads();
  uint32_t wave_pre = 0;
  for (int w = 0; w < wave; ++w) wave_pre += s_wcnt[w];
  const bool feas = i < m.n && ((ballot >> lane) & 1ull);

  unsigned long long key = 0;
  if (feas) {
    const uint32_t g = pre + wave_pre + wave_prefix_count(ballot, lane);  // rank in snapshot order
    const uint32_t pos = g >= ps_before ? g - ps_before : g + F - ps_before;  // rank in evaluation order
    const int64_t total = node_total(b, d, ns, cap, i, eval);
    if (eval) b.out_total[i] = total;
    if (d.flags & DF_OB) b.ob_heap[pos] = ObEnt{total, i, 0};  // the NodePluginScores list, feasible order
    key = pack_best(total, pos);
  }
  // the PTS/IPA histograms of this pod are dead now: zero them for the next pod on the stream
  for (int w = arena_base + threadIdx.x; w < d.arena_words; w += arena_stride) b.arena[w] = 0ull;
  key = wave_max_u64(key);
  __shared__ unsigned long long s_key[kBlock / 64];
  if (lane == 0) s_key[wave] = key;
  __syncthreads();

  // ---- one atomic per block, then the arrival ticket.  The only cross-block payload read in
  // this launch is ps->best, itself an agent-scope atomic: the atomicMax has returned before the
  // ticket add is issued, and the last block reads it with an agent-scope load -- no L2
  // write-back/invalidate fences needed (MI355X_MICROARCH.md, valid hand-off forms: 8-B agent
  // atomics both sides).  blk_cnt / fmask were written by the previous launch.
  __shared__ uint32_t s_last;
  if (threadIdx.x == 0) {
    unsigned long long k = 0;
    for (int w = 0; w < kBlock / 64; ++w) k = s_key[w] > k ? s_key[w] : k;
    if (k) (void)__hip_atomic_fetch_max(&ps->best, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t t = __hip_atomic_fetch_add(&ps->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == (uint32_t)nblocks - 1u) ? 1u : 0u;
  }
  __syncthreads();
  return s_last != 0;
}

// DevResult + AssumePod of the chosen node (schedule_one.go:1102-1137 -> NodeInfo.update,
// framework/types.go:445-468) on this replica of the mirror.  One thread.
// returns whether the AssumePod was applied to the mirror.  after/ipa_any (k_sched_loop): the
// node's core columns with the pod added, already known to the caller, are stored instead of
// read-modify-written, and the pod's ipa_any flags come from the caller (no load on the path).
__device__ __forceinline__ bool commit_result(const MirrorView& m, const BatchView& b, const uint8_t* base, const PodDesc& d,
                              PodStats* ps, int pod, uint32_t F, int node, unsigned long long best,
                              const NodeCore* after = nullptr, int ipa_any = -1) {
  const size_t cap = (size_t)m.cap;
  DevResult r;
  r.node = F > 0 ? node : -1;
  r.feasible = (int32_t)F;
  r.evaluated = 0;
  r.total = F > 0 ? (int64_t)(best >> kPreBits) : 0;
  r.key = best;
  r.status = F > 0 ? (int32_t)C_OK : (int32_t)C_UNSCHED;
  r.ipa_any = ipa_any >= 0 ? (uint32_t)ipa_any : ps->ipa_any;
  r.hinted = 0;
  r.pad = 0;
  if (d.flags & DF_ROTDEV) {  // k_sample_find's rotation bookkeeping
    r.evaluated = (int32_t)ps->processed;
    r.rot_next = ps->rot_out;
  }
  if (d.flags & DF_PREFILTER_REJECT) r.status = (int32_t)C_UNSCHED;
  if ((d.flags & DF_SCORE_ERROR) && F > 1) {  // prioritizeNodes error (schedule_one.go:600-603)
    r.status = (int32_t)C_ERROR;
    r.node = -1;
  }
  ps->feasible = F;
  if ((d.flags & DF_ASSUME) && r.node >= 0) {
    const int j = r.node;
    if (after) {
      m.req_cpu[j] = after->rcpu;
      m.req_mem[j] = after->rmem;
      m.req_eph[j] = after->reph;
      m.nz_cpu[j] = after->nzcpu;
      m.nz_mem[j] = after->nzmem;
      m.num_pods[j] = after->npods;
    } else {
      m.req_cpu[j] += d.a_cpu;
      m.req_mem[j] += d.a_mem;
      m.req_eph[j] += d.a_eph;
      m.nz_cpu[j] += d.a_nz_cpu;
      m.nz_mem[j] += d.a_nz_mem;
      m.num_pods[j] += 1;
    }
    const ScalarReq* sr = at<ScalarReq>(base, d.a_scalar_off);
    for (int k = 0; k < d.n_a_scalar; ++k) m.scalar_req[(size_t)sr[k].slot * cap + j] += sr[k].qty;
    const uint32_t* pp = at<uint32_t>(base, d.pod_ports_off);
    uint32_t* slots = m.ports + (size_t)j * m.port_slots;
    if (d.slot >= 0) m.pod_node[d.slot] = j;  // the pod joins NodeInfo.Pods (pod table)
    for (int k = 0; k < d.n_pod_ports; ++k) {  // HostPortInfo.Add: set semantics
      bool present = false;
      int empty = -1;
      for (int q = 0; q < m.port_slots; ++q) {  // the host sized the stride for every assume of the batch
        present |= slots[q] == pp[k];
        if (slots[q] == 0xffffffffu && empty < 0) empty = q;
      }
      if (!present && empty >= 0) slots[empty] = pp[k];
    }
  }
  b.results[pod] = r;
  return (d.flags & DF_ASSUME) && r.node >= 0;
}

__device__ __forceinline__ uint32_t winner_rank(unsigned long long best, uint32_t ps_before, uint32_t F) {
  // heap position of the winner -> global feasible rank g (undo the rotation)
  const uint32_t pos = preorder_pos((1u << kPreBits) - 1u - (uint32_t)(best & ((1ull << kPreBits) - 1ull)));
  uint32_t g = pos + ps_before;
  if (g >= F) g -= F;
  return g;
}

template <bool kLds>
__global__ __launch_bounds__(kBlock) void k_select(MirrorView m, BatchView b, int pod, int nblocks) {
  __shared__ __align__(16) uint8_t s_blob[kLds ? kBlobLds : 16];
  const uint8_t* base = b.descs + b.desc_off[pod];
  if constexpr (kLds) {
    stage_blob(base, reinterpret_cast<const PodDesc*>(base)->blob_bytes, s_blob);
    __syncthreads();
    base = s_blob;
  }
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if ((d.flags & DF_EARLY) && ps->ob_done) {  // placed by k_ob_hint / k_nominated: only the histograms to clear
    for (int w = blockIdx.x * kBlock + threadIdx.x; w < d.arena_words; w += nblocks * kBlock) b.arena[w] = 0ull;
    return;
  }

  // ---- global feasible count F, this block's exclusive prefix, and P(s) = feasible nodes
  // before the rotation start (nextStartNodeIndex, schedule_one.go:808) -- one strided pass
  const int s = (d.flags & DF_ROTDEV) ? (int)ps->rot : d.rot_start;
  const int sb = s / kBlock;
  __shared__ uint32_t s_red[kBlock / 64][3];
  uint32_t pre = 0, tot = 0, pres = 0;
  for (int k = threadIdx.x; k < nblocks; k += kBlock) {
    uint32_t c = b.blk_cnt[k];
    tot += c;
    if (k < (int)blockIdx.x) pre += c;
    if (k < sb) pres += c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pre += __shfl_xor(pre, o, 64);
    tot += __shfl_xor(tot, o, 64);
    pres += __shfl_xor(pres, o, 64);
  }
  if (lane == 0) { s_red[wave][0] = pre; s_red[wave][1] = tot; s_red[wave][2] = pres; }
  __syncthreads();
  pre = 0;
  tot = 0;
  pres = 0;
  for (int w = 0; w < kBlock / 64; ++w) { pre += s_red[w][0]; tot += s_red[w][1]; pres += s_red[w][2]; }
  const uint32_t F = tot;
  uint32_t ps_before = 0;
  if (s > 0 && F > 0) {
    const uint64_t* fw = b.fmask + (size_t)sb * (kBlock / 64);
    int rem = s - sb * kBlock;
    uint32_t acc = pres;
    for (int w = 0; w < kBlock / 64 && rem > 0; ++w) {
      int take = rem >= 64 ? 64 : rem;
      uint64_t msk = take == 64 ? ~0ull : ((1ull << take) - 1ull);
      acc += (uint32_t)__popcll(fw[w] & msk);
      rem -= take;
    }
    ps_before = acc;
  }
  NormStats ns;
  ns.mx_taint = dec_i64(ps->max_raw[P_TAINT]);
  ns.mx_na = dec_i64(ps->max_raw[P_NA]);
  ns.mx_pts = dec_i64(ps->max_raw[P_PTS]);
  ns.mn_pts = dec_i64(ps->min_raw[P_PTS]);
  ns.mx_ipa = dec_i64(ps->max_raw[P_IPA]);
  ns.mn_ipa = dec_i64(ps->min_raw[P_IPA]);
  ns.ipa_any = ps->ipa_any;
  if (!select_block(m, b, d, ps, ns, blockIdx.x, nblocks, pre, F, ps_before, blockIdx.x * kBlock, nblocks * kBlock))
    return;

  // ================= last block: winner lookup + AssumePod =================
  const unsigned long long best = __hip_atomic_load(&ps->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int node = -1;
  if (F > 0) node = find_rank_node(b, 0, nblocks, winner_rank(best, ps_before, F));
  if (threadIdx.x == 0) commit_result(m, b, base, d, ps, pod, F, node, best);
}

// ---- OpportunisticBatching (framework/runtime/batch.go:65-229, schedule_one.go:586-611,650-668) ----------------
// Go's container/heap down() over the stored NodePluginScores, nodeScoreHeap.Less = TotalScore > (Randomizer 0)
__device__ __forceinline__ void ob_down(ObEnt* h, int i, int n) {
  while (true) {
    const int j1 = 2 * i + 1;
    if (j1 >= n) break;
    int j = j1;
    if (j1 + 1 < n && h[j1 + 1].total > h[j1].total) j = j1 + 1;
    if (!(h[j].total > h[i].total)) break;
    const ObEnt t = h[i];
    h[i] = h[j];
    h[j] = t;
    i = j;
  }
}

constexpr int64_t kObMaxAgeNs = 500LL * 1000 * 1000;  // maxBatchAge (batch.go:57)

// k_ob_hint (one thread, after PreFilter and the pod's histograms): GetNodeHint (batch.go:65-95) --
// batchStateCompatible (:167-226: the host checked the signature, the cycle sequence and the nominated
// node; here the stored state, its age and whether the last chosen node now rejects the pod), the Pop --
// then evaluateNominatedNode with the hint (schedule_one.go:718-752): the hinted node's filters alone.
// Feasible: the pod is placed there (schedulePod's one-feasible-node path, :586-598) and
// StoreScheduleResults(hinted == chosen) keeps the rest of the heap (:110-118).
__global__ void k_ob_hint(MirrorView m, BatchView b, int pod) {
  if (threadIdx.x != 0) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  if (!(d.flags & DF_OB) || (d.flags & DF_PREFILTER_REJECT) || !d.ob_hint) return;
  ObState& st = *b.ob;
  if (st.len <= 0 || st.last_cycle != d.ob_cycle - 1 || d.ob_now > st.creation + kObMaxAgeNs || st.last_node < 0) return;
  int64_t rt = 0;
  const ArenaTopo at{ps, b.arena};
  if (run_filters(m, load_core(m, st.last_node), base, d, st.last_node, &rt, at, 0) == 0) return;  // not full
  ObEnt* h = b.ob_heap;
  const int n = st.len - 1;  // heap.Pop: swap(0, n), down(0, n), take the last
  const ObEnt top = h[0];
  h[0] = h[n];
  h[n] = top;
  ob_down(h, 0, n);
  st.len = n;
  const int hint = top.node;
  if (hint < 0 || hint >= m.n) return;  // no longer in the snapshot: an error, then the full pass
  if (run_filters(m, load_core(m, hint), base, d, hint, &rt, at, 0) != 0) {  // the full pass decides
    ps->nom_failed = (uint32_t)hint + 1u;  // its status is in NodeToStatus (k_sample_find counts it once)
    return;
  }
  if (d.flags & DF_ROTDEV) {  // the hint path leaves nextStartNodeIndex alone
    ps->rot_out = d.prev_pod < 0 ? ps->rot_in : b.stats[d.prev_pod].rot_out;
    ps->processed = 1;
  }
  commit_result(m, b, base, d, ps, pod, 1u, hint, 0ull);
  b.results[pod].hinted = 1u;
  b.results[pod].evaluated = 1;  // EvaluatedNodes = 1 + diagnosis.NodeToStatus.Len() (no failure)
  ps->ob_done = 1u;
  st.last_cycle = d.ob_cycle;
  st.last_node = hint;
}

// k_nominated (one thread, after PreFilter and the pod's histograms): evaluateNominatedNode (schedule_one.go:657-669,
// 714-745) for status.nominatedNodeName -- that node's filters alone (RunFilterPluginsWithNominatedPods: this
// context tracks no other pod's nomination).  Feasible: the pod is placed there (schedulePod's one-feasible-node
// path, :586-598; nextStartNodeIndex stays).  Else the node's status joins NodeToStatus (kept for evaluation
// output, counted once by k_sample_find) and the full pass follows.
__global__ void k_nominated(MirrorView m, BatchView b, int pod) {
  if (threadIdx.x != 0) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  if (!(d.flags & DF_NOMINATED) || (d.flags & DF_PREFILTER_REJECT)) return;
  const int nn = d.nominated_node;
  if (nn < 0 || nn >= m.n) return;
  int64_t rt = 0;
  const uint32_t st = run_filters(m, load_core(m, nn), base, d, nn, &rt, ArenaTopo{ps, b.arena}, 0);
  if (st != 0) {
    ps->nom_failed = (uint32_t)nn + 1u;
    if (d.flags & DF_EVAL_OUT) b.status[nn] = st;
    return;
  }
  if (d.flags & DF_ROTDEV) {
    ps->rot_out = d.prev_pod < 0 ? ps->rot_in : b.stats[d.prev_pod].rot_out;
    ps->processed = 1;
  }
  commit_result(m, b, base, d, ps, pod, 1u, nn, 0ull);
  b.results[pod].hinted = 2u;
  b.results[pod].evaluated = 1;  // EvaluatedNodes = 1 + diagnosis.NodeToStatus.Len() (no failure yet)
  ps->ob_done = 2u;
}

// k_ob_store (one workgroup, after k_select): StoreScheduleResults (batch.go:98-158) for a signed pod whose
// full evaluation placed it.  One feasible node: the state is dropped (nil list).  Otherwise the feasible
// list's (TotalScore, node) entries k_select wrote in feasible order become newSortedNodeScores' heap
// (heap.Init, one level at a time: a level's subtrees are disjoint and every deeper level is done first,
// which is the order Init's sequential loop visits them in) and the winner is popped.
__global__ __launch_bounds__(1024) void k_ob_store(BatchView b, int pod) {
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(b.descs + b.desc_off[pod]);
  PodStats* ps = b.stats + pod;
  if (!(d.flags & DF_OB) || ps->ob_done == 1u) return;  // (placed on its nominated node: the one-node path below)
  const DevResult r = b.results[pod];
  if (r.status != (int32_t)C_OK || r.node < 0) return;  // FitError / Error: nothing stored (schedulePod returns first)
  ObState& st = *b.ob;
  const int n = (int)ps->feasible;
  ObEnt* h = b.ob_heap;
  if (n >= 2) {
    const int last = n / 2 - 1;
    const int top_level = 31 - __clz(last + 1);
    for (int L = top_level; L >= 0; --L) {
      const int lo = (1 << L) - 1, hi = min((1 << (L + 1)) - 2, last);
      for (int i = lo + (int)threadIdx.x; i <= hi; i += (int)blockDim.x) ob_down(h, i, n);
      __syncthreads();
    }
  }
  if (threadIdx.x != 0) return;
  if (n >= 2) {
    const ObEnt top = h[0];
    h[0] = h[n - 1];
    h[n - 1] = top;
    ob_down(h, 0, n - 1);
    if (top.node != r.node && st.check == 0) st.check = (uint32_t)(1 + d.ob_cycle);  // never: k_select's pre-order rule
  }
  st.len = n >= 2 ? n - 1 : 0;
  st.creation = d.ob_now;
  st.last_cycle = d.ob_cycle;
  st.last_node = r.node;
}

// the host's remap after the snapshot's node list was rebuilt: old snapshot index -> new (-1: gone)
__global__ __launch_bounds__(kBlock) void k_ob_remap(ObState* st, ObEnt* h, const int32_t* map, int nold) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < st->len) {
    const int o = h[i].node;
    h[i].node = (o >= 0 && o < nold) ? map[o] : -1;
  }
  if (i == 0) {
    const int o = st->last_node;
    st->last_node = (o >= 0 && o < nold) ? map[o] : -1;
  }
}

// ---- percentageOfNodesToScore: the cut feasible list (schedule_one.go:778-884) ---------------------
// findNodesThatPassFilters checks nodes[(nextStartNodeIndex + i) % numAll] in order and stops at
// the (K+1)-th feasible node, K = numFeasibleNodesToFind (schedule_one.go:809-824, sequential
// Parallelizer semantics): the feasible list is the first K feasible nodes of the rotated order,
// processedNodes = K + the failures before that (K+1)-th node = its rotated position, and
// nextStartNodeIndex advances by it (:686-687).  Every node is still evaluated on the device (one
// pass is cheaper than a serial walk); the cut is the cyclic snapshot-index range [rot, samp_end).
__device__ __forceinline__ bool in_cyclic(int i, int lo, int hi) {  // lo != hi
  return lo < hi ? (i >= lo && i < hi) : (i >= lo || i < hi);
}

// k_sample_find (1 block): this pod's rotation start from the device-resident nextStartNodeIndex,
// the (K+1)-th feasible node of the rotated order, processedNodes and the next rotation.
__global__ __launch_bounds__(kBlock) void k_sample_find(MirrorView m, BatchView b, int pod, int nblocks) {
  if (ob_skip(b, pod)) return;  // k_ob_hint kept nextStartNodeIndex (rot_out)
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const int N = m.n;
  const uint32_t rot_in = d.prev_pod < 0 ? ps->rot_in : b.stats[d.prev_pod].rot_out;
  if (d.flags & DF_PREFILTER_REJECT) {  // the cycle ends before findNodesThatPassFilters (:635-648)
    if (threadIdx.x == 0) {
      ps->rot = 0;
      ps->rot_out = rot_in;
      ps->processed = 0;
      ps->samp_end = -1;
    }
    return;
  }
  const bool sub = (d.flags & DF_SUBSET) != 0;
  const int32_t* subset = at<int32_t>(base, d.subset_off);
  const int cnt = sub ? d.subset_cnt : N;  // numAllNodes = len(nodes)
  // nodes[(nextStartNodeIndex + i) % numAll]: the PreFilterResult list is in snapshot order
  const int s = cnt == 0 ? 0 : (sub ? subset[rot_in % (uint32_t)cnt] : (int)rot_in);
  __shared__ uint32_t s_tot[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t tot = 0;
  for (int k = threadIdx.x; k < nblocks; k += kBlock) tot += b.blk_cnt[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
  if (lane == 0) s_tot[wave] = tot;
  __syncthreads();
  uint32_t F = 0;
  for (int w = 0; w < kBlock / 64; ++w) F += s_tot[w];
  const uint32_t K = (uint32_t)d.num_to_find;
  int end = -1;
  uint32_t processed = (uint32_t)cnt;
  if (F > K) {
    const uint32_t below = s > 0 ? count_below(b, 0, nblocks, s) : 0u;  // feasible nodes before s
    end = find_rank_node(b, 0, nblocks, (below + K) % F);               // rotated rank K
    if (sub) {  // rotated position inside the PreFilterResult list
      __shared__ int s_pos[2];
      for (int q = threadIdx.x; q < cnt; q += kBlock) {
        if (subset[q] == s) s_pos[0] = q;
        if (subset[q] == end) s_pos[1] = q;
      }
      __syncthreads();
      processed = (uint32_t)((s_pos[1] - s_pos[0] + cnt) % cnt);
    } else {
      processed = (uint32_t)((end - s + N) % N);
    }
  }
  if (ps->nom_failed) {  // a nominated / hinted node that failed alone is in NodeToStatus: once more unless the
                         // full pass reached it (rotated position < processed; outside a PreFilterResult list: never)
    const int nf = (int)ps->nom_failed - 1;
    int pos = -1;
    if (!sub) {
      pos = (nf - s + N) % N;
    } else {
      __shared__ int s_nf;
      if (threadIdx.x == 0) s_nf = -1;
      __syncthreads();
      for (int q = threadIdx.x; q < cnt; q += kBlock)
        if (subset[q] == nf) s_nf = q;
      __syncthreads();
      if (s_nf >= 0) pos = (s_nf - (int)(rot_in % (uint32_t)cnt) + cnt) % cnt;
    }
    if (pos < 0 || pos >= (int)processed) ++processed;
  }
  if (threadIdx.x == 0) {
    ps->rot = (uint32_t)s;
    ps->samp_end = end;
    ps->processed = processed;
    ps->rot_out = N > 0 ? (uint32_t)(((uint64_t)rot_in + processed) % (uint64_t)N) : 0u;
  }
}

// k_sample_apply (node blocks): keep the feasible nodes in [rot, samp_end), rewrite this block's
// mask words and count, and do the feasible-list reductions k_filter_score skipped for a cut list:
// the normalising plugins' raw-score max/min, PodTopologySpread PreScore's ignored-node count and
// domain presence (podtopologyspread/scoring.go:61-115).  Evaluation output: nodes past the cut
// were never processed, so they carry no status (result[i] == nil, schedule_one.go:845-850).
// Node-sharded (shard != 0): the grid covers this rank's blocks from blk0, and the kept feasible
// nodes are k_sample_shard_b's intervals; the statuses of unprocessed nodes are cleared by
// k_select_shard once exchange A has carried the cut's end node to every rank.
__global__ __launch_bounds__(kBlock) void k_sample_apply(MirrorView m, BatchView b, int pod, int blk0, int shard) {
  if (ob_skip(b, pod)) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const int blk = blk0 + (int)blockIdx.x;
  const int i = blk * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t cap = (size_t)m.cap;
  const int end = ps->samp_end, s = (int)ps->rot;
  bool inproc;
  if (shard)
    inproc = i < m.n && ((i >= ps->keep[0] && i < ps->keep[1]) || (i >= ps->keep[2] && i < ps->keep[3]));
  else
    inproc = i < m.n && (end < 0 || in_cyclic(i, s, end));
  const unsigned long long word = b.fmask[(size_t)blk * (kBlock / 64) + wave];
  const bool kept = inproc && ((word >> lane) & 1ull);
  if (!shard && (d.flags & DF_EVAL_OUT) && i < m.n && !inproc && ps->nom_failed != (uint32_t)i + 1u) b.status[i] = 0u;
  const unsigned long long ballot = __ballot(kept);
  if (lane == 0) b.fmask[(size_t)blk * (kBlock / 64) + wave] = ballot;
  const uint32_t sm = d.score_mask;
  unsigned long long mt = 0, mn = 0, mi = 0, ni = ~0ull;
  if (kept) {
    if ((sm >> P_TAINT) & 1u) mt = enc_i64(b.raw[P_TAINT * cap + i]);
    if ((sm >> P_NA) & 1u) mn = enc_i64(b.raw[P_NA * cap + i]);
    if ((sm >> P_IPA) & 1u) mi = ni = enc_i64(b.raw[P_IPA * cap + i]);
  }
  bool pts = false;
  if ((sm >> P_PTS) & 1u) {
    const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
    pts = kept && !pts_ignored(m, d, cs, i);
    for (int32_t c = 0; c < d.n_ptss; ++c) {
      if (cs[c].hostname) continue;
      mark_domains(b.arena + cs[c].pres_base, pts ? pts_domain(m, cs[c], i) : 0, pts, &ps->pts_distinct[c]);
    }
  }
  mt = wave_max_u64(mt);
  mn = wave_max_u64(mn);
  mi = wave_max_u64(mi);
  ni = wave_min_u64(ni);
  const unsigned long long pball = __ballot(pts);
  __shared__ uint32_t s_cnt[kBlock / 64], s_pts[kBlock / 64];
  __shared__ unsigned long long s_max[3][kBlock / 64], s_min[kBlock / 64];
  if (lane == 0) {
    s_cnt[wave] = (uint32_t)__popcll(ballot);
    s_pts[wave] = (uint32_t)__popcll(pball);
    s_max[0][wave] = mt;
    s_max[1][wave] = mn;
    s_max[2][wave] = mi;
    s_min[wave] = ni;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0, pc = 0;
    unsigned long long a = 0, bb = 0, ia = 0, in = ~0ull;
    for (int w = 0; w < kBlock / 64; ++w) {
      c += s_cnt[w];
      pc += s_pts[w];
      a = s_max[0][w] > a ? s_max[0][w] : a;
      bb = s_max[1][w] > bb ? s_max[1][w] : bb;
      ia = s_max[2][w] > ia ? s_max[2][w] : ia;
      in = s_min[w] < in ? s_min[w] : in;
    }
    b.blk_cnt[blk] = c;
    if (c) {
      if ((sm >> P_TAINT) & 1u) atomicMax(&ps->max_raw[P_TAINT], a);
      if ((sm >> P_NA) & 1u) atomicMax(&ps->max_raw[P_NA], bb);
      if ((sm >> P_IPA) & 1u) {
        atomicMax(&ps->max_raw[P_IPA], ia);
        atomicMin(&ps->min_raw[P_IPA], in);
      }
      if (pc) atomicAdd(&ps->pts_nonignored, pc);
    }
  }
}

// ---- node-sharded path ----------------------------------------------------------------
// percentageOfNodesToScore on a node-sharded context.  The cut needs the global rotated prefix of
// feasible counts, so it costs one more all-reduce: k_sample_shard_a publishes this rank's feasible
// count and its feasible nodes before the rotation start (XS words); k_sample_shard_b cuts with the
// global figures.  The kept nodes are the global feasible ranks [below, below + K) mod F, the first
// K of the rotated order (schedule_one.go:809-824); intersected with this rank's ranks [P, P + c)
// they are at most two snapshot-index intervals, which k_sample_apply keeps.  The rank holding the
// (K+1)-th feasible node knows end and processedNodes and publishes them in exchange A (XA_END,
// XA_PROC); k_commit advances nextStartNodeIndex from them on every rank (:686-687).
__device__ __forceinline__ uint32_t pod_rot_in(const BatchView& b, const PodDesc& d, const PodStats* ps) {
  return d.prev_pod < 0 ? ps->rot_in : b.stats[d.prev_pod].rot_out;
}

__global__ __launch_bounds__(kBlock) void k_sample_shard_a(MirrorView m, BatchView b, ShardView sv, int pod) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  unsigned long long* x = sv.xs + (size_t)pod * XS_WORDS;
  const uint32_t rot_in = pod_rot_in(b, d, ps);
  if (d.flags & DF_PREFILTER_REJECT) {  // the cycle ends before findNodesThatPassFilters (:635-648)
    if (threadIdx.x == 0) {
      ps->rot = 0;
      ps->rot_out = rot_in;
      ps->processed = 0;
      ps->samp_end = -1;
    }
    if (threadIdx.x < XS_WORDS) x[threadIdx.x] = 0ull;
    return;
  }
  const bool sub = (d.flags & DF_SUBSET) != 0;
  const int32_t* subset = at<int32_t>(base, d.subset_off);
  const int cnt = sub ? d.subset_cnt : m.n;
  const int s = cnt == 0 ? 0 : (sub ? subset[rot_in % (uint32_t)cnt] : (int)rot_in);
  const int k0 = sv.blk0, k1 = sv.blk0 + sv.nblk;
  __shared__ uint32_t s_red[kBlock / 64];
  __shared__ uint32_t s_below;
  uint32_t c = 0;
  for (int k = k0 + threadIdx.x; k < k1; k += kBlock) c += b.blk_cnt[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = c;
  __syncthreads();
  c = 0;
  for (int w = 0; w < kBlock / 64; ++w) c += s_red[w];
  const uint32_t below = s > 0 ? count_below(b, k0, k1, s) : 0u;
  if (threadIdx.x == 0) {
    s_below = below;
    ps->rot = (uint32_t)s;
  }
  __syncthreads();
  if (threadIdx.x < XS_WORDS) {
    const int w = threadIdx.x;
    unsigned long long v = 0;
    if (w == XS_CNT + sv.rank) v = c;
    else if (w == XS_BELOW + sv.rank) v = s_below;
    x[w] = v;
  }
}

// cut = 0 (DF_ROTDEV without DF_SAMPLE): nothing is cut and no XS exchange ran; processedNodes is
// the whole list.
__global__ __launch_bounds__(kBlock) void k_sample_shard_b(MirrorView m, BatchView b, ShardView sv, int pod, int cut) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  if (d.flags & DF_PREFILTER_REJECT) return;
  const unsigned long long* x = sv.xs + (size_t)pod * XS_WORDS;
  const bool sub = (d.flags & DF_SUBSET) != 0;
  const int32_t* subset = at<int32_t>(base, d.subset_off);
  const int cnt = sub ? d.subset_cnt : m.n;
  const int N = m.n;
  const int s = (int)ps->rot;
  const uint32_t K = (uint32_t)d.num_to_find;
  uint32_t F = 0, below = 0, P = 0, c = 0;
  if (cut)
    for (int r = 0; r < sv.world; ++r) {
      const uint32_t cr = (uint32_t)x[XS_CNT + r];
      F += cr;
      below += (uint32_t)x[XS_BELOW + r];
      if (r < sv.rank) P += cr;
      if (r == sv.rank) c = cr;
    }
  if (!cut || F <= K) {  // every feasible node is kept
    if (threadIdx.x == 0) {
      ps->samp_end = -1;
      ps->processed = (uint32_t)cnt;
      ps->keep[0] = 0;
      ps->keep[1] = N;
      ps->keep[2] = ps->keep[3] = 0;
    }
    return;
  }
  const int k0 = sv.blk0, k1 = sv.blk0 + sv.nblk;
  const uint32_t gE = (below + K) % F;  // global feasible rank of the (K+1)-th node in rotated order
  const bool owner = gE >= P && gE < P + c;
  int end = -2;
  uint32_t processed = 0;
  if (owner) {
    end = find_rank_node(b, k0, k1, gE - P);
    __syncthreads();
    if (sub) {  // rotated position inside the PreFilterResult list
      __shared__ int s_pos[2];
      for (int q = threadIdx.x; q < cnt; q += kBlock) {
        if (subset[q] == s) s_pos[0] = q;
        if (subset[q] == end) s_pos[1] = q;
      }
      __syncthreads();
      processed = (uint32_t)((s_pos[1] - s_pos[0] + cnt) % cnt);
    } else {
      processed = (uint32_t)((end - s + N) % N);
    }
  }
  // kept global ranks: [below, min(below + K, F)) and [0, below + K - F) when it wraps
  const uint32_t lo[2] = {below, 0u};
  const uint32_t hi[2] = {below + K < F ? below + K : F, below + K > F ? below + K - F : 0u};
  int iv[4] = {0, 0, 0, 0};
  for (int j = 0; j < 2; ++j) {
    const uint32_t a = lo[j] > P ? lo[j] : P, e = hi[j] < P + c ? hi[j] : P + c;
    if (a < e) {  // uniform over the block
      __syncthreads();
      iv[2 * j] = find_rank_node(b, k0, k1, a - P);
      __syncthreads();
      iv[2 * j + 1] = find_rank_node(b, k0, k1, e - 1 - P) + 1;
    }
  }
  if (threadIdx.x == 0) {
    ps->samp_end = end;
    ps->processed = processed;
    for (int j = 0; j < 4; ++j) ps->keep[j] = iv[j];
  }
}

// k_xpack_a (1 block): this rank's share of the first exchange -- feasible count, feasible nodes
// before nextStartNodeIndex, PodTopologySpread non-ignored count, normalisation maxima/minima.
__global__ __launch_bounds__(kBlock) void k_xpack_a(BatchView b, ShardView sv, int pod) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  const PodStats* ps = b.stats + pod;
  const int k0 = sv.blk0, k1 = sv.blk0 + sv.nblk;
  __shared__ uint32_t s_red[kBlock / 64];
  uint32_t c = 0;
  for (int k = k0 + threadIdx.x; k < k1; k += kBlock) c += b.blk_cnt[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = c;
  __syncthreads();
  c = 0;
  for (int w = 0; w < kBlock / 64; ++w) c += s_red[w];
  const int s = (d.flags & DF_ROTDEV) ? (int)ps->rot : d.rot_start;
  const uint32_t below = s > 0 ? count_below(b, k0, k1, s) : 0u;
  const bool cut_owner = (d.flags & DF_ROTDEV) && ps->samp_end >= 0;  // this rank holds the cut's end node
  unsigned long long* x = sv.xa + (size_t)pod * XA_WORDS;
  if (threadIdx.x < XA_WORDS) {
    const int w = threadIdx.x;
    unsigned long long v = 0;
    if (w == XA_CNT + sv.rank) v = c;
    else if (w == XA_BELOW + sv.rank) v = below;
    else if (w == XA_NONIGN + sv.rank) v = ps->pts_nonignored;
    else if (w == XA_MAX_TAINT) v = ps->max_raw[P_TAINT];
    else if (w == XA_MAX_NA) v = ps->max_raw[P_NA];
    else if (w == XA_MAX_IPA) v = ps->max_raw[P_IPA];
    else if (w == XA_NMIN_IPA) v = ~ps->min_raw[P_IPA];
    else if (w == XA_END) v = cut_owner ? (unsigned long long)ps->samp_end + 1ull : 0ull;
    else if (w == XA_PROC) v = cut_owner ? (unsigned long long)ps->processed + 1ull : 0ull;
    x[w] = v;
  }
}

// k_unpack_pts (1 block): after the first exchange (and the all-reduce of the ScheduleAnyway
// domain-presence words), the global topology sizes PodTopologySpread.Score normalises with.
__global__ __launch_bounds__(kBlock) void k_unpack_pts(BatchView b, ShardView sv, int pod) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const unsigned long long* x = sv.xa + (size_t)pod * XA_WORDS;
  const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
  __shared__ uint32_t s_red[kBlock / 64];
  for (int32_t c = 0; c < d.n_ptss; ++c) {
    if (cs[c].hostname) continue;
    uint32_t n = 0;
    for (int v = threadIdx.x; v < cs[c].nvals; v += kBlock) n += b.arena[cs[c].pres_base + v] ? 1u : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kBlock / 64; ++w) t += s_red[w];
      ps->pts_distinct[c] = t;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int r = 0; r < sv.world; ++r) t += (uint32_t)x[XA_NONIGN + r];
    ps->pts_nonignored = t;
  }
}

// k_xpack_p (1 thread): PodTopologySpread raw-score max/min of this rank for the second exchange
__global__ void k_xpack_p(BatchView b, ShardView sv, int pod) {
  const PodStats* ps = b.stats + pod;
  unsigned long long* x = sv.xp + (size_t)pod * XP_WORDS;
  x[XP_MAX_PTS] = ps->max_raw[P_PTS];
  x[XP_NMIN_PTS] = ~ps->min_raw[P_PTS];
  x[2] = 0;
  x[3] = 0;
}

// k_select_shard: k_select over this rank's blocks with the all-reduced statistics; the last
// block writes this rank's best (key, node) into the final exchange vector.
__global__ __launch_bounds__(kBlock) void k_select_shard(MirrorView m, BatchView b, ShardView sv, int pod) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const unsigned long long* xa = sv.xa + (size_t)pod * XA_WORDS;
  const unsigned long long* xp = sv.xp + (size_t)pod * XP_WORDS;
  const int blk = sv.blk0 + blockIdx.x;
  if ((d.flags & (DF_EVAL_OUT | DF_SAMPLE)) == (DF_EVAL_OUT | DF_SAMPLE) && xa[XA_END] && sv.nblk > 0) {
    // a cut feasible list: nodes past the cut were never processed (result[i] == nil,
    // schedule_one.go:845-850)
    const int i = blk * kBlock + threadIdx.x;
    if (i < m.n && !in_cyclic(i, (int)ps->rot, (int)(xa[XA_END] - 1ull))) b.status[i] = 0u;
  }
  if (sv.nblk == 0) {  // an empty shard publishes an empty share and still zeroes its arena
    for (int w = threadIdx.x; w < d.arena_words; w += kBlock) b.arena[w] = 0ull;
    if (threadIdx.x < XB_WORDS) sv.xb[(size_t)pod * XB_WORDS + threadIdx.x] = 0ull;
    return;
  }
  uint32_t F = 0, shard_pre = 0, ps_before = 0;
  for (int r = 0; r < sv.world; ++r) {
    const uint32_t c = (uint32_t)xa[XA_CNT + r];
    F += c;
    if (r < sv.rank) shard_pre += c;
    ps_before += (uint32_t)xa[XA_BELOW + r];
  }
  __shared__ uint32_t s_red[kBlock / 64];
  uint32_t pre = 0;
  for (int k = sv.blk0 + threadIdx.x; k < blk; k += kBlock) pre += b.blk_cnt[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = pre;
  __syncthreads();
  pre = shard_pre;
  for (int w = 0; w < kBlock / 64; ++w) pre += s_red[w];
  NormStats ns;
  ns.mx_taint = dec_i64(xa[XA_MAX_TAINT]);
  ns.mx_na = dec_i64(xa[XA_MAX_NA]);
  ns.mx_ipa = dec_i64(xa[XA_MAX_IPA]);
  ns.mn_ipa = dec_i64(~xa[XA_NMIN_IPA]);
  ns.mx_pts = dec_i64(xp[XP_MAX_PTS]);
  ns.mn_pts = dec_i64(~xp[XP_NMIN_PTS]);
  ns.ipa_any = ps->ipa_any;
  if (!select_block(m, b, d, ps, ns, blk, sv.nblk, pre, F, ps_before, blockIdx.x * kBlock, sv.nblk * kBlock))
    return;
  const unsigned long long best = __hip_atomic_load(&ps->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int node = -1;
  if (best) node = find_rank_node(b, sv.blk0, sv.blk0 + sv.nblk, winner_rank(best, ps_before, F) - shard_pre);
  unsigned long long* xb = sv.xb + (size_t)pod * XB_WORDS;
  if (threadIdx.x < XB_WORDS) {
    const int w = threadIdx.x;
    unsigned long long v = 0;
    if (w == XB_KEY + sv.rank) v = best;
    else if (w == XB_NODE + sv.rank) v = node >= 0 ? (unsigned long long)(node + 1) : 0ull;
    xb[w] = v;
  }
}

// k_commit (1 thread): the winner over all ranks (distinct ranks hold distinct feasible
// positions, so the packed keys never tie), result + AssumePod on this replica.
__global__ void k_commit(MirrorView m, BatchView b, ShardView sv, int pod) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const unsigned long long* xa = sv.xa + (size_t)pod * XA_WORDS;
  const unsigned long long* xb = sv.xb + (size_t)pod * XB_WORDS;
  uint32_t F = 0;
  for (int r = 0; r < sv.world; ++r) F += (uint32_t)xa[XA_CNT + r];
  unsigned long long best = 0;
  int node = -1;
  for (int r = 0; r < sv.world; ++r)
    if (xb[XB_KEY + r] > best) {
      best = xb[XB_KEY + r];
      node = (int)xb[XB_NODE + r] - 1;
    }
  if ((d.flags & DF_ROTDEV) && !(d.flags & DF_PREFILTER_REJECT)) {  // nextStartNodeIndex (:686-687)
    if (xa[XA_PROC]) ps->processed = (uint32_t)(xa[XA_PROC] - 1ull);
    ps->rot_out = m.n > 0 ? (uint32_t)(((uint64_t)pod_rot_in(b, d, ps) + ps->processed) % (uint64_t)m.n) : 0u;
  }
  commit_result(m, b, base, d, ps, pod, F, node, best);
}

// k_max_reduce: the in-process (same-device) all-reduce of the local communicator:
// dst[w] = max over the ranks' vectors.  Safe in place: max is idempotent, so a rank reading a
// vector another rank has already overwritten with the result still reads the same maximum.
__global__ __launch_bounds__(kBlock) void k_max_reduce(unsigned long long* dst, RankPtrs src, int nsrc, int count) {
  for (int w = blockIdx.x * kBlock + threadIdx.x; w < count; w += gridDim.x * kBlock) {
    unsigned long long v = 0;
    for (int r = 0; r < nsrc; ++r) {
      const unsigned long long x = __hip_atomic_load(src.p[r] + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v = x > v ? x : v;
    }
    dst[w] = v;
  }
}

// =====================================================================================================
// k_sched_loop -- the persistent scheduling loop
// =====================================================================================================
// One launch schedules a run of consecutive pods (node-local plugins only: no pod-table
// aggregation).  Workgroup w owns the node blocks [k0, k1) (at most kLoopMaxBlk) for the whole
// run, so the AssumePod of a pod is applied by the owner of the chosen node and only ever read back
// by that same workgroup: the mirror needs no cross-workgroup hand-off.  Per pod:
//   stage    the pod program into LDS (issued for pod q+1 before pod q's second exchange)
//   phase 1  RunFilterPlugins + raw scores of my nodes; the fixed score and the raw normalising
//            scores stay in registers, the feasibility ballots in LDS
//   xchg A   every workgroup publishes two 8-byte granules {valid, feasible count | count before
//            nextStartNodeIndex} and {valid, max raw TaintToleration + 1 | max raw NodeAffinity + 1};
//            one wave per workgroup sweeps all of them (the data is the flag: R2 of the hand-off
//            recipe -- no fences, no counters)
//   phase 2  positions in the rotated feasible list, NormalizeScore + weights, packed
//            (TotalScore, heap pre-order key) max of my nodes
//   xchg B   one granule {valid, key} per workgroup, swept the same way; the thread holding the
//            global maximum applies AssumePod and writes the result.
// A granule is {tag(16) | payload(48)}: the tag is the batch's (host counter, never 0), so an array
// needs no zeroing between batches and a stale granule never matches.  Every granule is written
// exactly once per batch, into every rank's array (the local one, and the peers' over xGMI).
constexpr unsigned long long kPayload = kGranPayload;

// diagnostic phase stamps (config "loopStamps"): workgroup 0's lane 0, 100 MHz constant clock
__device__ __forceinline__ void stamp(const LoopView& lv, int q, int k) {
  if (lv.stamps && threadIdx.x == 0) lv.stamps[(size_t)q * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// publish one granule of pod q to every rank.  Unsharded: an agent-scope store.  Sharded: system
// scope into each rank's array (the peers' are IPC-mapped, uncached device memory).
__device__ __forceinline__ void gran_put(const LoopView& lv, int q, int gid, int slot, unsigned long long payload) {
  const int P = lv.world * lv.nwg;
  const unsigned long long v = gran_word(lv.tag, payload);
  const size_t at = ((size_t)q * P + gid) * kGran + slot;
  if (lv.world == 1) {
    __hip_atomic_store(lv.gran[0] + at, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  for (int r = 0; r < lv.world; ++r) __hip_atomic_store(lv.gran[r] + at, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The hardware registers a give-up record names (desc.h kFailWords): HW_ID (gfx9 layout: pipe [7:6], HQD
// [26:24], ME [31:30]) and XCC_ID, read with s_getreg (no memory access)
__device__ __forceinline__ uint32_t hw_id_reg() { return (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4); }
__device__ __forceinline__ uint32_t xcc_id_reg() { return (uint32_t)__builtin_amdgcn_s_getreg((15 << 11) | 20); }
// fail words 8..11: the launch's entry, by (the rank's) workgroup 0's first lane, unless a give-up is already recorded
__device__ __forceinline__ void loop_entry_record(uint32_t* fail, int w) {
  if (!fail || w != 0 || threadIdx.x != 0 || __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    return;
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(fail + 8, hw_id_reg(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 9, xcc_id_reg(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 10, (uint32_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 11, (uint32_t)(t >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// fail words 12..15: the give-up's time and the giving-up wave's hardware ids
__device__ __forceinline__ void give_up_record(uint32_t* fail) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __hip_atomic_store(fail + 12, (uint32_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 13, (uint32_t)(t >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 14, hw_id_reg(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(fail + 15, xcc_id_reg(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave: poll granules [slot0, slot0 + NS) of all P participants of pod q in the local array
// until every tag matches (relaxed loads, s_sleep between passes).  x[s][r] = payload of
// participant lane + 64 r; false on give-up.
constexpr int kMaxSweep = 4;  // P <= 256 participants
template <int NS, int MS>
__device__ __forceinline__ bool gran_sweep(const LoopView& lv, int q, int slot0, unsigned long long (&x)[NS][MS]) {
  const int lane = threadIdx.x & 63;
  const int P = lv.world * lv.nwg;
  const unsigned long long* g = lv.gran[lv.world == 1 ? 0 : lv.rank] + (size_t)q * P * kGran + slot0;
  const unsigned long long want = (unsigned long long)lv.tag;
  // give up after ~10 s of wall time (100 MHz constant clock): sharded ranks may start a launch
  // seconds apart (their hosts load the cluster independently)
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  for (uint32_t spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < MS; ++r) {
      const int v = lane + 64 * r;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        unsigned long long y = want << 48;
        if (v < P)
          y = lv.world == 1 ? __hip_atomic_load(g + (size_t)v * kGran + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : __hip_atomic_load(g + (size_t)v * kGran + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok &= (y >> 48) == want;
        x[k][r] = y & kPayload;
      }
    }
    if (__all(ok)) return true;
    if ((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t_start > 1000000000ull) {
      // give up: record which pod / granule / participant never came
      const unsigned long long miss = __ballot(!ok);
      if (lane == 0) {
        __hip_atomic_store(lv.fail + 1, (uint32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail + 2, (uint32_t)slot0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail + 3, (uint32_t)__builtin_ctzll(miss), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // k_sched_loop
        __hip_atomic_store(lv.fail + 5, (uint32_t)lv.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail + 6, (uint32_t)miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail + 7, (uint32_t)(miss >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        give_up_record(lv.fail);
        __hip_atomic_store(lv.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return false;
    }
    if ((spins & 63u) == 63u && __hip_atomic_load(lv.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// k_sched_loop's doorbell (desc.h PodRing::ctl), polled by one thread: the posted word, or kCtlStop (the
// host's stop, the pod limit, or `idle` ticks without a pod).
// (ctl: the host's word, or workgroup 0's relayed copy in device memory; exited, when given, records an idle exit)
__device__ __forceinline__ unsigned long long ring_wait_ctl(const unsigned long long* ctl, uint32_t* exited, int q,
                                                            int npods, unsigned long long idle) {
  if (q >= npods) return kCtlStop;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t spins = 0;; ++spins) {
    const unsigned long long v = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long posted = v & kCtlStop;
    if (posted == kCtlStop) return kCtlStop;
    if (posted > (unsigned long long)q) return v;
    if ((spins & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t0 > idle) {
      if (exited && blockIdx.x == 0) __hip_atomic_store(exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return kCtlStop;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
// k_agg_loop's doorbell (desc.h PodRing::ll, or the copy workgroup 0 relays in device memory, AggView::relay),
// polled by one wave: lanes 0..3 load the four tagged words in one instruction (one 32-byte read over PCIe
// per poll and workgroup; four single-word reads per poll crowd the link: C4's 59 workgroups took twice as
// long per call) until every tag reads q + 1; lane k's data word into *data.  -1: stop, idle or no pod left
// (`exited`, when given, records an idle exit for the host).
__device__ __forceinline__ int ring_wait_ll(const unsigned long long* ll, uint32_t* exited, int q, int npods,
                                            unsigned long long idle, int lane, uint32_t* data) {
  if (q >= npods) return -1;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t spins = 0;; ++spins) {
    const unsigned long long v = lane < kRingLL ? __hip_atomic_load(ll + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
    const uint32_t tag = (uint32_t)v;
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)tag) == kRingStop) return -1;
    const unsigned long long ok = __ballot(lane < kRingLL && tag == (uint32_t)(q + 1));
    if (ok == (1ull << kRingLL) - 1ull) {
      *data = (uint32_t)(v >> 32);
      return 0;
    }
    if ((spins & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t0 > idle) {
      if (exited && blockIdx.x == 0 && lane == 0) __hip_atomic_store(exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
// Resident mode: pod q's result to the host (the committing thread, after commit_result)
// The record goes to host memory with system-scope (write-through) stores; once they have completed
// (vmcnt), the sequence word follows in the same PCIe posted-write stream.  (A system-scope release here
// would write the whole L2 back first.)
__device__ __forceinline__ void ring_post_p(PodRing* ring, int q, const DevResult& r) {
  RingResult& o = ring->res[q % kRingSlots];
  static_assert(sizeof(DevResult) % 8 == 0, "DevResult is stored as 8-byte words");
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&r);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(&o.r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(DevResult) / 8); ++k)
    __hip_atomic_store(dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&o.seq, (uint32_t)(q + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ring_post(const LoopView& lv, int q, const DevResult& r) { ring_post_p(lv.ring, q, r); }

// NormalizeScore + weights for the loop's plugin set (TaintToleration, NodeAffinity normalised;
// Fit / BalancedAllocation / ImageLocality already in `fixed`) -- framework.go:1409-1452
__device__ __forceinline__ int64_t loop_total(const PodDesc& d, int64_t fixed, int64_t rt, int64_t rn, int64_t mx_t,
                                              int64_t mx_n) {
  if (d.flags & DF_NO_SCORE) return 1;
  int64_t total = fixed;
  const uint32_t sm = d.score_mask;
  if ((sm >> P_TAINT) & 1u) total += (mx_t == 0 ? 100 : 100 - go_div(100 * rt, mx_t)) * d.weight[P_TAINT];
  if ((sm >> P_NA) & 1u) total += (mx_n == 0 ? 0 : go_div(100 * rn, mx_n)) * d.weight[P_NA];
  return total;
}

// The loop's node cores live in LDS (structure of arrays, [block of my range][slot]): the
// evaluation waves read them every pod, the committing thread applies the AssumePod to them and
// to the mirror alike, and the selection wave reads its candidate's core for the pre-evaluation.
template <int U>
struct LoopCoresT {
  int64_t acpu[kLoopMaxBlk][U], amem[kLoopMaxBlk][U], aeph[kLoopMaxBlk][U];
  int64_t rcpu[kLoopMaxBlk][U], rmem[kLoopMaxBlk][U], reph[kLoopMaxBlk][U];
  int64_t nzcpu[kLoopMaxBlk][U], nzmem[kLoopMaxBlk][U];
  int64_t bwo[kLoopMaxBlk][U];  // BalancedAllocation without the pod (pod-independent)
  int32_t apods[kLoopMaxBlk][U], npods[kLoopMaxBlk][U];
  uint32_t flags[kLoopMaxBlk][U], tlo[kLoopMaxBlk][U], thi[kLoopMaxBlk][U];
  uint32_t ilo[kLoopMaxBlk][U], ihi[kLoopMaxBlk][U];
};
using LoopCores = LoopCoresT<kBlock>;  // k_agg_loop's layout (256-node blocks)
template <int U>
__device__ __forceinline__ NodeCore lds_core(const LoopCoresT<U>& L, int kk, int t) {
  NodeCore c;
  c.acpu = L.acpu[kk][t];
  c.amem = L.amem[kk][t];
  c.aeph = L.aeph[kk][t];
  c.rcpu = L.rcpu[kk][t];
  c.rmem = L.rmem[kk][t];
  c.reph = L.reph[kk][t];
  c.nzcpu = L.nzcpu[kk][t];
  c.nzmem = L.nzmem[kk][t];
  c.apods = L.apods[kk][t];
  c.npods = L.npods[kk][t];
  c.flags = L.flags[kk][t];
  c.tlo = L.tlo[kk][t];
  c.thi = L.thi[kk][t];
  c.ilo = L.ilo[kk][t];
  c.ihi = L.ihi[kk][t];
  return c;
}
template <int U>
__device__ __forceinline__ void lds_put_dynamic(LoopCoresT<U>& L, int kk, int t, const NodeCore& c) {
  L.rcpu[kk][t] = c.rcpu;
  L.rmem[kk][t] = c.rmem;
  L.reph[kk][t] = c.reph;
  L.nzcpu[kk][t] = c.nzcpu;
  L.nzmem[kk][t] = c.nzmem;
  L.npods[kk][t] = c.npods;
  L.bwo[kk][t] = bal2(c.rcpu, c.acpu, c.rmem, c.amem);
}
// AssumePod's NodeInfo.update on the core columns (framework/types.go:445-468), as commit_result
__device__ __forceinline__ void assume_core(NodeCore& c, const PodDesc& d) {
  c.rcpu += d.a_cpu;
  c.rmem += d.a_mem;
  c.reph += d.a_eph;
  c.nzcpu += d.a_nz_cpu;
  c.nzmem += d.a_nz_mem;
  c.npods += 1;
}

// exchange A's two granules from a workgroup's feasible count, count before nextStartNodeIndex and
// encoded maxima of the raw TaintToleration / NodeAffinity scores (raw scores are >= 0 and bounded,
// host-checked: +1 so that 0 means "no feasible node")
__device__ __forceinline__ void a_granules(uint32_t c, uint32_t bl, unsigned long long a, unsigned long long bb,
                                           unsigned long long* g0, unsigned long long* g1) {
  *g0 = gran_a_counts(c, bl);  // desc.h: the layout the host-side protocol test drives too
  *g1 = gran_a_maxima(c, a, bb);
}

// Can pod `nd`'s evaluation of a node be computed, before pod `d` is assumed, as it will be after?
// Default-plugin pods read nothing an AssumePod changes beyond the core columns, except host ports.
__device__ __forceinline__ bool post_ok(const PodDesc& d, const PodDesc& nd) {
  return (d.flags & DF_ASSUME) && (nd.flags & DF_FAST) && !(((nd.filter_mask >> P_PORTS) & 1u) && d.n_pod_ports > 0);
}

constexpr int kLoopThreads = kBlock + 128;  // NW = 4: four evaluation waves, one selection wave, one helper wave

// Role of each hardware wave of a k_sched_loop workgroup (roles: 0-3 evaluation, 4 selection, 5 helper).
// A workgroup's waves go to the CU's four SIMDs round robin, so waves w and w + 4 share a SIMD:
// map 0 pairs the selection wave with evaluation wave 0, map 1 with the helper, map 2 runs it alone
// (two evaluation waves then share a SIMD).
__constant__ int8_t kWaveMap[3][kLoopThreads / 64] = {{0, 1, 2, 3, 4, 5}, {4, 0, 1, 2, 5, 3}, {0, 1, 4, 3, 5, 2}};
// RING: the resident instance (pods through lv.ring, one run per pod); the batch instance has no run
// loop at all (its one run is the whole launch), so its code is what it was before the ring existed.
// MS: sweep rounds of 64 participants (the one-round instance for grids of at most 64: no masked-off rounds)
// (the body of k_sched_loop and k_sched_loop_group: w = the workgroup this block plays in its rank)
// (GRP: the group instance takes w from its block index; the others read blockIdx.x itself, as before the group
// instance existed -- their register allocation is that sensitive)
template <int NW, bool RING, int MS, bool GRP>
__device__ __forceinline__ void sched_loop_body(const MirrorView& m, const BatchView& b, const LoopView& lv, const int w_grp) {
  constexpr int U = NW * 64;                  // nodes per unit: one per evaluation-wave lane
  constexpr int kLoopThreads = U + 128;       // NW evaluation waves, one selection wave, one helper wave
  __shared__ __align__(16) uint8_t s_blob[3][kBlobLds];  // pod p's program in s_blob[p % 3]
  __shared__ LoopCoresT<U> s_core;
  __shared__ unsigned long long s_ball[2][kLoopMaxBlk][NW];  // [pod parity]
  // phase-1 slots: weighted fixed score, raw TaintToleration / NodeAffinity scores (< 2^31, host-checked)
  __shared__ int64_t s_fx[2][kLoopMaxBlk][U];
  __shared__ uint32_t s_rt[2][kLoopMaxBlk][U], s_rn[2][kLoopMaxBlk][U];
  // the same for pod q+1 on each node as if pod q were assumed there (default-plugin pods): the
  // chosen node's next evaluation is ready when the winner is known
  __shared__ int64_t s_fx2[kLoopMaxBlk][U], s_bwo2[kLoopMaxBlk][U];
  __shared__ uint32_t s_rt2[kLoopMaxBlk][U], s_rn2[kLoopMaxBlk][U];
  __shared__ unsigned long long s_ball2[kLoopMaxBlk][NW];
  __shared__ uint32_t s_u[2][2][NW];
  __shared__ unsigned long long s_x[2][2][NW];
  __shared__ uint32_t s_off[kLoopMaxPods], s_len[kLoopMaxPods];  // the run's program offsets / sizes
  __shared__ uint32_t s_ok, s_F, s_cand_ok;
  __shared__ int s_win, s_cand_q, s_cand_node, s_ipa, s_gnode;
  __shared__ unsigned long long s_tm[2][U], s_tn[2][U];  // per-slot maxima of phase 1 (encoded)
  __shared__ uint32_t s_e_done;  // evaluation waves that finished a phase 1 (monotonic)
  // the candidate's state if it wins, prepared by the helper wave: its core columns with the pod
  // added, and its evaluation wave's exchange-A partials for the next pod
  __shared__ unsigned long long s_cball, s_cmt, s_cmn;
  __shared__ unsigned long long s_ga[4];  // pod q+1's exchange-A granules: [0..1] candidate not chosen, [2..3] chosen
  __shared__ int s_ga_q;                  // the pod whose s_ga is ready
  __shared__ uint32_t s_ccnt, s_cbelow;
  __shared__ unsigned long long s_best;
  __shared__ unsigned long long s_ring_ctl;  // resident mode: the doorbell word (desc.h PodRing::ctl)
  __shared__ int s_pb;                       // resident mode: the last staged program's bytes
  // percentageOfNodesToScore (DF_ROTDEV): s_rot[p & 1] = pod p's rotation start (nextStartNodeIndex),
  // s_proc = the decided pod's processedNodes (schedule_one.go:686-687, 809-824)
  __shared__ uint32_t s_rot[2], s_proc;
  const int w = GRP ? w_grp : (int)blockIdx.x, G = lv.nwg;
  if constexpr (!RING) loop_entry_record(lv.fail, w);  // (the resident instance is never sharded)
  const int gid = lv.rank * G + w, P = lv.world * G;  // my participant index, participants (rank-major)
  // my node units [k0, k1) of the rank's range (lv.blk0 / lv.nblk count 256-node blocks)
  const int ub0 = lv.blk0 * (kBlock / U), unb = lv.nblk * (kBlock / U);
  const int k0 = ub0 + (int)((int64_t)unb * w / G), k1 = ub0 + (int)((int64_t)unb * (w + 1) / G);
  const int nk = k1 - k0;  // <= kLoopMaxBlk (host-checked)
  const int lane = threadIdx.x & 63;
  // my role (NW = 2: one wave per SIMD, no placement to choose)
  const int wave = NW == 4 ? __builtin_amdgcn_readfirstlane((int)kWaveMap[lv.wave_map][threadIdx.x >> 6])
                           : (int)(threadIdx.x >> 6);
  const int vt = wave * 64 + lane;           // my thread index in role order
  const bool sel = wave == NW;      // the selection wave: exchanges + phase 2
  const bool hlp = wave == NW + 1;  // the helper wave: candidate pre-evaluation + staging
  const int t = vt;                          // evaluation waves: my slot in each block of my range
  // diagnostic stamps (loopStamps): the resident instance has them in the diagnostic library only (registers)
#ifdef KSG_DIAG
  constexpr bool kSt = true;
#else
  constexpr bool kSt = !RING;
#endif
  auto stamp_s = [&](int q, int k) {       // diagnostic phase stamps: WG 0's selection lane 0
    if (kSt && lv.stamps && w == 0 && vt == U) lv.stamps[(size_t)q * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  // the committing thread: pod `pod`'s PodStats, with its rotation bookkeeping for commit_result (DF_ROTDEV)
  auto rot_stats = [&](int pod, int par) __attribute__((always_inline)) -> PodStats* {
    PodStats* ps = b.stats + pod;
    if (reinterpret_cast<const PodDesc*>(s_blob[(pod - lv.first_pod) % 3])->flags & DF_ROTDEV) {
      ps->rot = s_rot[par];
      ps->processed = s_proc;
      ps->rot_out = s_rot[par ^ 1];
    }
    return ps;
  };

  if (t < U) {  // evaluation waves
#pragma unroll
    for (int kk = 0; kk < kLoopMaxBlk; ++kk) {
      const int i = (k0 + kk) * U + t;
      if (kk < nk && i < m.n) {
        const NodeCore c = load_core(m, i);
        s_core.acpu[kk][t] = c.acpu;
        s_core.amem[kk][t] = c.amem;
        s_core.aeph[kk][t] = c.aeph;
        s_core.apods[kk][t] = c.apods;
        s_core.flags[kk][t] = c.flags;
        s_core.tlo[kk][t] = c.tlo;
        s_core.thi[kk][t] = c.thi;
        s_core.ilo[kk][t] = c.ilo;
        s_core.ihi[kk][t] = c.ihi;
        lds_put_dynamic(s_core, kk, t, c);
      }
    }
  }

  // ---- program staging by the helper wave: straight from global memory into a free LDS slot (no
  // register stage: one held across the helper's waits ended up in scratch)
  auto stage_prog = [&](int pod, int slot) __attribute__((always_inline)) {
    const uint4* src = reinterpret_cast<const uint4*>(b.descs + s_off[pod - lv.first_pod]);
    const uint32_t n16 = s_len[pod - lv.first_pod] / 16u;
    uint4* dst = reinterpret_cast<uint4*>(s_blob[slot]);
    for (uint32_t o = (uint32_t)lane; o < n16; o += 64u) dst[o] = src[o];
  };
  // resident mode: pod q's program from the ring (host memory: one round trip, every thread's 16 B)
  // (system-scope loads: they bypass the device caches, so a ring slot reused kRingSlots pods later is
  // never read stale -- the doorbell poll is relaxed, no acquire invalidates the caches)

  // ---- evaluation-wave state of the pod being prepared: per-thread maxima of the normalising raw
  // scores over my feasible nodes; per-wave feasible counts (all, and before nextStartNodeIndex)
  unsigned long long t_mt = 0, t_mn = 0;
  uint32_t w_cnt = 0, w_below = 0;
  auto below_mask_v = [&](int kk, int v, int srot) __attribute__((always_inline)) -> unsigned long long {
    const int lim = srot - ((k0 + kk) * U + v * 64);
    return lim <= 0 ? 0ull : lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
  };
  auto below_mask = [&](int kk, int srot) __attribute__((always_inline)) -> unsigned long long {
    return below_mask_v(kk, wave, srot);
  };
  // DF_ROTDEV pods: the rotation start is known only once the previous pod's processedNodes is, after
  // phase 1, so exchange A's "feasible before nextStartNodeIndex" is counted from the ballots then.
  // One wave: lane = (block of my range, evaluation wave); (fkw, fcw) takes ballot fball instead.
  auto below_wave = [&](int par, int srot, int fkw, int fcw, unsigned long long fball) __attribute__((always_inline))
      -> uint32_t {
    const int kk = lane / NW, v = lane % NW;
    uint32_t c = 0;
    if (kk < nk) {
      const unsigned long long bl = (kk == fkw && v == fcw) ? fball : s_ball[par][kk][v];
      c = (uint32_t)__popcll(bl & below_mask_v(kk, v, srot));
    }
    return wave_sum_u32(c);
  };
  auto publish_partials = [&](int par) __attribute__((always_inline)) {
    s_tm[par][t] = t_mt;
    s_tn[par][t] = t_mn;
    const unsigned long long mt = wave_max_u64(t_mt), mn = wave_max_u64(t_mn);
    if (lane == 0) {
      s_u[par][0][wave] = w_cnt;
      s_u[par][1][wave] = w_below;
      s_x[par][0][wave] = mt;
      s_x[par][1][wave] = mn;
    }
  };
  // phase 1: RunFilterPlugins + raw scores of my nodes for `pod`, against the cores as they are now
  auto phase1 = [&](int pod, int slot, int par, const PodDesc* dprev) __attribute__((always_inline)) {
    const uint8_t* base = s_blob[slot];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    const bool fast = (d.flags & DF_FAST) != 0;
    const bool post = dprev && post_ok(*dprev, d);
    const PodFast pf = load_fast(base, d);
    const bool bal = ((pf.sm >> P_BAL) & 1u) != 0;
    const bool same_bal = post && dprev->a_cpu == pf.bpr_cpu && dprev->a_mem == pf.bpr_mem;
    t_mt = t_mn = 0;
    w_cnt = w_below = 0;
    auto record = [&](int kk, const NodeEval& ne) __attribute__((always_inline)) {
      const bool feas = ne.st == 0;
      const unsigned long long ballot = __ballot(feas);
      if (lane == 0) s_ball[par][kk][wave] = ballot;
      w_cnt += (uint32_t)__popcll(ballot);
      w_below += (uint32_t)__popcll(ballot & below_mask(kk, d.rot_start));
      s_fx[par][kk][t] = ne.fixed;
      s_rt[par][kk][t] = (uint32_t)ne.rt;
      s_rn[par][kk][t] = (uint32_t)ne.rna;
      if (feas) {
        const unsigned long long et = enc_i64(ne.rt), en = enc_i64(ne.rna);
        t_mt = et > t_mt ? et : t_mt;
        t_mn = en > t_mn ? en : t_mn;
      }
    };
#pragma unroll
    for (int kk = 0; kk < kLoopMaxBlk; ++kk) {
      if (kk < nk) {
        const int i = (k0 + kk) * U + t;
        NodeEval ne{1u, false, 0, 0, 0, 0};
        if (post) {  // both evaluations, independent chains the compiler interleaves
          NodeEval ne2{1u, false, 0, 0, 0, 0};
          if (i < m.n) {
            const NodeCore c = lds_core(s_core, kk, t);
            NodeCore c2 = c;
            assume_core(c2, *dprev);
            // BalancedAllocation: the node with pod q+1 is the node with pod q when their requests
            // match (one template), so one bal2 serves both
            int64_t with1 = kNoBal, wo2;
            if (bal) with1 = bal2(c.rcpu + pf.bpr_cpu, c.acpu, c.rmem + pf.bpr_mem, c.amem);
            wo2 = bal && same_bal ? with1 : bal2(c2.rcpu, c2.acpu, c2.rmem, c2.amem);
            ne = eval_core_fast(m, c, s_core.bwo[kk][t], pf, base, d, i, with1);
            ne2 = eval_core_fast(m, c2, wo2, pf, base, d, i);
            s_bwo2[kk][t] = wo2;
          }
          const unsigned long long b2 = __ballot(ne2.st == 0);
          if (lane == 0) s_ball2[kk][wave] = b2;
          s_fx2[kk][t] = ne2.fixed;
          s_rt2[kk][t] = (uint32_t)ne2.rt;
          s_rn2[kk][t] = (uint32_t)ne2.rna;
        } else if (i < m.n) {
          ne = fast ? eval_core_fast(m, lds_core(s_core, kk, t), s_core.bwo[kk][t], pf, base, d, i)
                    : eval_node<false>(m, b, base, d, pod, i, true);
        }
        record(kk, ne);
      }
    }
    publish_partials(par);
    if (lane == 0) __hip_atomic_fetch_add(&s_e_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // phase 2 over the slots of evaluation waves [vlo, vhi) of every block of my range (the selection
  // wave takes all four: splitting it with the helper wave slowed phase 1 more than it saved): positions in
  // the rotated feasible list, NormalizeScore + weights, the best packed (TotalScore, pre-order) key
  // percentageOfNodesToScore: only the first K feasible nodes of the rotated order are the feasible list
  // (cutK = K, else ~0); endn gets the node at global feasible index gK, the (K+1)-th of the rotated order
  auto phase2_half = [&](int vlo, int vhi, uint32_t acc, uint32_t F, uint32_t ps_before, int64_t mx_t, int64_t mx_n,
                         const PodDesc& d, int par, unsigned long long* key, int* knode, uint32_t cutK, uint32_t gK,
                         int* endn) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < kLoopMaxBlk; ++kk) {
      if (kk < nk) {
        // every LDS read of the block issued up front (unconditional), then the arithmetic
        unsigned long long ballot[NW];
        int64_t fx[NW], rt[NW], rn[NW];
#pragma unroll
        for (int v = 0; v < NW; ++v) {
          ballot[v] = s_ball[par][kk][v];
          if (v >= vlo && v < vhi) {
            fx[v] = s_fx[par][kk][v * 64 + lane];
            rt[v] = s_rt[par][kk][v * 64 + lane];
            rn[v] = s_rn[par][kk][v * 64 + lane];
          }
        }
#pragma unroll
        for (int v = 0; v < NW; ++v) {  // branch-free: independent chains interleave
          if (v >= vlo && v < vhi) {
            const bool f = ((ballot[v] >> lane) & 1ull) != 0;
            const uint32_t g = acc + wave_prefix_count(ballot[v], lane);
            const uint32_t pos = g >= ps_before ? g - ps_before : g + F - ps_before;
            const unsigned long long kv =
                f && pos < cutK ? pack_best(loop_total(d, fx[v], rt[v], rn[v], mx_t, mx_n), pos) : 0ull;
            *endn = f && g == gK ? (k0 + kk) * U + v * 64 + lane : *endn;
            *knode = kv > *key ? (k0 + kk) * U + v * 64 + lane : *knode;
            *key = kv > *key ? kv : *key;
          }
          acc += (uint32_t)__popcll(ballot[v]);
        }
      }
    }
  };
  // the normalising plugins' raw maxima over my nodes in the cut feasible list (rotated position < K):
  // NormalizeScore runs over the kept list only (schedule_one.go:937-1048 scores feasibleNodes)
  auto kept_max = [&](uint32_t acc, uint32_t F, uint32_t ps_before, uint32_t K, int par, unsigned long long* mt,
                      unsigned long long* mn) __attribute__((always_inline)) {
    for (int kk = 0; kk < nk; ++kk) {
#pragma unroll
      for (int v = 0; v < NW; ++v) {
        const unsigned long long ballot = s_ball[par][kk][v];
        const bool f = ((ballot >> lane) & 1ull) != 0;
        const uint32_t g = acc + wave_prefix_count(ballot, lane);
        const uint32_t pos = g >= ps_before ? g - ps_before : g + F - ps_before;
        if (f && pos < K) {
          const unsigned long long et = enc_i64(s_rt[par][kk][v * 64 + lane]), en = enc_i64(s_rn[par][kk][v * 64 + lane]);
          *mt = et > *mt ? et : *mt;
          *mn = en > *mn ? en : *mn;
        }
        acc += (uint32_t)__popcll(ballot);
      }
    }
  };
  // exchange A of pod `pq` (program parity par): this workgroup's two granules from the four
  // evaluation waves' partials.  One thread.
  auto publish_a = [&](int pq, int par) __attribute__((always_inline)) {
    uint32_t c = 0, bl = 0;
    unsigned long long a = 0, bb = 0;
    for (int v = 0; v < NW; ++v) {
      c += s_u[par][0][v];
      bl += s_u[par][1][v];
      a = s_x[par][0][v] > a ? s_x[par][0][v] : a;
      bb = s_x[par][1][v] > bb ? s_x[par][1][v] : bb;
    }
    const PodDesc& dp = *reinterpret_cast<const PodDesc*>(s_blob[pq % 3]);
    if (RING || (dp.flags & DF_ROTDEV)) {  // counted from the ballots (resident: phase 1 may have run ahead)
      const int srot = (dp.flags & DF_ROTDEV) ? (int)s_rot[pq & 1] : dp.rot_start;
      bl = 0;
      for (int kk = 0; kk < nk; ++kk)
        for (int v = 0; v < NW; ++v) bl += (uint32_t)__popcll(s_ball[par][kk][v] & below_mask_v(kk, v, srot));
    }
    unsigned long long g0, g1;
    a_granules(c, bl, a, bb, &g0, &g1);
    gran_put(lv, pq, gid, 0, g0);
    gran_put(lv, pq, gid, 1, g1);
    if (kSt && lv.wstamps) lv.wstamps[((size_t)pq * G + w) * 8] = __builtin_amdgcn_s_memrealtime();
  };

  if (!RING)
    for (int k = vt; k < lv.npods; k += kLoopThreads) {
      s_off[k] = b.desc_off[lv.first_pod + k];
      s_len[k] = lv.desc_bytes[lv.first_pod + k];
    }
  if (threadIdx.x == 0) {
    s_cand_q = -1;
    s_ga_q = -1;
    s_e_done = 0;
  }
  __syncthreads();
  // A batch launch is one run of pods [0, npods).  Resident mode (lv.ring): every pod is a run of its
  // own, started when the host posts it; the pod index q (granules, stamps, results) keeps counting.
  // resident mode: the pod whose phase 1 was evaluated ahead of its doorbell (-1: none; see the run's end)
  int spec_for = -1;
  for (int run0 = 0;;) {
  int run_end = lv.npods;
  if constexpr (RING) {
    // the tagged doorbell (PodRing::ll); RING_SAME: the previous call's program but for the slot and the
    // rotation (the host compared the bytes), copied in LDS instead of read over PCIe
    // (relay: workgroup 0 polls the host and relays the word through device memory, where the other workgroups
    // poll: one PCIe poller instead of G; a staged program is still read from the host's ring by all)
    if (threadIdx.x == 0) {
      const bool hostp = lv.relay == nullptr || blockIdx.x == 0;  // (RING: never GRP)
      const unsigned long long v = ring_wait_ctl(hostp ? &lv.ring->ctl : lv.relay, hostp ? &lv.ring->exited : nullptr,
                                                 run0, lv.npods, lv.ring_idle);
      if (lv.relay && hostp) __hip_atomic_store(lv.relay, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // stops too
      s_ring_ctl = v;
      // (diagnostic build: stamp 7 of a resident pod = workgroup 0 saw its doorbell; the batch loop's phase-1 end)
      if (kSt && lv.stamps && w == 0 && (v & kCtlStop) != kCtlStop) lv.stamps[(size_t)run0 * 8 + 7] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const unsigned long long ctl = s_ring_ctl;
    if (ctl == kCtlStop) return;
    if ((ctl >> 11) & 1ull) {
      if (threadIdx.x < 64) {  // one wave (kBlobLds / 8 words at most)
        int o = (int)threadIdx.x;
        asm volatile("" : "+v"(o));
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(s_blob[(run0 + 2) % 3]);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(s_blob[run0 % 3]);
        for (; o < s_pb / 8; o += 64) dst[o] = src[o];
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        PodDesc& dn = *reinterpret_cast<PodDesc*>(s_blob[run0 % 3]);
        dn.slot = (int32_t)((ctl >> 12) & 0x7fffffull) - 1;
        dn.rot_start = (int32_t)(ctl >> 35);
      }
    } else {
      const int bytes = (int)((ctl >> 12) & 0xffffull);
      const unsigned long long* src = reinterpret_cast<const unsigned long long*>(lv.ring->blob[run0 % kRingSlots]);
      unsigned long long* dst = reinterpret_cast<unsigned long long*>(s_blob[run0 % 3]);
      for (uint32_t o = threadIdx.x; o < (uint32_t)bytes / 8u; o += (uint32_t)kLoopThreads)
        dst[o] = __hip_atomic_load(src + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (threadIdx.x == 0) s_pb = bytes;
    }
    run_end = run0 + 1;
  } else {
    if (run0 >= run_end) return;
    if (hlp && lv.npods > 0) {
      stage_prog(lv.first_pod, 0);
      if (lv.npods > 1) stage_prog(lv.first_pod + 1, 1);
    }
  }
  __syncthreads();
  // (resident: a RING_SAME pod -- the previous call's program but for its slot and rotation, which phase 1 does not
  // read -- whose phase 1 ran ahead, against these same cores, skips it; publish_a recounts its nodes before the
  // rotation start from the ballots)
  const bool ahead = RING && spec_for == run0 && ((s_ring_ctl >> 11) & 1ull);
  if (t < U && !ahead) phase1(lv.first_pod + run0, run0 % 3, run0 & 1, nullptr);
  __syncthreads();
  if (vt == U) {
    const PodDesc& d0 = *reinterpret_cast<const PodDesc*>(s_blob[run0 % 3]);
    if (d0.flags & DF_ROTDEV)  // the previous launched pod's nextStartNodeIndex, or the host's
      s_rot[run0 & 1] = RING ? (uint32_t)d0.rot_start  // resident: the host's, from the previous call's result
                             : d0.prev_pod < 0 ? b.stats[lv.first_pod + run0].rot_in : b.stats[d0.prev_pod].rot_out;
    publish_a(run0, run0 & 1);
  }

  for (int q = run0; q < run_end; ++q) {
    if (q == lv.give_up_at) {  // diagnostic: as if a workgroup never arrived (host recovery test)
      if (threadIdx.x == 0) {
        __hip_atomic_store(lv.fail + 1, (uint32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(lv.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    const int pod = lv.first_pod + q, par = q & 1, npar = par ^ 1;
    const int bq = q % 3, bn = (q + 1) % 3, bs = (q + 2) % 3;
    const bool more = !RING && q + 1 < run_end;  // resident mode: every pod is a run of its own
    const uint8_t* base = s_blob[bq];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);

    if (sel) {
      // ======== selection wave: exchange A, phase 2, exchange B, pre-evaluation, staging ========
      stamp_s(q, 0);  // exchange A of this pod was published at the end of the previous one
      if (kSt && lv.wstamps && lane == 0) lv.wstamps[((size_t)q * G + w) * 8 + 7] = __builtin_amdgcn_s_memrealtime();
      unsigned long long xa[2][MS];
      bool ok = gran_sweep<2, MS>(lv, q, 0, xa);
      uint32_t F = 0, wp = 0, bf = 0;
      unsigned long long tmax = 0, nmax = 0;
#pragma unroll
      for (int r = 0; r < MS; ++r) {
        const int v = lane + 64 * r;
        if (v < P) {
          const uint32_t c = gran_a_count(xa[0][r]);
          F += c;
          if (v < gid) wp += c;
          bf += gran_a_below(xa[0][r]);
          const unsigned long long tv = gran_a_tp1(xa[1][r]), nv = gran_a_np1(xa[1][r]);
          tmax = tv > tmax ? tv : tmax;
          nmax = nv > nmax ? nv : nmax;
        }
      }
      F = wave_sum_u32(F);
      const uint32_t ps_before = wave_sum_u32(bf);
      uint32_t acc = wave_sum_u32(wp);  // feasible nodes before my range
      tmax = wave_max_u64(tmax);
      nmax = wave_max_u64(nmax);
      stamp_s(q, 1);

      // percentageOfNodesToScore (DF_ROTDEV, unsharded): findNodesThatPassFilters keeps the first K
      // feasible nodes of the rotated order and stops at the (K+1)-th (schedule_one.go:809-824)
      const bool rotd = (d.flags & DF_ROTDEV) != 0;
      const uint32_t K = rotd ? (uint32_t)d.num_to_find : 0xffffffffu;
      const bool cut = rotd && F > K;
      const uint32_t gK = cut ? (ps_before + K) % F : 0xffffffffu;  // its global feasible index
      if (cut && ok && (tmax > 1 || nmax > 1)) {
        // some raw TaintToleration / NodeAffinity score is > 0: NormalizeScore's maxima are over the kept
        // nodes only -- one more exchange (M, at pod index q + kLoopMaxPods) of the kept maxima
        unsigned long long mt = 0, mn = 0, g0, g1;
        kept_max(acc, F, ps_before, K, par, &mt, &mn);
        mt = wave_max_u64(mt);
        mn = wave_max_u64(mn);
        a_granules(mt != 0ull ? 1u : 0u, 0u, mt, mn, &g0, &g1);
        if (lane == 0) gran_put(lv, q + kLoopMaxPods, gid, 1, g1);
        unsigned long long xm[1][MS];
        ok = gran_sweep<1, MS>(lv, q + kLoopMaxPods, 1, xm);
        tmax = nmax = 0;
#pragma unroll
        for (int r = 0; r < MS; ++r) {
          if (lane + 64 * r < P) {
            const unsigned long long tv = xm[0][r] & 0xffffffull, nv = (xm[0][r] >> 24) & 0xffffffull;
            tmax = tv > tmax ? tv : tmax;
            nmax = nv > nmax ? nv : nmax;
          }
        }
        tmax = wave_max_u64(tmax);
        nmax = wave_max_u64(nmax);
      }

      // ---- phase 2: positions, NormalizeScore + weights, my range's best packed key
      const int64_t mx_t = tmax ? (int64_t)tmax - 1 : 0, mx_n = nmax ? (int64_t)nmax - 1 : 0;
      unsigned long long key = 0;
      int knode = -1, endn = -1;
      if (ok) phase2_half(0, NW, acc, F, ps_before, mx_t, mx_n, d, par, &key, &knode, K, gK, &endn);
      const unsigned long long wkey = wave_max_u64(key);
      const unsigned long long hold = __ballot(key == wkey && key != 0ull);
      const int cand = hold ? __builtin_amdgcn_readlane(knode, (int)__builtin_ctzll(hold)) : -1;
      stamp_s(q, 2);
      // the holder of the (K+1)-th node: processedNodes = its rotated position (K + the failures before it)
      uint32_t myproc = 0;
      if (rotd) {
        const unsigned long long eh = __ballot(endn >= 0);
        if (eh) {
          const int en = __builtin_amdgcn_readlane(endn, (int)__builtin_ctzll(eh));
          myproc = (uint32_t)(((int64_t)en - (int64_t)s_rot[par] + m.n) % m.n) + 1u;
        }
      }
      if (lane == 0) {
        gran_put(lv, q, gid, 2, wkey);  // < 2^48: TotalScore < 2^19 (host-checked) << 29 | pre-order key
        if (lv.world > 1) gran_put(lv, q, gid, 3, (unsigned long long)(uint32_t)cand);
        else if (rotd) gran_put(lv, q, gid, 3, (unsigned long long)myproc);
        if (kSt && lv.wstamps) lv.wstamps[((size_t)q * G + w) * 8 + 1] = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(&s_cand_node, cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&s_cand_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      stamp_s(q, 3);
      unsigned long long xb[2][MS];
      if (lv.world == 1 && rotd) {  // the keys and the (K+1)-th node's processedNodes
        ok = ok && gran_sweep<2, MS>(lv, q, 2, xb);
      } else if (lv.world == 1) {  // unsharded: the owner is found locally, only the keys cross workgroups
        unsigned long long k1[1][MS];
        ok = ok && gran_sweep<1, MS>(lv, q, 2, k1);
#pragma unroll
        for (int r = 0; r < MS; ++r) {
          xb[0][r] = k1[0][r];
          xb[1][r] = 0;
        }
      } else {
        ok = ok && gran_sweep<2, MS>(lv, q, 2, xb);
      }
      unsigned long long bm = 0, pm = 0;
      int bnode = -1;
#pragma unroll
      for (int r = 0; r < MS; ++r) {
        const unsigned long long v = (lane + 64 * r) < P ? xb[0][r] : 0ull;
        if (v > bm) {
          bm = v;
          bnode = (int)(uint32_t)xb[1][r];
        }
        if (rotd && (lane + 64 * r) < P) pm = xb[1][r] > pm ? xb[1][r] : pm;
      }
      uint32_t rot_next = 0;
      if (rotd) {  // nextStartNodeIndex for the next pod (schedule_one.go:686-687); all processed without a cut
        pm = wave_max_u64(pm);
        const uint32_t proc = cut && pm ? (uint32_t)pm - 1u : (uint32_t)m.n;
        rot_next = m.n > 0 ? (uint32_t)(((uint64_t)s_rot[par] + proc) % (uint64_t)m.n) : 0u;
        if (lane == 0) {
          s_proc = proc;
          s_rot[npar] = rot_next;
        }
      }
      if (kSt && lv.wstamps && lane == 0) lv.wstamps[((size_t)q * G + w) * 8 + 4] = __builtin_amdgcn_s_memrealtime();
      const unsigned long long gbest = wave_max_u64(bm);
      const unsigned long long bh = __ballot(bm == gbest && gbest != 0ull);  // keys are unique
      const int gnode = bh ? __builtin_amdgcn_readlane(bnode, (int)__builtin_ctzll(bh)) : -1;
      bm = gbest;
      const int win = (F > 0 && wkey == bm && cand >= 0) ? cand : -1;
      if (lane == 0) {
        s_ok = ok ? 1u : 0u;
        s_best = bm;
        s_F = cut ? K : F;  // the feasible list's length
        s_win = win;
        s_gnode = F > 0 ? gnode : -1;
      }
      // exchange A of pod q+1, now: the pair the helper prepared for this outcome.  A chosen node
      // whose next evaluation was not prepared (generic pods) is fixed up after the barrier, and its
      // owner publishes then.
      if (more && ok) {
        while (__hip_atomic_load(&s_ga_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
          __builtin_amdgcn_s_sleep(1);
        const bool chosen = win >= 0 && (d.flags & DF_ASSUME);
        unsigned long long ga0 = s_ga[chosen ? 2 : 0];
        if (rotd && (!chosen || s_cand_ok)) {  // pod q+1's count before its rotation start, now known
          const int wsl = chosen ? win - k0 * U : -1;
          const uint32_t bl = below_wave(npar, (int)rot_next, chosen ? wsl / U : -1, chosen ? (wsl % U) >> 6 : -1,
                                         s_cball);
          ga0 = gran_a_counts(gran_a_count(ga0), bl);
        }
        if (lane == 0 && (!chosen || s_cand_ok)) {
          gran_put(lv, q + 1, gid, 0, ga0);
          gran_put(lv, q + 1, gid, 1, s_ga[chosen ? 3 : 1]);
          if (kSt && lv.wstamps) lv.wstamps[((size_t)(q + 1) * G + w) * 8] = __builtin_amdgcn_s_memrealtime();
        }
      }
      stamp_s(q, 4);
    } else if (hlp) {
      // ======== helper wave: stage pod q+2's program; once phase 1 of pod q+1 is done and the
      // selection wave's candidate known, prepare this workgroup's exchange-A granules of pod q+1
      // both ways -- the candidate not chosen (phase 1 as it is), and chosen (its next evaluation
      // with this pod assumed, computed in phase 1 for default-plugin pods) -- so the selection
      // wave publishes the right pair as soon as exchange B resolves.
      const bool stage = !RING && q + 2 < run_end;
      if (lane == 0) s_ipa = (int)b.stats[pod].ipa_any;  // for the result record (off the critical path)
      if (stage) stage_prog(pod + 2, bs);  // s_blob[(q + 2) % 3] held pod q-1, free since the last barrier
      while (__hip_atomic_load(&s_cand_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)  // posted every pod
        __builtin_amdgcn_s_sleep(1);
      const int cand = __hip_atomic_load(&s_cand_node, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint32_t cand_ok = 0;
      if (more) {
        const uint8_t* nb = s_blob[bn];
        const PodDesc& nd = *reinterpret_cast<const PodDesc*>(nb);
        cand_ok = cand >= 0 && post_ok(d, nd) ? 1u : 0u;
        while (__hip_atomic_load(&s_e_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
               (uint32_t)(NW) * (uint32_t)(q + 2))
          __builtin_amdgcn_s_sleep(1);
        // Everything both variants read is loaded at once (independent LDS reads, one round trip), and
        // the candidate's replacement values are formed in registers: this runs between phase 1 of pod
        // q+1 and exchange A, where the owner of the previous pod's node is already the latest.
        uint32_t u0[NW], u1[NW];
        unsigned long long x0[NW], x1[NW];
#pragma unroll
        for (int v = 0; v < NW; ++v) {
          u0[v] = s_u[npar][0][v];
          u1[v] = s_u[npar][1][v];
          x0[v] = s_x[npar][0][v];
          x1[v] = s_x[npar][1][v];
        }
        int cw = -1;
        unsigned long long tm = 0, tn = 0, nbal = 0;
        uint32_t ccnt = 0, cbelow = 0;
        if (cand_ok && (nd.flags & DF_RAW0)) {
          // every raw TaintToleration / NodeAffinity score is 0: a wave's maxima are enc(0) when it has a
          // feasible node, else 0 -- the chosen variant needs only the candidate's feasibility bit
          const int kw = cand / U - k0, sl = cand % U, cl = sl & 63;
          cw = sl >> 6;
          const unsigned long long b2 = s_ball2[kw][cw];
          unsigned long long old = 0;
#pragma unroll
          for (int kk = 0; kk < kLoopMaxBlk; ++kk)
            if (kk < nk && kk == kw) old = s_ball[npar][kk][cw];
          const bool cf = ((b2 >> cl) & 1ull) != 0;
          const unsigned long long bit = 1ull << cl;
          nbal = cf ? (old | bit) : (old & ~bit);
          const int lim = nd.rot_start - ((k0 + kw) * U + cw * 64);
          const unsigned long long bmk = lim <= 0 ? 0ull : lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
          uint32_t ucw0 = 0, ucw1 = 0;
#pragma unroll
          for (int v = 0; v < NW; ++v) {
            ucw0 = v == cw ? u0[v] : ucw0;
            ucw1 = v == cw ? u1[v] : ucw1;
          }
          ccnt = ucw0 - (uint32_t)__popcll(old) + (uint32_t)__popcll(nbal);
          cbelow = ucw1 - (uint32_t)__popcll(old & bmk) + (uint32_t)__popcll(nbal & bmk);
          tm = tn = ccnt > 0 ? enc_i64(0) : 0ull;
        } else if (cand_ok) {  // the candidate's evaluation wave, as its partials will be if it wins
          const int kw = cand / U - k0, sl = cand % U, cl = sl & 63;
          cw = sl >> 6;
          const unsigned long long b2 = s_ball2[kw][cw];
          const int64_t crt = s_rt2[kw][sl], crn = s_rn2[kw][sl];
          unsigned long long bk[kLoopMaxBlk];
          int64_t rtk[kLoopMaxBlk], rnk[kLoopMaxBlk];
#pragma unroll
          for (int kk = 0; kk < kLoopMaxBlk; ++kk) {
            bk[kk] = kk < nk ? s_ball[npar][kk][cw] : 0ull;
            rtk[kk] = kk < nk ? (int64_t)s_rt[npar][kk][sl] : 0;
            rnk[kk] = kk < nk ? (int64_t)s_rn[npar][kk][sl] : 0;
          }
          tm = s_tm[npar][cw * 64 + lane];
          tn = s_tn[npar][cw * 64 + lane];
          const bool cf = ((b2 >> cl) & 1ull) != 0;
          // the candidate lane's maxima over its blocks, block kw with the post-assume values (uniform)
          unsigned long long am = 0, an = 0, old = 0;
#pragma unroll
          for (int kk = 0; kk < kLoopMaxBlk; ++kk) {
            if (kk < nk) {
              const bool f = kk == kw ? cf : ((bk[kk] >> cl) & 1ull) != 0;
              const unsigned long long et = enc_i64(kk == kw ? crt : rtk[kk]);
              const unsigned long long en = enc_i64(kk == kw ? crn : rnk[kk]);
              am = f && et > am ? et : am;
              an = f && en > an ? en : an;
              old = kk == kw ? bk[kk] : old;
            }
          }
          if (lane == cl) {
            tm = am;
            tn = an;
          }
          tm = wave_max_u64(tm);
          tn = wave_max_u64(tn);
          const unsigned long long bit = 1ull << cl;
          nbal = cf ? (old | bit) : (old & ~bit);
          const int lim = nd.rot_start - ((k0 + kw) * U + cw * 64);
          const unsigned long long bmk = lim <= 0 ? 0ull : lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
          uint32_t ucw0 = 0, ucw1 = 0;
#pragma unroll
          for (int v = 0; v < NW; ++v) {
            ucw0 = v == cw ? u0[v] : ucw0;
            ucw1 = v == cw ? u1[v] : ucw1;
          }
          ccnt = ucw0 - (uint32_t)__popcll(old) + (uint32_t)__popcll(nbal);
          cbelow = ucw1 - (uint32_t)__popcll(old & bmk) + (uint32_t)__popcll(nbal & bmk);
        }
        if (lane == 0) {
          uint32_t c = 0, bl = 0, cc = 0, cbl = 0;
          unsigned long long xa = 0, xb = 0, ca = 0, cb = 0;
#pragma unroll
          for (int v = 0; v < NW; ++v) {
            c += u0[v];
            bl += u1[v];
            xa = x0[v] > xa ? x0[v] : xa;
            xb = x1[v] > xb ? x1[v] : xb;
            const uint32_t w0 = v == cw ? ccnt : u0[v], w1 = v == cw ? cbelow : u1[v];
            const unsigned long long y0 = v == cw ? tm : x0[v], y1 = v == cw ? tn : x1[v];
            cc += w0;
            cbl += w1;
            ca = y0 > ca ? y0 : ca;
            cb = y1 > cb ? y1 : cb;
          }
          if (cw >= 0) {  // the owner's commit installs these (after the barrier)
            s_cball = nbal;
            s_ccnt = ccnt;
            s_cbelow = cbelow;
            s_cmt = tm;
            s_cmn = tn;
          }
          a_granules(c, bl, xa, xb, &s_ga[0], &s_ga[1]);
          a_granules(cc, cbl, ca, cb, &s_ga[2], &s_ga[3]);
        }
      }
      if (lane == 0) {
        s_cand_ok = cand_ok;
        if (kSt && lv.wstamps) lv.wstamps[((size_t)q * G + w) * 8 + 5] = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(&s_ga_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }

    } else if (more) {
      // ======== evaluation waves: phase 1 of pod q+1 against the cores before this pod's assume.
      // Only the chosen node changes; its owner redoes it below.
      phase1(pod + 1, bn, npar, &d);
      if (kSt && lv.stamps && w == 0 && t == 0) lv.stamps[(size_t)q * 8 + 7] = __builtin_amdgcn_s_memrealtime();
      if (kSt && lv.wstamps && lane == 0)  // the last evaluation wave's phase-1 end
        atomicMax(&lv.wstamps[((size_t)q * G + w) * 8 + 6], __builtin_amdgcn_s_memrealtime());
    }
    __syncthreads();
    if (!s_ok) return;
    stamp_s(q, 5);

    // ---- the winning node's owner fixes up pod q+1's phase 1, publishes its exchange A, then
    // assumes + reports this pod; every other workgroup's selection wave publishes A at once
    {
      const uint32_t F = s_F;
      const int win = s_win;
      const int wsl = win >= 0 ? win - k0 * U : -1;  // kk * U + slot
      const bool owner_wg = F > 0 && wsl >= 0 && (d.flags & DF_ASSUME);
      const int gnode = s_gnode;
      const bool remote = lv.world > 1 && F > 0 && (gnode < lv.blk0 * kBlock || gnode >= (lv.blk0 + lv.nblk) * kBlock);
      if (!owner_wg) {  // exchange A of pod q+1 already published by the selection wave
        if (F == 0) {
          if (w == 0 && t == 0) {
            commit_result(m, b, base, d, rot_stats(pod, par), pod, F, -1, s_best, nullptr, s_ipa);
            if constexpr (RING) ring_post(lv, q, b.results[pod]);
          }
        } else if (wsl >= 0 && t == wsl % U) {  // chosen here, not assumed
          commit_result(m, b, base, d, rot_stats(pod, par), pod, F, win, s_best, nullptr, s_ipa);
          if constexpr (RING) ring_post(lv, q, b.results[pod]);
        } else if (remote && w == 0 && t == 0) {  // chosen on another rank: the result and this replica's assume
          commit_result(m, b, base, d, rot_stats(pod, par), pod, F, gnode, s_best, nullptr, s_ipa);
        }
      } else if (s_cand_ok) {  // the helper prepared everything: LDS stores, then publish
        if (t == wsl % U) {
          const int kw = wsl / U, cw = t >> 6;
          if (kSt && lv.wstamps) lv.wstamps[((size_t)q * G + w) * 8 + 2] = __builtin_amdgcn_s_memrealtime();
          NodeCore c = lds_core(s_core, kw, t);
          assume_core(c, d);
          s_core.rcpu[kw][t] = c.rcpu;
          s_core.rmem[kw][t] = c.rmem;
          s_core.reph[kw][t] = c.reph;
          s_core.nzcpu[kw][t] = c.nzcpu;
          s_core.nzmem[kw][t] = c.nzmem;
          s_core.npods[kw][t] = c.npods;
          s_core.bwo[kw][t] = s_bwo2[kw][t];
          s_fx[npar][kw][t] = s_fx2[kw][t];
          s_rt[npar][kw][t] = s_rt2[kw][t];
          s_rn[npar][kw][t] = s_rn2[kw][t];
          s_ball[npar][kw][cw] = s_cball;
          s_u[npar][0][cw] = s_ccnt;
          s_u[npar][1][cw] = s_cbelow;
          s_x[npar][0][cw] = s_cmt;
          s_x[npar][1][cw] = s_cmn;
          if (kSt && lv.wstamps) lv.wstamps[((size_t)q * G + w) * 8 + 3] = __builtin_amdgcn_s_memrealtime();
          commit_result(m, b, base, d, rot_stats(pod, par), pod, F, win, s_best, &c, s_ipa);
          if constexpr (RING) ring_post(lv, q, b.results[pod]);
        }
      } else if (t < U && wave == ((wsl % U) >> 6)) {  // generic pods: re-evaluate here
        const int kw = wsl / U, owner = wsl % 64;
        const uint8_t* nb = s_blob[bn];
        const PodDesc& nd = *reinterpret_cast<const PodDesc*>(nb);
        bool feas = ((s_ball[npar][kw][wave] >> lane) & 1ull) != 0;
        if (lane == owner) {
          NodeCore c = lds_core(s_core, kw, t);
          assume_core(c, d);
          commit_result(m, b, base, d, rot_stats(pod, par), pod, F, win, s_best, &c, s_ipa);  // before the re-read
          if constexpr (RING) ring_post(lv, q, b.results[pod]);
          lds_put_dynamic(s_core, kw, t, c);
          if (more) {
            const NodeEval ne = (nd.flags & DF_FAST)
                                    ? eval_core_fast(m, c, s_core.bwo[kw][t], load_fast(nb, nd), nb, nd, win)
                                    : eval_node<false>(m, b, nb, nd, pod + 1, win, true);
            feas = ne.st == 0;
            s_fx[npar][kw][t] = ne.fixed;
            s_rt[npar][kw][t] = (uint32_t)ne.rt;
            s_rn[npar][kw][t] = (uint32_t)ne.rna;
            t_mt = t_mn = 0;  // my maxima again, over my (possibly changed) feasible nodes
            for (int kk = 0; kk < nk; ++kk) {
              const bool f = kk == kw ? feas : ((s_ball[npar][kk][wave] >> lane) & 1ull) != 0;
              if (f) {
                const unsigned long long et = enc_i64(s_rt[npar][kk][t]), en = enc_i64(s_rn[npar][kk][t]);
                t_mt = et > t_mt ? et : t_mt;
                t_mn = en > t_mn ? en : t_mn;
              }
            }
          }
        }
        if (more) {
          const unsigned long long old = s_ball[npar][kw][wave];
          const unsigned long long nbal = __ballot(feas);
          const unsigned long long bmk = below_mask(kw, nd.rot_start);
          w_cnt = w_cnt - (uint32_t)__popcll(old) + (uint32_t)__popcll(nbal);
          w_below = w_below - (uint32_t)__popcll(old & bmk) + (uint32_t)__popcll(nbal & bmk);
          if (lane == 0) s_ball[npar][kw][wave] = nbal;
          publish_partials(npar);
          if (lane == 0) publish_a(q + 1, npar);  // the other waves' partials are final since the barrier
        }
      }
    }
    DIAG_FLUSH();
    __syncthreads();  // pod q+1's phase-1 state is final; s_blob[q % 3] is free again
    stamp_s(q, 6);
  }
  if constexpr (!RING) return;
  // Resident: the next call's pod is most often of this one's template (kube-scheduler pops a ReplicaSet's pods
  // one after another).  Its phase 1 against the cores as this commit left them runs now, before its doorbell,
  // and is used if the doorbell says RING_SAME.  Default-plugin pods only (the fast path reads no HBM column).
  if (lv.ring_ahead && (reinterpret_cast<const PodDesc*>(s_blob[run0 % 3])->flags & DF_FAST) && run_end < lv.npods) {
    if (t < U) phase1(lv.first_pod + run_end, run0 % 3, run_end & 1, nullptr);
    spec_for = run_end;
  } else {
    spec_for = -1;
  }
  run0 = run_end;
  }
}
// The views are read where the kernel arguments lie (the kernarg segment, laid out as LoopGroupArg): binding the
// by-value parameters to the body's references made the compiler copy them into registers up front (scratch spills)
template <int NW, bool RING, int MS = kMaxSweep>
__global__ __launch_bounds__(NW * 64 + 128) void k_sched_loop(MirrorView m, BatchView b, LoopView lv) {
  const LoopGroupArg& a = *(const LoopGroupArg*)__builtin_amdgcn_kernarg_segment_ptr();
  sched_loop_body<NW, RING, MS, false>(a.m, a.b, a.lv, 0);
}
// In-process rank groups (localGroup: W contexts on one device): every rank's loop in ONE dispatch, block
// r * G + w playing rank r's workgroup w with rank r's views.  Loops of separate dispatches on separate
// hardware queues are not co-scheduled by the command processor (one rank's loop entered only
// when its peers gave up); the workgroups of one dispatch that fits the device are.
template <int NW, int MS>
__global__ __launch_bounds__(NW * 64 + 128) void k_sched_loop_group(const LoopGroupArg* __restrict__ ga, int G) {
  const int r = (int)blockIdx.x / G;
  const LoopGroupArg& a = ga[r];
  sched_loop_body<NW, false, MS, true>(a.m, a.b, a.lv, (int)blockIdx.x - r * G);
}


// =====================================================================================================
// k_agg_loop -- the persistent loop for pods with pod-table aggregation
// =====================================================================================================
// PodTopologySpread / InterPodAffinity pods (SchedulingPodAffinity, TopologySpreading, the mixed
// cluster) in one launch, instead of k_aggregate + k_filter_score + k_select per pod.  Geometry as
// k_sched_loop: G resident workgroups, workgroup w owns the node blocks [k0, k1) for the whole run
// and keeps their cores in LDS.  It also owns the pod-table slots and existing affinity terms of the
// pods bound to those nodes (scanned once per launch; the owner of a chosen node appends the
// assumed pod and its terms).  Per pod q, three granule exchanges (Z, A, B):
//   aggregation  node role (DoNotSchedule eligibility, shared-domain presence), pod role (the
//                pod's selectors against my pods), term role (my existing terms against the pod).
//                Counts on a key whose values are each on one node (kubernetes.io/hostname) are
//                complete here: they stay in LDS, one per node.  Counts on shared keys (zones)
//                are partial: staged in LDS, added to the pod's compact region in HBM.
//   xchg Z       {IPA any bits}, {min count | eligible nodes} of each node-local DoNotSchedule
//                constraint over my nodes.  After it: the region's totals into LDS, and each
//                shared DoNotSchedule constraint's minimum over its present domains.
//   phase 1      RunFilterPlugins + raw scores of my nodes (LDS cores, LDS counts)
//   xchg A       {feasible | before nextStartNodeIndex}, {max raw TT + 1 | max raw NA + 1},
//                max and min raw InterPodAffinity (biased)
//   phase 2      positions in the rotated feasible list, NormalizeScore + weights, best packed key
//   xchg B       {key}; the owner of the maximum commits (AssumePod on the LDS core + mirror).
struct AggTopo {
  const unsigned long long* gh;  // shared-region totals of the pod
  const int32_t* lh;             // node-local counts [histogram][kAggSlots]
  const long long* mn;           // DoNotSchedule minimum per constraint
  const uint32_t* nd;            // DoNotSchedule domains per constraint
  uint32_t ipa_any;
  __device__ __forceinline__ int64_t cnt(int32_t, int32_t lref, int32_t v, int ls) const;
  __device__ __forceinline__ int64_t pmin(int c) const { return mn[c]; }
  __device__ __forceinline__ uint32_t pndom(int c) const { return nd[c]; }
  __device__ __forceinline__ uint32_t any() const { return ipa_any; }
};
constexpr int kAggSlots = kAggSlotsC;  // node slots per workgroup
__device__ __forceinline__ int64_t AggTopo::cnt(int32_t, int32_t lref, int32_t v, int ls) const {
  return lref >= 0 ? (int64_t)gh[lref + v] : (int64_t)lh[(size_t)(-1 - lref) * kAggSlots + ls];
}

// RunFilterPlugins + raw scores of node i for the loop (eval_node's plugin set minus the
// PodTopologySpread score, which the loop does not take)
// DF_LFAST: the node-local plugins by eval_core_fast (bal_wo: the core's BalancedAllocation without
// the pod), then the PodTopologySpread / InterPodAffinity filters.
__device__ __forceinline__ NodeEval eval_agg(const MirrorView& m, const NodeCore& nc, int64_t bal_wo, const PodFast& pf,
                                             const uint8_t* base, const PodDesc& d, int i, const AggTopo& tp, int ls) {
  NodeEval r{1u, false, 0, 0, 0, 0};
  const uint32_t sm = d.score_mask;
  if (pf.flags & DF_LFAST) {
    r = eval_core_fast(m, nc, bal_wo, pf, base, d, i);
    if (r.st == 0) r.st = topo_filters(m, base, d, i, tp, ls);
    if (r.st) return r;
  } else {
    int64_t raw_taint = 0;
    const uint32_t st = run_filters(m, nc, base, d, i, &raw_taint, tp, ls);
    r.st = st;
    if (st) return r;
    int64_t fixed = 0;
    if ((sm >> P_TAINT) & 1u) r.rt = raw_taint;
    if ((sm >> P_NA) & 1u) {
      int64_t sc = 0;
      if (d.flags & DF_HAS_ADDED_PREF) sc += prog_weight(m, base, d, d.na_added_pref, i);
      if (d.flags & DF_HAS_PREF_NA) sc += prog_weight(m, base, d, d.na_preferred, i);
      r.rna = sc;
    }
    if ((sm >> P_FIT) & 1u) fixed += fit_score(m, nc, base, d, i) * d.weight[P_FIT];
    if ((sm >> P_BAL) & 1u) fixed += balanced_alloc_score(m, nc, base, d, i) * d.weight[P_BAL];
    if ((sm >> P_IMG) & 1u) fixed += image_score_range(m, base, d, nc.ilo, nc.ihi) * d.weight[P_IMG];
    r.fixed = fixed;
  }
  if ((sm >> P_IPA) & 1u) {  // InterPodAffinity.Score (interpodaffinity/scoring.go:240-255)
    const KeyHist* tk = at<KeyHist>(base, d.topokeys_off);
    int64_t sc = 0;
    for (int32_t k = 0; k < d.n_topokeys; ++k) {
      const int32_t v = node_label(m, tk[k].slot, i);
      if (v >= 0) sc += tp.cnt(tk[k].base, tk[k].lref, v, ls);
    }
    r.ripa = sc;
  }
  return r;
}

// NormalizeScore + weights (framework.go:1409-1452): node_total's arithmetic on the loop's values
__device__ __forceinline__ int64_t agg_total(const PodDesc& d, int64_t fixed, int64_t rt, int64_t rn, int64_t ri,
                                             int64_t mx_t, int64_t mx_n, int64_t mx_i, int64_t mn_i, uint32_t any) {
  if (d.flags & DF_NO_SCORE) return 1;
  int64_t total = loop_total(d, fixed, rt, rn, mx_t, mx_n);
  if ((d.score_mask >> P_IPA) & 1u) {  // interpodaffinity/scoring.go:258-290
    int64_t v = ri;
    if (any & 8u) {
      const int64_t diff = mx_i - mn_i;
      double f = 0.0;
      if (diff > 0) f = 100.0 * ((double)(ri - mn_i) / (double)diff);
      v = (int64_t)f;
    }
    total += v * d.weight[P_IPA];
  }
  return total;
}

// publish granule `slot` of participant gid (rank-major) for pod q: unsharded, an agent-scope store;
// node-sharded, a system-scope store into every rank's array (k_sched_loop's gran_put)
template <bool SHARD>
__device__ __forceinline__ void agran_put(const AggView& av, int q, int gid, int slot, unsigned long long payload) {
  const size_t at = ((size_t)q * (SHARD ? av.world : 1) * av.nwg + gid) * kAGran + slot;
  const unsigned long long v = gran_word(av.tag, payload);
  if constexpr (!SHARD) {
    __hip_atomic_store(av.gran + at, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
#pragma unroll
    for (int r = 0; r < kMaxShards; ++r)
      if (r < av.world) __hip_atomic_store(av.grans[r] + at, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// One wave: poll granules [slot0, slot0 + nact) of every participant for pod q until all tags match, and hand
// each round of 64 participants' payloads to visit(r, x).  Round by round (ALL false): a round is visited as soon
// as it is all there, so no round's payloads stay live (MS rounds of NS 64-bit granules held together were the
// batch loop's register peak; the later rounds have usually arrived by then).  ALL: every round polled together,
// then visited (the resident instance, whose register allocation fits that form).
template <bool SHARD, int NS, int MS, bool ALL, class V>
__device__ __forceinline__ bool agran_sweep(const AggView& av, int q, int slot0, V&& visit, int nact = NS) {
  const int lane = threadIdx.x & 63;
  const int P = (SHARD ? av.world : 1) * av.nwg;
  const unsigned long long* g = av.gran + (size_t)q * P * kAGran + slot0;
  const unsigned long long want = (unsigned long long)av.tag;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  constexpr int kR = ALL ? MS : 1;  // rounds polled together
  uint32_t spins = 0;
#pragma unroll 1
  for (int r0 = 0; r0 < MS; r0 += kR) {
    if (64 * r0 >= P) break;
    unsigned long long x[kR][NS];
    for (;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int v = lane + 64 * (r0 + r);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          unsigned long long y = want << 48;
          if (v < P && k < nact)
            y = SHARD ? __hip_atomic_load(g + (size_t)v * kAGran + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                      : __hip_atomic_load(g + (size_t)v * kAGran + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (y >> 48) == want;
          x[r][k] = y & kPayload;
        }
      }
      if (__all(ok)) break;
      if ((spins & 255u) == 255u && __builtin_amdgcn_s_memrealtime() - t_start > 1000000000ull) {
        const unsigned long long miss = __ballot(!ok);
        uint32_t first = 0u;  // the first failure's record is kept (a later give-up is its consequence)
        if (lane == 0 && __hip_atomic_compare_exchange_strong(av.fail, &first, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(av.fail + 1, (uint32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(av.fail + 2, (uint32_t)slot0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(av.fail + 3, (uint32_t)__builtin_ctzll(miss), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(av.fail + 4, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // k_agg_loop
          __hip_atomic_store(av.fail + 5, (uint32_t)av.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(av.fail + 6, (uint32_t)miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(av.fail + 7, (uint32_t)(miss >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          give_up_record(av.fail);
        }
        return false;
      }
      if ((spins & 63u) == 63u && __hip_atomic_load(av.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int r = 0; r < kR; ++r)
      if (64 * (r0 + r) < P) visit(r0 + r, x[r]);
  }
  return true;
}

// k_agg_loop's resident mode: the committed pod's pod-table entry (RingEntry, staged in LDS) into the
// device pod table -- what Cluster::upload_pod_table would write for it -- so that the pods after it
// count it (the owner of its node appends it to its lists).  One thread; pod_node is commit_result's.
__device__ __forceinline__ void apply_entry(const MirrorView& m, const uint8_t* e) {
  const RingEntry& h = *reinterpret_cast<const RingEntry*>(e);
  if (h.slot < 0) return;
  const size_t s = (size_t)h.slot;
  const_cast<int32_t*>(m.pod_ns)[s] = h.ns;
  const_cast<uint32_t*>(m.pod_flags)[s] = h.flags;
  const_cast<uint32_t*>(m.pod_lbl_off)[s] = h.lbl_off;
  const_cast<uint32_t*>(m.pod_lbl_cnt)[s] = h.lbl_cnt;
  const unsigned long long* lb = reinterpret_cast<const unsigned long long*>(e + sizeof(RingEntry));
  unsigned long long* pool = const_cast<unsigned long long*>(m.lbl_pool) + h.lbl_off;
  for (uint32_t k = 0; k < h.lbl_cnt; ++k) pool[k] = lb[k];
  const int32_t* tw = reinterpret_cast<const int32_t*>(lb + h.lbl_cnt);
  int32_t* tp = const_cast<int32_t*>(m.term_pool) + h.tpool_off;
  for (int32_t k = 0; k < h.tpool_cnt; ++k) tp[k] = tw[k];
  const RingTerm* rt = reinterpret_cast<const RingTerm*>(tw + ((h.tpool_cnt + 1) & ~1));
  DTerm* terms = const_cast<DTerm*>(m.terms);
  for (int32_t k = 0; k < h.nterms; ++k) terms[rt[k].j] = rt[k].d;
}

// SHARD: node-sharded over the device exchange (av.world > 1); the unsharded instance compiles none of it.
// PTSS: some pod of the run has PodTopologySpread scoring (ScheduleAnyway constraints); the instance
// without it leaves that code out (its registers and issue slots cost the other pods ~1 us).
// RING: the resident instance (ksg_schedule_one of PodTopologySpread / InterPodAffinity pods):
// pods through av.ring, each a run of its own -- gathered when it arrives (or, same template, folded at the
// end of the pod before it), no staging ahead.
// MS: sweep rounds of 64 participants (kMaxSweep = 4: up to 256; the 1-round instance for grids of at most 64
// workgroups holds a quarter of the exchange registers, which pays for the PodTopologySpread PX skip, as in RING)
// (the body of k_agg_loop and k_agg_loop_group: w = the workgroup this block plays in its rank)
template <bool SHARD, bool PTSS, bool RING, int MS, bool GRP>
__device__ __forceinline__ void agg_loop_body(const MirrorView& m, const BatchView& b, const AggView& av, const int w_grp) {
  constexpr bool kPxa = RING || MS < kMaxSweep;  // phase 1 guesses the PTS raw scores (AG_PXA)
  constexpr int kBlob = RING ? kBlobLds : kAggBlobLds;       // program slot bytes (desc.h)
  constexpr uint32_t kLp = RING ? kAggRingPods : kAggPods;     // LDS list entries (the rest spill to HBM)
  constexpr uint32_t kLt = RING ? kAggRingTerms : kAggTerms;
  __shared__ __align__(16) uint8_t s_blob[3][kBlob];  // pod p's program in s_blob[p % 3]
  __shared__ LoopCores s_core;
  // phase-1 slots: {weighted fixed score, raw TaintToleration, raw NodeAffinity} in one 16-byte
  // record (one LDS read in phase 2), raw InterPodAffinity apart (read only when it scores)
  struct SlotVal { int64_t fixed; uint32_t rt, rn; };
  __shared__ __align__(16) SlotVal s_sv[kAggSlots];
  __shared__ int64_t s_ri[kAggSlots];
  __shared__ unsigned long long s_ball[kAggThreads / 64];  // [wave] feasibility ballots
  __shared__ int32_t s_lh[kAggLocal * kAggSlots];          // node-local histograms
  __shared__ unsigned long long s_gh[kAggGWords];          // shared-region partials, then totals
  __shared__ __align__(16) uint16_t s_elig[kAggSlots];     // eligibility per node: DoNotSchedule c (bit c),
                                                           // ScheduleAnyway c (bit 8 + c)
  __shared__ uint32_t s_pc[kAggScoreCons][kAggSlots];      // PodTopologySpread score: count at my node's
                                                           // domain per constraint (~0u: the node lacks the key)
  __shared__ uint32_t s_pods[kLp], s_terms[kLt];  // (slot | term) << 9 | node slot
  __shared__ uint32_t s_np, s_nt;
  __shared__ uint32_t s_off[kLoopMaxPods];
  __shared__ long long s_pmin[kAggMaxCons];
  __shared__ uint32_t s_pndom[kAggMaxCons];
  __shared__ uint32_t s_any, s_gany, s_ok, s_F, s_psb, s_acc, s_gbar;
  __shared__ long long s_lmin[kAggLocalCons];
  __shared__ uint32_t s_lcnt[kAggLocalCons];
  __shared__ uint32_t s_latm[kAggLocalCons];   // my eligible nodes at my minimum (exchange Z)
  __shared__ uint32_t s_lmult[kAggLocalCons];  // eligible nodes at the global minimum (exchange Z, then the folds)
  __shared__ uint32_t s_bc[kAggLocalCons];     // the chosen node's counts under them before the fold (exchange B)
  __shared__ uint32_t s_lstale;                // a fold took the last node off a minimum: exchange Z again
  __shared__ unsigned long long s_wx[kAggThreads / 64][4];
  __shared__ uint32_t s_wu[kAggThreads / 64][3];           // feasible, before the start, PTS non-ignored
  __shared__ unsigned long long s_wp[kAggThreads / 64][2]; // PTS domain presence bits [0, 64), [64, 128)
  __shared__ uint32_t s_psz[kAggScoreCons];                // PTS topology sizes of the pod being decided
  __shared__ uint32_t s_psz_used[kAggScoreCons];           // ... of the previous PTS-scored pod (~0: none),
  __shared__ double s_pwt[kAggScoreCons];                  //   their weights log(size + 2),
  __shared__ uint32_t s_praw[PTSS && kPxa ? kAggThreads : 1];  // phase 1's raw scores with them (~0: not scored)
  __shared__ unsigned long long s_wq[kAggThreads / 64][2]; //   and their per-wave {max + 1, 2^24 - 1 - min}
  __shared__ unsigned long long s_pxm[2];                  // wave 1 -> 0: its half's raw PTS max+1 / reversed min
  __shared__ int s_px_q, s_pxd_q;                          // wave 1 -> 0: half done; wave 0 -> 1: exchange PX done
  __shared__ int64_t s_pts_mx, s_pts_mn;                   // PTS NormalizeScore max / min of the pod
  __shared__ int s_gnode, s_pend_ls;  // the chosen node of the pod just decided; my pending list append
  __shared__ unsigned long long s_best;
  // the fold plan of pod q into pod q+1 (built while pod q is decided): what q+1's aggregation would
  // add for pod q at its node, keyed by the label slot it is counted under
  struct FoldItem { int32_t lref, slot, cons, wt; uint32_t anyb; int32_t absent; };  // cons >= 8: score constraint
  constexpr int kFoldMax = 80;
  __shared__ FoldItem s_fi[kFoldMax];
  __shared__ int32_t s_fv[kFoldMax];  // the chosen node's value id of each item's slot
  __shared__ uint32_t s_nfi;
  __shared__ int s_pw;                // participant whose key won the pod just decided
  __shared__ int s_rnode;             // node-sharded: that participant's chosen node (global snapshot index)
  __shared__ uint32_t s_el;           // the chosen node's DoNotSchedule eligibility for the next pod
  __shared__ int s_bn_q;              // the pod whose chosen node (s_gnode, s_el) wave 0 has resolved
  __shared__ int s_a_q, s_p2_q;       // wave 0 -> 1: exchange A of pod q swept; wave 1 -> 0: its phase-2 half done
  __shared__ int s_elig_q;            // the pod whose DoNotSchedule eligibility s_elig holds
  __shared__ unsigned long long s_p2k;
  __shared__ int s_p2n;
  __shared__ int64_t s_mx[4];
  __shared__ uint32_t s_pmult[kAggMaxCons];  // DoNotSchedule: present domains at the minimum
  __shared__ uint32_t s_ll[kRingLL];          // resident mode: the doorbell's data words (desc.h PodRing::ll)
  __shared__ int s_ring_end;                  // resident mode: -1: the launch ends
  __shared__ int s_pb, s_eb;                  // resident mode: the last staged program's / entry's bytes
  __shared__ int s_spec_q;                    // resident mode: the counts hold pod s_spec_q's plus its placement
  __shared__ int s_ahead_q;                   // resident mode: phase 1 of pod s_ahead_q's program again is in LDS
  __shared__ unsigned long long s_patch[kPatchWords];  // resident mode: a RING_TERMS doorbell's patch
  __shared__ int32_t s_tc_off[kAggTc];        // template cache: each written slot's template (a pod's program offset)
  __shared__ int s_gprev, s_lprev;            // template cache: pod q-1's node (-1: not placed), my slot of it (-1)
  __shared__ uint32_t s_tcq;                  // template cache: pod q's decisions (kTq*, slots, fold mask)
  __shared__ uint32_t s_gbar5;                // template cache: waves 3..7's barrier (monotonic)
  __shared__ uint32_t s_tcr[4];               // template cache: TcWord of pod p in s_tcr[p % 4] (pods q-1 .. q+2)
  // (the batch instance's template cache borrows a resident-mode doorbell word: pod q-1's node's eligibility under
  // q+1's template)
  uint32_t& s_elp = s_ll[0];
  const int w = GRP ? w_grp : (int)blockIdx.x, G = av.nwg;
  loop_entry_record(av.fail, w);
  const int P = SHARD ? av.world * G : G, gid = SHARD ? av.rank * G + w : w;  // participants (rank-major), mine
  const int k0 = av.blk0 + (int)((int64_t)av.nblk * w / G), k1 = av.blk0 + (int)((int64_t)av.nblk * (w + 1) / G);
  const int nk = k1 - k0;  // <= kLoopMaxBlk (host-checked)
  const int nlo = k0 * kBlock, nhi = k1 * kBlock < m.n ? k1 * kBlock : m.n;
  // my pod / term lists: the first kLp / kLt entries in LDS, the rest in my HBM spill rows
  uint32_t* const spl = av.spill + (size_t)w * (size_t)(av.spill_pods + av.spill_terms);
  const uint32_t pcap = kLp + (uint32_t)av.spill_pods, tcap = kLt + (uint32_t)av.spill_terms;
  auto put_pod = [&](uint32_t k, uint32_t e) __attribute__((always_inline)) {
    if (k < kLp) s_pods[k] = e;
    else spl[k - kLp] = e;
  };
  auto put_term = [&](uint32_t k, uint32_t e) __attribute__((always_inline)) {
    if (k < kLt) s_terms[k] = e;
    else spl[(uint32_t)av.spill_pods + k - kLt] = e;
  };
  const int t = (int)threadIdx.x, lane = t & 63, wave = t >> 6;
  const int kk = t / kBlock, tt = t % kBlock;  // my node slot t = kk * kBlock + tt
  const int my_i = (k0 + kk) * kBlock + tt;
  const bool my_node = kk < nk && my_i < m.n;
  auto stamp = [&](int q, int k) {
#ifndef KSG_DIAG
    if constexpr (kPxa) return;  // the resident / 1-round instances' stamps: the diagnostic build (registers)
#endif
    if (av.stamps && w == 0 && t == 0) av.stamps[(size_t)q * kAggStamps + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto gstamp = [&](int q, int k) {  // the gathering waves (wave 2's lane 0) of workgroup 0
#ifndef KSG_DIAG
    if constexpr (kPxa) return;
#endif
    if (av.stamps && w == 0 && t == 128) av.stamps[(size_t)q * kAggStamps + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto wstamp = [&](int q, int k) {  // thread 0 of every workgroup
#ifndef KSG_DIAG
    if constexpr (kPxa) return;
#endif
    if (av.wstamps && t == 0) av.wstamps[((size_t)q * G + w) * 4 + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto fail = [&](uint32_t code) {
    uint32_t first = 0u;
    if (__hip_atomic_compare_exchange_strong(av.fail, &first, 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      uint32_t wv = (uint32_t)w;  // (formed here: a copy hoisted out of the pod loop would hold a register)
      asm volatile("" : "+v"(wv));
      __hip_atomic_store(av.fail + 1, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(av.fail + 2, wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  auto stage_prog = [&](int q, int tid, int nthr) __attribute__((always_inline)) {
    const uint4* src = reinterpret_cast<const uint4*>(b.descs + s_off[q]);
    const uint32_t n16 = av.desc_bytes[av.first_pod + q] / 16u;
    uint4* dst = reinterpret_cast<uint4*>(s_blob[q % 3]);
    for (uint32_t o = (uint32_t)tid; o < n16; o += (uint32_t)nthr) dst[o] = src[o];
  };
  // spec(q): pod q's counts may be gathered before pod q-1 is placed, and pod q-1 folded in after
  // (no node-local DoNotSchedule minimum, which would need the chosen node's own count)
  auto spec = [&](const PodDesc& dn) { return dn.agg_local_cons == 0 && !(av.debug & 1); };

  // ---- aggregation of pod q by threads [0, nthr) of a group (tid = my index in it), meeting at
  // gbar(): the pod's selectors against my pods, my pods' terms against the pod, my nodes'
  // DoNotSchedule eligibility; partials of shared keys into the pod's region; Z published by tid 0.
  // (gather false: the counts are in LDS already -- the template cache -- and only the node-local DoNotSchedule
  // minima and exchange Z remain, with the any bits as they stand)
  auto aggregate = [&](int q, int tid, int nthr, auto&& gbar, bool gather = true) __attribute__((always_inline)) {
    const uint8_t* base = s_blob[q % 3];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    unsigned long long* region = av.region + (size_t)q * av.gwords;
    const int gw = gather ? d.agg_gwords : 0, nl = gather ? d.agg_nlocal : 0;
    const PtsCons* cf = at<PtsCons>(base, d.ptsf_off);
    const int32_t* sp = at<int32_t>(base, d.sel_pool_off);
    for (int x = tid; x < nl * kAggSlots; x += nthr) s_lh[x] = 0;
    for (int x = tid; x < gw; x += nthr) s_gh[x] = 0ull;
    if (tid == 0) {
      s_gany = gather ? 0u : s_any;
      s_lmin[0] = s_lmin[1] = 0x7fffffffffffffffll;
      s_lcnt[0] = s_lcnt[1] = 0;
      s_latm[0] = s_latm[1] = 0;
    }
    gbar();
    // node role: DoNotSchedule eligibility (nodeLabelsMatchSpreadConstraints + inclusion policies,
    // podtopologyspread/common.go:43-80) and the shared domains it makes present (filtering.go:255-311)
    const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
    for (int ls = tid; ls < (gather ? kAggSlots : 0); ls += nthr) {
      const int i = nlo + ls;
      uint32_t el = 0;
      if (ls < nk * kBlock && i < m.n && d.n_ptsf) {
        el = pts_eligible(m, base, d, cf, d.n_ptsf, i);
        for (int32_t c = 0; c < d.n_ptsf; ++c)
          if (((el >> c) & 1u) && cf[c].lref >= 0) s_gh[cf[c].pref + node_label(m, cf[c].slot, i)] = 1ull;
      }
      // processAllNode's node test for the ScheduleAnyway counts (scoring.go:164-181)
      if (PTSS && ls < nk * kBlock && i < m.n && d.n_ptss)
        el |= pts_eligible(m, base, d, cs, d.n_ptss, i, (d.flags & DF_PTS_ANYTOPO) == 0) << 8;
      s_elig[ls] = (uint16_t)el;
    }
    gbar();
    if (tid == 0) __hip_atomic_store(&s_elig_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t any = 0;
    auto add = [&](int32_t lref, int32_t v, int ls, long long wt) __attribute__((always_inline)) {
      if (lref >= 0) atomicAdd(&s_gh[lref + v], (unsigned long long)wt);
      else atomicAdd(&s_lh[(-1 - lref) * kAggSlots + ls], (int32_t)wt);
    };
    const uint32_t np = s_np, nitems = !gather ? 0u : s_np + ((d.ipa_flags & (IPA_EXIST_FILTER | IPA_EXIST_SCORE)) ? s_nt : 0u);
    // a pod with no selector of its own (only existing pods' terms to test, e.g. a plain pod beside
    // anti-affinity pods) has nothing to do in the pod role: its scan starts at the term role
    const bool pod_role = d.n_ptsf || (PTSS && d.n_ptss) || d.n_raff || d.n_ranti || (d.ipa_flags & IPA_PREF);
    for (uint32_t k = (pod_role ? 0u : np) + (uint32_t)tid; k < nitems; k += (uint32_t)nthr) {
      if (k < np) {
        // pod role: the pod's selectors against one pod on my nodes (k_aggregate's pod role)
        const uint32_t e = k < kLp ? s_pods[k] : spl[k - kLp];
        const int s = (int)(e >> 9), ls = (int)(e & 511u), n = nlo + ls;
        const int32_t pns = m.pod_ns[s];
        const bool term = (m.pod_flags[s] & 1u) != 0;
        const unsigned long long* pl = m.lbl_pool + m.pod_lbl_off[s];
        const int32_t pn = (int32_t)m.pod_lbl_cnt[s];
        if (!term && pns == d.ns_id && d.n_ptsf) {  // calPreFilterState counts (filtering.go:255-300)
          const uint32_t el = s_elig[ls];
          for (int32_t c = 0; c < d.n_ptsf; ++c)
            if (((el >> c) & 1u) && !lsel_empty(sp + cf[c].sel) && lsel_match(sp + cf[c].sel, pl, pn))
              add(cf[c].lref, node_label(m, cf[c].slot, n), ls, 1);
        }
        if (PTSS && !term && pns == d.ns_id && d.n_ptss) {  // PreScore counts (scoring.go:155-189), hostname per node (:207-214)
          const uint32_t el = s_elig[ls] >> 8;
          for (int32_t c = 0; c < d.n_ptss; ++c) {
            if (lsel_empty(sp + cs[c].sel) || !lsel_match(sp + cs[c].sel, pl, pn)) continue;
            if (cs[c].hostname) add(cs[c].lref, 0, ls, 1);
            else if ((el >> c) & 1u) add(cs[c].lref, pts_domain(m, cs[c], n), ls, 1);
          }
        }
        if (d.n_raff) {  // affinityCounts (filtering.go:256-266)
          const IpaTerm* ts = at<IpaTerm>(base, d.raff_off);
          bool all = true;
          for (int32_t k2 = 0; k2 < d.n_raff; ++k2) all = all && term_matches_pod(sp, ts[k2], pns, pl, pn);
          if (all)
            for (int32_t k2 = 0; k2 < d.n_raff; ++k2) {
              const int32_t v = node_label(m, ts[k2].slot, n);
              if (v >= 0) {
                add(ts[k2].lref, v, ls, 1);
                any |= 1u;
              }
            }
        }
        if (d.n_ranti) {  // antiAffinityCounts (filtering.go:268-276)
          const IpaTerm* ts = at<IpaTerm>(base, d.ranti_off);
          for (int32_t k2 = 0; k2 < d.n_ranti; ++k2)
            if (term_matches_pod(sp, ts[k2], pns, pl, pn)) {
              const int32_t v = node_label(m, ts[k2].slot, n);
              if (v >= 0) {
                add(ts[k2].lref, v, ls, 1);
                any |= 2u;
              }
            }
        }
        if (d.ipa_flags & IPA_PREF) {  // the incoming pod's soft terms (scoring.go:98-110)
          const IpaTerm* ta = at<IpaTerm>(base, d.paff_off);
          for (int32_t k2 = 0; k2 < d.n_paff; ++k2)
            if (term_matches_pod(sp, ta[k2], pns, pl, pn)) {
              const int32_t v = node_label(m, ta[k2].slot, n);
              if (v >= 0) {
                add(ta[k2].lref, v, ls, ta[k2].weight);
                any |= 8u;
              }
            }
          const IpaTerm* tn = at<IpaTerm>(base, d.panti_off);
          for (int32_t k2 = 0; k2 < d.n_panti; ++k2)
            if (term_matches_pod(sp, tn[k2], pns, pl, pn)) {
              const int32_t v = node_label(m, tn[k2].slot, n);
              if (v >= 0) {
                add(tn[k2].lref, v, ls, -(long long)tn[k2].weight);
                any |= 8u;
              }
            }
        }
      } else {
        // term role: one existing affinity term of a pod on my nodes against the incoming pod
        const uint32_t kt2 = k - np;
        const uint32_t e = kt2 < kLt ? s_terms[kt2] : spl[(uint32_t)av.spill_pods + kt2 - kLt];
        const int j = (int)(e >> 9), ls = (int)(e & 511u), n = nlo + ls;
        const DTerm tm = m.terms[j];
        if (tm.key >= d.n_keytab) continue;
        const int32_t* kt = at<int32_t>(base, d.keytab_off) + (size_t)tm.key * kKeytabStride;
        const bool anti = tm.kind == T_REQ_ANTI;
        const int32_t hb = anti ? ((d.ipa_flags & IPA_EXIST_FILTER) ? kt[1] : -1)
                                : ((d.ipa_flags & IPA_EXIST_SCORE) ? kt[2] : -1);
        long long wt = 0;
        if (tm.kind == T_REQ_AFF) wt = d.hard_weight;  // HardPodAffinityWeight (scoring.go:112-117)
        else if (tm.kind == T_PREF_AFF) wt = tm.weight;
        else if (tm.kind == T_PREF_ANTI) wt = -(long long)tm.weight;
        else wt = 1;
        if (hb < 0 || wt == 0) continue;
        const int32_t* tp = m.term_pool;
        const unsigned long long* il = at<unsigned long long>(base, d.lbl_off);
        const unsigned long long* nsl = at<unsigned long long>(base, d.nslbl_off);
        // AffinityTerm.Matches(incoming pod, namespace labels) (types.go:391-396)
        const bool match = (id_in(tp + tm.ns_off, tm.ns_cnt, d.ns_id) || lsel_match(tp + tm.nssel, nsl, d.n_nslbl)) &&
                           lsel_match(tp + tm.sel, il, d.n_lbl);
        const int32_t v = match ? node_label(m, kt[0], n) : -1;
        if (v >= 0) {
          add(anti ? kt[3] : kt[4], v, ls, wt);
          any |= anti ? 4u : 8u;
        }
      }
    }
    if (any) atomicOr(&s_gany, any);
    gbar();
    // my partials of the shared region; node-local DoNotSchedule minima over my eligible nodes
    for (int x = tid; x < gw; x += nthr)
      if (s_gh[x]) {
        if constexpr (!SHARD) {
          atomicAdd(region + x, s_gh[x]);
        } else {  // node-sharded: the sums are global in every rank's region
          for (int r = 0; r < av.world; ++r)
            __hip_atomic_fetch_add(av.regions[r] + (size_t)q * av.gwords + x, s_gh[x], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    if (d.agg_local_cons) {
      int li = 0;
      for (int32_t c = 0; c < d.n_ptsf && li < kAggLocalCons; ++c) {
        if (!((d.agg_local_cons >> c) & 1)) continue;
        long long mn = 0x7fffffffffffffffll;
        uint32_t cnt = 0;
        for (int ls = tid; ls < kAggSlots; ls += nthr)
          if ((s_elig[ls] >> c) & 1u) {
            const long long x = s_lh[(size_t)(-1 - cf[c].lref) * kAggSlots + ls];
            mn = x < mn ? x : mn;
            ++cnt;
          }
        if (cnt) {
          atomicMin(&s_lmin[li], mn);
          atomicAdd(&s_lcnt[li], cnt);
        }
        ++li;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my region atomics performed before Z
    if constexpr (SHARD) __threadfence_system();       // ... at the peers too
    gbar();
    if (d.agg_local_cons) {  // my eligible nodes at my minimum (exchange Z sums those of the global one)
      int li = 0;
      for (int32_t c = 0; c < d.n_ptsf && li < kAggLocalCons; ++c) {
        if (!((d.agg_local_cons >> c) & 1)) continue;
        const long long mn = s_lmin[li];
        uint32_t k = 0;
        for (int ls = tid; ls < kAggSlots; ls += nthr)
          if (((s_elig[ls] >> c) & 1u) && (long long)s_lh[(size_t)(-1 - cf[c].lref) * kAggSlots + ls] == mn) ++k;
        if (k) atomicAdd(&s_latm[li], k);
        ++li;
      }
      gbar();
    }
    if (tid == 0) {  // every Z granule is published (zero for an absent constraint)
      unsigned long long z[2] = {0, 0};
      for (int li = 0; li < kAggLocalCons; ++li) {
        const long long mn = s_lmin[li];
        const unsigned long long m24 = mn > 0xffffffll ? 0xffffffull : (unsigned long long)mn;
        // no eligible node: min 2^24-1
        z[li] = ((unsigned long long)(s_latm[li] & 0xfffu) << 36) | ((unsigned long long)(s_lcnt[li] & 0xfffu) << 24) | m24;
      }
      agran_put<SHARD>(av, q, gid, AG_Z0, s_gany);
      agran_put<SHARD>(av, q, gid, AG_Z1, z[0]);
      agran_put<SHARD>(av, q, gid, AG_Z2, z[1]);
    }
  };
  // exchange Z of pod q (wave 0): OR of the any bits, node-local minima and domain counts
  auto sweep_z = [&](int q) __attribute__((always_inline)) {
    uint32_t a = 0, c1 = 0, c2 = 0, k1 = 0, k2 = 0;
    unsigned long long m1 = 0xffffffull, m2 = 0xffffffull;
    const bool ok = agran_sweep<SHARD, 3, MS, RING>(av, q, AG_Z0, [&](int r, const unsigned long long (&z)[3]) {
      if (lane + 64 * r < P) {
        a |= (uint32_t)z[0];
        const unsigned long long x1 = z[1] & 0xffffffull, x2 = z[2] & 0xffffffull;
        const uint32_t a1 = (uint32_t)(z[1] >> 36) & 0xfffu, a2 = (uint32_t)(z[2] >> 36) & 0xfffu;
        c1 += (uint32_t)(z[1] >> 24) & 0xfffu;
        c2 += (uint32_t)(z[2] >> 24) & 0xfffu;
        k1 = x1 < m1 ? a1 : x1 == m1 ? k1 + a1 : k1;  // nodes at my lane's minimum so far
        k2 = x2 < m2 ? a2 : x2 == m2 ? k2 + a2 : k2;
        m1 = x1 < m1 ? x1 : m1;
        m2 = x2 < m2 ? x2 : m2;
      }
    });
    unsigned long long g1 = m1, g2 = m2;
    for (int o = 32; o > 0; o >>= 1) {
      a |= (uint32_t)__shfl_xor((int)a, o, 64);
      const unsigned long long y1 = __shfl_xor(g1, o, 64), y2 = __shfl_xor(g2, o, 64);
      g1 = y1 < g1 ? y1 : g1;
      g2 = y2 < g2 ? y2 : g2;
    }
    c1 = wave_sum_u32(c1);
    c2 = wave_sum_u32(c2);
    k1 = wave_sum_u32(m1 == g1 ? k1 : 0u);  // the global minimum's multiplicity
    k2 = wave_sum_u32(m2 == g2 ? k2 : 0u);
    if (lane == 0) {
      if (!ok) s_ok = 0u;
      s_any = a;
      s_lmin[0] = (long long)g1;
      s_lmin[1] = (long long)g2;
      s_lcnt[0] = c1;
      s_lcnt[1] = c2;
      s_lmult[0] = k1;
      s_lmult[1] = k2;
      s_lstale = 0u;
    }
  };
  // the region's totals into LDS (all threads; then a barrier)
  auto load_totals = [&](int q, int tid, int nthr) __attribute__((always_inline)) {
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(s_blob[q % 3]);
    const unsigned long long* region = av.region + (size_t)q * av.gwords;
    for (int x = tid; x < d.agg_gwords; x += nthr)
      s_gh[x] = SHARD ? __hip_atomic_load(region + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                      : __hip_atomic_load(region + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // DoNotSchedule minima (criticalPaths, filtering.go:64-124): shared constraints over their present
  // domains (one wave each), node-local ones from exchange Z (all threads; then a barrier)
  auto minima = [&](int q) __attribute__((always_inline)) {
    const uint8_t* base = s_blob[q % 3];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    const PtsCons* cf = at<PtsCons>(base, d.ptsf_off);
    int li = 0;
    for (int32_t c = 0; c < d.n_ptsf; ++c) {
      if ((d.agg_local_cons >> c) & 1) {
        if (t == 0) {
          s_pmin[c] = li < kAggLocalCons ? s_lmin[li] : 0;
          s_pndom[c] = li < kAggLocalCons ? s_lcnt[li] : 0;
        }
        ++li;
        continue;
      }
      if (wave != (c & 7)) continue;
      long long mn = 0x7fffffffffffffffll;
      uint32_t cnt = 0;
      for (int v = lane; v < cf[c].nvals; v += 64)
        if (s_gh[cf[c].pref + v]) {
          const long long x = (long long)s_gh[cf[c].lref + v];
          mn = x < mn ? x : mn;
          ++cnt;
        }
      mn = (long long)dec_i64(~wave_max_u64(~enc_i64(mn)));
      cnt = wave_sum_u32(cnt);
      if (lane == 0) {
        s_pmin[c] = mn;
        s_pndom[c] = cnt;
      }
    }
  };
  // minima() for a folded pod, by the gathering group's waves (wave index gw of gnw): per shared
  // DoNotSchedule constraint its minimum, present domains and how many of them sit at the minimum
  // (node-local constraints: the minimum, domains and multiplicity exchange Z gave)
  auto minima_grp = [&](int q, int gwv, int gnw, bool local = true) __attribute__((always_inline)) {
    const uint8_t* base = s_blob[q % 3];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    const PtsCons* cf = at<PtsCons>(base, d.ptsf_off);
    for (int32_t c = gwv; c < d.n_ptsf; c += gnw) {
      if ((d.agg_local_cons >> c) & 1) {
        const int li = __popc((uint32_t)d.agg_local_cons & ((1u << c) - 1u));
        if (lane == 0 && local) {
          s_pmin[c] = li < kAggLocalCons ? s_lmin[li] : 0;
          s_pndom[c] = li < kAggLocalCons ? s_lcnt[li] : 0;
        }
        continue;
      }
      long long mn = 0x7fffffffffffffffll;
      uint32_t cnt = 0;
      for (int v = lane; v < cf[c].nvals; v += 64)
        if (s_gh[cf[c].pref + v]) {
          const long long x = (long long)s_gh[cf[c].lref + v];
          mn = x < mn ? x : mn;
          ++cnt;
        }
      mn = (long long)dec_i64(~wave_max_u64(~enc_i64(mn)));
      cnt = wave_sum_u32(cnt);
      uint32_t mult = 0;
      for (int v = lane; v < cf[c].nvals; v += 64)
        if (s_gh[cf[c].pref + v] && (long long)s_gh[cf[c].lref + v] == mn) ++mult;
      mult = wave_sum_u32(mult);
      if (lane == 0) {
        s_pmin[c] = mn;
        s_pndom[c] = cnt;
        s_pmult[c] = mult;
      }
    }
  };
  // The fold plan of pod q into pod q + 1 (one wave, lanes gl): pod q as an existing pod of q+1 --
  // its labels against q+1's selectors, its own terms against q+1 -- exactly what q+1's aggregation
  // would count for it, less the chosen node's label values (looked up once the node is known).
  // (plan_fold_b: the placed pod's program bp, the next pod's base)
  // (emit(lref, label slot, constraint, weight, any bit, absent value) takes each item)
  // (ent: the placed pod's RingEntry in LDS -- its own terms and their term-pool words as the owner's commit writes
  // them to the device tables, which only the owner may read back (resident mode); nullptr: read the tables)
  auto plan_fold_e = [&](const uint8_t* bp, const uint8_t* base, int gl, const uint8_t* ent, auto&& emit)
                         __attribute__((always_inline)) {
    asm volatile("" : "+v"(gl));  // lane-dependent item selection stays in the loop (register pressure)
    const PodDesc& dp = *reinterpret_cast<const PodDesc*>(bp);
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    const int32_t* sp = at<int32_t>(base, d.sel_pool_off);
    const unsigned long long* pl = at<unsigned long long>(bp, dp.lbl_off);
    const int32_t pn = dp.n_lbl, pns = dp.ns_id;
    const bool term = (dp.flags & DF_TERMINATING) != 0;
    auto push = [&](int32_t lref, int32_t slot, int32_t cons, int32_t wt, uint32_t anyb) __attribute__((always_inline)) {
      emit(lref, slot, cons, wt, anyb, -1);
    };
    // lane 0: PodTopologySpread + required affinity; 1..8 ranti; 9..16 paff; 17..24 panti; 32.. own terms
    if (gl == 0) {
      if (!term && pns == d.ns_id && d.n_ptsf) {
        const PtsCons* cf = at<PtsCons>(base, d.ptsf_off);
        for (int32_t c = 0; c < d.n_ptsf; ++c)
          if (!lsel_empty(sp + cf[c].sel) && lsel_match(sp + cf[c].sel, pl, pn)) push(cf[c].lref, cf[c].slot, c, 1, 0u);
      }
      if (d.n_raff) {
        const IpaTerm* ts = at<IpaTerm>(base, d.raff_off);
        bool all = true;
        for (int32_t k2 = 0; k2 < d.n_raff; ++k2) all = all && term_matches_pod(sp, ts[k2], pns, pl, pn);
        if (all)
          for (int32_t k2 = 0; k2 < d.n_raff; ++k2) push(ts[k2].lref, ts[k2].slot, -1, 1, 1u);
      }
    } else if (gl <= 8) {
      const int k2 = gl - 1;
      const IpaTerm* ts = at<IpaTerm>(base, d.ranti_off);
      if (k2 < d.n_ranti && term_matches_pod(sp, ts[k2], pns, pl, pn)) push(ts[k2].lref, ts[k2].slot, -1, 1, 2u);
    } else if (gl <= 24) {
      const bool aff = gl <= 16;
      const int k2 = aff ? gl - 9 : gl - 17;
      const IpaTerm* ts = at<IpaTerm>(base, aff ? d.paff_off : d.panti_off);
      if ((d.ipa_flags & IPA_PREF) && k2 < (aff ? d.n_paff : d.n_panti) && term_matches_pod(sp, ts[k2], pns, pl, pn))
        push(ts[k2].lref, ts[k2].slot, -1, aff ? ts[k2].weight : -ts[k2].weight, 8u);
    } else if (PTSS && gl >= 25 && gl < 25 + kAggScoreCons) {  // ScheduleAnyway constraint gl - 25 of pod q+1
      const int c = gl - 25;
      const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
      if (c < d.n_ptss && !term && pns == d.ns_id && !lsel_empty(sp + cs[c].sel) && lsel_match(sp + cs[c].sel, pl, pn))
        // hostname: every node counts (no eligibility); else node test bit 8 + c
        emit(cs[c].lref, cs[c].slot, cs[c].hostname ? -1 : 8 + c, 1, 0u, cs[c].hostname ? 0 : cs[c].absent);
    } else if (gl >= 32 && (d.ipa_flags & (IPA_EXIST_FILTER | IPA_EXIST_SCORE))) {
      const int32_t* own = at<int32_t>(bp, dp.own_terms_off);
      // (the entry lists the terms in the program's order: both are the slot's pt_terms, engine.cpp / podtable.cpp)
      const RingEntry* he = reinterpret_cast<const RingEntry*>(ent);
      const int32_t* etw = ent ? reinterpret_cast<const int32_t*>(ent + sizeof(RingEntry) + (size_t)he->lbl_cnt * 8) : nullptr;
      const RingTerm* ert = ent ? reinterpret_cast<const RingTerm*>(etw + ((he->tpool_cnt + 1) & ~1)) : nullptr;
      for (int k2 = gl - 32; k2 < dp.n_own_terms; k2 += 32) {
        const DTerm tm = ent ? ert[k2].d : m.terms[own[k2]];
        if (tm.key >= d.n_keytab) continue;
        const int32_t* kt = at<int32_t>(base, d.keytab_off) + (size_t)tm.key * kKeytabStride;
        const bool anti = tm.kind == T_REQ_ANTI;
        const int32_t hb = anti ? ((d.ipa_flags & IPA_EXIST_FILTER) ? kt[1] : -1)
                                : ((d.ipa_flags & IPA_EXIST_SCORE) ? kt[2] : -1);
        int32_t wt = 0;
        if (tm.kind == T_REQ_AFF) wt = d.hard_weight;
        else if (tm.kind == T_PREF_AFF) wt = tm.weight;
        else if (tm.kind == T_PREF_ANTI) wt = -tm.weight;
        else wt = 1;
        if (hb < 0 || wt == 0) continue;
        // (the entry holds the term-pool words [tpool_off, tpool_off + tpool_cnt): the offsets are rebased, never the
        // pointer -- an LDS pointer moved below its start is outside the LDS aperture once it is a flat address)
        const int32_t* tp = ent ? etw : m.term_pool;
        const int32_t tb = ent ? he->tpool_off : 0;
        const unsigned long long* il = at<unsigned long long>(base, d.lbl_off);
        const unsigned long long* nsl = at<unsigned long long>(base, d.nslbl_off);
        if ((id_in(tp + (tm.ns_off - tb), tm.ns_cnt, d.ns_id) || lsel_match(tp + (tm.nssel - tb), nsl, d.n_nslbl)) &&
            lsel_match(tp + (tm.sel - tb), il, d.n_lbl))
          push(anti ? kt[3] : kt[4], kt[0], -1, wt, anti ? 4u : 8u);
      }
    }
  };
  // the plan into LDS (s_fi / s_nfi; s_nfi was reset after the previous fold: a reset here by one lane would race
  // the others' pushes)
  auto plan_fold_b = [&](const uint8_t* bp, const uint8_t* base, int gl, const uint8_t* ent = nullptr)
                         __attribute__((always_inline)) {
    plan_fold_e(bp, base, gl, ent,
                [&](int32_t lref, int32_t slot, int32_t cons, int32_t wt, uint32_t anyb, int32_t absent)
                    __attribute__((always_inline)) {
                      const uint32_t k = atomicAdd(&s_nfi, 1u);
                      if (k < (uint32_t)kFoldMax) s_fi[k] = FoldItem{lref, slot, cons, wt, anyb, absent};
                    });
  };
  auto plan_fold = [&](int q, int gl) __attribute__((always_inline)) { plan_fold_b(s_blob[q % 3], s_blob[(q + 1) % 3], gl); };
  // the owner of pod q's node adds it (and its own terms) to my lists: one thread
  auto append = [&](int q, int lq) __attribute__((always_inline)) {
    const uint8_t* bp = s_blob[q % 3];
    const PodDesc& dp = *reinterpret_cast<const PodDesc*>(bp);
    const uint32_t np = s_np, nt = s_nt;
    put_pod(np, ((uint32_t)dp.slot << 9) | (uint32_t)lq);
    const int32_t* own = at<int32_t>(bp, dp.own_terms_off);
    uint32_t k2 = 0;
    for (; k2 < (uint32_t)dp.n_own_terms && nt + k2 < tcap; ++k2) put_term(nt + k2, ((uint32_t)own[k2] << 9) | (uint32_t)lq);
    s_np = np + 1;
    s_nt = nt + k2;
    if (np >= pcap || k2 < (uint32_t)dp.n_own_terms) fail(0xfffffffdu);  // host-checked
  };
  // fold the placed pod (the plan in s_fi, the chosen node's label values in s_fv, its eligibility s_el) into
  // the next pod's counts: shared ones everywhere, node-local ones at the owner (local slot lq); one wave
  // (fold_at: the placed pod at node nq with eligibility el under the counts' template; adj: the DoNotSchedule
  // minima in s_pmin / s_pmult are current and move with the counts)
  auto fold_at = [&](int lq, int nq, uint32_t el, bool adj, int q1) __attribute__((always_inline)) {
    if (nq < 0) return;
    const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
    uint32_t any = 0;
    for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) {
      const FoldItem it = s_fi[k];
      const int32_t v = s_fv[k] >= 0 ? s_fv[k] : it.absent;  // absent: the "" domain (DF_PTS_ANYTOPO)
      if (v < 0 || (it.cons >= 0 && !((el >> it.cons) & 1u))) continue;
      if (adj && it.lref < 0 && it.cons >= 0 && it.cons < 8) {
        // a node-local DoNotSchedule count went up by one at the chosen node (its count before: exchange B):
        // the minimum moves only if that node was the last one holding it
        const PodDesc& dn = *reinterpret_cast<const PodDesc*>(s_blob[q1 % 3]);
        const int li = __popc((uint32_t)dn.agg_local_cons & ((1u << it.cons) - 1u));
        if (li < kAggLocalCons && (long long)s_bc[li] == s_lmin[li]) {
          if (s_lmult[li] > 1u) s_lmult[li] -= 1u;
          else {
            s_lmin[li] += 1;
            s_pmin[it.cons] = s_lmin[li];
            s_lstale = 1u;  // its multiplicity is unknown until exchange Z
          }
        }
      }
      if (it.lref >= 0) {
        const unsigned long long old = atomicAdd(&s_gh[it.lref + v], (unsigned long long)(long long)it.wt);
        if (adj && it.cons >= 0 && it.cons < 8) {  // a DoNotSchedule domain count went up by one: its minimum moves
          const int c = it.cons;  // only if this was the minimum's one domain (one item per constraint)
          if ((long long)old == s_pmin[c]) {
            if (s_pmult[c] == 1u) s_pmin[c] = (long long)old + 1;
            else s_pmult[c] -= 1u;
          }
        }
      } else if (lq >= 0) {
        atomicAdd(&s_lh[(-1 - it.lref) * kAggSlots + lq], it.wt);
      }
      any |= it.anyb;
    }
    for (int o = 32; o > 0; o >>= 1) any |= (uint32_t)__shfl_xor((int)any, o, 64);
    if (lane == 0) s_any |= any;
  };
  auto fold_pod = [&](int lq, int q1) __attribute__((always_inline)) { fold_at(lq, s_gnode, s_el, true, q1); };

  // ---- the template cache (the batch instance; av.tcw nullptr: off).  A pod's counts are its template's
  // counts after every placement before it.  While pod q is decided, the gathering waves write the counts of
  // q's template back to its slot when q+1 is of another template, load q+1's from its slot when they are
  // cached (a hit: no gather) and fold pod q-1's placement into the other cached templates' slots.
  // (not the PodTopologySpread-scoring instances: their registers have no room for it, and the workloads that
  // score spreading -- system default constraints -- stamp their pods from one template)
  constexpr bool kTc = !SHARD && !RING && !PTSS;
  // kTqOne: q+1's counts are loaded and its template has one node-local DoNotSchedule constraint -- its minimum
  // rides exchange B (each workgroup's part in AG_BC beside the chosen node's count), no exchange Z
  constexpr uint32_t kTqWb = 1u, kTqHit = 2u, kTqLite = 4u, kTqOne = 8u, kTqEw = 16u;
  // (the cache's addresses are formed where used -- opaque, so none of them is hoisted out of the pod loop and
  // kept live across it: the loop has no registers to spare)
  auto tc_word = [&](int q) -> uint32_t {
    const uint32_t* p = av.tcw;
    asm volatile("" : "+s"(p));
    return p ? p[av.first_pod + q] : 0u;
  };
  auto tc_at = [&](int sl) {
    unsigned long long* p = av.tcache;
    asm volatile("" : "+s"(p));
    return p + ((size_t)w * kAggTc + (size_t)sl) * kTcWords;
  };
  // pod q's counts in LDS (through pod q-1) into slot sl: threads [0, nthr) of a group
  // (ew: the eligibility too -- static per template, stored once per slot assignment)
  auto tc_store = [&](int q, int sl, int tid, int nthr, bool ew) __attribute__((always_inline)) {
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(s_blob[q % 3]);
    unsigned long long* cb = tc_at(sl);
    for (int x = tid; x < d.agg_gwords; x += nthr) cb[x] = s_gh[x];
    uint32_t* lh = reinterpret_cast<uint32_t*>(cb + kTcLh);
    for (int x = tid; x < d.agg_nlocal * kAggSlots; x += nthr) lh[x] = (uint32_t)s_lh[x];
    uint32_t* el = reinterpret_cast<uint32_t*>(cb + kTcElig);
    const uint32_t* se = reinterpret_cast<const uint32_t*>(s_elig);
    for (int x = tid; x < (ew ? kAggSlots / 2 : 0); x += nthr) el[x] = se[x];
    if (tid == 0) {
      cb[kTcAny] = s_any;
      s_tc_off[sl] = (int32_t)s_off[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // slot sl into LDS as pod q1's counts (agent-scope loads: this CU's L1 may hold the lines from an earlier pod)
  auto tc_load = [&](int q1, int sl, int tid, int nthr) __attribute__((always_inline)) {
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(s_blob[q1 % 3]);
    const unsigned long long* cb = tc_at(sl);
    for (int x = tid; x < d.agg_gwords; x += nthr)
      s_gh[x] = __hip_atomic_load(cb + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t* lh = reinterpret_cast<const uint32_t*>(cb + kTcLh);
    for (int x = tid; x < d.agg_nlocal * kAggSlots; x += nthr)
      s_lh[x] = (int32_t)__hip_atomic_load(lh + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t* el = reinterpret_cast<const uint32_t*>(cb + kTcElig);
    uint32_t* se = reinterpret_cast<uint32_t*>(s_elig);
    for (int x = tid; x < kAggSlots / 2; x += nthr) se[x] = __hip_atomic_load(el + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) s_any = (uint32_t)__hip_atomic_load(cb + kTcAny, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // node nq's eligibility under the template of program base (aggregate's node role)
  auto elig_of = [&](const uint8_t* base, int nq) __attribute__((always_inline)) -> uint32_t {
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    uint32_t el = d.n_ptsf ? pts_eligible(m, base, d, at<PtsCons>(base, d.ptsf_off), d.n_ptsf, nq) : 0u;
    if (PTSS && d.n_ptss)
      el |= pts_eligible(m, base, d, at<PtsCons>(base, d.ptss_off), d.n_ptss, nq, (d.flags & DF_PTS_ANYTOPO) == 0) << 8;
    return el;
  };
  // pod q-1's placement into the counts just loaded for pod q+1 (one wave; the minima come after)
  // (prep: the plan, the node's label values and eligibility -- before the load; apply: after it)
  // (wave 2 plans and reads the label values, wave 3 the eligibility)
  auto fold_prev_prep = [&](int q, int gl) __attribute__((always_inline)) {
    const int nq = s_gprev;
    if (nq < 0) return;
    const uint8_t* base = s_blob[(q + 1) % 3];
    if (wave == 3) {
      const uint32_t el = elig_of(base, nq);
      if (gl == 0) s_elp = el;
      return;
    }
    plan_fold_b(s_blob[(q + 2) % 3], base, gl);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
    for (uint32_t k = (uint32_t)gl; k < nfi; k += 64) s_fv[k] = node_label(m, s_fi[k].slot, nq);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };
  auto fold_prev_apply = [&](int q, int gl) __attribute__((always_inline)) {
    const int nq = s_gprev;
    if (nq < 0) return;
    fold_at(s_lprev, nq, s_elp, false, q + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (gl == 0) s_nfi = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // pod q-1's placement into cached slot sl (one wave; base: the slot's template program, in HBM)
  auto fold_prev_tc = [&](int q, int sl, int gl, const uint8_t* base) __attribute__((always_inline)) {
    const int nq = s_gprev, lq = s_lprev;
    unsigned long long* cb = tc_at(sl);
    int32_t* lh = reinterpret_cast<int32_t*>(cb + kTcLh);
    const uint32_t el = elig_of(base, nq);
    uint32_t any = 0;
    plan_fold_e(s_blob[(q + 2) % 3], base, gl, nullptr,
                [&](int32_t lref, int32_t slot, int32_t cons, int32_t wt, uint32_t anyb, int32_t absent)
                    __attribute__((always_inline)) {
                      int32_t v = node_label(m, slot, nq);
                      if (v < 0) v = absent;  // absent: the "" domain (DF_PTS_ANYTOPO)
                      if (v < 0 || (cons >= 0 && !((el >> cons) & 1u))) return;
                      if (lref >= 0) atomicAdd(cb + lref + v, (unsigned long long)(long long)wt);
                      else if (lq >= 0) atomicAdd(lh + (size_t)(-1 - lref) * kAggSlots + lq, wt);
                      any |= anyb;
                    });
    for (int o = 32; o > 0; o >>= 1) any |= (uint32_t)__shfl_xor((int)any, o, 64);
    if (gl == 0 && any) atomicOr(reinterpret_cast<uint32_t*>(cb + kTcAny), any);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto wg_bar = [&]() __attribute__((always_inline)) { __syncthreads(); };

  // ---- launch prologue: node cores, program offsets, my pods and terms, the first pod's counts
  if (my_node) {
    const NodeCore c = load_core(m, my_i);
    s_core.acpu[kk][tt] = c.acpu;
    s_core.amem[kk][tt] = c.amem;
    s_core.aeph[kk][tt] = c.aeph;
    s_core.apods[kk][tt] = c.apods;
    s_core.flags[kk][tt] = c.flags;
    s_core.tlo[kk][tt] = c.tlo;
    s_core.thi[kk][tt] = c.thi;
    s_core.ilo[kk][tt] = c.ilo;
    s_core.ihi[kk][tt] = c.ihi;
    lds_put_dynamic(s_core, kk, tt, c);
  }
  if (!RING)
    for (int k = t; k < av.npods; k += kAggThreads) s_off[k] = b.desc_off[av.first_pod + k];
  if (t == 0) {
    s_np = 0;
    s_nt = 0;
    s_gbar = 0;
    s_ok = 1;
    s_pend_ls = -1;
    s_nfi = 0;
    s_bn_q = -1;
    s_a_q = -1;
    s_p2_q = -1;
    s_px_q = -1;
    s_pxd_q = -1;
    s_elig_q = -1;
    s_spec_q = -1;
    s_ahead_q = -1;
    s_gprev = -1;
    s_lprev = -1;
    s_tcq = 0;
    s_gbar5 = 0;
    s_lstale = 0u;
    s_bc[0] = s_bc[1] = 0u;
    s_lmult[0] = s_lmult[1] = 0u;
    s_pb = 0;
    s_eb = 0;
    for (int c = 0; c < kAggScoreCons; ++c) s_psz_used[c] = ~0u;
  }
  __syncthreads();
  for (int s = t; s < m.pods_hw; s += kAggThreads) {
    const int n = m.pod_node[s];
    if (n >= nlo && n < nhi) {
      const uint32_t k = atomicAdd(&s_np, 1u);
      if (k < pcap) put_pod(k, ((uint32_t)s << 9) | (uint32_t)(n - nlo));
    }
  }
  for (int j = t; j < m.n_terms; j += kAggThreads) {
    const DTerm tm = m.terms[j];
    const int n = tm.kind >= 0 ? m.pod_node[tm.owner] : -1;
    if (n >= nlo && n < nhi) {
      const uint32_t k = atomicAdd(&s_nt, 1u);
      if (k < tcap) put_term(k, ((uint32_t)j << 9) | (uint32_t)(n - nlo));
    }
  }
  if (!RING && av.npods > 0) stage_prog(0, t, kAggThreads);
  if (!RING && av.npods > 1) stage_prog(1, t, kAggThreads);
  if (kTc && t < 2) s_tcr[t] = t < av.npods ? tc_word(t) : 0u;  // (then pod q+2's while pod q is decided)
  __syncthreads();
  if (s_np > pcap || s_nt > tcap) {  // host-checked; never taken
    if (t == 0) fail(0xfffffffeu);
    return;
  }
  if (SHARD && av.npods > 0) {
    // every rank zeroed its regions before its launch (stream order): no workgroup adds into a peer's
    // region before every participant has started (one granule row past the pods, kAggStartRow)
    if (t == 0) agran_put<SHARD>(av, kAggStartRow, gid, 0, 1ull);
    if (wave == 0) {
      if (!agran_sweep<SHARD, 1, MS, RING>(av, kAggStartRow, 0, [](int, const unsigned long long (&)[1]) {}) && lane == 0)
        s_ok = 0u;
    }
    __syncthreads();
    if (!s_ok) return;
  }
  if (!RING && av.npods > 0) {
    aggregate(0, t, kAggThreads, wg_bar);
    if (wave == 0) sweep_z(0);
    __syncthreads();
    if (!s_ok) return;
    load_totals(0, t, kAggThreads);
    __syncthreads();
    if constexpr (kTc) minima_grp(0, wave, kAggThreads / 64);  // (with multiplicities: a fold may follow)
    else minima(0);
    __syncthreads();
  }
  uint32_t gtarget = 0;  // waves 1..7: arrivals their group barrier waits for (s_gbar is monotonic)
  uint32_t gtarget5 = 0;  // waves 3..7: likewise for s_gbar5
  auto grp_bar = [&]() __attribute__((always_inline)) {
    gtarget += kAggThreads / 64 - 2;  // waves 2..7
    if (lane == 0) __hip_atomic_fetch_add(&s_gbar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&s_gbar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gtarget)
      __builtin_amdgcn_s_sleep(1);
  };

  for (int q = 0; q < av.npods; ++q) {
    bool ahead = false;  // resident: this pod's phase 1 ran at the end of the pod before (below)
    if constexpr (RING) {
      // ======== resident mode: pod q from the ring (host memory, bypassing the device caches): its program
      // into s_blob[q % 3], its pod-table entry into s_blob[(q + 1) % 3]; then its counts ========
      // (relay: workgroup 0 polls the host and relays the doorbell -- with the program and entry when they are
      // staged -- through device memory, where the other workgroups poll: one PCIe reader instead of G)
      const bool relay = av.relay != nullptr, hostp = !relay || w == 0;
      if (wave == 0) {
        uint32_t v = 0;
        const int r = ring_wait_ll(hostp ? av.ring->ll : av.relay, hostp ? &av.ring->exited : nullptr, q, av.npods,
                                   av.ring_idle, lane, &v);
        if (lane < kRingLL) s_ll[lane] = v;
        if (lane == 0) s_ring_end = r;
      }
      stamp(q, 9);
      __syncthreads();
      if (s_ring_end < 0) {
        if (relay && w == 0 && t == 0)  // the others leave too
          __hip_atomic_store(av.relay, (unsigned long long)kRingStop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      const uint32_t rmode = s_ll[0];
      auto relay_doorbell = [&]() __attribute__((always_inline)) {  // workgroup 0, after any relayed bytes landed
        if (relay && w == 0 && t < kRingLL)
          __hip_atomic_store(av.relay + t, (unsigned long long)(uint32_t)(q + 1) | ((unsigned long long)s_ll[t] << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      };
      if (rmode & RING_SAME) {
        if (rmode & RING_TERMS) {  // the patch words, one per lane of wave 0 (workgroup 0 of a relay passes them on)
          if (wave == 0) {
            const unsigned long long* src = hostp ? av.ring->patch[q % kRingSlots] : av.relay + kRingLL;
            unsigned long long x = 0;
            if (lane < kPatchWords) x = __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (lane < kPatchWords) s_patch[lane] = x;
            if (relay && hostp) {
              if (lane < kPatchWords) __hip_atomic_store(av.relay + kRingLL + lane, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the relayed words landed before the doorbell
            }
          }
        }
        relay_doorbell();
        // pod q-1's program and entry but for the slot, the rotation and the label-pool offset (the host
        // compared the rest byte for byte): copied in LDS -- the entry first, its buffer takes the program
        const int pw8 = s_pb / 8, ew8 = s_eb / 8;
        unsigned long long* ed = reinterpret_cast<unsigned long long*>(s_blob[(q + 1) % 3]);
        const unsigned long long* es_ = reinterpret_cast<const unsigned long long*>(s_blob[q % 3]);
        for (int k = t; k < ew8; k += kAggThreads) ed[k] = es_[k];
        __syncthreads();
        unsigned long long* pd = reinterpret_cast<unsigned long long*>(s_blob[q % 3]);
        const unsigned long long* ps_ = reinterpret_cast<const unsigned long long*>(s_blob[(q + 2) % 3]);
        for (int k = t; k < pw8; k += kAggThreads) pd[k] = ps_[k];
        __syncthreads();
        if (t == 0) {
          PodDesc& dn = *reinterpret_cast<PodDesc*>(s_blob[q % 3]);
          dn.slot = (int32_t)s_ll[1];
          dn.rot_start = (int32_t)s_ll[2];
          dn.flags = (dn.flags & ~DF_AGG_SAME) | ((rmode & RING_AGG_SAME) ? DF_AGG_SAME : 0u);
          RingEntry& en = *reinterpret_cast<RingEntry*>(ed);
          en.slot = ew8 ? (int32_t)s_ll[1] : -1;
          en.lbl_off = s_ll[3];
          if (rmode & RING_TERMS) {  // (the host replayed this patch on pod q-1's bytes and compared the result)
            const int32_t toff = (int32_t)(uint32_t)s_patch[0], n = (int32_t)(s_patch[0] >> 32);
            const int32_t* js = reinterpret_cast<const int32_t*>(&s_patch[1]);
            int32_t* own = reinterpret_cast<int32_t*>(s_blob[q % 3] + dn.own_terms_off);
            const int32_t dt = toff - en.tpool_off;
            RingTerm* rt = reinterpret_cast<RingTerm*>(reinterpret_cast<uint8_t*>(ed) + sizeof(RingEntry) +
                                                       (size_t)en.lbl_cnt * 8 + (size_t)((en.tpool_cnt + 1) & ~1) * 4);
            en.tpool_off = toff;
            for (int32_t k = 0; k < n && k < 2 * (kPatchWords - 1); ++k) {
              own[k] = js[k];
              rt[k].j = js[k];
              rt[k].d.owner = en.slot;
              rt[k].d.sel += dt;
              rt[k].d.nssel += dt;
              rt[k].d.ns_off += dt;
            }
          }
        }
      } else {
        const int pw8 = (int)s_ll[1] / 8, ew8 = (int)s_ll[2] / 8;
        const unsigned long long* ps_ = reinterpret_cast<const unsigned long long*>(av.ring->blob[q % kRingSlots]);
        const unsigned long long* es_ = reinterpret_cast<const unsigned long long*>(av.ring->entry[q % kRingSlots]);
        unsigned long long* pd = reinterpret_cast<unsigned long long*>(s_blob[q % 3]);
        unsigned long long* ed = reinterpret_cast<unsigned long long*>(s_blob[(q + 1) % 3]);
        // (workgroup 0 of a relay reads the host's copy and writes the device's; the others read the device's)
        const unsigned long long* sp_ = hostp ? ps_ : av.relay + kRingLL;
        const unsigned long long* se_ = hostp ? es_ - pw8 : av.relay + kRingLL;
        const bool put = relay && hostp;
        // every word of a thread's share in flight at once (one round trip each), then stored
        constexpr int kStageW = (kBlobLds + kRingEntryBytes) / 8 / kAggThreads;
        static_assert(kStageW * 8 * kAggThreads == kBlobLds + kRingEntryBytes, "staging share");
        unsigned long long xs[kStageW];
#pragma unroll
        for (int i = 0; i < kStageW; ++i) {
          const int k = t + i * kAggThreads;
          xs[i] = 0;
          if (k < pw8 + ew8) xs[i] = __hip_atomic_load((k < pw8 ? sp_ : se_) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
#pragma unroll
        for (int i = 0; i < kStageW; ++i) {
          const int k = t + i * kAggThreads;
          if (k >= pw8 + ew8) break;
          if (k < pw8) pd[k] = xs[i];
          else ed[k - pw8] = xs[i];
          if (put) __hip_atomic_store(av.relay + kRingLL + k, xs[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (put) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the relayed bytes landed before the doorbell
          __syncthreads();
          relay_doorbell();
        }
        if (t == 0) {
          if (ew8 == 0) reinterpret_cast<RingEntry*>(ed)->slot = -1;
          s_pb = pw8 * 8;
          s_eb = ew8 * 8;
        }
      }
      __syncthreads();
      stamp(q, 13);
      // the same template as pod q-1 (host: DF_AGG_SAME): pod q's counts are q-1's plus q-1's placement,
      // folded into the counts in LDS at the end of pod q-1 already (s_spec_q)
      const PodDesc& dq = *reinterpret_cast<const PodDesc*>(s_blob[q % 3]);
      ahead = (rmode & RING_SAME) && (dq.flags & DF_AGG_SAME) && s_spec_q == q - 1 && s_ahead_q == q - 1 && q > 0;
      if (!((dq.flags & DF_AGG_SAME) && s_spec_q == q - 1 && q > 0)) {
        aggregate(q, t, kAggThreads, wg_bar);
        if (wave == 0) sweep_z(q);
        __syncthreads();
        if (!s_ok) return;
        stamp(q, 14);
        load_totals(q, t, kAggThreads);
        __syncthreads();
        stamp(q, 15);
        minima(q);
        __syncthreads();
      }
    }
    if (q == av.give_up_at) {  // diagnostic: as if a workgroup never arrived (host recovery test)
      if (t == 0) fail((uint32_t)q);
      return;
    }
    const int pod = av.first_pod + q;
    const uint8_t* base = s_blob[q % 3];
    const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
    PodStats* ps = b.stats + pod;
    const bool more = !RING && q + 1 < av.npods;
    const bool sp1 = more && spec(*reinterpret_cast<const PodDesc*>(s_blob[(q + 1) % 3]));
    // pod q+1's counts are defined as pod q's (host: DF_AGG_SAME): they are q's counts plus q's placement, so
    // nothing is gathered for it -- the fold below runs on the counts in LDS, then its minima are recomputed
    const bool same1 = sp1 && (reinterpret_cast<const PodDesc*>(s_blob[(q + 1) % 3])->flags & DF_AGG_SAME) &&
                       !(av.debug & 4);
    // the template cache: write pod q's counts back (q+1 is of another template), load q+1's (a hit), or keep
    // them (same template) -- for a next pod with node-local DoNotSchedule minima too (lite1: no gather, only
    // exchange Z after the placement)
    // (decided by thread 0 into s_tcq, read where used: kept live across the pod they spill registers)
    if (kTc && t == 0) {
      const uint32_t tc0 = s_tcr[q & 3], tc1 = more ? s_tcr[(q + 1) & 3] : 0u, tcm = q > 0 ? s_tcr[(q - 1) & 3] : 0u;
      const int ts0 = tc_slot(tc0), ts1 = tc_slot(tc1);
      const bool wb = more && ts0 >= 0 && ts1 != ts0;
      const bool hit1 = more && ts1 >= 0 && ts1 != ts0 && tc_hit(tc1);
      const bool lite = more && !sp1 && !(av.debug & 1) && ts1 >= 0 && (ts1 == ts0 || hit1);
      const bool one = lite && hit1 && !(av.debug & 64) &&
                       __popc((uint32_t)reinterpret_cast<const PodDesc*>(s_blob[(q + 1) % 3])->agg_local_cons) == 1;
      s_tcq = (wb ? kTqWb : 0u) | (hit1 ? kTqHit : 0u) | (lite ? kTqLite : 0u) | (one ? kTqOne : 0u) |
              (wb && tc_elig(tc0) ? kTqEw : 0u) | ((uint32_t)(ts0 & 15) << 8) |
              ((uint32_t)(ts1 & 15) << 12) | (tc_fold(tc0) << 16) | ((tcm & 15u) << 24);
    }
    stamp(q, 0);
    wstamp(q, 0);

    // ======== phase 1: my node (LDS core, LDS counts) ========
    // (a lambda: the resident instance also runs it at the end of the pod before, for a next pod of the same
    // program -- `ahead`)
    auto phase1 = [&]() __attribute__((always_inline)) {
      {
        const AggTopo tp{s_gh, s_lh, s_pmin, s_pndom, s_any};
        NodeEval ne{1u, false, 0, 0, 0, 0};
        PodFast pf;
        if ((d.flags & DF_LFAST) && !(av.debug & 2)) pf = load_fast(base, d);
        else pf.flags = d.flags & ~DF_LFAST;
        // opaque per pod: keeps the compiler from hoisting my node's column addresses out of the pod
        // loop, where they would stay live (and spill) across the exchanges
        int my_iq = my_i;
        asm volatile("" : "+v"(my_iq));
        if (my_node) ne = eval_agg(m, lds_core(s_core, kk, tt), s_core.bwo[kk][tt], pf, base, d, my_iq, tp, t);
        const bool feas = ne.st == 0;
        const unsigned long long ballot = __ballot(feas);
        // PodTopologySpread score inputs (scoring.go:61-115, 199-226): the count at my node's domain per
        // constraint (the weights need exchange A's topology sizes), and the domains of my feasible,
        // non-ignored nodes as presence bits
        unsigned long long pb0 = 0, pb1 = 0;
        bool pts_on = false;
        if (PTSS && ((d.score_mask >> P_PTS) & 1u)) {
          const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
          const bool anytopo = (d.flags & DF_PTS_ANYTOPO) != 0;
          bool ign = false;
          uint32_t cnt[kAggScoreCons];
  #pragma unroll
          for (int c = 0; c < kAggScoreCons; ++c) {
            cnt[c] = ~0u;
            if (c < d.n_ptss && my_node) {
              const int32_t v = node_label(m, cs[c].slot, my_iq);
              if (v >= 0) cnt[c] = (uint32_t)tp.cnt(cs[c].hist_base, cs[c].lref, cs[c].hostname ? 0 : v, t);
              else ign |= !anytopo;
            }
            s_pc[c][t] = cnt[c];
          }
          pts_on = feas && !ign;
          if (pts_on)
  #pragma unroll
            for (int c = 0; c < kAggScoreCons; ++c)
              if (c < d.n_ptss && !cs[c].hostname) {
                const int b = cs[c].pbit + pts_domain(m, cs[c], my_iq);
                if (b < 64) pb0 |= 1ull << b;
                else pb1 |= 1ull << (b - 64);
              }
  #pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            pb0 |= __shfl_xor(pb0, o, 64);
            pb1 |= __shfl_xor(pb1, o, 64);
          }
        }
        const unsigned long long pball = __ballot(pts_on);
        const int lim = d.rot_start - (nlo + wave * 64);
        const unsigned long long bm = lim <= 0 ? 0ull : lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
        s_sv[t] = SlotVal{ne.fixed, (uint32_t)ne.rt, (uint32_t)ne.rna};
        s_ri[t] = ne.ripa;
        unsigned long long et = 0, en = 0, ei = 0, ni = ~0ull;
        if (feas) {
          et = enc_i64(ne.rt);
          en = enc_i64(ne.rna);
          ei = enc_i64(ne.ripa);
          ni = ei;
        }
        et = wave_max_u64(et);
        en = wave_max_u64(en);
        ei = wave_max_u64(ei);
        ni = ~wave_max_u64(~ni);
        if (lane == 0) {
          s_ball[wave] = ballot;
          s_wu[wave][0] = (uint32_t)__popcll(ballot);
          s_wu[wave][1] = (uint32_t)__popcll(ballot & bm);
          s_wu[wave][2] = (uint32_t)__popcll(pball);
          s_wp[wave][0] = pb0;
          s_wp[wave][1] = pb1;
          s_wx[wave][0] = et;
          s_wx[wave][1] = en;
          s_wx[wave][2] = ei;
          s_wx[wave][3] = ni;
        }
      }
      __syncthreads();
      if (PTSS && kPxa && ((d.score_mask >> P_PTS) & 1u) && s_psz_used[0] != ~0u) {
        // each slot's raw PodTopologySpread score with the previous scored pod's topology sizes (the
        // arithmetic of the score pass after exchange A, below); exchange A checks the sizes and carries
        // the max / min (AG_PXA)
        const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
        const bool anytopo = (d.flags & DF_PTS_ANYTOPO) != 0;
        int tq = t;  // opaque per pod: the slot addresses are not hoisted out of the pod loop (registers)
        asm volatile("" : "+v"(tq));
        bool ign = false, have = true;
        double score = 0.0;
  #pragma unroll
        for (int c = 0; c < kAggScoreCons; ++c) {
          if (c >= d.n_ptss) continue;
          have = have && s_psz_used[c] != ~0u;
          const uint32_t cnt = s_pc[c][tq];
          if (cnt == ~0u) {
            ign |= !anytopo;
            continue;
          }
          if (!have) continue;
          const double prod = (double)cnt * s_pwt[c];
          const double term = prod + (double)(cs[c].max_skew - 1);
          score = score + term;
        }
        const bool scored = have && ((s_ball[tq >> 6] >> (tq & 63)) & 1ull) && !ign;
        const uint32_t raw = scored ? (uint32_t)(int64_t)round(score) : 0u;
        s_praw[tq] = scored ? raw : ~0u;
        unsigned long long hx = scored ? (unsigned long long)raw + 1ull : 0ull;
        unsigned long long hn = scored ? (1ull << 24) - 1ull - raw : 0ull;
        hx = wave_max_u64(hx);
        hn = wave_max_u64(hn);
        if (lane == 0) {
          s_wq[wave][0] = hx;
          s_wq[wave][1] = hn;
        }
        __syncthreads();
      }
    };
    if (!ahead) {
      phase1();
    } else {
      // the same program's phase 1 against the cores and the folded counts this pod sees ran at the end of pod
      // q-1 (the host compared the program bytes: only the slot, the rotation and the label-pool offset differ,
      // and phase 1 reads the rotation alone): the count before the new rotation start, from the ballots
      if (lane == 0) {
        const int lim = d.rot_start - (nlo + wave * 64);
        const unsigned long long bm = lim <= 0 ? 0ull : lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
        s_wu[wave][1] = (uint32_t)__popcll(s_ball[wave] & bm);
      }
      __syncthreads();
    }
    stamp(q, 1);
    const uint32_t ipa_any = s_any;

    if (wave <= 1) {
      // ======== waves 0-1: exchange A (wave 0), phase 2 (both halves), exchange B + commit (wave 0) ========
      if (wave == 0) {
        if (lane == 0) {
          uint32_t c = 0, bl = 0;
          unsigned long long a = 0, bb = 0, mi = 0, ni = ~0ull;
          for (int v = 0; v < kAggThreads / 64; ++v) {
            c += s_wu[v][0];
            bl += s_wu[v][1];
            a = s_wx[v][0] > a ? s_wx[v][0] : a;
            bb = s_wx[v][1] > bb ? s_wx[v][1] : bb;
            mi = s_wx[v][2] > mi ? s_wx[v][2] : mi;
            ni = s_wx[v][3] < ni ? s_wx[v][3] : ni;
          }
          unsigned long long g0, g1;
          a_granules(c, bl, a, bb, &g0, &g1);
          // raw InterPodAffinity biased into [1, 2^47): max as is, min reversed (max of 2^47 - x)
          const unsigned long long bi = c ? (unsigned long long)(dec_i64(mi) + kAggIpaBias) + 1ull : 0ull;
          const unsigned long long bn = c ? (1ull << 47) - (unsigned long long)(dec_i64(ni) + kAggIpaBias) : 0ull;
          agran_put<SHARD>(av, q, gid, AG_A0, g0);
          agran_put<SHARD>(av, q, gid, AG_A1, g1);
          agran_put<SHARD>(av, q, gid, AG_A2, bi);
          agran_put<SHARD>(av, q, gid, AG_A3, bn);
          if (PTSS && ((d.score_mask >> P_PTS) & 1u)) {  // PodTopologySpread: domain presence, non-ignored count
            uint32_t ni = 0;
            unsigned long long p0 = 0, p1 = 0;
            for (int v = 0; v < kAggThreads / 64; ++v) {
              ni += s_wu[v][2];
              p0 |= s_wp[v][0];
              p1 |= s_wp[v][1];
            }
            agran_put<SHARD>(av, q, gid, AG_P0, p0 & ((1ull << 48) - 1ull));
            agran_put<SHARD>(av, q, gid, AG_P1, (unsigned long long)(ni & 0xfffffu) |
                                           ((((p0 >> 48) | (p1 << 16)) & ((1ull << 28) - 1ull)) << 20));
            unsigned long long hx = 0, hn = 0;
            for (int v = 0; v < kAggThreads / 64 && s_psz_used[0] != ~0u; ++v) {
              hx = s_wq[v][0] > hx ? s_wq[v][0] : hx;
              hn = s_wq[v][1] > hn ? s_wq[v][1] : hn;
            }
            if (kPxa) agran_put<SHARD>(av, q, gid, AG_PXA, (hx << 24) | hn);
          }
          wstamp(q, 1);
        }
        const bool pts_q = PTSS && ((d.score_mask >> P_PTS) & 1u) != 0;
        uint32_t F = 0, wp = 0, bf = 0, ni = 0;
        unsigned long long tmax = 0, nmax = 0, imax = 0, inmax = 0, p0 = 0, p1 = 0;
        const bool ok = agran_sweep<SHARD, PTSS ? 6 : 4, MS, RING || !PTSS>(av, q, AG_A0, [&](int r, const auto& xa) {
          const int v = lane + 64 * r;
          if (v < P) {
            const uint32_t c = gran_a_count(xa[0]);
            F += c;
            if (v < gid) wp += c;
            bf += gran_a_below(xa[0]);
            const unsigned long long tv = gran_a_tp1(xa[1]), nv = gran_a_np1(xa[1]);
            tmax = tv > tmax ? tv : tmax;
            nmax = nv > nmax ? nv : nmax;
            imax = xa[2] > imax ? xa[2] : imax;
            inmax = xa[3] > inmax ? xa[3] : inmax;
            if constexpr (PTSS) {  // PodTopologySpread: non-ignored nodes, domain presence
              ni += (uint32_t)(xa[5] & 0xfffffull);
              p0 |= xa[4];
              p1 |= xa[5] >> 20;
            }
          }
        }, pts_q ? 6 : 4);
        F = wave_sum_u32(F);
        bf = wave_sum_u32(bf);
        wp = wave_sum_u32(wp);
        tmax = wave_max_u64(tmax);
        nmax = wave_max_u64(nmax);
        imax = wave_max_u64(imax);
        inmax = wave_max_u64(inmax);
        if (pts_q) {  // the topology sizes (initPreScoreState, scoring.go:82-115)
          ni = wave_sum_u32(ni);
          for (int o = 32; o > 0; o >>= 1) {
            p0 |= __shfl_xor(p0, o, 64);
            p1 |= __shfl_xor(p1, o, 64);
          }
          // bits [0, 48) in p0, [48, 76) in p1
          if (lane < kAggScoreCons && lane < d.n_ptss) {
            const PtsCons& pc = at<PtsCons>(base, d.ptss_off)[lane];
            uint32_t sz = ni;  // hostname: len(filteredNodes) - len(IgnoredNodes)
            if (!pc.hostname) {
              sz = 0;
              for (int bb = pc.pbit; bb < pc.pbit + pc.nvals; ++bb)
                sz += (uint32_t)((bb < 48 ? (p0 >> bb) : (p1 >> (bb - 48))) & 1ull);
            }
            s_psz[lane] = sz;
          }
        }
        if (lane == 0) {
          s_F = F;
          s_psb = bf;
          s_acc = wp;
          s_mx[0] = tmax ? (int64_t)tmax - 1 : 0;
          s_mx[1] = nmax ? (int64_t)nmax - 1 : 0;
          s_mx[2] = imax ? (int64_t)(imax - 1ull) - kAggIpaBias : 0;
          s_mx[3] = inmax ? (int64_t)((1ull << 47) - inmax) - kAggIpaBias : 0;
          if (!ok) s_ok = 0u;
          __hip_atomic_store(&s_a_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        stamp(q, 2);
      } else {
        while (__hip_atomic_load(&s_a_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
          __builtin_amdgcn_s_sleep(1);
      }
      constexpr int kH = kAggThreads / 128;
      bool spec = false;
      if (PTSS && ((d.score_mask >> P_PTS) & 1u) && s_ok) {
        // ---- PodTopologySpread.Score of my half's feasible nodes with the global topology sizes
        // (scoring.go:199-226; k_pts_score's arithmetic), into s_pc[0]; NormalizeScore's max / min over
        // every workgroup's scored nodes by exchange PX (scoring.go:229-268).  When the sizes are the ones
        // phase 1 guessed (s_psz_used), its raw scores stand and exchange A carried the max / min (AG_PXA).
        spec = kPxa && __ballot(lane < d.n_ptss && lane < kAggScoreCons && s_psz[lane] != s_psz_used[lane]) == 0ull &&
               !(av.debug & 16);
        const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
        const bool anytopo = (d.flags & DF_PTS_ANYTOPO) != 0;
        double wt[kAggScoreCons];
#pragma unroll
        for (int c = 0; c < kAggScoreCons; ++c) wt[c] = c < d.n_ptss ? m.log_tab[s_psz[c] + 2] : 0.0;
        unsigned long long hmx = 0, hmn = 0;
#pragma unroll
        for (int vv = 0; vv < kH && !spec; ++vv) {
          const int v = wave * kH + vv, ls = v * 64 + lane;
          const bool f = ((s_ball[v] >> lane) & 1ull) != 0;
          bool ign = false;
          double score = 0.0;
#pragma unroll
          for (int c = 0; c < kAggScoreCons; ++c) {
            if (c >= d.n_ptss) continue;
            const uint32_t cnt = s_pc[c][ls];
            if (cnt == ~0u) {
              ign |= !anytopo;
              continue;
            }
            const double prod = (double)cnt * wt[c];
            const double term = prod + (double)(cs[c].max_skew - 1);
            score = score + term;
          }
          const bool scored = f && !ign;
          const uint32_t raw = (uint32_t)(int64_t)round(score);  // math.Round: half away from zero
          s_pc[0][ls] = scored ? raw : ~0u;
          if (scored) {
            hmx = (unsigned long long)raw + 1ull > hmx ? (unsigned long long)raw + 1ull : hmx;
            const unsigned long long r = (1ull << 24) - 1ull - raw;
            hmn = r > hmn ? r : hmn;
          }
        }
        hmx = wave_max_u64(hmx);
        hmn = wave_max_u64(hmn);
        if (wave == 1) {
          if (lane == 0 && !spec) {
            s_pxm[0] = hmx;
            s_pxm[1] = hmn;
            __hip_atomic_store(&s_px_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          while (__hip_atomic_load(&s_pxd_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
            __builtin_amdgcn_s_sleep(1);
        } else {
          if (!spec) {
            while (__hip_atomic_load(&s_px_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
              __builtin_amdgcn_s_sleep(1);
            hmx = s_pxm[0] > hmx ? s_pxm[0] : hmx;
            hmn = s_pxm[1] > hmn ? s_pxm[1] : hmn;
            if (lane == 0) agran_put<SHARD>(av, q, gid, AG_PX, (hmx << 24) | hmn);
          }
          unsigned long long gx = 0, gn = 0;
          const bool okp = agran_sweep<SHARD, 1, MS, RING>(av, q, spec ? AG_PXA : AG_PX, [&](int r, const unsigned long long (&xp)[1]) {
            if (lane + 64 * r < P) {
              const unsigned long long a = xp[0] >> 24, bb = xp[0] & 0xffffffull;
              gx = a > gx ? a : gx;
              gn = bb > gn ? bb : gn;
            }
          });
          gx = wave_max_u64(gx);
          gn = wave_max_u64(gn);
          // the next pod's guess (wave 1 decided spec before this: on a mismatch it published PX first, and on a
          // match the update writes the values it compared)
          if (kPxa && lane < d.n_ptss && lane < kAggScoreCons) {
            s_psz_used[lane] = s_psz[lane];
            s_pwt[lane] = m.log_tab[s_psz[lane] + 2];
          }
          if (lane == 0) {
            s_pts_mx = gx ? (int64_t)gx - 1 : 0;  // maxScore starts at 0 (scoring.go:239)
            s_pts_mn = gn ? (int64_t)(((1ull << 24) - 1ull) - gn) : 0;
            if (!okp) s_ok = 0u;
            __hip_atomic_store(&s_pxd_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
      // ---- phase 2 over my half of the slots (wave v: ballots [4v, 4v + 4)): positions in the rotated
      // feasible list, NormalizeScore + weights, the best packed key
      const bool ok = s_ok != 0u;
      const uint32_t F = s_F, ps_before = s_psb;
      const int64_t mx_t = s_mx[0], mx_n = s_mx[1], mx_i = s_mx[2], mn_i = s_mx[3];
      uint32_t acc = s_acc;
      if (wave == 1)
        for (int v = 0; v < kAggThreads / 128; ++v) acc += (uint32_t)__popcll(s_ball[v]);
      unsigned long long key = 0;
      int knode = -1;
      if (ok) {
        // every LDS read of my half issued up front, then the arithmetic
        unsigned long long ballot[kH];
        SlotVal sv[kH];
        int64_t ri[kH];
        uint32_t rp[kH];
        const bool ipa = ((d.score_mask >> P_IPA) & 1u) != 0, pts = PTSS && ((d.score_mask >> P_PTS) & 1u) != 0;
        const int64_t pmx = s_pts_mx, pmn = s_pts_mn;
#pragma unroll
        for (int vv = 0; vv < kH; ++vv) {
          const int v = wave * kH + vv;
          ballot[vv] = s_ball[v];
          sv[vv] = s_sv[v * 64 + lane];
          ri[vv] = ipa ? s_ri[v * 64 + lane] : 0;
          rp[vv] = pts ? (spec ? s_praw[v * 64 + lane] : s_pc[0][v * 64 + lane]) : 0u;
        }
        // branch-free: the four chains are independent, so the compiler interleaves them
#pragma unroll
        for (int vv = 0; vv < kH; ++vv) {
          const int ls = (wave * kH + vv) * 64 + lane;
          const bool f = ((ballot[vv] >> lane) & 1ull) != 0;
          const uint32_t g = acc + wave_prefix_count(ballot[vv], lane);
          const uint32_t pos = g >= ps_before ? g - ps_before : g + F - ps_before;
          int64_t total = agg_total(d, sv[vv].fixed, sv[vv].rt, sv[vv].rn, ri[vv], mx_t, mx_n, mx_i, mn_i, ipa_any);
          if (pts && !(d.flags & DF_NO_SCORE)) {  // PodTopologySpread NormalizeScore (scoring.go:250-266)
            const int64_t sc = rp[vv] == ~0u ? 0 : pmx == 0 ? 100 : go_div(100 * (pmx + pmn - (int64_t)rp[vv]), pmx);
            total += sc * d.weight[P_PTS];
          }
          const unsigned long long kv = f ? pack_best(total, pos) : 0ull;
          knode = kv > key ? nlo + ls : knode;
          key = kv > key ? kv : key;
          acc += (uint32_t)__popcll(ballot[vv]);
        }
      }
      unsigned long long wk = wave_max_u64(key);
      const unsigned long long hold = __ballot(key == wk && key != 0ull);
      int wn = hold ? __builtin_amdgcn_readlane(knode, (int)__builtin_ctzll(hold)) : -1;
      stamp(q, 10);
      if (wave == 1) {
        if (lane == 0) {
          s_p2k = wk;
          s_p2n = wn;
          __hip_atomic_store(&s_p2_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      } else {
        while (__hip_atomic_load(&s_p2_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
          __builtin_amdgcn_s_sleep(1);
        stamp(q, 11);
        if (s_p2k > wk) {  // keys are unique
          wk = s_p2k;
          wn = s_p2n;
        }
        if (lane == 0) {
          agran_put<SHARD>(av, q, gid, AG_B, wk);  // < 2^48: TotalScore < 2^19 (host-checked) << 29 | pre-order key
          wstamp(q, 2);
          stamp(q, 12);
          // my candidate and its DoNotSchedule eligibility for pod q+1 (the gathering group's node
          // role computed it for all my nodes): if it wins, every workgroup folds pod q in there
          uint32_t el = 0;
          if ((sp1 || (kTc && (s_tcq & kTqLite))) && wn >= 0) {
            const PodDesc& dn = *reinterpret_cast<const PodDesc*>(s_blob[(q + 1) % 3]);
            if (dn.n_ptsf || dn.n_ptss) {
              while (__hip_atomic_load(&s_elig_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q + 1)
                __builtin_amdgcn_s_sleep(1);
              el = s_elig[wn - nlo];
            }
          } else if (RING && wn >= 0 && (d.n_ptsf || d.n_ptss)) {
            el = s_elig[wn - nlo];  // resident: a fold into the next pod is of this pod's template
          }
          agran_put<SHARD>(av, q, gid, AG_BN, (unsigned long long)(uint32_t)(wn + 1) | ((unsigned long long)el << 32));
          if (kTc && (s_tcq & kTqLite)) {
            // my candidate's counts under pod q+1's node-local DoNotSchedule constraints (its counts are in LDS:
            // s_elig_q said so), for the fold's minima
            unsigned long long bc = 0;
            if (wn >= 0) {
              const uint8_t* bn = s_blob[(q + 1) % 3];
              const PodDesc& dn = *reinterpret_cast<const PodDesc*>(bn);
              const PtsCons* cf = at<PtsCons>(bn, dn.ptsf_off);
              int li = 0;
              for (int32_t c = 0; c < dn.n_ptsf && li < kAggLocalCons; ++c) {
                if (!((dn.agg_local_cons >> c) & 1)) continue;
                const int32_t x = s_lh[(size_t)(-1 - cf[c].lref) * kAggSlots + (wn - nlo)];
                bc |= (unsigned long long)(x > 0xffffff ? 0xffffff : x) << (24 * li);
                ++li;
              }
            }
            if (s_tcq & kTqOne)  // {my candidate's count (14) | my minimum (14) | nodes at it (10) | nodes (10)}
              bc = (bc & 0x3fffull) | ((unsigned long long)(s_lmin[0] > 0x3fff ? 0x3fff : s_lmin[0]) << 14) |
                   ((unsigned long long)(s_latm[0] & 0x3ffu) << 28) | ((unsigned long long)(s_lcnt[0] & 0x3ffu) << 38);
            agran_put<SHARD>(av, q, gid, AG_BC, bc);
          }
        }
        stamp(q, 3);
        unsigned long long bmx = 0, bnx = 0, bcx = 0;
        int bpart = -1;
        // B, BN (, the template cache's BC: the next pod's node-local counts at the chosen node)
        constexpr int kBs = kTc ? 3 : 2;
        const uint32_t tqb = kTc ? s_tcq : 0u;
        unsigned long long zm = 0x3fffull;  // (kTqOne: the merged minimum of AG_BC's parts, nodes at it, nodes)
        uint32_t zk = 0, zc = 0;
        const bool okb = ok && agran_sweep<SHARD, kBs, MS, RING || !PTSS>(av, q, AG_B, [&](int r, const unsigned long long (&xb)[kBs]) {
          const unsigned long long v = (lane + 64 * r) < P ? xb[0] : 0ull;
          if (v > bmx) {
            bmx = v;
            bnx = xb[1];
            if constexpr (kBs > 2) bcx = xb[2];
            bpart = lane + 64 * r;
          }
          if constexpr (kBs > 2) {
            if ((tqb & kTqOne) && lane + 64 * r < P) {
              const unsigned long long x = (xb[2] >> 14) & 0x3fffull;
              const uint32_t a = (uint32_t)(xb[2] >> 28) & 0x3ffu;
              zc += (uint32_t)(xb[2] >> 38) & 0x3ffu;
              zk = x < zm ? a : x == zm ? zk + a : zk;
              zm = x < zm ? x : zm;
            }
          }
        }, (tqb & kTqLite) ? 3 : 2);
        const unsigned long long gbest = wave_max_u64(bmx);
        const unsigned long long bh = __ballot(bmx == gbest && gbest != 0ull);
        const int hl = bh ? (int)__builtin_ctzll(bh) : 0;
        const int pw = (F > 0 && bh) ? __builtin_amdgcn_readlane(bpart, hl) : -1;
        const uint32_t bnlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bnx, hl);
        const uint32_t bnhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bnx >> 32), hl);
        if (kTc && (tqb & kTqLite)) {
          const bool one = (tqb & kTqOne) != 0;
          const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bcx & (one ? 0x3fffull : 0xffffffull)), hl);
          const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((bcx >> 24) & 0xffffffull), hl);
          if (one) {  // pod q+1's node-local minimum, its multiplicity and domains (through pod q-1)
            unsigned long long g = zm;
            for (int o = 32; o > 0; o >>= 1) {
              const unsigned long long y = __shfl_xor(g, o, 64);
              g = y < g ? y : g;
            }
            zc = wave_sum_u32(zc);
            zk = wave_sum_u32(zm == g ? zk : 0u);
            if (lane == 0) {
              const uint8_t* bn = s_blob[(q + 1) % 3];
              const int c = __builtin_ctz((uint32_t)reinterpret_cast<const PodDesc*>(bn)->agg_local_cons);
              s_lmin[0] = (long long)g;
              s_lcnt[0] = zc;
              s_lmult[0] = zk;
              s_lstale = 0u;
              s_pmin[c] = (long long)g;
              s_pndom[c] = zc;
            }
          }
          if (lane == 0) {
            s_bc[0] = b0;
            s_bc[1] = one ? 0u : b1;
          }
        }
        const int gnode = (F > 0 && pw == gid) ? wn : -1;  // the chosen node, if it is mine
        // ======== commit (lane 0): the owner of the chosen node applies AssumePod to its LDS core and
        // the mirror; the pod joins my lists before the next pod that counts it ========
        if (lane == 0) {
          if (!okb) s_ok = 0u;
          s_best = gbest;
          s_pw = pw;
          if (SHARD) s_rnode = (int)bnlo - 1;  // the chosen node (global index), for a replica's commit
          s_pend_ls = -1;
          if (okb) {
            if (F == 0) {
              if (w == 0) {
                commit_result(m, b, base, d, ps, pod, 0, -1, gbest, nullptr, (int)ipa_any);
                if constexpr (RING) ring_post_p(av.ring, q, b.results[pod]);
              }
            } else if (gnode >= nlo && gnode < nhi) {
              const int ls = gnode - nlo;
              if (d.flags & DF_ASSUME) {
                NodeCore c = lds_core(s_core, ls / kBlock, ls % kBlock);
                assume_core(c, d);
                commit_result(m, b, base, d, ps, pod, F, gnode, gbest, &c, (int)ipa_any);
                lds_put_dynamic(s_core, ls / kBlock, ls % kBlock, c);
                if (d.slot >= 0) s_pend_ls = ls;
                if constexpr (RING) apply_entry(m, s_blob[(q + 1) % 3]);
              } else {
                commit_result(m, b, base, d, ps, pod, F, gnode, gbest, nullptr, (int)ipa_any);
              }
              if constexpr (RING) ring_post_p(av.ring, q, b.results[pod]);
            }
          }
          // the chosen node and its eligibility for the fold, to the gathering group
          if (sp1 || RING || kTc) {
            const bool placed = okb && F > 0 && pw >= 0 && (d.flags & DF_ASSUME) && d.slot >= 0;
            s_gnode = placed ? (int)bnlo - 1 : -1;
            s_el = placed ? bnhi : 0u;
            __hip_atomic_store(&s_bn_q, q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        stamp(q, 4);
        if (lane == 0) wstamp(q, 3);
      }
    } else {
      // ======== waves 2..7: pod q+1's counts before pod q is placed (folded in below), its
      // DoNotSchedule minima, then the program of pod q+2 ========
      const int gt = t - 128, gn = kAggThreads - 128;
      const uint32_t tq = kTc ? (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tcq) : 0u;
      if (kTc && t == 128) s_tcr[(q + 2) & 3] = q + 2 < av.npods ? tc_word(q + 2) : 0u;  // (read at pod q+1's top)
      const bool tc_hit1 = (tq & kTqHit) != 0, lite1 = (tq & kTqLite) != 0;
      const int ts1 = (int)((tq >> 12) & 15u);
      // the template cache, first: pod q's counts (through pod q-1) written back to its slot, q+1's loaded
      // (through pod q-2's placement) and pod q-1's placement folded in (wave 2, both programs in LDS)
      const bool prep = tc_hit1 && s_gprev >= 0;
      if ((tq & kTqWb) || prep) {
        if (prep && wave <= 3) fold_prev_prep(q, lane);
        if ((tq & kTqWb) && (!prep || wave > 2)) tc_store(q, (int)((tq >> 8) & 15u), prep ? gt - 64 : gt, prep ? gn - 64 : gn, (tq & kTqEw) != 0);
        grp_bar();
      }
      gstamp(q, 13);
      if (tc_hit1) {
        tc_load(q + 1, ts1, gt, gn);
        grp_bar();
        if (wave == 2) fold_prev_apply(q, lane);
      }
      gstamp(q, 14);
      // (then pod q-1 into the other cached templates' slots, on waves 3..7 beside wave 2's work below)
      const uint32_t fo = (tq >> 16) & 63u & ~(tc_hit1 ? 1u << ts1 : 0u);
      auto fold_others = [&]() __attribute__((always_inline)) {
        if (!fo || s_gprev < 0 || wave < 3) return;
        uint32_t f = fo;
        for (int k = 0; f; ++k) {
          const int sl = __builtin_ctz(f);
          f &= f - 1u;
          // (the slot of pod q-1's own template: its program is pod q-1's, still in LDS)
          if (k % (kAggThreads / 64 - 3) == wave - 3)
            fold_prev_tc(q, sl, lane, (int)((tq >> 24) & 15u) == sl + 1 ? s_blob[(q + 2) % 3] : b.descs + s_tc_off[sl]);
        }
      };
      // waves 3..7, while wave 2 finishes pod q's fold plan: the other slots' folds, then pod q+2's program into
      // pod q-1's slot (nothing reads pod q-1's program after them)
      bool staged = false;
      auto fold_stage = [&]() __attribute__((always_inline)) {
        fold_others();
        if (kTc && !RING && q + 2 < av.npods) {
          if (wave >= 3) {
            if (fo && s_gprev >= 0) {
              gtarget5 += kAggThreads / 64 - 3;
              if (lane == 0) __hip_atomic_fetch_add(&s_gbar5, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
              while (__hip_atomic_load(&s_gbar5, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gtarget5)
                __builtin_amdgcn_s_sleep(1);
            }
            stage_prog(q + 2, t - 192, kAggThreads - 192);
          }
          staged = true;
        }
      };
      if (same1) {
        if (wave == 2) {
          if (lane == 0) __hip_atomic_store(&s_elig_q, q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          plan_fold(q, lane);
          // the chosen node's value of every fold item's label (once wave 0 has resolved the node)
          while (__hip_atomic_load(&s_bn_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
            __builtin_amdgcn_s_sleep(1);
          const int nq = s_gnode;
          const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
          for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) s_fv[k] = nq >= 0 ? node_label(m, s_fi[k].slot, nq) : -1;
        }
        fold_stage();
      } else if (sp1 && tc_hit1) {
        // cached: q+1's counts are loaded (through pod q-1's placement); its minima by every gathering wave
        if (wave == 2 && lane == 0) __hip_atomic_store(&s_elig_q, q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        grp_bar();  // (pod q-1 folded in)
        minima_grp(q + 1, wave - 2, kAggThreads / 64 - 2);
        if (wave == 2) {
          plan_fold(q, lane);
          while (__hip_atomic_load(&s_bn_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
            __builtin_amdgcn_s_sleep(1);
          const int nq = s_gnode;
          const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
          for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) s_fv[k] = nq >= 0 ? node_label(m, s_fi[k].slot, nq) : -1;
        }
        fold_stage();
      } else if (sp1) {
        fold_others();
        if (fo && s_gprev >= 0) grp_bar();  // (the gather below uses every gathering wave)
        aggregate(q + 1, gt, gn, grp_bar);
        if (wave == 2) {
          plan_fold(q, lane);
          sweep_z(q + 1);  // every workgroup's counts of q+1 (without pod q) are in the region
        }
        grp_bar();
        load_totals(q + 1, gt, gn);
        grp_bar();
        minima_grp(q + 1, wave - 2, kAggThreads / 64 - 2);
        if (wave == 2) {
          // the chosen node's value of every fold item's label (once wave 0 has resolved the node)
          while (__hip_atomic_load(&s_bn_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
            __builtin_amdgcn_s_sleep(1);
          const int nq = s_gnode;
          const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
          for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) s_fv[k] = nq >= 0 ? node_label(m, s_fi[k].slot, nq) : -1;
        }
      } else if (lite1) {
        // node-local DoNotSchedule minima: the counts in LDS now -- kept (same template: the minima and their
        // multiplicities too), or loaded: then exchange Z gives those (through pod q-1), here or (aggLoopDebug 64)
        // after the placement; pod q's fold moves them
        // (loaded: exchange Z after the placement gives them -- or, one such constraint (kTqOne), exchange B
        // carries each workgroup's minimum, its nodes and those at it, from wave 2 here)
        if (tc_hit1) grp_bar();  // (pod q-1 folded in)
        if (wave == 2) {
          if (tq & kTqOne) {
            const uint8_t* bn = s_blob[(q + 1) % 3];
            const PodDesc& dn = *reinterpret_cast<const PodDesc*>(bn);
            const int c = __builtin_ctz((uint32_t)dn.agg_local_cons);
            const int32_t* lh = s_lh + (size_t)(-1 - at<PtsCons>(bn, dn.ptsf_off)[c].lref) * kAggSlots;
            long long mn = 0x7fffffffffffffffll;
            uint32_t cnt = 0;
            for (int ls = lane; ls < kAggSlots; ls += 64)
              if ((s_elig[ls] >> c) & 1u) {
                mn = lh[ls] < mn ? lh[ls] : mn;
                ++cnt;
              }
            mn = (long long)dec_i64(~wave_max_u64(~enc_i64(mn)));
            cnt = wave_sum_u32(cnt);
            uint32_t atm = 0;
            for (int ls = lane; ls < kAggSlots; ls += 64)
              if (((s_elig[ls] >> c) & 1u) && (long long)lh[ls] == mn) ++atm;
            atm = wave_sum_u32(atm);
            if (lane == 0) {
              s_lmin[0] = mn;
              s_lcnt[0] = cnt;
              s_latm[0] = atm;
            }
          }
          if (lane == 0) __hip_atomic_store(&s_elig_q, q + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          plan_fold(q, lane);
        }
        fold_stage();
        if (wave == 2) {
          while (__hip_atomic_load(&s_bn_q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != q)
            __builtin_amdgcn_s_sleep(1);
          const int nq = s_gnode;
          const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
          for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) s_fv[k] = nq >= 0 ? node_label(m, s_fi[k].slot, nq) : -1;
        }
      } else {
        fold_others();
        if (fo && s_gprev >= 0) grp_bar();  // before pod q-1's program slot takes q+2's
      }
      gstamp(q, 15);
      if (!RING && q + 2 < av.npods && !staged) stage_prog(q + 2, gt, gn);  // s_blob[(q+2)%3] held pod q-1
    }
    __syncthreads();
    if (!s_ok) return;
    if (SHARD && t == 0 && w == 0 && s_F > 0 && s_pw >= 0 && s_pw / G != av.rank) {
      // chosen on another rank: the result, and the pod joins this replica's pod table (the k_aggregate
      // pod role of later launch-path pods reads it).  The node's mirror columns are not mine in this
      // launch; the host uploads them with the next cycle's node updates (Cluster::add_pod).
      DevResult r;
      r.node = s_rnode;
      r.feasible = (int32_t)s_F;
      r.evaluated = 0;
      r.total = (int64_t)(s_best >> kPreBits);
      r.key = s_best;
      r.status = (int32_t)C_OK;
      r.ipa_any = ipa_any;
      b.results[pod] = r;
      if ((d.flags & DF_ASSUME) && d.slot >= 0) m.pod_node[d.slot] = s_rnode;
    }
    stamp(q, 5);

    // ======== pod q+1's counts, final ========
    if (more) {
      const int lq = s_pend_ls;
      if (sp1) {
        stamp(q, 6);
        stamp(q, 7);
        if (wave == 0) {
          fold_pod(lq, q + 1);
          if (same1) {  // the minima over the folded counts (no gathered ones to adjust)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            minima_grp(q + 1, 0, 1);
          }
          if (lane == 0) {
            if (lq >= 0) append(q, lq);
            s_nfi = 0;  // the next plan starts empty
          }
        }
        __syncthreads();
      } else if (kTc && (s_tcq & kTqLite)) {
        // pod q into q+1's counts: a node-local minimum moves by the chosen node's count (exchange B) and its
        // multiplicity; exchange Z again only when the fold took the last node off it
        const bool zend = (s_tcq & kTqHit) && !(s_tcq & kTqOne);  // (loaded, exchange Z not run yet)
        if (wave == 0) {
          fold_at(lq, s_gnode, s_el, !zend, q + 1);
          if (!zend) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            minima_grp(q + 1, 0, 1);
          }
          if (lane == 0) {
            if (lq >= 0) append(q, lq);
            s_nfi = 0;
          }
        }
        __syncthreads();
        if (zend || s_lstale) {
          aggregate(q + 1, t, kAggThreads, wg_bar, false);
          if (wave == 0) sweep_z(q + 1);
          __syncthreads();
          if (!s_ok) return;
          minima_grp(q + 1, wave, kAggThreads / 64);
          __syncthreads();
        }
      } else {
        if (t == 0 && lq >= 0) append(q, lq);
        __syncthreads();
        aggregate(q + 1, t, kAggThreads, wg_bar);
        if (wave == 0) sweep_z(q + 1);
        __syncthreads();
        if (!s_ok) return;
        load_totals(q + 1, t, kAggThreads);
        __syncthreads();
        if constexpr (kTc) minima_grp(q + 1, wave, kAggThreads / 64);  // (with multiplicities: a fold may follow)
        else minima(q + 1);
        __syncthreads();
      }
    } else if (RING) {
      // the next pod arrives through the ring: pod q joins its node owner's lists now, and its entry
      // (written by the owner's committing thread) is read by the owner's gathers of the pods after it.  While the host
      // turns around, pod q is folded into the counts in LDS as a next pod of its own template would count
      // it (the plan against q's own program): a next pod marked DF_AGG_SAME starts from them, any other
      // gathers afresh.  (q's own terms come from its entry in LDS, not the tables the owner wrote.)
      if (wave == 0) {
        // (q's own terms from its entry in LDS: the device term table is the owner's to read back)
        const RingEntry& he = *reinterpret_cast<const RingEntry*>(s_blob[(q + 1) % 3]);
        const bool sp = (d.flags & DF_AGGREGATE) && spec(d) && !(av.debug & 4) &&
                        (d.n_own_terms == 0 || (he.slot >= 0 && he.nterms == d.n_own_terms));
        if (sp) {
          plan_fold_b(s_blob[q % 3], s_blob[q % 3], lane, s_blob[(q + 1) % 3]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const int nq = s_gnode;
          const uint32_t nfi = s_nfi < (uint32_t)kFoldMax ? s_nfi : (uint32_t)kFoldMax;
          for (uint32_t k = (uint32_t)lane; k < nfi; k += 64) s_fv[k] = nq >= 0 ? node_label(m, s_fi[k].slot, nq) : -1;
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          fold_pod(s_pend_ls, q);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          minima_grp(q, 0, 1);
        }
        if (lane == 0) {
          if (s_pend_ls >= 0) append(q, s_pend_ls);
          s_nfi = 0;
          s_spec_q = sp ? q : -1;
        }
      }
      // (no agent-scope fence: the entry the owner wrote is read back only by the owner's own gathers -- its
      // lists -- within this launch; an agent-scope release / acquire here wrote back and invalidated the L2 of
      // every workgroup's XCD each pod: 11 µs per call at 100 000 nodes)
      __syncthreads();
      // and phase 1 of pod q's program again, against the cores this commit left and the folded counts: a next
      // pod of the same program (RING_SAME + DF_AGG_SAME, as a binding pops a ReplicaSet's pods) skips it
      if (!(av.debug & 128) && s_spec_q == q) {
        phase1();
        if (t == 0) s_ahead_q = q;
      }
    }
    if (kTc && t == 0) {  // pod q's placement, for the next pod's folds into the cached templates
      s_gprev = s_gnode;
      s_lprev = s_pend_ls;
    }
    stamp(q, 8);
  }
}
template <bool SHARD, bool PTSS, bool RING = false, int MS = kMaxSweep>
__global__ __launch_bounds__(kAggThreads) void k_agg_loop(MirrorView m, BatchView b, AggView av) {
  const AggGroupArg& a = *(const AggGroupArg*)__builtin_amdgcn_kernarg_segment_ptr();  // (k_sched_loop)
  agg_loop_body<SHARD, PTSS, RING, MS, false>(a.m, a.b, a.av, 0);
}
// In-process rank groups: every rank's node-sharded k_agg_loop in one dispatch (k_sched_loop_group)
__global__ __launch_bounds__(kAggThreads) void k_agg_loop_group(const AggGroupArg* __restrict__ ga, int G) {
  const int r = (int)blockIdx.x / G;
  const AggGroupArg& a = ga[r];
  agg_loop_body<true, true, false, kMaxSweep, true>(a.m, a.b, a.av, (int)blockIdx.x - r * G);
}

}  // namespace ksg

// ---- host-side launchers (C++ linkage, called by the host library) ------------------------------
namespace ksg {
// t0/t1 non-null: the events are attached to the dispatch packet itself (hipExtLaunchKernel), so
// their elapsed time is the kernel's own begin/end -- the same interval rocprofv3 reports.
// blk0/nblk: the node blocks to evaluate (nblk < 0: all of them).
hipError_t launch_filter_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, hipEvent_t t0,
                               hipEvent_t t1, int blk0, int nblk, bool lds) {
  if (nblk < 0) nblk = (m.n + kBlock - 1) / kBlock;
  if (nblk == 0) return hipSuccess;
  if (lds) {
    if (t0)
      hipExtLaunchKernelGGL(k_filter_score<true>, dim3(nblk), dim3(kBlock), 0, s, t0, t1, 0, m, b, pod, blk0);
    else
      hipLaunchKernelGGL(k_filter_score<true>, dim3(nblk), dim3(kBlock), 0, s, m, b, pod, blk0);
  } else {
    if (t0)
      hipExtLaunchKernelGGL(k_filter_score<false>, dim3(nblk), dim3(kBlock), 0, s, t0, t1, 0, m, b, pod, blk0);
    else
      hipLaunchKernelGGL(k_filter_score<false>, dim3(nblk), dim3(kBlock), 0, s, m, b, pod, blk0);
  }
  return hipGetLastError();
}
hipError_t launch_select(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, bool lds) {
  const int nb = (m.n + kBlock - 1) / kBlock;
  if (lds)
    hipLaunchKernelGGL(k_select<true>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, nb);
  else
    hipLaunchKernelGGL(k_select<false>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, nb);
  return hipGetLastError();
}
hipError_t launch_ob_hint(const MirrorView& m, const BatchView& b, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_ob_hint, dim3(1), dim3(64), 0, s, m, b, pod);
  return hipGetLastError();
}
hipError_t launch_nominated(const MirrorView& m, const BatchView& b, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_nominated, dim3(1), dim3(64), 0, s, m, b, pod);
  return hipGetLastError();
}
hipError_t launch_ob_store(const BatchView& b, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_ob_store, dim3(1), dim3(1024), 0, s, b, pod);
  return hipGetLastError();
}
hipError_t launch_ob_remap(ObState* st, ObEnt* h, const int32_t* map, int nold, int maxlen, hipStream_t s) {
  hipLaunchKernelGGL(k_ob_remap, dim3((maxlen + kBlock - 1) / kBlock > 0 ? (maxlen + kBlock - 1) / kBlock : 1),
                     dim3(kBlock), 0, s, st, h, map, nold);
  return hipGetLastError();
}
// ---- incremental mirror ingestion (Cache.UpdateNode, cache.go UpdateNode + UpdateSnapshot's
// generation diff): one thread per updated node writes its static columns in place.
__global__ __launch_bounds__(kBlock) void k_node_update(MirrorView m, const NodeUpdate* u, const uint32_t* ids,
                                                       const LabelEntry* lbl, const ScalarEntry* sc, int count) {
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= count) return;
  const NodeUpdate r = u[k];
  const int i = r.node;
  if (i < 0 || i >= m.n) return;
  const size_t cap = (size_t)m.cap;
  const_cast<int64_t*>(m.alloc_cpu)[i] = r.alloc_cpu;
  const_cast<int64_t*>(m.alloc_mem)[i] = r.alloc_mem;
  const_cast<int64_t*>(m.alloc_eph)[i] = r.alloc_eph;
  const_cast<int32_t*>(m.alloc_pods)[i] = r.alloc_pods;
  const_cast<uint32_t*>(m.flags)[i] = r.flags;
  for (int q = 0; q < m.scalar_cols; ++q) const_cast<int64_t*>(m.scalar_alloc)[(size_t)q * cap + i] = 0;
  for (uint32_t q = 0; q < r.sc_cnt; ++q)
    const_cast<int64_t*>(m.scalar_alloc)[(size_t)sc[r.sc_off + q].slot * cap + i] = sc[r.sc_off + q].value;
  for (int q = 0; q < r.n_taint; ++q) const_cast<uint32_t*>(m.taint_ids)[r.taint_off + q] = ids[r.id_off + q];
  for (int q = 0; q < r.n_img; ++q) const_cast<uint32_t*>(m.img_ids)[r.img_off + q] = ids[r.id_off + r.n_taint + q];
  for (int q = 0; q < r.lbl_cnt; ++q) {
    const LabelEntry e = lbl[r.lbl_off + q];
    const size_t o = (size_t)e.slot * cap + i;
    const_cast<int32_t*>(m.labels)[o] = e.value;
    const_cast<int64_t*>(m.label_num)[o] = e.num;
    const_cast<uint8_t*>(m.label_num_ok)[o] = (uint8_t)e.ok;
  }
}
hipError_t launch_node_update(const MirrorView& m, const NodeUpdate* u, const uint32_t* ids, const LabelEntry* lbl,
                              const ScalarEntry* sc, int count, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_node_update, dim3((count + kBlock - 1) / kBlock), dim3(kBlock), 0, s, m, u, ids, lbl, sc, count);
  return hipGetLastError();
}
// ---- node add / remove without a full re-layout (Cluster::relayout_gather): every surviving node's
// columns move to its new snapshot index in one gather per column block; new or changed nodes are
// then written by k_node_update / k_node_dyn.  dst[r][i] = src[r][idx[i]] for idx[i] >= 0
// (rows x cap elements of esz bytes, row stride cap elements).
__global__ __launch_bounds__(kBlock) void k_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* idx, int n,
                                                        int cap, int esz) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const int r = blockIdx.y;
  if (i >= n) return;
  const int s = idx[i];
  if (s < 0) return;
  const size_t ro = (size_t)r * (size_t)cap;
  if (esz == 8) {
    reinterpret_cast<uint64_t*>(dst)[ro + i] = reinterpret_cast<const uint64_t*>(src)[ro + s];
  } else if (esz == 4) {
    reinterpret_cast<uint32_t*>(dst)[ro + i] = reinterpret_cast<const uint32_t*>(src)[ro + s];
  } else if (esz == 1) {
    dst[ro + i] = src[ro + s];
  } else {  // ports: port_slots uint32 per node
    for (int k = 0; k < esz / 4; ++k)
      reinterpret_cast<uint32_t*>(dst)[(ro + i) * (size_t)(esz / 4) + k] =
          reinterpret_cast<const uint32_t*>(src)[(ro + s) * (size_t)(esz / 4) + k];
  }
}
// CSR ids (taints, images): node i's run moves from old_off[idx[i]] to new_off[i]
__global__ __launch_bounds__(kBlock) void k_gather_csr(uint32_t* dst, const uint32_t* src, const int32_t* idx,
                                                       const uint32_t* old_off, const uint32_t* new_off, int n) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int s = idx[i];
  if (s < 0) return;
  const uint32_t lo = old_off[s], cnt = old_off[s + 1] - lo, to = new_off[i];
  for (uint32_t k = 0; k < cnt; ++k) dst[to + k] = src[lo + k];
}
hipError_t launch_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* idx, int n, int cap, int rows, int esz,
                              hipStream_t s) {
  if (n <= 0 || rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_rows, dim3((n + kBlock - 1) / kBlock, rows), dim3(kBlock), 0, s, dst, src, idx, n, cap, esz);
  return hipGetLastError();
}
hipError_t launch_gather_csr(uint32_t* dst, const uint32_t* src, const int32_t* idx, const uint32_t* old_off,
                             const uint32_t* new_off, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_csr, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, dst, src, idx, old_off, new_off, n);
  return hipGetLastError();
}

// pod events (NodeInfo.update via AddPod / RemovePod / ForgetPod): one thread per queued node
// writes its dynamic columns in place
__global__ __launch_bounds__(kBlock) void k_node_dyn(MirrorView m, const NodeDyn* d, const uint32_t* port_pool,
                                                     const ScalarEntry* sc, int count) {
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= count) return;
  const NodeDyn& r = d[k];
  const int i = r.node;
  if (i < 0 || i >= m.n) return;
  const size_t cap = (size_t)m.cap;
  m.req_cpu[i] = r.req_cpu;
  m.req_mem[i] = r.req_mem;
  m.req_eph[i] = r.req_eph;
  m.nz_cpu[i] = r.nz_cpu;
  m.nz_mem[i] = r.nz_mem;
  m.num_pods[i] = r.num_pods;
  for (int q = 0; q < m.scalar_cols; ++q) m.scalar_req[(size_t)q * cap + i] = 0;
  for (uint32_t q = 0; q < r.sc_cnt; ++q) m.scalar_req[(size_t)sc[r.sc_off + q].slot * cap + i] = sc[r.sc_off + q].value;
  for (int q = 0; q < m.port_slots; ++q)
    m.ports[(size_t)i * m.port_slots + q] = (uint32_t)q < r.port_cnt ? port_pool[r.port_off + q] : 0xffffffffu;
}
hipError_t launch_node_dyn(const MirrorView& m, const NodeDyn* d, const uint32_t* port_pool, const ScalarEntry* sc,
                           int count, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_node_dyn, dim3((count + kBlock - 1) / kBlock), dim3(kBlock), 0, s, m, d, port_pool, sc, count);
  return hipGetLastError();
}
hipError_t launch_sample(const MirrorView& m, const BatchView& b, int pod, bool cut, hipStream_t s) {
  const int nb = (m.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_sample_find, dim3(1), dim3(kBlock), 0, s, m, b, pod, nb);
  if (cut && nb > 0) hipLaunchKernelGGL(k_sample_apply, dim3(nb), dim3(kBlock), 0, s, m, b, pod, 0, 0);
  return hipGetLastError();
}
hipError_t launch_sample_shard_a(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_sample_shard_a, dim3(1), dim3(kBlock), 0, s, m, b, sv, pod);
  return hipGetLastError();
}
hipError_t launch_sample_shard_b(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, bool cut,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_sample_shard_b, dim3(1), dim3(kBlock), 0, s, m, b, sv, pod, cut ? 1 : 0);
  if (cut && sv.nblk > 0)
    hipLaunchKernelGGL(k_sample_apply, dim3(sv.nblk), dim3(kBlock), 0, s, m, b, pod, sv.blk0, 1);
  return hipGetLastError();
}
hipError_t launch_xpack_a(const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_xpack_a, dim3(1), dim3(kBlock), 0, s, b, sv, pod);
  return hipGetLastError();
}
hipError_t launch_unpack_pts(const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack_pts, dim3(1), dim3(kBlock), 0, s, b, sv, pod);
  return hipGetLastError();
}
hipError_t launch_xpack_p(const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_xpack_p, dim3(1), dim3(1), 0, s, b, sv, pod);
  return hipGetLastError();
}
// nblk == 0 (an empty shard) still launches one block: the rank must publish its (empty) share
hipError_t launch_select_shard(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  ShardView v = sv;
  hipLaunchKernelGGL(k_select_shard, dim3(v.nblk > 0 ? v.nblk : 1), dim3(kBlock), 0, s, m, b, v, pod);
  return hipGetLastError();
}
hipError_t launch_commit(const MirrorView& m, const BatchView& b, const ShardView& sv, int pod, hipStream_t s) {
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, s, m, b, sv, pod);
  return hipGetLastError();
}
hipError_t launch_max_reduce(unsigned long long* dst, const RankPtrs& src, int nsrc, int count, hipStream_t s) {
  const int nb = (count + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_max_reduce, dim3(nb < 64 ? (nb > 0 ? nb : 1) : 64), dim3(kBlock), 0, s, dst, src, nsrc, count);
  return hipGetLastError();
}
// unit 128: 128-node workgroups (two evaluation waves, every role on a SIMD of its own); 256: four
hipError_t launch_sched_loop(const MirrorView& m, const BatchView& b, const LoopView& lv, hipStream_t s,
                             hipEvent_t t0, hipEvent_t t1, int unit) {
  if (lv.ring) {  // resident (no timing events: the launch spans many calls)
    if (unit == 128 && lv.world * lv.nwg <= 64)
      hipLaunchKernelGGL((k_sched_loop<2, true, 1>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, m, b, lv);
    else if (unit == 128)
      hipLaunchKernelGGL((k_sched_loop<2, true>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, m, b, lv);
    else
      hipLaunchKernelGGL((k_sched_loop<4, true>), dim3(lv.nwg), dim3(kLoopThreads), 0, s, m, b, lv);
  } else if (unit == 128 && lv.world * lv.nwg <= 64) {  // one sweep round (C2's 40 workgroups)
    if (t0)
      hipExtLaunchKernelGGL((k_sched_loop<2, false, 1>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, t0, t1, 0, m, b, lv);
    else
      hipLaunchKernelGGL((k_sched_loop<2, false, 1>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, m, b, lv);
  } else if (unit == 128) {
    if (t0)
      hipExtLaunchKernelGGL((k_sched_loop<2, false>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, t0, t1, 0, m, b, lv);
    else
      hipLaunchKernelGGL((k_sched_loop<2, false>), dim3(lv.nwg), dim3(2 * 64 + 128), 0, s, m, b, lv);
  } else {
    if (t0)
      hipExtLaunchKernelGGL((k_sched_loop<4, false>), dim3(lv.nwg), dim3(kLoopThreads), 0, s, t0, t1, 0, m, b, lv);
    else
      hipLaunchKernelGGL((k_sched_loop<4, false>), dim3(lv.nwg), dim3(kLoopThreads), 0, s, m, b, lv);
  }
  return hipGetLastError();
}
hipError_t launch_agg_loop(const MirrorView& m, const BatchView& b, const AggView& av, hipStream_t s, hipEvent_t t0,
                           hipEvent_t t1) {
  auto go = [&](auto kern) {
    if (t0)
      hipExtLaunchKernelGGL(kern, dim3(av.nwg), dim3(kAggThreads), 0, s, t0, t1, 0, m, b, av);
    else
      hipLaunchKernelGGL(kern, dim3(av.nwg), dim3(kAggThreads), 0, s, m, b, av);
  };
  if (av.ring) {
    go(k_agg_loop<false, true, true>);  // the resident instance (unsharded)
  } else if (av.world > 1) {
    go(k_agg_loop<true, true>);  // (the sharded instance without PTSS spills registers: not built)
  } else {
    if (av.ptss && av.nwg <= 64) go(k_agg_loop<false, true, false, 1>);
    else if (av.ptss) go(k_agg_loop<false, true>);
    else if (av.nwg <= 64) go(k_agg_loop<false, false, false, 1>);  // one sweep round (C3, C4)
    else go(k_agg_loop<false, false>);  // up to four rounds, polled together (C5)
  }
  return hipGetLastError();
}
// A rank's group launch arguments into the leader's device array, stream-ordered (the kernel arguments are
// copied at enqueue time, and the loop before it on the stream has ended before this overwrites its slot)
template <class A>
__global__ void k_put_group_arg(A a, A* dst) {
  if (threadIdx.x == 0) *dst = a;
}
hipError_t launch_put_group_arg(const LoopGroupArg& a, LoopGroupArg* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_put_group_arg<LoopGroupArg>, dim3(1), dim3(64), 0, s, a, dst);
  return hipGetLastError();
}
hipError_t launch_put_group_arg(const AggGroupArg& a, AggGroupArg* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_put_group_arg<AggGroupArg>, dim3(1), dim3(64), 0, s, a, dst);
  return hipGetLastError();
}
// In-process rank groups: every rank's loop in one dispatch of world * nwg workgroups (ga: [world] in device
// memory; the same instance choice as launch_sched_loop / launch_agg_loop's node-sharded batch instances)
hipError_t launch_sched_loop_group(const LoopGroupArg* ga, int world, int nwg, hipStream_t s, hipEvent_t t0,
                                   hipEvent_t t1, int unit) {
  const dim3 grid(world * nwg);
  if (unit == 128 && world * nwg <= 64)
    hipExtLaunchKernelGGL((k_sched_loop_group<2, 1>), grid, dim3(2 * 64 + 128), 0, s, t0, t1, 0, ga, nwg);
  else if (unit == 128)
    hipExtLaunchKernelGGL((k_sched_loop_group<2, kMaxSweep>), grid, dim3(2 * 64 + 128), 0, s, t0, t1, 0, ga, nwg);
  else
    hipExtLaunchKernelGGL((k_sched_loop_group<4, kMaxSweep>), grid, dim3(kLoopThreads), 0, s, t0, t1, 0, ga, nwg);
  return hipGetLastError();
}
hipError_t launch_agg_loop_group(const AggGroupArg* ga, int world, int nwg, hipStream_t s, hipEvent_t t0, hipEvent_t t1) {
  hipExtLaunchKernelGGL(k_agg_loop_group, dim3(world * nwg), dim3(kAggThreads), 0, s, t0, t1, 0, ga, nwg);
  return hipGetLastError();
}
// Workgroups of each persistent loop one CU holds at once (the loops' grids must be resident as a whole:
// every workgroup spins on the others' granules): [0] k_sched_loop 128-node unit, [1] 256-node unit,
// [2] k_agg_loop, [3] its node-sharded instance.  0 means the kernel cannot be resident at all.
hipError_t loop_occupancy(int (&occ)[4]) {
  struct K { const void* f; int threads; } ks[4] = {
      {reinterpret_cast<const void*>(&k_sched_loop<2, false>), 2 * 64 + 128},
      {reinterpret_cast<const void*>(&k_sched_loop<4, false>), kLoopThreads},
      {reinterpret_cast<const void*>(&k_agg_loop<false, true>), kAggThreads},
      {reinterpret_cast<const void*>(&k_agg_loop<true, true>), kAggThreads}};
  for (int i = 0; i < 4; ++i) {
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[i], ks[i].f, ks[i].threads, 0);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
// Loads the module's code object onto the current device now (hipFuncGetAttributes), so that no
// first launch inside a batch does it while an in-process peer's persistent loop is running.
hipError_t warm_kernels() {
  hipFuncAttributes a;
  const void* fs[] = {reinterpret_cast<const void*>(&k_filter_score<true>), reinterpret_cast<const void*>(&k_filter_score<false>),
                      reinterpret_cast<const void*>(&k_select<true>),       reinterpret_cast<const void*>(&k_select<false>),
                      reinterpret_cast<const void*>(&k_xpack_a),            reinterpret_cast<const void*>(&k_unpack_pts),
                      reinterpret_cast<const void*>(&k_xpack_p),            reinterpret_cast<const void*>(&k_select_shard),
                      reinterpret_cast<const void*>(&k_commit),             reinterpret_cast<const void*>(&k_max_reduce),
                      reinterpret_cast<const void*>(&k_sched_loop<4, false>), reinterpret_cast<const void*>(&k_sched_loop<2, false>),
                      reinterpret_cast<const void*>(&k_sched_loop<4, true>), reinterpret_cast<const void*>(&k_sched_loop<2, true>),
                      reinterpret_cast<const void*>(&k_sched_loop<2, false, 1>), reinterpret_cast<const void*>(&k_sched_loop<2, true, 1>),         reinterpret_cast<const void*>(&k_sample_find),
                      reinterpret_cast<const void*>(&k_sample_apply),        reinterpret_cast<const void*>(&k_sample_shard_a),
                      reinterpret_cast<const void*>(&k_sample_shard_b),        reinterpret_cast<const void*>(&k_node_update),
                      reinterpret_cast<const void*>(&k_node_dyn),           reinterpret_cast<const void*>(&k_agg_loop<false, false>),
                      reinterpret_cast<const void*>(&k_agg_loop<false, true>),
                      reinterpret_cast<const void*>(&k_agg_loop<true, true>),
                      reinterpret_cast<const void*>(&k_agg_loop<false, true, true>),
                      reinterpret_cast<const void*>(&k_agg_loop<false, true, false, 1>),
                      reinterpret_cast<const void*>(&k_agg_loop<false, false, false, 1>),
                      reinterpret_cast<const void*>(&k_gather_rows),        reinterpret_cast<const void*>(&k_gather_csr),
                      reinterpret_cast<const void*>(&k_ob_hint),            reinterpret_cast<const void*>(&k_ob_store),
                      reinterpret_cast<const void*>(&k_nominated),
                      reinterpret_cast<const void*>(&k_sched_loop_group<2, 1>),
                      reinterpret_cast<const void*>(&k_sched_loop_group<2, kMaxSweep>),
                      reinterpret_cast<const void*>(&k_sched_loop_group<4, kMaxSweep>),
                      reinterpret_cast<const void*>(&k_agg_loop_group),
                      reinterpret_cast<const void*>(&k_put_group_arg<LoopGroupArg>),
                      reinterpret_cast<const void*>(&k_put_group_arg<AggGroupArg>),
                      reinterpret_cast<const void*>(&k_ob_remap)};
  for (const void* f : fs) {
    const hipError_t e = hipFuncGetAttributes(&a, f);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
#ifdef KSG_DIAG
hipError_t set_diag(unsigned long long* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &p, sizeof(p)); }
#endif

// =====================================================================================================
// k_preempt / k_preempt_seg: DefaultPreemption.SelectVictimsOnNode (default_preemption.go:252-354) for every
// node the dry run may check (findCandidates' NodesForStatusCode(Unschedulable), preemption.go:174-196, or
// every node), one thread per node, the preemptor's cycle status in b.status (k_filter_score, evaluation
// output).  The node's state is the mirror minus the victims: the filters a removal can change run on it --
// NodePorts, NodeResourcesFit (the static filters before them passed or fail unchanged), then
// PodTopologySpread / InterPodAffinity with the victims' RemovePod / AddPod effect on the cycle's counts
// (PreemptTopo) -- and the victims are added back one at a time in reprieve order, each kept removed only
// when the preemptor no longer fits with it (reprievePod, :316-343).
// =====================================================================================================
// The cycle's PodTopologySpread counts as the preemption dry run sees them at node i: the preFilterState
// clone with the victims' RemovePod / AddPod applied (podtopologyspread/filtering.go:157-212).  Every
// victim is on node i, so only the count of node i's own domain moves; the domain minimum becomes the
// smaller of that count and the minimum over the other domains -- what criticalPaths.update tracks
// exactly for a sequence of updates to one domain.  InterPodAffinity's counts move the same way
// (filtering.go:75-85 updateWithPod): group 0 the preemptor's required affinity terms, group 1 its required
// anti-affinity terms, group 2 the existing-anti keys, each entry the count of node i's own domain.
//
// The tracked state lives in one of two stores.  PreemptRegs: up to kPreemptCons entries of each kind in
// registers (every loop over them is unrolled, so every index is static).  PreemptWide: any count the pod
// compiler accepts, in a per-node workspace laid out field-major and node-minor ([field][n]), so a wave's
// lanes touch consecutive words.
struct PreemptRegs {
  static constexpr bool kWide = false;
  static constexpr int kCap = kPreemptCons;
  mutable int64_t hb_[kCap], vi_[kCap], cnt0_[kCap], dlt_[kCap], excl_[kCap], atot_[kCap];
  mutable int32_t ihb_[3 * kCap], ivi_[3 * kCap], idl_[3 * kCap];
  __device__ __forceinline__ void bind(const PreemptIn&, int, int) {}
  __device__ __forceinline__ int64_t& hb(int c) const { return hb_[c]; }
  __device__ __forceinline__ int64_t& vi(int c) const { return vi_[c]; }
  __device__ __forceinline__ int64_t& cnt0(int c) const { return cnt0_[c]; }
  __device__ __forceinline__ int64_t& dlt(int c) const { return dlt_[c]; }
  __device__ __forceinline__ int64_t& excl(int c) const { return excl_[c]; }
  __device__ __forceinline__ int64_t& atot(int k) const { return atot_[k]; }
  __device__ __forceinline__ int32_t& ihb(int g, int k) const { return ihb_[g * kCap + k]; }
  __device__ __forceinline__ int32_t& ivi(int g, int k) const { return ivi_[g * kCap + k]; }
  __device__ __forceinline__ int32_t& idl(int g, int k) const { return idl_[g * kCap + k]; }
};
struct PreemptWide {
  static constexpr bool kWide = true;
  long long* w;  // this node's word of field 0
  size_t st;     // words between fields (the node count)
  int C, G;
  __device__ __forceinline__ void bind(const PreemptIn& in, int i, int n) {
    w = in.wide + i;
    st = (size_t)n;
    C = in.wide_c;
    G = in.wide_g;
  }
  __device__ __forceinline__ int64_t& f(int k) const { return *reinterpret_cast<int64_t*>(w + (size_t)k * st); }
  __device__ __forceinline__ int64_t& hb(int c) const { return f(c); }
  __device__ __forceinline__ int64_t& vi(int c) const { return f(C + c); }
  __device__ __forceinline__ int64_t& cnt0(int c) const { return f(2 * C + c); }
  __device__ __forceinline__ int64_t& dlt(int c) const { return f(3 * C + c); }
  __device__ __forceinline__ int64_t& excl(int c) const { return f(4 * C + c); }
  __device__ __forceinline__ int64_t& atot(int k) const { return f(5 * C + k); }
  __device__ __forceinline__ int64_t& ihb(int g, int k) const { return f(5 * C + G + g * G + k); }
  __device__ __forceinline__ int64_t& ivi(int g, int k) const { return f(5 * C + 4 * G + g * G + k); }
  __device__ __forceinline__ int64_t& idl(int g, int k) const { return f(5 * C + 7 * G + g * G + k); }
};
// f(k) for k < n: a plain loop over the workspace, an unrolled guarded one over the registers
template <class S, class F>
__device__ __forceinline__ void each_k(int n, F&& f) {
  if constexpr (S::kWide) {
    for (int k = 0; k < n; ++k) f(k);
  } else {
#pragma unroll
    for (int k = 0; k < S::kCap; ++k)
      if (k < n) f(k);
  }
}
template <class S>
struct PreemptTopo {
  ArenaTopo a;
  S s;
  int32_t nc;     // DoNotSchedule constraints (an entry with hb < 0: node i is not eligible for it)
  int32_t ng[3];  // entries per InterPodAffinity group
  // a preemptor matching its own required affinity terms (filtering.go:404-415): whether affinityCounts is
  // empty depends on every count, not only node i's -- the cycle's total per term (atot) with the victims'
  // deltas at node i's domains; nra < 0: not tracked (the cycle's bit)
  int32_t nra;
  __device__ __forceinline__ int64_t cnt(int32_t hist_base, int32_t lref, int32_t v, int ls) const {
    int64_t x = a.cnt(hist_base, lref, v, ls);
    each_k<S>(nc, [&](int c) {
      if (s.hb(c) == hist_base && s.vi(c) == v) x += s.dlt(c);
    });
#pragma unroll
    for (int g = 0; g < 3; ++g)
      each_k<S>(ng[g], [&](int k) {
        if (s.ihb(g, k) == hist_base && s.ivi(g, k) == v) x += s.idl(g, k);
      });
    return x;
  }
  __device__ __forceinline__ int64_t pmin(int c) const {
    int64_t r = a.pmin(c);
    auto own = [&](int k) {
      const int64_t o = s.cnt0(k) + s.dlt(k);
      r = o < s.excl(k) ? o : s.excl(k);
    };
    if constexpr (S::kWide) {
      if (c < nc && s.hb(c) >= 0) own(c);
    } else {
      each_k<S>(nc, [&](int k) {
        if (k == c && s.hb(k) >= 0) own(k);
      });
    }
    return r;
  }
  __device__ __forceinline__ uint32_t pndom(int c) const { return a.pndom(c); }
  __device__ __forceinline__ uint32_t any() const {
    const uint32_t a0 = a.any();
    if (nra < 0) return a0;
    bool nonempty = false;  // affinityCounts after the removals / reprieves: some term's total is not 0
    each_k<S>(nra, [&](int k) {
      int64_t x = s.atot(k);
      each_k<S>(nra, [&](int j) {
        if (s.ihb(0, j) == s.ihb(0, k) && s.ivi(0, j) >= 0) x += s.idl(0, j);
      });
      nonempty |= x != 0;
    });
    return (a0 & ~1u) | (nonempty ? 1u : 0u);
  }
};

// Per required affinity term of the preemptor: the cycle's total count over the term's
// histogram (k_aggregate's arena) -- whether affinityCounts is empty once victims are removed (PreemptTopo::any).
__global__ __launch_bounds__(kBlock) void k_aff_totals(BatchView b, int pod, long long* out) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  const int k = blockIdx.x;
  if (k >= d.n_raff) return;
  const IpaTerm t = at<IpaTerm>(base, d.raff_off)[k];
  long long x = 0;
  for (int v = threadIdx.x; v < t.nvals; v += kBlock) x += (long long)b.arena[t.hist_base + v];
  __shared__ long long s[kBlock];
  s[threadIdx.x] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long y = 0;
    for (int q = 0; q < kBlock; ++q) y += s[q];
    out[k] = y;
  }
}
hipError_t launch_aff_totals(const BatchView& b, int pod, int nterms, long long* out, hipStream_t s) {
  if (nterms <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_aff_totals, dim3(nterms), dim3(kBlock), 0, s, b, pod, out);
  return hipGetLastError();
}

// Per DoNotSchedule constraint (one workgroup each): the minimum count over the present domains, how many
// domains hold it, and the next larger count -- the minimum over "every domain but one holding the
// minimum", which PreemptTopo needs for the node whose own domain is that one.
__global__ __launch_bounds__(kBlock) void k_pts_minima(BatchView b, int pod, long long* mm) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  const int c = blockIdx.x;
  if (c >= d.n_ptsf) return;
  const PtsCons cs = at<PtsCons>(base, d.ptsf_off)[c];
  const long long INF = 0x7fffffffffffffffll;
  long long mn = INF, nx = INF, cnt = 0;
  for (int v = threadIdx.x; v < cs.nvals; v += kBlock) {
    if (!b.arena[cs.pres_base + v]) continue;
    const long long x = (long long)b.arena[cs.hist_base + v];
    if (x < mn) {
      nx = mn;
      mn = x;
      cnt = 1;
    } else if (x == mn) {
      ++cnt;
    } else if (x < nx) {
      nx = x;
    }
  }
  __shared__ long long s[3][kBlock];
  s[0][threadIdx.x] = mn;
  s[1][threadIdx.x] = cnt;
  s[2][threadIdx.x] = nx;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long m0 = INF, c0 = 0, n0 = INF;
    for (int t = 0; t < kBlock; ++t) {
      const long long m1 = s[0][t], c1 = s[1][t], n1 = s[2][t];
      if (c1 == 0) continue;
      if (m1 < m0) {
        n0 = m0 < n1 ? m0 : n1;
        m0 = m1;
        c0 = c1;
      } else if (m1 == m0) {
        c0 += c1;
        n0 = n0 < n1 ? n0 : n1;
      } else {
        n0 = n0 < m1 ? n0 : m1;
      }
    }
    mm[3 * c] = m0;
    mm[3 * c + 1] = c0;
    mm[3 * c + 2] = n0;
  }
}

hipError_t launch_pts_minima(const BatchView& b, int pod, int ncons, long long* mm, hipStream_t s) {
  if (ncons <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pts_minima, dim3(ncons), dim3(kBlock), 0, s, b, pod, mm);
  return hipGetLastError();
}

// The existing pods' required anti-affinity terms that match the preemptor (the term role of k_aggregate,
// AffinityTerm.Matches, types.go:391-396), counted per owning pod-table slot and existing-anti key: what a
// victim's RemovePod takes out of existingAntiAffinityCounts at its node (filtering.go:75-85).
__global__ __launch_bounds__(kBlock) void k_preempt_terms(MirrorView m, BatchView b, int pod, int32_t* contrib) {
  const int j = (int)blockIdx.x * kBlock + (int)threadIdx.x;
  if (j >= m.n_terms) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  const DTerm t = m.terms[j];
  if (t.kind != T_REQ_ANTI || m.pod_node[t.owner] < 0 || t.key >= d.n_keytab) return;
  const int32_t* kt = at<int32_t>(base, d.keytab_off) + (size_t)t.key * kKeytabStride;
  const int32_t hb = (d.ipa_flags & IPA_EXIST_FILTER) ? kt[1] : -1;
  if (hb < 0) return;
  const int32_t* tp = m.term_pool;
  const unsigned long long* il = at<unsigned long long>(base, d.lbl_off);
  const unsigned long long* nl = at<unsigned long long>(base, d.nslbl_off);
  const bool match = (id_in(tp + t.ns_off, t.ns_cnt, d.ns_id) || lsel_match(tp + t.nssel, nl, d.n_nslbl)) &&
                     lsel_match(tp + t.sel, il, d.n_lbl);
  if (!match) return;
  const KeyHist* ek = at<KeyHist>(base, d.exkeys_off);
  for (int e = 0; e < d.n_exkeys; ++e)
    if (ek[e].base == hb) {
      atomicAdd(&contrib[(size_t)t.owner * (size_t)d.n_exkeys + e], 1);
      return;
    }
}
hipError_t launch_preempt_terms(const MirrorView& m, const BatchView& b, int pod, int32_t* contrib, hipStream_t s) {
  if (m.n_terms <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_preempt_terms, dim3((m.n_terms + kBlock - 1) / kBlock), dim3(kBlock), 0, s, m, b, pod, contrib);
  return hipGetLastError();
}


// Fit with the victims removed (fit.go:593-734, as run_filters): nc holds the node's Requested less the
// removed victims; sreq (nullptr: no extended resources) the same for each of the preemptor's scalar
// resources, add (nullptr: none) a victim's request of them being tried back (reprieve)
__device__ __forceinline__ uint32_t preempt_node_filters(const MirrorView& m, const NodeCore& nc, const int64_t* sreq,
                                                         const int64_t* add, const uint8_t* base, const PodDesc& d,
                                                         int i, bool port) {
  const uint32_t fm = d.filter_mask;
  if (((fm >> P_PORTS) & 1u) && port) return pack_status(C_UNSCHED, P_PORTS, KSG_R_NODE_PORTS);
  if ((fm >> P_FIT) & 1u) {
    uint32_t reasons = 0;
    bool unresolvable = false;
    if ((int64_t)nc.npods + 1 > (int64_t)nc.apods) reasons |= KSG_R_TOO_MANY_PODS;
    if (d.fit_any) {
      if (d.req_cpu > 0 && d.req_cpu > nc.acpu - nc.rcpu) {
        reasons |= KSG_R_INSUFFICIENT_CPU;
        unresolvable |= d.req_cpu > nc.acpu;
      }
      if (d.req_mem > 0 && d.req_mem > nc.amem - nc.rmem) {
        reasons |= KSG_R_INSUFFICIENT_MEMORY;
        unresolvable |= d.req_mem > nc.amem;
      }
      if (d.req_eph > 0 && d.req_eph > nc.aeph - nc.reph) {
        reasons |= KSG_R_INSUFFICIENT_EPHEMERAL;
        unresolvable |= d.req_eph > nc.aeph;
      }
      const ScalarReq* sr = at<ScalarReq>(base, d.scalar_off);
      for (int k = 0; sreq && k < d.n_scalar; ++k) {
        const int64_t a = m.scalar_alloc[(size_t)sr[k].slot * (size_t)m.cap + (size_t)i];
        const int64_t used = sreq[k] + (add ? add[k] : 0);
        if (sr[k].qty > a - used) {
          reasons |= KSG_R_INSUFFICIENT_SCALAR;
          unresolvable |= sr[k].qty > a;
        }
      }
    }
    if (reasons) return pack_status(unresolvable ? C_UU : C_UNSCHED, P_FIT, reasons);
  }
  return 0u;
}

// The victims' topology effects at node i, as both dry-run kernels track them
template <class S>
struct TopoTrack {
  PreemptTopo<S> tp;
  uint32_t elig;  // DoNotSchedule constraints node i is eligible for (pts_eligible)
};
template <class S>
__device__ __forceinline__ void topo_track_init(const MirrorView& m, const BatchView& b, int pod, const uint8_t* base,
                                                const PodDesc& d, int i, const PreemptIn& in, TopoTrack<S>& T,
                                                uint32_t* flags) {
  PreemptTopo<S>& tp = T.tp;
  const S& st = tp.s;
  tp.a = ArenaTopo{b.stats + pod, b.arena};
  tp.s.bind(in, i, m.n);
  const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
  tp.nc = in.pts_check ? d.n_ptsf : 0;
  tp.ng[0] = in.ipa_check ? d.n_raff : 0;
  tp.ng[1] = in.ipa_check ? d.n_ranti : 0;
  tp.ng[2] = (in.ipa_check && in.ex_contrib) ? d.n_exkeys : 0;
  if constexpr (!S::kWide) {
    // the host sends a preemptor beyond the registers to the workspace-resident dry run; a mismatch is an
    // internal error the pick reports (PSegOut flag bit 0), never a wrong result
    if (tp.nc > S::kCap || tp.ng[0] > S::kCap || tp.ng[1] > S::kCap || tp.ng[2] > S::kCap) {
      *flags |= 1u;
      tp.nc = tp.ng[0] = tp.ng[1] = tp.ng[2] = 0;
    }
  }
  T.elig = tp.nc ? pts_eligible(m, base, d, cs, d.n_ptsf, i) : 0u;
  each_k<S>(tp.nc, [&](int c) {
    st.hb(c) = st.vi(c) = -1;
    st.cnt0(c) = st.dlt(c) = st.excl(c) = 0;
    if ((T.elig >> c) & 1u) {
      const int32_t v = node_label(m, cs[c].slot, i);
      st.hb(c) = cs[c].hist_base;
      st.vi(c) = v;
      st.cnt0(c) = (int64_t)b.arena[cs[c].hist_base + v];
      const long long* mm = in.pts_mm + 3 * c;
      st.excl(c) = (st.cnt0(c) == mm[0] && mm[1] == 1) ? mm[2] : mm[0];
    }
  });
  const IpaTerm* raff = at<IpaTerm>(base, d.raff_off);
  const IpaTerm* ranti = at<IpaTerm>(base, d.ranti_off);
  const KeyHist* ek = at<KeyHist>(base, d.exkeys_off);
  each_k<S>(tp.ng[0], [&](int k) {
    st.ihb(0, k) = raff[k].hist_base;
    st.ivi(0, k) = node_label(m, raff[k].slot, i);
    st.idl(0, k) = 0;
  });
  each_k<S>(tp.ng[1], [&](int k) {
    st.ihb(1, k) = ranti[k].hist_base;
    st.ivi(1, k) = node_label(m, ranti[k].slot, i);
    st.idl(1, k) = 0;
  });
  each_k<S>(tp.ng[2], [&](int k) {
    st.ihb(2, k) = ek[k].base;
    st.ivi(2, k) = node_label(m, ek[k].slot, i);
    st.idl(2, k) = 0;
  });
  tp.nra = -1;
  if (in.ipa_check && in.aff_tot && (d.ipa_flags & IPA_SELF_ALL)) {
    tp.nra = tp.ng[0];
    each_k<S>(tp.nra, [&](int k) { st.atot(k) = (int64_t)in.aff_tot[k]; });
  }
}
// The victim in pod-table slot `slot` removed (sg = -1) or added back (+1) at node i; false: no count moves.
// PodTopologySpread (updateWithPod, podtopologyspread/filtering.go:181-212): a victim in the preemptor's
// namespace that matches a DoNotSchedule constraint's selector, at a node eligible for it.
// InterPodAffinity (filtering.go:75-85): the preemptor's affinity terms count it when it matches all of
// them, its anti-affinity terms each when it matches, and its own required anti-affinity terms that match
// the preemptor count at their keys.  (A preemptor matching its own terms: affinityCounts emptied by the
// removal flips the "no pod matches anywhere" rule, filtering.go:404-415 -- PreemptTopo::any.)
template <class S>
__device__ __forceinline__ bool topo_victim(const MirrorView& m, const uint8_t* base, const PodDesc& d,
                                            const PreemptIn& in, TopoTrack<S>& T, int32_t slot, int sg) {
  const S& st = T.tp.s;
  const int32_t ns = m.pod_ns[slot];
  const unsigned long long* lb = m.lbl_pool + m.pod_lbl_off[slot];
  const int32_t ln = (int32_t)m.pod_lbl_cnt[slot];
  const int32_t* sp = at<int32_t>(base, d.sel_pool_off);
  bool moved = false;
  if (T.elig && ns == d.ns_id) {
    const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
    each_k<S>(T.tp.nc, [&](int c) {
      if (((T.elig >> c) & 1u) && lsel_match(sp + cs[c].sel, lb, ln)) {
        st.dlt(c) += sg;
        moved = true;
      }
    });
  }
  const int nra = T.tp.ng[0], nrn = T.tp.ng[1], nex = T.tp.ng[2];
  if (nra == 0 && nrn == 0 && nex == 0) return moved;
  const IpaTerm* raff = at<IpaTerm>(base, d.raff_off);
  const IpaTerm* ranti = at<IpaTerm>(base, d.ranti_off);
  bool all = nra > 0;
  each_k<S>(nra, [&](int k) { all = all && term_matches_pod(sp, raff[k], ns, lb, ln); });
  if (all)
    each_k<S>(nra, [&](int k) {
      if (st.ivi(0, k) >= 0) {
        st.idl(0, k) += sg;
        moved = true;
      }
    });
  each_k<S>(nrn, [&](int k) {
    if (st.ivi(1, k) >= 0 && term_matches_pod(sp, ranti[k], ns, lb, ln)) {
      st.idl(1, k) += sg;
      moved = true;
    }
  });
  each_k<S>(nex, [&](int k) {
    if (st.ivi(2, k) >= 0) {
      const int32_t cn = in.ex_contrib[(size_t)slot * in.ex_stride + k];
      if (cn) {
        st.idl(2, k) += sg * cn;
        moved = true;
      }
    }
  });
  return moved;
}
// the node's Requested of the preemptor's extended resources, in its scratch row (nullptr: none)
__device__ __forceinline__ int64_t* preempt_sreq(const MirrorView& m, const uint8_t* base, const PodDesc& d,
                                                 const PreemptIn& in, int i) {
  if (!in.sreq || d.n_scalar == 0) return nullptr;
  int64_t* row = in.sreq + (size_t)i * (size_t)d.n_scalar;
  const ScalarReq* sr = at<ScalarReq>(base, d.scalar_off);
  for (int k = 0; k < d.n_scalar; ++k) row[k] = m.scalar_req[(size_t)sr[k].slot * (size_t)m.cap + (size_t)i];
  return row;
}

// Host-staged victims (PNode / PVictim: the host sorted them and grouped them by PDB violation)
template <class S>
__global__ __launch_bounds__(kBlock) void k_preempt(MirrorView m, BatchView b, int pod, const PNode* pn,
                                                    const PVictim* pv, uint8_t* vout, POut* out, int all_nodes,
                                                    PreemptIn in) {
  const int i = (int)blockIdx.x * kBlock + (int)threadIdx.x;
  if (i >= m.n) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  POut o{PS_NOT_CHECKED, 0, 0, 0};
  const uint32_t st0 = b.status[i];
  const PNode nd = pn[i];
  if (!all_nodes && status_code(st0) != C_UNSCHED) {
    out[i] = o;
    return;
  }
  if (nd.vcnt == 0) {  // "No preemption victims found for incoming pod" (:291-294)
    o.st = PS_NO_VICTIMS;
    out[i] = o;
    return;
  }
  // a status from a filter that reads no pod (or a PreFilter rejection) holds with the victims removed too
  const uint32_t p0 = status_plugin(st0);
  if (st0 != 0 && (p0 == P_UNSCHED || p0 == P_NODENAME || p0 == P_TAINT || p0 == P_NA || p0 == 15u)) {
    o.st = st0;
    out[i] = o;
    return;
  }
  NodeCore nc = load_core(m, i);
  int64_t* sreq = preempt_sreq(m, base, d, in, i);
  const int ns = d.n_scalar;
  TopoTrack<S> T;
  topo_track_init(m, b, pod, base, d, i, in, T, &o.flags);
  const PVictim* v = pv + nd.voff;
  bool moves = false;  // some victim moves a topology count: the topology filters re-run on every reprieve
  for (int q = 0; q < nd.vcnt; ++q) {  // removePod of every potential victim (:285-289)
    nc.rcpu -= v[q].cpu;
    nc.rmem -= v[q].mem;
    nc.reph -= v[q].eph;
    if (sreq)
      for (int k = 0; k < ns; ++k) sreq[k] -= in.vsc[(size_t)v[q].slot * ns + k];
    moves |= topo_victim(m, base, d, in, T, v[q].slot, -1);
  }
  nc.npods -= nd.vcnt;
  bool port = (nd.flags & PN_BASE_PORT) != 0;
  uint32_t st = preempt_node_filters(m, nc, sreq, nullptr, base, d, i, port);
  if (st == 0) st = topo_filters(m, base, d, i, T.tp, 0);
  o.st = st;
  if (st == 0) {
    for (int q = 0; q < nd.vcnt; ++q) {  // reprieve in the host's order (:331-343)
      const PVictim x = v[q];
      NodeCore t = nc;
      t.rcpu += x.cpu;
      t.rmem += x.mem;
      t.reph += x.eph;
      t.npods += 1;
      const int64_t* add = sreq ? in.vsc + (size_t)x.slot * ns : nullptr;
      const bool tpo = port || (x.flags & PV_PORT) != 0;
      // tried back: the counts move now and move back if the preemptor no longer fits
      const bool mv = moves && topo_victim(m, base, d, in, T, x.slot, +1);
      bool fits = preempt_node_filters(m, t, sreq, add, base, d, i, tpo) == 0;
      if (fits && mv) fits = topo_filters(m, base, d, i, T.tp, 0) == 0;
      if (fits) {
        nc = t;
        if (sreq)
          for (int k = 0; k < ns; ++k) sreq[k] += add[k];
        port = tpo;
        vout[nd.voff + q] = 0;
      } else {
        if (mv) topo_victim(m, base, d, in, T, x.slot, -1);
        vout[nd.voff + q] = 1;
        o.nvictims += 1;
        o.nviolating += (x.flags & PV_VIOL) ? 1 : 0;
      }
    }
  }
  out[i] = o;
}

hipError_t launch_preempt(const MirrorView& m, const BatchView& b, int pod, const PNode* pn, const PVictim* pv,
                          uint8_t* vout, POut* out, int all_nodes, const PreemptIn& in, hipStream_t s) {
  const int nb = (m.n + kBlock - 1) / kBlock;
  if (nb == 0) return hipSuccess;
  if (in.wide)
    hipLaunchKernelGGL(k_preempt<PreemptWide>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, pn, pv, vout, out, all_nodes, in);
  else
    hipLaunchKernelGGL(k_preempt<PreemptRegs>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, pn, pv, vout, out, all_nodes, in);
  return hipGetLastError();
}

// k_preempt_seg: k_preempt over the device-resident pod segments (PreemptView).  The filter re-runs and
// the reprieve are k_preempt's; what the host staged per call there is derived here: the potential
// victims (the segment suffix below the preemptor's priority), filterPodsWithPDBViolation
// (default_preemption.go:406-452: selector programs against the pod table's labels, budgets in
// registers), the victims' host-port conflicts and the node's remaining conflicting ports.
template <class S>
__global__ __launch_bounds__(kBlock) void k_preempt_seg(MirrorView m, BatchView b, int pod, PreemptView pv) {
  const int i = (int)blockIdx.x * kBlock + (int)threadIdx.x;
  if (i >= m.n) return;
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PSegOut o{};
  o.st = PS_NOT_CHECKED;
  const uint32_t st0 = b.status[i];
  if (!pv.all_nodes && status_code(st0) != C_UNSCHED) {
    pv.out[i] = o;
    return;
  }
  const int cnt = pv.cnt[i];
  const PRec* r = pv.seg + (size_t)i * kSegCap;
  int first = cnt;
  for (int q = 0; q < cnt; ++q)
    if (r[q].prio < pv.prio) {
      first = q;
      break;
    }
  if (first == cnt) {  // "No preemption victims found for incoming pod"
    o.st = PS_NO_VICTIMS;
    pv.out[i] = o;
    return;
  }
  const uint32_t p0 = status_plugin(st0);
  if (st0 != 0 && (p0 == P_UNSCHED || p0 == P_NODENAME || p0 == P_TAINT || p0 == P_NA || p0 == 15u)) {
    o.st = st0;
    pv.out[i] = o;
    return;
  }
  const PreemptIn& in = pv.in;
  TopoTrack<S> T;
  topo_track_init(m, b, pod, base, d, i, in, T, &o.flags);
  const int ns = d.n_scalar;
  // filterPodsWithPDBViolation over the importance-ordered potential victims
  unsigned long long viol0 = 0ull, viol1 = 0ull;  // two words, no dynamically indexed array (scratch)
  if (pv.npdb > 0) {
    int32_t allowed[kMaxPdb];
#pragma unroll
    for (int k = 0; k < kMaxPdb; ++k) allowed[k] = k < pv.npdb ? pv.pdb[k].allowed : 0;
    for (int q = first; q < cnt; ++q) {
      const int32_t slot = r[q].slot;
      const int32_t ln = (int32_t)m.pod_lbl_cnt[slot];
      if (ln == 0) continue;  // a pod with no labels matches no PDB
      const unsigned long long* lb = m.lbl_pool + m.pod_lbl_off[slot];
      const int32_t pns = m.pod_ns[slot];
      const uint32_t dis = pv.disrupted ? pv.disrupted[slot] : 0u;
      bool v = false;
#pragma unroll
      for (int k = 0; k < kMaxPdb; ++k) {
        if (k >= pv.npdb) break;
        const PdbDev pb = pv.pdb[k];
        if (!pb.ok || pb.ns != pns || !lsel_match(pv.pdb_pool + pb.sel, lb, ln) || ((dis >> k) & 1u)) continue;
        if (--allowed[k] < 0) v = true;
      }
      if (v) (q < 64 ? viol0 : viol1) |= 1ull << (q & 63);
    }
  }
  const bool ports_on = ((d.filter_mask >> P_PORTS) & 1u) != 0;
  auto conf = [&](uint32_t pid) {
    return ports_on && pid != 0xffffffffu && bit(base, d.port_conflict_off, pid, d.n_port_words);
  };
  bool port = false;  // a conflicting port no potential victim holds (NodeInfo.RemovePod drops shared ones too)
  if (ports_on)
    for (int s = 0; s < m.port_slots; ++s) {
      const uint32_t pid = m.ports[(size_t)i * m.port_slots + s];
      if (!conf(pid)) continue;
      bool held = false;
      for (int q = first; q < cnt; ++q) held |= r[q].port[0] == pid || r[q].port[1] == pid;
      port |= !held;
    }
  NodeCore nc = load_core(m, i);
  int64_t* sreq = preempt_sreq(m, base, d, in, i);
  auto vsc = [&](const PRec& x) -> const int64_t* {  // the victim's request of the preemptor's scalars
    return sreq && (x.flags & PR_SCALAR) ? in.vsc + (size_t)x.slot * ns : nullptr;
  };
  bool moves = false;  // some victim moves a topology count: the topology filters re-run on every reprieve
  for (int q = first; q < cnt; ++q) {
    nc.rcpu -= r[q].cpu;
    nc.rmem -= r[q].mem;
    nc.reph -= r[q].eph;
    if (const int64_t* a = vsc(r[q]))
      for (int k = 0; k < ns; ++k) sreq[k] -= a[k];
    moves |= topo_victim(m, base, d, in, T, r[q].slot, -1);
  }
  nc.npods -= cnt - first;
  uint32_t st = preempt_node_filters(m, nc, sreq, nullptr, base, d, i, port);
  if (st == 0) st = topo_filters(m, base, d, i, T.tp, 0);
  o.st = st;
  unsigned long long vm0 = 0ull, vm1 = 0ull, vv0 = 0ull, vv1 = 0ull;
  if (st == 0) {
    for (int pass = 0; pass < 2; ++pass)  // the violating group first, then the others (:331-343)
      for (int q = first; q < cnt; ++q) {
        const bool isv = (((q < 64 ? viol0 : viol1) >> (q & 63)) & 1ull) != 0;
        if (isv != (pass == 0)) continue;
        const PRec x = r[q];
        NodeCore t = nc;
        t.rcpu += x.cpu;
        t.rmem += x.mem;
        t.reph += x.eph;
        t.npods += 1;
        const int64_t* add = vsc(x);
        const bool tpo = port || conf(x.port[0]) || conf(x.port[1]);
        const bool mv = moves && topo_victim(m, base, d, in, T, x.slot, +1);
        bool fits = preempt_node_filters(m, t, sreq, add, base, d, i, tpo) == 0;
        if (fits && mv) fits = topo_filters(m, base, d, i, T.tp, 0) == 0;
        if (fits) {
          nc = t;
          if (add)
            for (int kk = 0; kk < ns; ++kk) sreq[kk] += add[kk];
          port = tpo;
        } else {
          if (mv) topo_victim(m, base, d, in, T, x.slot, -1);
          (q < 64 ? vm0 : vm1) |= 1ull << (q & 63);
          o.nvictims += 1;
          if (isv) {
            (q < 64 ? vv0 : vv1) |= 1ull << (q & 63);
            o.nviolating += 1;
          }
        }
      }
  }
  o.vmask[0] = vm0;
  o.vmask[1] = vm1;
  o.violmask[0] = vv0;
  o.violmask[1] = vv1;
  // the selection criteria: the victims' most important member leads either victim order (importance
  // order, or reprieve order within one PDB group, both led by the segment's earliest victim)
  o.hiprio = INT32_MIN;
  o.sumprio = 0;
  o.earliest = INT64_MAX;
  for (int q = first; q < cnt; ++q) {
    if (!((((q < 64 ? vm0 : vm1) >> (q & 63)) & 1ull))) continue;
    const int64_t t = r[q].start == INT64_MAX ? pv.now : r[q].start;
    if (o.hiprio == INT32_MIN || r[q].prio > o.hiprio) {
      o.hiprio = r[q].prio;
      o.earliest = t;
    } else if (r[q].prio == o.hiprio && t < o.earliest) {
      o.earliest = t;
    }
    o.sumprio += (int64_t)r[q].prio + 2147483648LL;
  }
  pv.out[i] = o;
}

// DryRunPreemption's candidate cut with sequential Parallelizer semantics (preemption.go:404-457) and
// SelectCandidate / pickOneNodeForPreemption (:262-397) over k_preempt_seg's per-node results, in one
// workgroup: the potential nodes (snapshot order) are ranked by a block scan, walked from the offset in
// rotated order with running non-violating / violating candidate counts (each list capped at
// numCandidates, candidateList.add), cut where a non-violating candidate is held and the two reach
// numCandidates, and the candidates reduced by the five criteria (ties: earliest in candidate order,
// non-violating list first).
constexpr int kPickThreads = 1024;
__device__ __forceinline__ int block_excl_scan(int v, int* tot, int* s_w) {  // kPickThreads, returns exclusive prefix
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int k = 0; k < kPickThreads / 64; ++k) {
      const int t = s_w[k];
      s_w[k] = acc;
      acc += t;
    }
    s_w[kPickThreads / 64] = acc;
  }
  __syncthreads();
  const int r = s_w[w] + x - v;
  *tot = s_w[kPickThreads / 64];
  __syncthreads();
  return r;
}
struct PickKey {  // larger is better, lexicographic
  int64_t a, b, c, d, e;
  int32_t idx;  // candidate-order index (smaller wins a full tie)
  int32_t node;
};
__device__ __forceinline__ bool pick_better(const PickKey& x, const PickKey& y) {
  if (x.node < 0) return false;
  if (y.node < 0) return true;
  if (x.a != y.a) return x.a > y.a;
  if (x.b != y.b) return x.b > y.b;
  if (x.c != y.c) return x.c > y.c;
  if (x.d != y.d) return x.d > y.d;
  if (x.e != y.e) return x.e > y.e;
  return x.idx < y.idx;
}
__global__ __launch_bounds__(kPickThreads) void k_preempt_pick(const PSegOut* out, int n, int64_t offset_in, int64_t pct,
                                                               int64_t absn, int32_t* pot, PickOut* res) {
  __shared__ int s_w[kPickThreads / 64 + 1];
  __shared__ int s_cut, s_unsup;
  __shared__ PickKey s_k[kPickThreads];
  const int t = threadIdx.x;
  if (t == 0) s_unsup = 0;
  __syncthreads();
  // potential ranks (snapshot order) -> pot[rank] = node
  int P = 0;
  for (int b0 = 0; b0 < n; b0 += kPickThreads) {
    const int i = b0 + t;
    const int f = (i < n && out[i].st != PS_NOT_CHECKED) ? 1 : 0;
    int tot;
    const int r = block_excl_scan(f, &tot, s_w);
    if (f) pot[P + r] = i;
    P += tot;
  }
  __syncthreads();
  if (P == 0) {
    if (t == 0) {
      res->potential = res->ncand = res->ncandidates = 0;
      res->best = -1;
      res->offset = 0;
      res->unsupported = s_unsup;
    }
    return;
  }
  const int offset = (int)(((offset_in % P) + P) % P);
  int64_t nc = (int64_t)P * pct / 100;
  if (nc < absn) nc = absn;
  if (nc > P) nc = P;
  const int ncand = (int)nc;
  // one pass in rotated order: running non-violating / violating counts (block scans), the cut -- the first
  // position whose candidate brings min(NV, nc) >= 1 and min(NV, nc) + min(VV, nc) >= nc -- and every
  // thread's best candidate up to it.  Candidate order: the non-violating list, then the violating one,
  // each in rotated order (the tie-break index needs no list sizes: class in the high bits).
  auto cls = [&](int j) {  // 1: non-violating candidate, 2: violating candidate, 0: neither
    const PSegOut& o = out[pot[(offset + j) % P]];
    if (o.st != 0 || o.nvictims == 0) return 0;
    return o.nviolating == 0 ? 1 : 2;
  };
  __shared__ int s_nvc, s_vvc;
  if (t == 0) {
    s_cut = INT32_MAX;
    s_nvc = s_vvc = 0;
  }
  __syncthreads();
  PickKey best{0, 0, 0, 0, 0, 0, -1};
  int NV = 0, VV = 0;
  for (int b0 = 0; b0 < P; b0 += kPickThreads) {
    const int j = b0 + t;
    const int c = j < P ? cls(j) : 0;
    int tn, tv;
    const int en = block_excl_scan(c == 1 ? 1 : 0, &tn, s_w);
    const int ev = block_excl_scan(c == 2 ? 1 : 0, &tv, s_w);
    const int nvi = NV + en + (c == 1 ? 1 : 0), vvi = VV + ev + (c == 2 ? 1 : 0);  // inclusive counts
    const int64_t nvc = nvi < nc ? nvi : nc, vvc = vvi < nc ? vvi : nc;
    if (c != 0 && nvc >= 1 && nvc + vvc >= nc) atomicMin(&s_cut, j);
    __syncthreads();
    const int cut = s_cut;
    // a node whose result the device could not compute (PSegOut flag bit 0) matters only if the dry
    // run reaches it: a potential node at or before the cut (DryRunPreemption stops there)
    if (j < P && j <= cut && (out[pot[(offset + j) % P]].flags & 1u)) s_unsup = 1;
    if (c != 0 && j <= cut) {
      int idx = -1;
      if (c == 1 && nvi - 1 < ncand) idx = nvi - 1;
      if (c == 2 && vvi - 1 < ncand) idx = (1 << 24) + vvi - 1;
      if (idx >= 0) {
        const int node = pot[(offset + j) % P];
        const PSegOut& o = out[node];
        PickKey k{-(int64_t)o.nviolating, -(int64_t)o.hiprio, -o.sumprio, -(int64_t)o.nvictims, o.earliest, idx, node};
        if (pick_better(k, best)) best = k;
      }
    }
    if (j == cut) {
      s_nvc = (int)nvc;
      s_vvc = (int)vvc;
    }
    NV += tn;
    VV += tv;
    if (cut != INT32_MAX) break;  // uniform: every lane read the shared value after the barrier
  }
  __syncthreads();
  if (s_cut == INT32_MAX && t == 0) {  // no cut: every potential node was checked
    s_nvc = NV < ncand ? NV : ncand;
    s_vvc = VV < ncand ? VV : ncand;
  }
  __syncthreads();
  const int nvtot = s_nvc, vvtot = s_vvc;
  s_k[t] = best;
  __syncthreads();
  for (int w = kPickThreads / 2; w > 0; w >>= 1) {
    if (t < w && pick_better(s_k[t + w], s_k[t])) s_k[t] = s_k[t + w];
    __syncthreads();
  }
  if (t == 0) {
    res->potential = P;
    res->ncand = ncand;
    res->ncandidates = nvtot + vvtot;
    res->best = s_k[0].node;
    res->offset = offset;
    res->unsupported = s_unsup;
    if (s_k[0].node >= 0) res->best_out = out[s_k[0].node];
  }
}

hipError_t launch_preempt_pick(const PSegOut* out, int n, int64_t offset, int64_t pct, int64_t absn, int32_t* pot,
                               PickOut* res, hipStream_t s) {
  hipLaunchKernelGGL(k_preempt_pick, dim3(1), dim3(kPickThreads), 0, s, out, n, offset, pct, absn, pot, res);
  return hipGetLastError();
}

hipError_t launch_preempt_seg(const MirrorView& m, const BatchView& b, int pod, const PreemptView& pv, hipStream_t s) {
  const int nb = (m.n + kBlock - 1) / kBlock;
  if (nb == 0) return hipSuccess;
  if (pv.in.wide)
    hipLaunchKernelGGL(k_preempt_seg<PreemptWide>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, pv);
  else
    hipLaunchKernelGGL(k_preempt_seg<PreemptRegs>, dim3(nb), dim3(kBlock), 0, s, m, b, pod, pv);
  return hipGetLastError();
}


// Evaluation output of a node-sharded context: each rank scatters the per-node vectors of its own block
// range into a zeroed full-length buffer, which an all-reduce (MAX) over the ranks then completes on
// every rank -- statuses and the weighted normalised scores are all non-negative, so 0 is the identity.
// Layout: [n] status | [kNumPlugins][n] plugin scores | [n] TotalScore.
__global__ __launch_bounds__(kBlock) void k_eval_pack(BatchView b, int n, int cap, int lo, int hi,
                                                      unsigned long long* g) {
  const int i = lo + (int)blockIdx.x * kBlock + (int)threadIdx.x;
  if (i >= hi || i >= n) return;
  g[i] = b.status[i];
#pragma unroll
  for (int q = 0; q < kNumPlugins; ++q) g[(size_t)(1 + q) * n + i] = (unsigned long long)b.out_scores[(size_t)q * cap + i];
  g[(size_t)(1 + kNumPlugins) * n + i] = (unsigned long long)b.out_total[i];
}
hipError_t launch_eval_pack(const BatchView& b, int n, int cap, int lo, int hi, unsigned long long* g, hipStream_t s) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_eval_pack, dim3((hi - lo + kBlock - 1) / kBlock), dim3(kBlock), 0, s, b, n, cap, lo, hi, g);
  return hipGetLastError();
}

}  // namespace ksg
