// aggregate.hip -- PodTopologySpread / InterPodAffinity per-domain counts on gfx950.
//
// k_aggregate runs once per pod before the node pass when the pod (or the cluster) has spread
// constraints or affinity terms.  One launch, three block roles:
//   node blocks  : domain presence per DoNotSchedule constraint -- the keys of
//                  TpValueToMatchNum (podtopologyspread/filtering.go:255-311)
//   pod blocks   : one thread per pod-table slot; the incoming pod's selectors against every
//                  existing pod: countPodsMatchSelector for PTS (common.go:145-160), the incoming
//                  pod's required / preferred (anti-)affinity terms (interpodaffinity/
//                  filtering.go:246-283, scoring.go:98-110)
//   term blocks  : one thread per existing affinity term against the incoming pod
//                  (existing anti-affinity, filtering.go:216-240; hard/soft symmetric weights,
//                  scoring.go:112-124)
// Counts land in an int64 arena indexed by (histogram base + topology value id).  Small arenas
// are staged in LDS (one LDS atomic per update, one global atomic per touched entry per
// block); the last block to arrive reduces each constraint's critical-path minimum.
// k_pts_score then evaluates PodTopologySpread.Score for the feasible nodes (scoring.go:199-226).
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace ksg {

constexpr int kLdsArena = 2048;  // int64 entries staged in LDS (16 KiB)


__global__ __launch_bounds__(kBlock) void k_aggregate(MirrorView m, BatchView b, int pod, int nb_node, int nb_pod,
                                                        int nb_term) {
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const int blk = blockIdx.x, tid = threadIdx.x;
  const int32_t* sp = at<int32_t>(base, d.sel_pool_off);
  const bool lds = d.arena_words <= kLdsArena;
  __shared__ unsigned long long s_arena[kLdsArena];
  __shared__ uint32_t s_any;
  if (lds)
    for (int w = tid; w < d.arena_words; w += kBlock) s_arena[w] = 0ull;
  if (tid == 0) s_any = 0;
  __syncthreads();
  auto add = [&](int32_t idx, long long v) {
    if (lds) atomicAdd(&s_arena[idx], (unsigned long long)v);
    else atomicAdd(&b.arena[idx], (unsigned long long)v);
  };

  if (blk < nb_node) {
    // ---- node role: domain presence (an entry exists even with zero matching pods)
    const int i = blk * kBlock + tid;
    if (i < m.n && d.n_ptsf) {
      const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
      const uint32_t el = pts_eligible(m, base, d, cs, d.n_ptsf, i);
      for (int32_t c = 0; c < d.n_ptsf; ++c) {
        const bool on = ((el >> c) & 1u) != 0;
        mark_domains(b.arena + cs[c].pres_base, on ? node_label(m, cs[c].slot, i) : 0, on, &ps->pts_ndom[c]);
      }
    }
  } else if (blk < nb_node + nb_pod) {
    // ---- pod role
    const int s = (blk - nb_node) * kBlock + tid;
    const int n = s < m.pods_hw ? m.pod_node[s] : -1;
    if (n >= 0) {
      const int32_t pns = m.pod_ns[s];
      const bool term = (m.pod_flags[s] & 1u) != 0;
      const unsigned long long* pl = m.lbl_pool + m.pod_lbl_off[s];
      const int32_t pn = (int32_t)m.pod_lbl_cnt[s];
      if (!term && pns == d.ns_id) {
        if (d.n_ptsf) {  // calPreFilterState counts (filtering.go:255-300)
          const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
          const uint32_t el = pts_eligible(m, base, d, cs, d.n_ptsf, n);
          for (int32_t c = 0; c < d.n_ptsf; ++c)
            if (((el >> c) & 1u) && !lsel_empty(sp + cs[c].sel) && lsel_match(sp + cs[c].sel, pl, pn))
              add(cs[c].hist_base + node_label(m, cs[c].slot, n), 1);
        }
        if (d.n_ptss) {  // processAllNode (scoring.go:155-189) + per-node hostname counts (:207-214)
          const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
          const uint32_t el = pts_eligible(m, base, d, cs, d.n_ptss, n, (d.flags & DF_PTS_ANYTOPO) == 0);
          for (int32_t c = 0; c < d.n_ptss; ++c) {
            if (lsel_empty(sp + cs[c].sel) || !lsel_match(sp + cs[c].sel, pl, pn)) continue;
            if (cs[c].hostname) add(cs[c].hist_base + n, 1);
            else if ((el >> c) & 1u) add(cs[c].hist_base + pts_domain(m, cs[c], n), 1);
          }
        }
      }
      uint32_t any = 0;
      if (d.n_raff) {  // affinityCounts: existing pods matching ALL required affinity terms (filtering.go:256-266)
        const IpaTerm* ts = at<IpaTerm>(base, d.raff_off);
        bool all = true;
        for (int32_t k = 0; k < d.n_raff; ++k) all = all && term_matches_pod(sp, ts[k], pns, pl, pn);
        if (all)
          for (int32_t k = 0; k < d.n_raff; ++k) {
            const int32_t v = node_label(m, ts[k].slot, n);
            if (v >= 0) {
              add(ts[k].hist_base + v, 1);
              any |= 1u;
            }
          }
      }
      if (d.n_ranti) {  // antiAffinityCounts (filtering.go:268-276)
        const IpaTerm* ts = at<IpaTerm>(base, d.ranti_off);
        for (int32_t k = 0; k < d.n_ranti; ++k)
          if (term_matches_pod(sp, ts[k], pns, pl, pn)) {
            const int32_t v = node_label(m, ts[k].slot, n);
            if (v >= 0) {
              add(ts[k].hist_base + v, 1);
              any |= 2u;
            }
          }
      }
      if (d.ipa_flags & IPA_PREF) {  // the incoming pod's soft terms (scoring.go:98-110)
        const IpaTerm* ta = at<IpaTerm>(base, d.paff_off);
        for (int32_t k = 0; k < d.n_paff; ++k)
          if (term_matches_pod(sp, ta[k], pns, pl, pn)) {
            const int32_t v = node_label(m, ta[k].slot, n);
            if (v >= 0) {
              add(ta[k].hist_base + v, ta[k].weight);
              any |= 8u;
            }
          }
        const IpaTerm* tn = at<IpaTerm>(base, d.panti_off);
        for (int32_t k = 0; k < d.n_panti; ++k)
          if (term_matches_pod(sp, tn[k], pns, pl, pn)) {
            const int32_t v = node_label(m, tn[k].slot, n);
            if (v >= 0) {
              add(tn[k].hist_base + v, -(long long)tn[k].weight);
              any |= 8u;
            }
          }
      }
      if (any) atomicOr(&s_any, any);
    }
  } else {
    // ---- term role: existing pods' terms against the incoming pod
    const int j = (blk - nb_node - nb_pod) * kBlock + tid;
    if (j < m.n_terms) {
      const DTerm t = m.terms[j];
      const int n = t.kind >= 0 ? m.pod_node[t.owner] : -1;
      if (n >= 0 && t.key < d.n_keytab) {
        const int32_t* kt = at<int32_t>(base, d.keytab_off) + (size_t)t.key * kKeytabStride;
        const bool anti = t.kind == T_REQ_ANTI;
        const int32_t hb = anti ? ((d.ipa_flags & IPA_EXIST_FILTER) ? kt[1] : -1)
                                : ((d.ipa_flags & IPA_EXIST_SCORE) ? kt[2] : -1);
        long long w = 0;
        if (t.kind == T_REQ_AFF) w = d.hard_weight;  // HardPodAffinityWeight (scoring.go:112-117)
        else if (t.kind == T_PREF_AFF) w = t.weight;
        else if (t.kind == T_PREF_ANTI) w = -(long long)t.weight;
        else w = 1;
        if (hb >= 0 && w != 0) {
          const int32_t* tp = m.term_pool;
          const unsigned long long* il = at<unsigned long long>(base, d.lbl_off);
          const unsigned long long* nl = at<unsigned long long>(base, d.nslbl_off);
          // AffinityTerm.Matches(incoming pod, namespace labels) (types.go:391-396)
          const bool match = (id_in(tp + t.ns_off, t.ns_cnt, d.ns_id) || lsel_match(tp + t.nssel, nl, d.n_nslbl)) &&
                             lsel_match(tp + t.sel, il, d.n_lbl);
          const int32_t v = match ? node_label(m, kt[0], n) : -1;
          if (v >= 0) {
            add(hb + v, w);
            atomicOr(&s_any, anti ? 4u : 8u);
          }
        }
      }
    }
  }

  // ---- flush the LDS histogram + flags, then the arrival ticket
  __syncthreads();
  if (lds)
    for (int w = tid; w < d.arena_words; w += kBlock)
      if (s_arena[w]) atomicAdd(&b.arena[w], s_arena[w]);
  if (tid == 0 && s_any) atomicOr(&ps->ipa_any, s_any);
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's atomics performed before the ticket
  __syncthreads();
  if (tid == 0) {
    // every count/flag this block published is an agent-scope atomic: wait for them to be
    // performed, then take the ticket (no L2 write-back fence; the last block reads the arena
    // with agent-scope atomic loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = __hip_atomic_fetch_add(&ps->done_agg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == (uint32_t)(nb_node + nb_pod + nb_term) - 1u) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last || d.n_ptsf == 0) return;
  // critical-path minimum over the present domains of each DoNotSchedule constraint
  // (criticalPaths, filtering.go:64-110; minMatchNum :111-124)
  const PtsCons* cs = at<PtsCons>(base, d.ptsf_off);
  __shared__ long long s_min[kBlock / 64];
  for (int32_t c = 0; c < d.n_ptsf; ++c) {
    long long mn = 0x7fffffffffffffffll;
    for (int v = tid; v < cs[c].nvals; v += kBlock) {
      const unsigned long long pres = __hip_atomic_load(b.arena + cs[c].pres_base + v, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
      if (pres) {
        const long long x = (long long)__hip_atomic_load(b.arena + cs[c].hist_base + v, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        mn = x < mn ? x : mn;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const long long y = __shfl_xor(mn, o, 64);
      mn = y < mn ? y : mn;
    }
    if ((tid & 63) == 0) s_min[tid >> 6] = mn;
    __syncthreads();
    if (tid == 0) {
      long long r = s_min[0];
      for (int w = 1; w < kBlock / 64; ++w) r = s_min[w] < r ? s_min[w] : r;
      ps->pts_min[c] = r;
    }
    __syncthreads();
  }
}

// PodTopologySpread.Score for every feasible node (podtopologyspread/scoring.go:199-226): raw = round(
// sum_c cnt_c * log(topoSize_c + 2) + (maxSkew_c - 1)), -1 for ignored nodes; min/max for NormalizeScore.
__global__ __launch_bounds__(kBlock) void k_pts_score(MirrorView m, BatchView b, int pod, int blk0) {
  {  // OpportunisticBatching: placed by k_ob_hint, no scores (kernels.hip ob_skip)
    const PodDesc* pd = reinterpret_cast<const PodDesc*>(b.descs + b.desc_off[pod]);
    if ((pd->flags & DF_EARLY) && b.stats[pod].ob_done) return;
  }
  const uint8_t* base = b.descs + b.desc_off[pod];
  const PodDesc& d = *reinterpret_cast<const PodDesc*>(base);
  PodStats* ps = b.stats + pod;
  const int blk = blk0 + (int)blockIdx.x;
  const int i = blk * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t cap = (size_t)m.cap;
  bool scored = false;
  int64_t raw = 0;
  if (i < m.n && ((b.fmask[(size_t)blk * (kBlock / 64) + wave] >> lane) & 1ull)) {
    const PtsCons* cs = at<PtsCons>(base, d.ptss_off);
    if (pts_ignored(m, d, cs, i)) {
      raw = -1;
    } else {
      double score = 0.0;
      for (int32_t c = 0; c < d.n_ptss; ++c) {
        const int32_t v = node_label(m, cs[c].slot, i);
        if (v < 0) continue;  // only keys the node carries score (scoring.go:213-222)
        long long cnt;
        int32_t sz;
        if (cs[c].hostname) {
          cnt = (long long)b.arena[cs[c].hist_base + i];
          sz = (int32_t)ps->pts_nonignored;  // len(filteredNodes) - len(IgnoredNodes)
        } else {
          cnt = (long long)b.arena[cs[c].hist_base + v];
          sz = (int32_t)ps->pts_distinct[c];
        }
        const double w = m.log_tab[sz + 2];  // topologyNormalizingWeight (scoring.go:293-299)
        const double prod = (double)cnt * w;
        const double term = prod + (double)(cs[c].max_skew - 1);
        score = score + term;
      }
      raw = (int64_t)round(score);  // math.Round: half away from zero
      scored = true;
    }
    b.raw[P_PTS * cap + i] = raw;
  }
  unsigned long long mx = scored ? enc_i64(raw) : 0ull, mn = scored ? enc_i64(raw) : ~0ull;
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mx, o, 64), c = __shfl_xor(mn, o, 64);
    mx = a > mx ? a : mx;
    mn = c < mn ? c : mn;
  }
  __shared__ unsigned long long s_mx[kBlock / 64], s_mn[kBlock / 64];
  if (lane == 0) {
    s_mx[wave] = mx;
    s_mn[wave] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) {
      mx = s_mx[w] > mx ? s_mx[w] : mx;
      mn = s_mn[w] < mn ? s_mn[w] : mn;
    }
    mx = s_mx[0] > mx ? s_mx[0] : mx;
    mn = s_mn[0] < mn ? s_mn[0] : mn;
    if (mn != ~0ull) {
      atomicMax(&ps->max_raw[P_PTS], mx);
      atomicMin(&ps->min_raw[P_PTS], mn);
    }
  }
}

hipError_t launch_aggregate(const MirrorView& m, const BatchView& b, int pod, const PodDesc& d, hipStream_t s) {
  const int nb_node = d.n_ptsf ? (m.n + kBlock - 1) / kBlock : 0;
  const bool pod_work = d.n_ptsf || d.n_ptss || d.n_raff || d.n_ranti || (d.ipa_flags & IPA_PREF);
  const int nb_pod = pod_work ? (m.pods_hw + kBlock - 1) / kBlock : 0;
  const bool term_work = (d.ipa_flags & (IPA_EXIST_FILTER | IPA_EXIST_SCORE)) != 0;
  const int nb_term = term_work ? (m.n_terms + kBlock - 1) / kBlock : 0;
  int total = nb_node + nb_pod + nb_term;
  if (total == 0) total = 1;  // still run the ticket/critical-path epilogue
  hipLaunchKernelGGL(k_aggregate, dim3(total), dim3(kBlock), 0, s, m, b, pod, nb_node, nb_pod,
                     total - nb_node - nb_pod);
  return hipGetLastError();
}

hipError_t warm_aggregate() {
  hipFuncAttributes a;
  hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_aggregate));
  if (e == hipSuccess) e = hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_pts_score));
  return e;
}

hipError_t launch_pts_score(const MirrorView& m, const BatchView& b, int pod, hipStream_t s, int blk0, int nblk) {
  if (nblk < 0) nblk = (m.n + kBlock - 1) / kBlock;
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pts_score, dim3(nblk), dim3(kBlock), 0, s, m, b, pod, blk0);
  return hipGetLastError();
}

}  // namespace ksg
