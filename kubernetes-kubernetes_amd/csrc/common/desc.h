// desc.h -- device-visible data layout shared by the host library and the HIP kernels.
//
// Two kinds of data live in HBM:
//  * the node mirror: a structure-of-arrays copy of the scheduler snapshot's NodeInfo
//    fields the node-local plugins read (framework/types.go:172-220), indexed by
//    snapshot position (nodeTree order, backend/cache/node_tree.go:119-143);
//  * per-pod "programs": a PodDesc header followed by a byte blob of compiled
//    selectors / bitmaps / resource vectors, produced once per pod on the host
//    (the work upstream does in PreFilter/PreScore) and consumed by every node thread.
// Plain C++ PODs only -- this header is included by .cpp (g++/hipcc host) and .hip files.
#pragma once
#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC__)
#define KSG_HD __host__ __device__
#else
#define KSG_HD
#endif

namespace ksg {

constexpr int kNumPlugins = 10;  // KSG_NUM_PLUGINS
constexpr int kBlock = 256;      // threads per block of the per-node kernels (4 waves)
constexpr int kMaxScalar = 16;   // interned extended/scalar resource columns
constexpr int kPortSlots = 8;    // used-port slots per node (grown by the host if exceeded)

// ---- selector programs (labels.Selector / nodeaffinity terms compiled to slots) ----------
enum SelOp : int32_t {
  SEL_IN = 0,        // node value id in vals
  SEL_NOTIN = 1,     // absent or value not in vals
  SEL_EXISTS = 2,
  SEL_DNE = 3,       // DoesNotExist
  SEL_GT = 4,        // numeric label > num
  SEL_LT = 5,        // numeric label < num
  SEL_NODE_EQ = 6,   // matchFields metadata.name == node[num]
  SEL_NODE_NE = 7,
  SEL_TRUE = 8,
  SEL_FALSE = 9,
};
struct SelReq {
  int32_t slot;     // label column slot (SEL_IN..SEL_LT)
  int32_t op;
  int32_t nvals;    // SEL_IN / SEL_NOTIN: value ids at vals_off (int32 each)
  int32_t vals_off;
  int64_t num;      // SEL_GT/LT threshold, SEL_NODE_* node index
};
struct SelTerm {   // AND of reqs [req_off, req_off + nreq)
  int32_t req_off;
  int32_t nreq;
  int32_t weight;  // preferred terms
  int32_t parse_err;  // a term with a parse error never matches (nodeaffinity.go:190-193)
};
struct SelProg {   // OR over terms (required) or sum of matching weights (preferred)
  int32_t term_off;
  int32_t nterm;
};

// ---- NodeResourcesFit / BalancedAllocation scoring resources ------------------------------
enum ResKind : int32_t { RES_SKIP = 0, RES_CPU = 1, RES_MEM = 2, RES_EPH = 3, RES_SCALAR = 4 };
struct ScoreRes {
  int32_t kind;     // RES_SKIP: pod requests 0 of a scalar resource (resource_allocation.go:180-182)
  int32_t slot;     // scalar column
  int64_t weight;
  int64_t pod_req;  // calculatePodResourceRequest (resource_allocation.go:236-259)
};
struct ScalarReq {
  int32_t slot;
  int32_t pad;
  int64_t qty;
};
struct ImageTerm {  // one image id the pod references that exists in the cluster
  int32_t image;
  int32_t mult;     // how many of the pod's containers/volumes name it
  int64_t scaled;   // scaledImageScore: int64(float64(size) * numNodes/totalNodes) (image_locality.go:141-148)
};

enum DescFlags : uint32_t {
  DF_TOLERATES_UNSCHED = 1u << 0,  // pod tolerates node.kubernetes.io/unschedulable:NoSchedule
  DF_HAS_SELECTOR = 1u << 1,       // RequiredNodeAffinity.labelSelector (pod.spec.nodeSelector)
  DF_HAS_REQUIRED_NA = 1u << 2,    // RequiredNodeAffinity.nodeSelector
  DF_HAS_ADDED_NA = 1u << 3,       // NodeAffinityArgs.addedAffinity.required
  DF_ALL_FEASIBLE = 1u << 4,       // plugin-eval mode: skip filters, score every node
  DF_EVAL_OUT = 1u << 5,           // write per-node status / per-plugin score vectors
  DF_ASSUME = 1u << 6,             // device-side AssumePod of the winner
  DF_SUBSET = 1u << 7,             // PreFilterResult restricts nodes to the sorted list at subset_off
  DF_NO_SCORE = 1u << 8,           // no score plugin: every TotalScore is 1 (schedule_one.go:948-957)
  DF_PREFILTER_REJECT = 1u << 9,   // PreFilter rejected the pod: every node gets prefilter_code
  DF_HAS_PREF_NA = 1u << 10,       // pod preferred node affinity present
  DF_HAS_ADDED_PREF = 1u << 11,    // NodeAffinityArgs.addedAffinity.preferred present
  DF_SCORE_ERROR = 1u << 12,       // PreScore/Score returns Error: the cycle fails iff scoring runs (F > 1)
  DF_NODE_LIST = 1u << 13,         // plugin-eval mode: only the nodes in the bitmap at node_list_off are listed
};

struct PodDesc {
  uint32_t blob_bytes;   // header + blob, 16-byte multiple
  uint32_t flags;        // DescFlags
  uint32_t filter_mask;  // bit p: Filter of plugin p runs (PreFilter did not Skip)
  uint32_t score_mask;   // bit p: Score of plugin p runs (PreScore did not Skip)
  int32_t node_name;     // NodeName: -1 none, -2 unknown name (never matches), else snapshot index
  int32_t rot_start;     // snapshot index where findNodesThatPassFilters starts (nextStartNodeIndex)
  int32_t prefilter_code;
  int32_t subset_cnt;
  int32_t subset_off;    // int32 node indices, ascending
  int32_t prefilter_plugin;
  int64_t weight[kNumPlugins];
  // NodeResourcesFit filter: preFilterState (fit.go:317-335)
  int64_t req_cpu, req_mem, req_eph;
  int32_t fit_any;       // any of cpu/mem/eph/scalar requested (fit.go:661-666)
  int32_t n_scalar;      // ScalarReq at scalar_off (ignored resources removed)
  int32_t scalar_off;
  int32_t fit_strategy;  // 0 Least 1 Most 2 RequestedToCapacityRatio
  int32_t n_fit_res, fit_res_off;  // ScoreRes
  int32_t n_rtcr, rtcr_off;        // int64 pairs (utilization, score) for the broken-linear shape
  int32_t n_bal_res, bal_res_off;  // ScoreRes (pod_req = Requested, useRequested=true)
  // TaintToleration: bitmaps over distinct taint ids
  int32_t n_taint_words, untol_ns_off, intol_pns_off, node_list_off;
  // NodeAffinity
  SelProg na_required;   // pod required terms (OR)
  SelProg na_selector;   // nodeSelector as a single AND term
  SelProg na_added;      // addedAffinity required terms (OR)
  SelProg na_preferred;  // pod preferred terms (sum of weights)
  SelProg na_added_pref; // addedAffinity preferred terms
  int32_t req_off, vals_off;  // SelReq array / int32 value-id pool (absolute blob offsets)
  // NodePorts: conflict bitmap over distinct port ids
  int32_t n_port_words, port_conflict_off;
  int32_t n_pod_ports, pod_ports_off;  // port ids added to the node on assume
  // ImageLocality
  int32_t n_img, img_off;  // ImageTerm
  int64_t img_count;       // containers + initContainers + image volumes
  // AssumePod payload: PodInfo.CalculateResource (framework/types.go:1035-1076)
  int64_t a_cpu, a_mem, a_eph, a_nz_cpu, a_nz_mem;
  int32_t n_a_scalar, a_scalar_off;  // ScalarReq
};

// Per-pod device result (ScheduleResult + diagnostics), written by the select kernel.
struct DevResult {
  int32_t status;     // KSG_CODE_*
  int32_t node;       // chosen snapshot index or -1
  int32_t feasible;
  int32_t evaluated;
  int64_t total;
  uint64_t key;       // winning packed key (debug)
};

// Per-pod scratch (zeroed by the host before each batch).
struct PodStats {
  unsigned long long best;  // packed (TotalScore, heap pre-order key) max
  unsigned long long max_raw[kNumPlugins];  // enc_i64, init enc_i64(INT64_MIN) for max
  unsigned long long min_raw[kNumPlugins];  // enc_i64, init enc_i64(INT64_MAX) for min
  uint32_t done;            // arrival ticket of the select kernel's blocks
  uint32_t feasible;
  uint32_t pad[2];
};

// Node mirror view passed to kernels by value.
struct MirrorView {
  int32_t n;        // nodes in snapshot order
  int32_t cap;      // column stride
  const int64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int64_t* alloc_eph;
  const int32_t* alloc_pods;
  const uint32_t* flags;          // bit0 unschedulable
  const int64_t* scalar_alloc;    // [kMaxScalar][cap]
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* req_eph;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* num_pods;
  int64_t* scalar_req;            // [kMaxScalar][cap]
  const uint32_t* taint_off;      // [n+1]
  const uint32_t* taint_ids;
  const uint32_t* img_off;        // [n+1]
  const uint32_t* img_ids;        // sorted per node
  const int32_t* labels;          // [slots][cap] local value id, -1 absent
  const int64_t* label_num;       // [slots][cap] parsed integer value
  const uint8_t* label_num_ok;    // [slots][cap]
  uint32_t* ports;                // [cap][kPortSlots] port id, 0xffffffff empty
};

// Everything a per-pod kernel launch needs besides the mirror.
struct BatchView {
  const uint8_t* descs;   // concatenated PodDesc+blob
  const uint32_t* desc_off;  // byte offset of pod i
  PodStats* stats;        // [pods]
  DevResult* results;     // [pods]
  uint32_t* status;       // [cap] per-node packed status of the pod being evaluated
  uint64_t* fmask;        // [cap/64] feasibility bits
  uint32_t* blk_cnt;      // [blocks] feasible nodes per block
  int64_t* fixed;         // [cap] weighted sum of the non-normalised plugin scores
  int64_t* raw;           // [kNumPlugins][cap] raw scores of normalising plugins (+ eval mode: all)
  int64_t* out_scores;    // eval mode: [kNumPlugins][cap] weighted normalised scores
  int64_t* out_total;     // eval mode: [cap]
};

// packed per-node status word: code(4) | plugin(4, 15 = none) | reasons(24)
KSG_HD inline uint32_t pack_status(uint32_t code, uint32_t plugin, uint32_t reasons) {
  return code | (plugin << 4) | (reasons << 8);
}
KSG_HD inline uint32_t status_code(uint32_t s) { return s & 15u; }
KSG_HD inline uint32_t status_plugin(uint32_t s) { return (s >> 4) & 15u; }
KSG_HD inline uint32_t status_reasons(uint32_t s) { return s >> 8; }

// container/heap pre-order key of feasible-list position p (0-based): the heap root
// after heap.Init with a strict ">" Less is, among the maximal TotalScores, the entry
// whose position comes first in pre-order of the implicit binary tree.
// x = p+1 aligned to 24 bits, ties (ancestor vs leftmost descendant) by depth.
constexpr int kPreBits = 29;
KSG_HD inline uint32_t preorder_key(uint32_t p) {
  uint32_t x = p + 1;
  uint32_t len = 32u - (uint32_t)__builtin_clz(x);
  return ((x << (24u - len)) << 5) | len;
}
KSG_HD inline uint32_t preorder_pos(uint32_t key) {  // inverse of preorder_key
  uint32_t len = key & 31u;
  uint32_t x = (key >> 5) >> (24u - len);
  return x - 1;
}
KSG_HD inline unsigned long long pack_best(int64_t total, uint32_t p) {
  return ((unsigned long long)total << kPreBits) | (unsigned long long)((1u << kPreBits) - 1u - preorder_key(p));
}
// order-preserving int64 <-> uint64 (so signed min/max use unsigned atomics)
KSG_HD inline unsigned long long enc_i64(int64_t v) { return (unsigned long long)v ^ 0x8000000000000000ull; }
KSG_HD inline int64_t dec_i64(unsigned long long u) { return (int64_t)(u ^ 0x8000000000000000ull); }

}  // namespace ksg
