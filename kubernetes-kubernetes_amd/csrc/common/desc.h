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
#include <stddef.h>
#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC__)
#define KSG_HD __host__ __device__
#else
#define KSG_HD
#endif

namespace ksg {

constexpr int kNumPlugins = 10;  // KSG_NUM_PLUGINS
constexpr int kBlock = 256;      // threads per block of the per-node kernels (4 waves)
constexpr int kMaxScalar = 16;   // minimum extended/scalar resource columns (MirrorView::scalar_cols grows)
constexpr int kPortSlots = 8;    // minimum used-port slots per node (MirrorView::port_slots grows with the cluster)
constexpr int kMaxCons = 32;      // PodTopologySpread constraints per kind per pod (eligibility is a 32-bit mask)
constexpr int kMaxPodTerms = 64;  // InterPodAffinity terms per kind per pod
constexpr int kAggMaxCons = 8;    // k_agg_loop: constraints / terms per kind of a looped pod (LDS minima, the
constexpr int kAggMaxTerms = 8;   // fold plan's lane layout); pods with more take the launch path
constexpr int kMaxShards = 8;    // node shards (GPUs) of one node-sharded scheduler
constexpr int kBlobLds = 16384;  // pod programs up to this size are staged in LDS by the kernels
constexpr int kLoopMaxPods = 1024;  // k_sched_loop: pods per launch (their program offsets are staged in LDS)
constexpr int kLoopMaxBlk = 2;   // k_sched_loop: node blocks per workgroup (cores and scores kept in LDS)

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

// ---- metav1.LabelSelector programs (labels.Selector over pod / namespace labels) -----------
// int32 stream: [nothing, nreq, {key, op, nvals, value ids...} x nreq]; label sets are sorted
// uint64 (key id << 32 | value id) arrays.  apimachinery/pkg/labels/selector.go:247-294,419-426
enum LSelOp : int32_t { LS_IN = 0, LS_NOTIN = 1, LS_EXISTS = 2, LS_DNE = 3 };

// PodTopologySpread constraint as compiled by the host (podtopologyspread/common.go:87-128)
struct PtsCons {
  int32_t slot;         // label column of the topology key
  int32_t max_skew;
  int32_t min_domains;
  int32_t self_match;   // the incoming pod matches its own selector (filtering.go:338-341)
  int32_t aff_honor;    // NodeAffinityPolicy == Honor
  int32_t taint_honor;  // NodeTaintsPolicy == Honor
  int32_t hostname;     // score: kubernetes.io/hostname counts per node (scoring.go:207-214)
  int32_t sel;          // selector program offset (int32 units, pod selector pool)
  int32_t hist_base;    // arena entries: per-domain (or per-node) matching pod counts
  int32_t pres_base;    // arena entries: domain presence flags
  int32_t nvals;        // domains (label values of the key)
  int32_t lref;         // k_agg_loop: where hist_base's counts live (AggRef)
  int32_t pref;         // k_agg_loop: where pres_base's flags live (AggRef; unused for node-local keys)
  int32_t absent;       // DF_PTS_ANYTOPO score constraints: the domain of a node without the key (the ""
                        // value's id, or an extra entry past the values), -1 otherwise
  int32_t pbit;         // k_agg_loop score constraints: first bit of its domains in the presence vector
  int32_t pad;
};
// an InterPodAffinity term of the incoming pod (interpodaffinity/filtering.go:246-283, scoring.go:81-125)
struct IpaTerm {
  int32_t slot;         // label column of the topology key
  int32_t weight;
  int32_t hist_base;    // arena base of this topology key's counts
  int32_t sel;          // selector program offset
  int32_t ns_off, ns_cnt;  // namespace ids (pod selector pool, int32 units)
  int32_t all_ns;       // namespaceSelector matches the empty label set
  int32_t lref;         // k_agg_loop: where hist_base's counts live (AggRef)
  int32_t nvals;        // values of the topology key: the histogram's length
  int32_t pad_;
};
struct KeyHist { int32_t slot; int32_t base; int32_t lref; int32_t pad; };
// k_agg_loop's placement of one arena histogram ("AggRef"): >= 0, the histogram's first word in the
// pod's compact shared region (a topology key whose values several nodes share: zones); < 0, the
// node-local histogram -1 - lref, one count per node of the workgroup's range (a key whose every
// value is on one node only, like kubernetes.io/hostname: the owner of the node holds every count).
constexpr int kKeytabStride = 5;  // keytab entry: slot, existing-anti base, topology base, their AggRefs
// an existing pod's affinity term (device term table, kube-scheduler/framework/types.go:380-396)
enum TermKind : int32_t { T_DEAD = -1, T_REQ_AFF = 0, T_REQ_ANTI = 1, T_PREF_AFF = 2, T_PREF_ANTI = 3 };
struct DTerm {
  int32_t owner;        // pod-table slot
  int32_t kind;         // TermKind
  int32_t weight;
  int32_t key;          // topology key id
  int32_t sel;          // term pool offsets (int32 units)
  int32_t nssel;
  int32_t ns_off, ns_cnt;
};
enum IpaFlags : uint32_t {
  IPA_SELF_ALL = 1u << 0,   // the incoming pod matches all its own required affinity terms
  IPA_PREF = 1u << 1,       // incoming preferred terms are processed against every pod (hasConstraints)
  IPA_EXIST_FILTER = 1u << 2,  // existing required anti-affinity terms are checked (Filter active)
  IPA_EXIST_SCORE = 1u << 3,   // existing pods' terms contribute to the score (PreScore active)
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
  DF_AGGREGATE = 1u << 14,         // PTS/IPA counts: k_aggregate runs before the node pass
  DF_FAST = 1u << 15,              // default-plugin shape: straight-line cpu/mem Fit + BalancedAllocation (eval_node_fast)
  DF_ROTDEV = 1u << 16,            // nextStartNodeIndex is device-resident: k_sample_find derives this pod's rotation
  DF_SAMPLE = 1u << 17,            // numFeasibleNodesToFind < nodes: the feasible list is cut (k_sample_apply)
  DF_LFAST = 1u << 18,             // DF_FAST's shape for the node-local plugins (k_agg_loop: eval_core_fast + the
                                   // PodTopologySpread / InterPodAffinity filters and score after it)
  DF_TERMINATING = 1u << 19,       // the pod has a deletionTimestamp (its pod-table slot's flag)
  DF_PTS_ANYTOPO = 1u << 20,       // PodTopologySpread scores with system-default constraints: requireAllTopologies
                                   // is false (podtopologyspread/scoring.go:141-144), no node is ignored and a node
                                   // without a constraint's key is in its "" domain (PtsCons::absent)
  DF_AGG_SAME = 1u << 21,          // k_agg_loop: this pod's counts are defined exactly as the previous pod's of the
                                   // batch (same program but for slot / rotation / own terms): its counts are that
                                   // pod's plus its placement (fold), no gather (set by the host at staging)
  DF_RAW0 = 1u << 22,              // every node's raw TaintToleration and NodeAffinity scores are 0 (no intolerable
                                   // PreferNoSchedule taint exists, no preferred terms): k_sched_loop's helper forms
                                   // the chosen variant's maxima from the counts alone
  DF_OB = 1u << 23,                // OpportunisticBatching: a signed pod (SignPod non-nil, framework.go:884-924) --
                                   // k_ob_hint may place it on the stored heap's next node, k_ob_store keeps its
                                   // cycle's sorted nodes for the next pod (framework/runtime/batch.go:65-229)
  DF_NOMINATED = 1u << 24,         // status.nominatedNodeName names a snapshot node (nominated_node): k_nominated
                                   // runs that node's filters alone first (evaluateNominatedNode, schedule_one.go:
                                   // 657-669,714-745); feasible: the pod goes there, else the full pass follows
};
// a pod the per-pod path may place before its full evaluation (PodStats::ob_done: 1 hint, 2 nominated node)
constexpr uint32_t DF_EARLY = DF_OB | DF_NOMINATED;

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
  // ---- PodTopologySpread / InterPodAffinity (pod-table aggregation)
  int32_t ns_id, slot;               // incoming pod's namespace id; reserved pod-table slot (assume)
  int32_t n_lbl, lbl_off;            // incoming pod labels (uint64 pairs, sorted)
  int32_t n_nslbl, nslbl_off;        // labels of the incoming pod's namespace
  int32_t sel_pool_off;              // int32 pool: selector programs + namespace id lists
  int32_t n_ptsf, ptsf_off, n_ptss, ptss_off;  // PtsCons (DoNotSchedule / ScheduleAnyway)
  uint32_t ipa_flags;
  int32_t hard_weight;
  int32_t n_raff, raff_off, n_ranti, ranti_off, n_paff, paff_off, n_panti, panti_off;  // IpaTerm
  int32_t n_keytab, keytab_off;      // int32 [key id][kKeytabStride]: slot, existing-anti / topology-score arena base (-1 none), their AggRefs
  int32_t n_exkeys, exkeys_off;      // KeyHist: existing anti-affinity counts (Filter)
  int32_t n_topokeys, topokeys_off;  // KeyHist: topology scores (Score)
  int32_t arena_words;               // arena entries this pod uses (zeroed again by k_select)
  // ---- percentageOfNodesToScore (schedule_one.go:778-782,858-884), DF_ROTDEV / DF_SAMPLE
  int32_t num_to_find;               // numFeasibleNodesToFind (or 1 without score plugins)
  int32_t prev_pod;                  // previous launched pod of the batch (its rot_out), -1: PodStats::rot_in
  // ---- k_agg_loop (the persistent loop for pods with pod-table aggregation)
  int32_t n_own_terms, own_terms_off;  // int32 term-table entries of this pod's own affinity terms (the
                                       // owner adds them to its term list when the pod is assumed)
  int32_t agg_gwords;                  // words of the compact shared region (AggRef >= 0)
  int32_t agg_nlocal;                  // node-local histograms (AggRef < 0)
  int32_t agg_local_cons;              // bit c: DoNotSchedule constraint c counts on a node-local histogram
  // ---- OpportunisticBatching (DF_OB; zero otherwise, so programs of unsigned pods compare as before)
  int32_t ob_hint;                     // 1: the previous cycle of this context was a pod of the same signature
                                       // without a nominated node -- GetNodeHint may find the state usable
  int64_t ob_cycle;                    // SchedulingQueue.SchedulingCycle() of this pod's cycle
  int64_t ob_now;                      // time.Now() of this cycle, ns (maxBatchAge, batch.go:57,208)
  // ---- evaluateNominatedNode (DF_NOMINATED)
  int32_t nominated_node;              // snapshot index of status.nominatedNodeName
  int32_t nom_pad;
};

// ---- DefaultPreemption: SelectVictimsOnNode per node, one thread each ----------
// The host lays out, per snapshot node, the pods isPreemptionAllowed admits (lower priority than the
// preemptor) in reprieve order: sorted by MoreImportantPod, the PDB-violating group first
// (default_preemption.go:280-343).  k_preempt removes them all, re-runs the filters the removal can
// change (NodePorts, NodeResourcesFit, then PodTopologySpread / InterPodAffinity with the victims'
// effect on the cycle's counts, PreemptIn), and reprieves them one by one.
enum PVFlags : uint32_t {
  PV_PORT = 1u,  // the victim holds a host port the preemptor's ports conflict with
  PV_VIOL = 2u,  // the victim is in the PDB-violating group (filterPodsWithPDBViolation)
};
struct PVictim {
  int64_t cpu, mem, eph;          // Resource it adds to NodeInfo.Requested (PodInfo.CalculateResource)
  uint32_t flags;                 // PVFlags
  int32_t slot;                   // pod-table slot (namespace, labels, terms; PreemptIn::vsc row)
};
enum PNFlags : uint32_t {
  PN_BASE_PORT = 1u,  // a conflicting host port stays on the node with every victim removed
};
struct PNode {
  int32_t voff, vcnt;  // the node's victims in the PVictim array
  uint32_t flags;      // PNFlags
  int32_t pad;
};
enum PStat : uint32_t { PS_NOT_CHECKED = 0xffffffffu, PS_NO_VICTIMS = 0xfffffffeu };
struct POut {
  uint32_t st;         // packed Filter status with the victims removed (0: fits), or a PStat
  int32_t nvictims;    // victims that stay removed (flag 1 in the per-victim output)
  int32_t nviolating;  // of them, from the PDB-violating group (numViolatingVictim)
  uint32_t flags;      // as PSegOut::flags
};

// The device-resident form (k_preempt_seg): every node's pods as an importance-ordered segment of
// kSegCap records, kept up to date by the cache events (only the nodes whose pods changed are
// re-sorted and re-uploaded).  The pods isPreemptionAllowed admits are then the segment's suffix with
// priority below the preemptor's, and the PDB grouping runs on the device against the pod table's labels.
constexpr int kSegCap = 128;  // records per node segment (a node with more pods takes the host-staged path)
constexpr int kMaxPdb = 8;    // PodDisruptionBudgets the device groups by (more: host-staged path)
enum PRFlags : uint32_t { PR_MANY_PORTS = 1u, PR_SCALAR = 2u };
struct PRec {
  int64_t cpu, mem, eph;  // PodInfo.CalculateResource
  int64_t start;          // status.startTime (Unix ns), INT64_MAX without one (the call's clock)
  int32_t prio, slot;     // corev1helpers.PodPriority; pod-table slot (namespace, labels)
  uint32_t port[2];       // host port ids (0xffffffff: none)
  uint32_t flags;         // PRFlags
  int32_t pad;
};
struct PdbDev { int32_t ns, sel, allowed, ok; };  // namespace id, selector program offset, DisruptionsAllowed
struct PSegOut {
  uint32_t st;                  // as POut
  int32_t nvictims, nviolating;
  uint32_t flags;               // bit 0: a potential victim matches a DoNotSchedule spread selector (unsupported)
  unsigned long long vmask[2];  // segment positions kept removed (victims)
  unsigned long long violmask[2];  // segment positions in the PDB-violating group
  // pickOneNodeForPreemption's criteria over the victims (preemption.go:322-357)
  int32_t hiprio;               // priority of the most important victim
  int32_t pad;
  int64_t sumprio;              // sum of (priority + MaxInt32 + 1)
  int64_t earliest;             // GetEarliestPodStartTime: earliest start among the highest-priority victims
};
// k_preempt_pick's answer: DryRunPreemption's cut and SelectCandidate over the per-node results
struct PickOut {
  int32_t potential, ncand, ncandidates, best;  // best: snapshot index, -1 if no candidate
  int32_t offset, unsupported, pad[2];          // unsupported: some node's PSegOut flag bit 0
  PSegOut best_out;                             // the chosen node's result (victim masks)
};
// DoNotSchedule constraints / affinity terms / existing-anti keys the register-resident dry run tracks per
// kind; a preemptor with more takes the workspace-resident one (PreemptIn::wide), up to the compile's caps
constexpr int kPreemptCons = 8;
// What both dry-run kernels (k_preempt_seg, k_preempt) read about the victims' effects beyond Requested:
// their scalar resources and the PodTopologySpread / InterPodAffinity counts they move.
struct PreemptIn {
  int32_t pts_check, ipa_check;
  const long long* pts_mm;   // [n_ptsf][3]: per DoNotSchedule constraint the domain minimum, its
                             // multiplicity and the next larger count (k_pts_minima)
  const int32_t* ex_contrib; // [slot][ex_stride]: the pod's required anti-affinity terms that match the
                             // preemptor, per existing-anti key (k_preempt_terms); nullptr: none
  const long long* aff_tot;  // [n_raff]: per required affinity term of a self-matching preemptor the
                             // cycle's total count over its histogram (k_aff_totals); nullptr: not needed
  // the preemptor's extended resources (PodDesc scalar order, n_scalar of them, any number):
  const int64_t* vsc;        // [slot][n_scalar]: each pod's request of them (CalculateResource), 0 rows elsewhere
  int64_t* sreq;             // [n][n_scalar]: per node, the dry run's Requested of them (the kernel's scratch)
  // the workspace-resident dry run (PreemptWide): per node 5 wide_c + 10 wide_g words, field-major and
  // node-minor ([field][n]); wide_c = n_ptsf, wide_g = max(n_raff, n_ranti, n_exkeys); nullptr: registers
  long long* wide;
  int32_t wide_c, wide_g, ex_stride, pad;
};
struct PreemptView {
  const PRec* seg;           // [n][kSegCap]
  const int32_t* cnt;        // [n] records in use
  const PdbDev* pdb;         // [npdb]
  const int32_t* pdb_pool;   // their selector programs
  const uint8_t* disrupted;  // [slot] bit k: the pod is in PDB k's DisruptedPods (nullptr: none)
  PSegOut* out;              // [n]
  int32_t npdb, prio, all_nodes, pad;
  int64_t now;               // GetPodStartTime for pods without a start time
  PreemptIn in;
};

// Per-pod device result (ScheduleResult + diagnostics), written by the select kernel.
struct DevResult {
  int32_t status;     // KSG_CODE_*
  int32_t node;       // chosen snapshot index or -1
  int32_t feasible;
  int32_t evaluated;
  int64_t total;
  uint64_t key;       // winning packed key (debug)
  uint32_t ipa_any;   // PodStats::ipa_any (PreFilter / PreScore Skip decisions taken on the device)
  uint32_t rot_next;  // DF_ROTDEV: nextStartNodeIndex after this pod
  uint32_t hinted;    // 1: the pod took the OpportunisticBatching hint, 2: its nominated node (no full evaluation)
  uint32_t pad;
};

// Per-pod scratch (zeroed by the host before each batch).
struct PodStats {
  unsigned long long best;  // packed (TotalScore, heap pre-order key) max
  unsigned long long max_raw[kNumPlugins];  // enc_i64, init enc_i64(INT64_MIN) for max
  unsigned long long min_raw[kNumPlugins];  // enc_i64, init enc_i64(INT64_MAX) for min
  uint32_t done;            // arrival ticket of the select kernel's blocks
  uint32_t feasible;
  uint32_t done_agg;        // arrival ticket of k_aggregate's blocks
  uint32_t ipa_any;         // bit0 affinity counts, bit1 anti counts, bit2 existing anti, bit3 topology score
  long long pts_min[kMaxCons];        // critical-path minimum per DoNotSchedule constraint
  uint32_t pts_ndom[kMaxCons];        // domains per DoNotSchedule constraint
  uint32_t pts_distinct[kMaxCons];    // feasible, non-ignored domains per ScheduleAnyway constraint
  uint32_t pts_nonignored;            // feasible nodes carrying every ScheduleAnyway key
  // device-resident nextStartNodeIndex (DF_ROTDEV, k_sample_find)
  uint32_t rot_in;                    // first launched pod of the batch: the host's nextStartNodeIndex
  uint32_t rot;                       // this pod's rotation start (snapshot index)
  uint32_t rot_out;                   // nextStartNodeIndex after this pod (schedule_one.go:686-687)
  uint32_t processed;                 // nodes processed by findNodesThatPassFilters
  int32_t samp_end;                   // snapshot index of the (K+1)-th feasible node in rotated order, -1: none
                                      // (node-sharded: -2 on the ranks that do not hold it)
  int32_t keep[4];                    // node-sharded cut: this rank's kept nodes are the feasible ones in
                                      // [keep[0], keep[1]) or [keep[2], keep[3]) (k_sample_shard_b)
  uint32_t ob_done;                   // DF_EARLY: k_ob_hint (1) or k_nominated (2) placed the pod; the full-evaluation
                                      // kernels return at once
  uint32_t nom_failed;                // 1 + the snapshot index of a nominated / hinted node whose filters failed alone
                                      // (its status is in NodeToStatus: processedNodes counts it once), 0: none
  uint32_t pad;
};

// OpportunisticBatching's state on the device (framework/runtime/batch.go:31-58): the sorted nodes a signed
// pod's cycle left (sortedNodeScores after heap.Init and the winner's Pop: a Go container/heap of
// (TotalScore, node) entries in heap order, ObEnt[len]), its creation time and the last cycle.  Written by
// k_ob_store / k_ob_hint only; node indices are snapshot indices (the host remaps them when the node list is
// rebuilt, -1: a node no longer in the snapshot).
struct ObEnt {
  int64_t total;
  int32_t node;
  int32_t pad;
};
struct ObState {
  int64_t creation;    // batchState.creationTime (ns, the cycle's clock)
  int64_t last_cycle;  // lastCycle.cycleCount of the last StoreScheduleResults
  int32_t last_node;   // lastCycle.chosenNode (-1: none / gone)
  int32_t len;         // sortedNodes.Len(); 0: stateEmpty (nil state, nil or empty list)
  uint32_t check;      // k_ob_store: 1 + the first cycle whose heap pop disagreed with k_select's winner
  uint32_t pad;
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
  const int64_t* scalar_alloc;    // [scalar_cols][cap]
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* req_eph;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* num_pods;
  int64_t* scalar_req;            // [scalar_cols][cap]
  const uint32_t* taint_off;      // [n+1]
  const uint32_t* taint_ids;
  const uint32_t* img_off;        // [n+1]
  const uint32_t* img_ids;        // sorted per node
  const int32_t* labels;          // [slots][cap] local value id, -1 absent
  const int64_t* label_num;       // [slots][cap] parsed integer value
  const uint8_t* label_num_ok;    // [slots][cap]
  uint32_t* ports;                // [cap][port_slots] port id, 0xffffffff empty
  // pod table (NodeInfo.Pods of every node, flattened; slots indexed by the host)
  int32_t pods_hw;                // slots in use (high-water mark)
  int32_t n_terms;                // term table entries in use
  int32_t* pod_node;              // [slot] snapshot index, -1 free / not assumed
  const int32_t* pod_ns;          // [slot] namespace id
  const uint32_t* pod_flags;      // [slot] bit0 terminating
  const uint32_t* pod_lbl_off;    // [slot] offset into lbl_pool
  const uint32_t* pod_lbl_cnt;    // [slot]
  const unsigned long long* lbl_pool;  // (key << 32 | value) sorted per pod
  const DTerm* terms;             // existing pods' affinity terms
  const int32_t* term_pool;       // their selector programs / namespace id lists
  const double* log_tab;          // go math.Log(k) for k in [0, log_n)
  int32_t log_n;
  int32_t port_slots;             // `ports` row stride: >= every node's host ports + what a batch can assume
  int32_t scalar_cols;            // scalar resource columns (>= the interned extended resources)
  int32_t pad_;
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
  int64_t* out_scores;    // eval mode: [kNumPlugins][cap] normalised scores, unweighted
  int64_t* out_total;     // eval mode: [cap]
  unsigned long long* arena;  // PTS/IPA histograms (zero between pods)
  ObState* ob;            // OpportunisticBatching state (DF_OB pods)
  ObEnt* ob_heap;         // [cap] its sorted nodes (heap order)
};

// ---- node-sharded evaluation ----------------------------------------------------
// Every rank holds the whole mirror (replicated by the informer feed) and evaluates the nodes of
// its contiguous block range.  Per pod, fixed-layout uint64 vectors are all-reduced with MAX:
// per-rank slots (zero elsewhere) carry counts, encoded int64 maxima carry the normalisation
// maxima, and bitwise-NOT of encoded minima carry the minima (0 is the identity of every slot).
enum XaWord : int {
  XA_CNT = 0,                   // [kMaxShards] feasible nodes of rank r
  XA_BELOW = kMaxShards,        // [kMaxShards] feasible nodes of rank r before nextStartNodeIndex
  XA_NONIGN = 2 * kMaxShards,   // [kMaxShards] PodTopologySpread non-ignored feasible nodes of rank r
  XA_MAX_TAINT = 3 * kMaxShards,
  XA_MAX_NA,
  XA_MAX_IPA,
  XA_NMIN_IPA,
  XA_END,                       // percentageOfNodesToScore cut: 1 + the (K+1)-th feasible node, from its rank
  XA_PROC,                      // 1 + processedNodes, from the same rank (0: every rank knows it)
  XA_WORDS = 4 * kMaxShards,
};
static_assert(XA_PROC < XA_WORDS, "XA layout");
// The cut's pre-exchange (k_sample_shard_a): per-rank feasible counts before the cut
enum XsWord : int { XS_CNT = 0, XS_BELOW = kMaxShards, XS_WORDS = 2 * kMaxShards };
enum XpWord : int { XP_MAX_PTS = 0, XP_NMIN_PTS = 1, XP_WORDS = 4 };
enum XbWord : int { XB_KEY = 0, XB_NODE = kMaxShards, XB_WORDS = 2 * kMaxShards };
struct RankPtrs { unsigned long long* p[kMaxShards]; };  // every rank's exchange vector (local transport)
// One node's static columns (NodeInfo.node) for an in-place update of the mirror, flushed in bulk
// at the next cycle (Cluster::flush_node_updates -> k_node_update).  Variable parts live in pools
// after the records: taint / image ids (uint32) at id_off, label entries at lbl_off (lbl_cnt of
// them: slot, value id, Gt/Lt integer, parse ok).
struct NodeUpdate {
  int32_t node, n_taint, n_img, lbl_cnt;
  uint32_t taint_off, img_off;      // the node's CSR offsets on the device
  uint32_t id_off, lbl_off;         // into the id / label pools of the flush
  int64_t alloc_cpu, alloc_mem, alloc_eph;
  int32_t alloc_pods;
  uint32_t flags;
  uint32_t sc_off, sc_cnt;          // the node's scalar allocatable in the flush's ScalarEntry pool
};
struct LabelEntry { int32_t slot, value; int64_t num; int32_t ok, pad; };
struct ScalarEntry { int32_t slot, pad; int64_t value; };  // one non-zero scalar resource column of a node
// One node's dynamic columns (NodeInfo.Requested / NonZeroRequested / len(Pods) / UsedPorts)
// after pod events, flushed in bulk at the next cycle (Cluster::flush_node_dynamic -> k_node_dyn).
struct NodeDyn {
  int32_t node, num_pods;
  int64_t req_cpu, req_mem, req_eph, nz_cpu, nz_mem;
  uint32_t sc_off, sc_cnt;      // the node's scalar requests in the flush's ScalarEntry pool
  uint32_t port_off, port_cnt;  // the node's UsedPorts ids in the flush's id pool
};

struct ShardView {
  int32_t world, rank;
  int32_t blk0, nblk;         // this rank's kBlock-node blocks [blk0, blk0 + nblk)
  unsigned long long* xa;     // [pods][XA_WORDS]
  unsigned long long* xp;     // [pods][XP_WORDS]
  unsigned long long* xb;     // [pods][XB_WORDS]
  unsigned long long* xs;     // [pods][XS_WORDS]
};

// ---- persistent scheduling loop (k_sched_loop) -------------------------------------
// One launch evaluates a run of consecutive pods: `nwg` resident workgroups each own a contiguous
// range of node blocks for the whole run and meet at two device-scope arrival counters per pod.
// ---- the resident loops' pod ring (single-pod calls) -----------------------------------
// Host-pinned, device-mapped, fine-grained (uncached on the device).  The host posts pod q's program
// into blob[q % kRingSlots] (unless RING_SAME, below), then the doorbell ll; the loop's workgroups poll
// it, take the program into LDS and schedule the pod; the committing thread writes res[q % kRingSlots]
// and, last, its seq = q + 1.  A stop (ll[0]'s tag kRingStop) ends the launch; so does kLoopMaxPods pods
// or ring_idle of s_memrealtime ticks without a pod (the host relaunches first when it has been idle for
// half that: the loop never outlives its process).
constexpr int kRingSlots = 2;
constexpr uint32_t kRingStop = 0xffffffffu;
struct alignas(16) RingResult {
  uint32_t seq, pad[3];
  DevResult r;
};
// k_agg_loop's resident instance also takes the pod's pod-table entry through the ring (entry[q %
// kRingSlots], its size in ll[2]): the owner of the chosen node writes it into the device
// pod table when it commits the pod, so the pods after it count it.  The host laid the
// entry out in its shadow (Cluster::pod_table_put) and checked that the device arrays hold it.
struct RingEntry {
  int32_t slot;                // pod-table slot (-1: none; nothing is written)
  int32_t ns;
  uint32_t flags, lbl_off, lbl_cnt;
  int32_t tpool_off, tpool_cnt;  // term-pool words [tpool_off, tpool_off + tpool_cnt)
  int32_t nterms;
  // followed by unsigned long long labels[lbl_cnt], int32_t tpool[tpool_cnt] (padded to 8 bytes),
  // RingTerm terms[nterms]
};
struct RingTerm {
  int32_t j, pad;  // term-table index
  DTerm d;
};
constexpr int kRingEntryBytes = 8192;  // (staged into one of the resident k_agg_loop's program slots)
// The doorbell is four self-tagged words (ll[k] = {tag = q + 1 | data << 32}, each 8-byte store atomic on
// its own, so the loop takes them in one poll without a second read over PCIe):
//   ll[0] data: RING_SAME (pod q is pod q-1's program -- and, k_agg_loop, its entry -- but for the fields
//               below: nothing is staged, the loop copies q-1's in LDS and patches them) | RING_AGG_SAME
//               (k_agg_loop: the program's DF_AGG_SAME);
//   ll[1..3]:   RING_SAME: {slot, rot_start, entry lbl_off}; else {program bytes, entry bytes, 0}.
//   RING_TERMS (with RING_SAME): the pod's own affinity terms are pod q-1's but for their term-table indices and
//               the term-pool offset of their words (a pod stamped from the same template): PodRing::patch[q %
//               kRingSlots] holds {new tpool_off | n << 32} and the n indices (int32 pairs); the loop rewrites the
//               program's own-term list and the entry's terms (index, owner, word offsets) in LDS.
// A stop is ll[0]'s tag kRingStop.
enum : uint32_t { RING_SAME = 1u, RING_AGG_SAME = 2u, RING_TERMS = 4u };
constexpr int kPatchWords = 1 + 4 * kAggMaxTerms / 2;  // RING_TERMS: the header and up to 4 * kAggMaxTerms indices
constexpr int kRingLL = 4;
constexpr int kRelayWords = kRingLL + kBlobLds / 8 + kRingEntryBytes / 8;  // AggView::relay
// k_sched_loop polls one word instead (its registers leave no room for four): ctl = {q + 1 (bits 0-10) |
// RING_SAME << 11 | RING_SAME ? slot + 1 << 12 (23 bits), rot_start << 35 (25 bits) : program bytes << 12};
// q + 1 = kCtlStop ends the launch.
constexpr unsigned long long kCtlStop = 0x7ffull;
struct alignas(128) PodRing {
  unsigned long long ctl;          // [host] k_sched_loop's doorbell
  unsigned long long ll[kRingLL];  // [host] k_agg_loop's doorbell (above)
  uint32_t pad0[22];
  uint32_t exited;         // [device] 1: the loop left on its own (idle / pod limit)
  uint32_t pad1[31];
  RingResult res[kRingSlots];
  alignas(128) uint8_t blob[kRingSlots][kBlobLds];
  alignas(128) uint8_t entry[kRingSlots][kRingEntryBytes];
  alignas(128) unsigned long long patch[kRingSlots][kPatchWords];  // [host] RING_TERMS
};

struct LoopView {
  int32_t first_pod, npods;  // pods [first_pod, first_pod + npods) of the batch
  int32_t nwg;               // workgroups of this rank (all resident; one per CU at most)
  int32_t blk0, nblk;        // this rank's kBlock-node blocks [blk0, blk0 + nblk) (all of them unsharded)
  int32_t world, rank;       // node shards: participants are world * nwg workgroups, rank-major
  uint32_t tag;              // this batch's granule tag (1..65535; 0 never valid)
  unsigned long long* gran[kMaxShards];  // every rank's granule array, [pods][world * nwg][kGran]; [rank] is local
  uint32_t* fail;            // set when a spin gives up (a workgroup never arrived)
  unsigned long long* stamps;  // diagnostic: [npods][8] s_memrealtime per phase (nullptr)
  const uint32_t* desc_bytes;  // [batch pods] program sizes (indexed like BatchView::desc_off)
  unsigned long long* wstamps;  // diagnostic: [npods][nwg][8] exchange / owner times (nullptr)
  int32_t give_up_at;        // diagnostic: every workgroup gives up at this pod of the run (-1: never)
  int32_t wave_map;          // which hardware wave plays which role (k_sched_loop kWaveMap; 0: identity)
  PodRing* ring;             // resident mode (nullptr: a batch run): pods arrive one by one through the ring
  unsigned long long ring_idle;  // resident mode: s_memrealtime ticks (100 MHz) without a pod before leaving
  int32_t ring_ahead;        // resident mode: evaluate the next pod's phase 1 ahead of its doorbell (config residentAhead)
  int32_t pad_ring;
  // resident mode with many workgroups: workgroup 0 alone polls the host's ctl and relays the word through
  // device memory (relay[0]), where the others poll (nullptr: every workgroup polls the host)
  unsigned long long* relay;
};
// exchange granules per participant per pod: A0 {count, count before nextStartNodeIndex},
// A1 {max raw TT + 1, max raw NA + 1}, B {packed key < 2^48}, B_node (sharded only) -- four words used, the row
// padded to 16 (one 128-byte line per participant, no line written by two workgroups): k_sched_loop 5.33 -> 5.28 us
// per pod at C2, 5.28 -> 5.25 at C1 (interleaved A/B, profiles/r06g_granule_stride_ab.txt).  The same padding of
// k_agg_loop's 14-word rows measured slower (DTS 16.13 -> 16.43 us per pod) and was not kept.
constexpr int kGran = 16;
// A persistent loop's give-up record (LoopView::fail / AggView::fail): [0] flag, [1] pod of the run
// (the granule row; or a k_agg_loop check code), [2] granule (or workgroup), [3] first missing sweep
// lane, [4] loop (1 k_sched_loop, 2 k_agg_loop), [5] its granule tag, [6, 7] the sweep's missing-lane
// ballot at the give-up (lane l: some participant l + 64 k had not published); the launch's entry, written by
// workgroup 0 while no give-up is recorded: [8] its HW_ID register (ME / pipe / HQD it was dispatched from),
// [9] its XCC, [10, 11] s_memrealtime at entry; [12, 13] s_memrealtime at the give-up, [14] the giving-up
// wave's HW_ID, [15] its XCC (a rank whose loop entered after a peer gave up was not resident with it)
constexpr int kFailWords = 16;
constexpr int kFailBytes = kFailWords * 4;

// ---- persistent loop for pods with pod-table aggregation (k_agg_loop) ---------------
// Same workgroup geometry as k_sched_loop (unsharded).  Each workgroup also owns the pod-table slots
// and existing affinity terms of the pods bound to its nodes.
constexpr int kAggThreads = 512;   // one node slot per thread (8 waves)
constexpr int kAggLocal = 4;       // node-local histograms per pod
constexpr int kAggGWords = 1024;   // compact shared-region words per pod (staged in LDS)
constexpr int kAggLocalCons = 2;   // DoNotSchedule constraints on node-local histograms per pod
constexpr int kAggPods = 5120;     // batch k_agg_loop: pod-table slots per workgroup in LDS (its nodes' pods; the
                                   // rest spill to HBM)
constexpr int kAggTerms = 5120;    // batch k_agg_loop: existing affinity terms per workgroup in LDS (likewise)
constexpr int kAggBlobLds = 8192;  // batch k_agg_loop's three program slots: its pods' programs up to this size
                                   // (larger pods take the launch path); the 24 KB this frees over kBlobLds hold
                                   // 6144 more list entries, so C5's fill-front workgroup stays in LDS
constexpr int kAggRingPods = 2048;   // the resident instance keeps kBlobLds program slots (its registers leave no
constexpr int kAggRingTerms = 2048;  // room for the longer LDS offsets) and the shorter lists
static_assert(kRingEntryBytes <= kBlobLds, "a ring entry is staged into a k_agg_loop program slot");
constexpr int kAggSpillMax = 1 << 20;  // pod / term list entries past those per workgroup (HBM spill rows)
constexpr int kAGran = 14;         // granules per participant per pod
constexpr int kAggStartRow = 1024; // k_agg_loop (node-sharded): the start barrier's granule row (= kLoopMaxPods)
enum AggGran : int {
  AG_Z0 = 0,   // {InterPodAffinity "any" bits}: every count of the pod is in the shared region
  AG_Z1 = 1,   // node-local DoNotSchedule constraint 0: {min count over my eligible nodes (24) | eligible nodes (12) |
               //  of them at that minimum (12)}
  AG_Z2 = 2,   // ... constraint 1
  AG_A0 = 3,   // {feasible | feasible before nextStartNodeIndex}
  AG_A1 = 4,   // {max raw TaintToleration + 1 | max raw NodeAffinity + 1}
  AG_A2 = 5,   // max raw InterPodAffinity (biased, 0 = none)
  AG_A3 = 6,   // min raw InterPodAffinity (biased and reversed, 0 = none)
  AG_P0 = 7,   // PodTopologySpread scoring: presence bits [0, 48) of my feasible, non-ignored nodes' domains
  AG_P1 = 8,   // {non-ignored feasible nodes (20) | presence bits [48, 76) (28)}
  AG_PXA = 9,  // AG_PX of the raw scores phase 1 computed with the previous pod's topology sizes: exact,
               // and exchange PX skipped, when this pod's sizes (from P0 / P1) equal them
  AG_B = 10,   // packed (TotalScore, pre-order) key
  AG_BN = 11,  // the snapshot index + 1 of the workgroup's best node (every workgroup folds the
               // chosen pod into the next pod's counts)
  AG_BC = 12,  // the template cache: my best node's counts under the next pod's node-local DoNotSchedule
               // constraints {constraint 0 (24) | constraint 1 (24)} (the fold moves their minima without exchange Z)
  AG_PX = 13,  // PodTopologySpread raw-score {max + 1 (24) | 2^24 - 1 - min (24)} over my scored nodes
};
constexpr int kAggScoreCons = 2;   // k_agg_loop: ScheduleAnyway constraints of a looped pod (per-node counts in LDS)
constexpr int kAggPresBits = 76;   // k_agg_loop: presence bits of its non-hostname score constraints' domains
constexpr int64_t kAggPtsRawMax = ((int64_t)1 << 24) - 2;  // raw PodTopologySpread scores the granules carry
constexpr int64_t kAggIpaBias = (int64_t)1 << 46;  // |raw InterPodAffinity| < 2^46 (host-checked)
constexpr int kAggStamps = 16;                     // diagnostic stamps per pod (AggView::stamps)
struct AggView {
  int32_t first_pod, npods;   // pods [first_pod, first_pod + npods) of the batch
  int32_t nwg;                // resident workgroups
  int32_t blk0, nblk;         // node blocks [blk0, blk0 + nblk)
  uint32_t tag;               // granule tag (1..65535)
  int32_t gwords;             // region words per pod (max agg_gwords of the run)
  int32_t debug;              // diagnostic (config "aggLoopDebug"): bit 0 never fold (gather every pod after
                              // the previous one is placed), bit 1 never DF_LFAST, bit 2 no same-template
                              // shortcut (DF_AGG_SAME), bit 3 (host) no RING_SAME -- the resident loops stage
                              // every pod over PCIe, bit 4 the resident loop always runs exchange PX,
                              // bit 7 (host: residentAhead false) no phase 1 ahead of the doorbell
  unsigned long long* gran;   // [npods][world * nwg][kAGran] (this rank's)
  unsigned long long* region; // [npods][gwords]: shared-region sums (zeroed by the host; this rank's)
  // node shards: participants are world * nwg workgroups, rank-major.  Every granule and
  // every shared-region partial goes into each rank's array (the peers' are IPC-mapped, uncached).
  // (the peers' pointers live in device memory, not in the kernel arguments: SGPR pressure)
  int32_t world, rank;
  unsigned long long* const* grans;    // [world] every rank's granule array
  unsigned long long* const* regions;  // [world] every rank's regions
  uint32_t* fail;             // set when a spin gives up
  const uint32_t* desc_bytes; // [batch pods] program sizes
  unsigned long long* stamps; // diagnostic: [npods][kAggStamps] (nullptr)
  unsigned long long* wstamps;  // diagnostic: [npods][nwg][4] phase-1 start, A publish, B publish, commit end
  int32_t give_up_at;         // diagnostic: every workgroup gives up at this pod of the run (-1: never)
  int32_t ptss;               // some pod of the run has PodTopologySpread scoring (the k_agg_loop<., true> instance)
  // a workgroup's pod / term lists past kAggPods / kAggTerms entries (nodes that gathered many pods):
  // [nwg][spill_pods + spill_terms] in HBM, this rank's workgroups
  uint32_t* spill;
  int32_t spill_pods, spill_terms;
  // resident instance (k_agg_loop<false, true, true>): pods through the ring, one run per pod
  PodRing* ring;
  unsigned long long ring_idle;  // s_memrealtime ticks without a pod before the launch ends by itself
  // resident mode with many workgroups: workgroup 0 alone polls the host doorbell and relays it -- and a
  // staged program and entry -- through device memory (kRelayWords: the doorbell's four tagged words, then the
  // program, then the entry); the others poll that (nullptr: every workgroup polls the host)
  unsigned long long* relay;
  // the template cache (batch instance): per workgroup kAggTc slots of kTcWords words, each a
  // template's counts as this workgroup holds them; tcw[batch pod] the host's plan (TcWord; nullptr: off)
  unsigned long long* tcache;
  const uint32_t* tcw;
};
// In-process rank groups (localGroup, one device) run every rank's persistent loop in one dispatch
// (k_sched_loop_group / k_agg_loop_group): rank r's launch arguments, [world] of them in device
// memory, staged by the group's leader.
struct LoopGroupArg {
  MirrorView m;
  BatchView b;
  LoopView lv;
};
struct AggGroupArg {
  MirrorView m;
  BatchView b;
  AggView av;
};
// (the single-device loop kernels read their three by-value arguments through these layouts: the kernarg segment
// places each argument at the next multiple of its alignment, as a struct places its members)
static_assert(offsetof(LoopGroupArg, b) == sizeof(MirrorView) && offsetof(LoopGroupArg, lv) == sizeof(MirrorView) + sizeof(BatchView) &&
              offsetof(AggGroupArg, av) == sizeof(MirrorView) + sizeof(BatchView) && alignof(MirrorView) == 8 &&
              alignof(BatchView) == 8 && alignof(LoopView) == 8 && alignof(AggView) == 8, "kernel argument layout");
// k_agg_loop's template cache: a pod's counts are a function of its template (the program but for the fields
// agg_same masks) and of the pods placed before it.  Each workgroup keeps the counts of up to kAggTc templates
// in HBM, current through the last placement, so a pod of a cached template loads them instead of gathering.
constexpr int kAggTc = 6;
constexpr int kAggSlotsC = kLoopMaxBlk * kBlock;             // node slots per k_agg_loop workgroup
constexpr int kTcLh = kAggGWords;                             // slot layout (words): shared-region totals,
constexpr int kTcElig = kTcLh + kAggLocal * kAggSlotsC / 2;   // node-local histograms (int32),
constexpr int kTcAny = kTcElig + kAggSlotsC / 4;              // eligibility (uint16), the IPA any bits
constexpr int kTcWords = (kTcAny + 1 + 7) & ~7;
// TcWord (per pod of a run): bits 0-3 slot + 1 (0: the pod's counts are not cached), bit 4 hit (the slot holds
// its template's counts: loaded, not gathered), bit 5 the write-back while this pod is decided stores the
// template's node eligibility too (static: once per slot assignment), bits 8-13 the slots the loop folds the
// previous pod's placement into while it decides this pod
KSG_HD inline int tc_slot(uint32_t w) { return (int)(w & 15u) - 1; }
KSG_HD inline bool tc_hit(uint32_t w) { return (w & 16u) != 0; }
KSG_HD inline bool tc_elig(uint32_t w) { return (w & 32u) != 0; }
KSG_HD inline uint32_t tc_fold(uint32_t w) { return (w >> 8) & 63u; }

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
// ---- label sets and selector programs (shared by the host compiler and the kernels) -------
KSG_HD inline int32_t lset_find(const unsigned long long* set, int32_t n, uint32_t key) {
  int32_t lo = 0, hi = n;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if ((uint32_t)(set[mid] >> 32) < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < n && (uint32_t)(set[lo] >> 32) == key) ? (int32_t)(uint32_t)set[lo] : -1;
}
// labels.Selector.Matches over a sorted label set (selector.go:247-294, 419-426)
KSG_HD inline bool lsel_match(const int32_t* prog, const unsigned long long* set, int32_t n) {
  if (prog[0]) return false;  // nothingSelector
  const int32_t nreq = prog[1];
  const int32_t* r = prog + 2;
  for (int32_t q = 0; q < nreq; ++q) {
    const int32_t key = r[0], op = r[1], nv = r[2];
    const int32_t v = lset_find(set, n, (uint32_t)key);
    bool ok;
    if (op == LS_IN || op == LS_NOTIN) {
      bool has = false;
      if (v >= 0)
        for (int32_t k = 0; k < nv; ++k) has |= r[3 + k] == v;
      ok = op == LS_IN ? (v >= 0 && has) : (v < 0 || !has);
    } else if (op == LS_EXISTS) {
      ok = v >= 0;
    } else {
      ok = v < 0;
    }
    if (!ok) return false;
    r += 3 + nv;
  }
  return true;
}
KSG_HD inline bool lsel_empty(const int32_t* prog) { return prog[0] == 0 && prog[1] == 0; }
KSG_HD inline bool id_in(const int32_t* ids, int32_t n, int32_t x) {
  for (int32_t k = 0; k < n; ++k)
    if (ids[k] == x) return true;
  return false;
}

// order-preserving int64 <-> uint64 (so signed min/max use unsigned atomics)
KSG_HD inline unsigned long long enc_i64(int64_t v) { return (unsigned long long)v ^ 0x8000000000000000ull; }
KSG_HD inline int64_t dec_i64(unsigned long long u) { return (int64_t)(u ^ 0x8000000000000000ull); }

// ---- persistent-loop exchange granules: 8 bytes, {launch tag (16) | payload (48)} ----
constexpr unsigned long long kGranPayload = (1ull << 48) - 1ull;
KSG_HD inline unsigned long long gran_word(uint32_t tag, unsigned long long payload) {
  return ((unsigned long long)tag << 48) | (payload & kGranPayload);
}
// k_sched_loop exchange A, granule 0: {feasible nodes before nextStartNodeIndex (20) | feasible nodes (20)}
KSG_HD inline unsigned long long gran_a_counts(uint32_t cnt, uint32_t below) {
  return ((unsigned long long)below << 20) | cnt;  // counts < 2^20 (host-checked)
}
// granule 1: {max raw NodeAffinity + 1 (24) | max raw TaintToleration + 1 (24)} over the feasible nodes (0: none);
// the maxima arrive order-encoded (enc_i64), raw scores are < 2^24 - 1 (host-checked)
KSG_HD inline unsigned long long gran_a_maxima(uint32_t cnt, unsigned long long enc_t, unsigned long long enc_n) {
  const unsigned long long tp1 = cnt ? (unsigned long long)dec_i64(enc_t) + 1ull : 0ull;
  const unsigned long long np1 = cnt ? (unsigned long long)dec_i64(enc_n) + 1ull : 0ull;
  return (np1 << 24) | tp1;
}
KSG_HD inline uint32_t gran_a_count(unsigned long long g) { return (uint32_t)(g & 0xfffffull); }
KSG_HD inline uint32_t gran_a_below(unsigned long long g) { return (uint32_t)((g >> 20) & 0xfffffull); }
KSG_HD inline unsigned long long gran_a_tp1(unsigned long long g) { return g & 0xffffffull; }
KSG_HD inline unsigned long long gran_a_np1(unsigned long long g) { return (g >> 24) & 0xffffffull; }

}  // namespace ksg
