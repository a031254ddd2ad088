// host.hpp -- host side of the MI355X node-evaluation engine.
//
// Layers (bottom-up):
//   objects  : v1.Node / v1.Pod / v1.Namespace decoded from JSON into scheduler-facing specs
//   Cluster  : the scheduler cache mirror on the host -- interning tables (label keys/values,
//              taints, images, host ports, extended resources), NodeInfo shadows, bound pods,
//              nodeTree order (backend/cache/node_tree.go) -- plus the HBM mirror it feeds
//   Engine   : per-pod compilation (PreFilter/PreScore work that is O(pod), not O(nodes)) into
//              PodDesc programs, batch launch of the per-node kernels, result readback
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <chrono>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../common/desc.h"
#include "json.hpp"
#include "ksg.h"

namespace ksg {

// ===================================================================================
// objects
// ===================================================================================
using StrMap = std::vector<std::pair<std::string, std::string>>;  // sorted by key

struct ResAmount {  // v1.ResourceList entry, quantity in milli-units (Quantity.MilliValue())
  std::string name;
  int64_t milli;
};
using ResVec = std::vector<ResAmount>;

bool parse_quantity(const std::string& s, int64_t* milli);
int64_t milli_ceil(int64_t m);  // Quantity.Value() from milli-units (rounds up)
bool parse_go_int(const std::string& s, int64_t* v);  // strconv.ParseInt(s, 10, 64)
bool parse_rfc3339(const std::string& s, int64_t* unix_ns);  // metav1.Time (RFC 3339, optional fraction)
bool valid_label_key(const std::string& k);            // validation.IsQualifiedName
bool valid_label_value(const std::string& v);          // validation.IsValidLabelValue
bool scalar_resource(const std::string& n);            // scheduler/util/utils.go:200-203

struct Expr { std::string key, op; std::vector<std::string> values; };
struct NSTerm { std::vector<Expr> exprs, fields; };
struct LabelSel {  // metav1.LabelSelector; present=false is a nil selector
  bool present = false;
  StrMap match;
  std::vector<Expr> exprs;
};
struct PATerm {
  LabelSel sel;
  std::vector<std::string> namespaces;
  LabelSel ns_sel;
  std::string topo;
  int32_t weight = 0;
};
struct Tol { std::string key, op, value, effect; };
struct HostPort { std::string ip, proto; int32_t port; };
struct Container {
  std::string name, image;
  ResVec req;
  std::vector<HostPort> ports;
  bool sidecar = false;
  // InPlacePodVerticalScaling (GA, kube_features.go:1479-1483): the container status of the same name
  // (status.containerStatuses, then initContainerStatuses) with resources != nil -- its actuated
  // requests (resources.requests) and allocatedResources (component-helpers resource/helpers.go:199-215)
  bool has_status = false;
  ResVec st_req, st_alloc;
};
struct Spread {
  int32_t max_skew = 0;
  std::string key, when;
  LabelSel sel;
  int32_t min_domains = 1;
  bool aff_honor = true, taint_honor = false;
  std::vector<std::string> match_label_keys;
};

// A pod's pod-table entry compiled once, when the pod is queued (Cluster::pod_table_precompile), as
// the reference parses a pod's affinity terms once in framework.NewPodInfo (types.go:422-448): its
// label set and each affinity term's selector programs as interned ids (stable for the context's
// life), so reserving its slot in a batch is a copy.
struct PodTablePre {
  std::vector<unsigned long long> labels;
  std::vector<int32_t> words;  // every kept term's selector, namespace selector and namespace ids
  struct Term { int32_t kind, weight, key, sel, nssel, ns_off, ns_cnt; };  // offsets into `words`
  std::vector<Term> terms;     // in pod_table_put's order; a category with an invalid selector is absent
};
struct PodSpec {
  std::string name, ns, uid;
  StrMap labels;
  bool terminating = false;
  std::string node_name;
  bool has_node_selector = false;
  StrMap node_selector;
  bool has_required_na = false;
  std::vector<NSTerm> required_na;
  bool has_preferred_na = false;
  std::vector<std::pair<int32_t, NSTerm>> preferred_na;
  bool has_pod_affinity = false, has_pod_anti = false;
  std::vector<PATerm> aff_req, anti_req, aff_pref, anti_pref;
  std::vector<Tol> tolerations;
  std::vector<Container> containers, init_containers;
  bool has_overhead = false;
  ResVec overhead, pod_requests;
  // in-place resize state (helpers.go:160-170, 299-320; InPlacePodLevelResourcesVerticalScaling is on
  // by default, kube_features.go:1474-1477): status.resources != nil with its requests and
  // status.allocatedResources, and the first PodResizePending condition's reason == Infeasible
  bool has_pod_status_res = false;
  ResVec pod_st_req, pod_st_alloc;
  bool resize_infeasible = false;
  bool has_status_res = false;  // some container, or the pod, carries status resources
  std::vector<Spread> spreads;
  std::vector<std::string> image_volumes;
  // why a pod to schedule is outside the device's plugin set ("" if it is not): volumes or resource
  // claims whose plugins (VolumeBinding, VolumeRestrictions, NodeVolumeLimits, VolumeZone,
  // DynamicResources) would not Skip their PreFilter for it
  std::string unsupported;
  // metav1.GetControllerOfNoCopy: the ownerReference with controller == true (helper/spread.go:51-55)
  bool has_controller = false;
  std::string owner_api, owner_kind, owner_name;
  // DefaultPreemption inputs (corev1helpers.PodPriority, util.GetPodStartTime, preemption/util.go:23-35)
  int32_t priority = 0;          // spec.priority (0 when nil)
  bool has_start = false;        // status.startTime != nil
  int64_t start_ns = 0;          // status.startTime, Unix nanoseconds
  bool preempt_never = false;    // spec.preemptionPolicy == Never
  std::string nominated_node;    // status.nominatedNodeName
  bool preempt_terminating = false;  // PodTerminatingByPreemption
  mutable std::shared_ptr<const PodTablePre> pt_pre;  // Cluster::pod_table_precompile (same context only)
  // every request / overhead names cpu, memory or ephemeral-storage only (1), or not (0); -1: not yet
  // known.  Set by decode_pod, so a batch's pipeline check does not re-compare resource names.
  int8_t scalar_free = -1;
  // OpportunisticBatching: the pod's SignPod fragments (staging/src/k8s.io/kube-scheduler/framework/signers.go
  // and the plugins' SignPod), each a canonical text that is equal for two pods iff json.Marshal of the
  // reference's value is; Engine::sign combines them with the profile (framework.go:884-924)
  struct Sign {
    std::string sched, tols, labels, ports, na, nsel, images, vols;
    bool claims = false;
  } sign;
  // NodeDeclaredFeatures' PreFilter would not Skip: the pod needs a declared node feature
  // (component-helpers/nodedeclaredfeatures: RestartAllContainers rules, hostNetwork with hostUsers false)
  bool needs_features = false;
};
bool pod_scalar_free(const PodSpec& p);  // the check behind PodSpec::scalar_free
struct NodeImage { std::vector<std::string> names; int64_t size; };
struct NodeSpec {
  std::string name;
  StrMap labels;
  bool unschedulable = false;
  std::vector<std::array<std::string, 3>> taints;  // key, value, effect
  ResVec alloc;
  std::vector<NodeImage> images;
};
struct NamespaceSpec { std::string name; StrMap labels; };
// The objects PodTopologySpread's default constraints derive a pod's selector from
// (helper.DefaultSelector, plugins/helper/spread.go:37-95): Services and ReplicationControllers carry a
// map selector (present = non-nil), ReplicaSets and StatefulSets a metav1.LabelSelector.
enum ObjKind : int { OBJ_SERVICE = 0, OBJ_RC = 1, OBJ_RS = 2, OBJ_SS = 3 };
struct SelectorObj {
  int kind = OBJ_SERVICE;
  std::string ns, name;
  LabelSel sel;  // map selectors are sel.match (exprs empty); sel.present = selector != nil
};

bool decode_pod(const char* p, size_t n, PodSpec* out, std::string* err);
bool decode_node(const char* p, size_t n, NodeSpec* out, std::string* err);
bool decode_namespace(const char* p, size_t n, NamespaceSpec* out, std::string* err);
bool decode_selector_obj(const char* p, size_t n, SelectorObj* out, std::string* err);
int obj_kind(const std::string& kind);  // -1: not one of the four

// pod requests (component-helpers/resource/helpers.go:151-291) for the scheduler's uses
struct PodResources {
  int64_t cpu = 0, mem = 0, eph = 0;  // Requested contribution (Resource.Add semantics)
  std::vector<std::pair<std::string, int64_t>> scalar;
  int64_t nz_cpu = 0, nz_mem = 0;
  // Fit filter max-request vector (SetMaxResource) -- identical values in practice
};
// resource.PodRequests; use_status: PodResourcesOptions.UseStatusResources (CalculateResource and the
// score plugins' calculatePodResourceRequest set it, Fit's PreFilter does not: fit.go:317-325)
ResVec pod_requests(const PodSpec& p, const ResVec* non_missing, bool use_status);
PodResources calc_resources(const PodSpec& p);
// Fit's PreFilter request (computePodResourceRequest, fit.go:317-325: no status resources), in
// calc_resources' units (non-zero fields unused)
PodResources calc_fit_request(const PodSpec& p);
double go_log(double x);  // Go's math.Log (podtable.cpp)
bool tolerates(const Tol& t, const std::string& key, const std::string& value, const std::string& effect,
               bool cmp_ops);

// ===================================================================================
// config (KubeSchedulerConfiguration subset)
// ===================================================================================
struct Config {
  int pct = 100;
  bool enabled[kNumPlugins];
  int64_t weight[kNumPlugins];
  int fit_strategy = 0;
  std::vector<std::pair<std::string, int64_t>> fit_res{{"cpu", 1}, {"memory", 1}};
  std::vector<std::pair<int64_t, int64_t>> rtcr;
  std::set<std::string> ignored_res, ignored_groups;
  std::vector<std::pair<std::string, int64_t>> bal_res{{"cpu", 1}, {"memory", 1}};
  int32_t hard_weight = 1;
  bool ignore_pref_existing = false;
  bool taint_cmp_ops = false;
  bool ob_gate = true;  // featureGates.OpportunisticBatching (framework/runtime/batch.go)
  bool has_added_required = false;
  std::vector<NSTerm> added_required;
  bool has_added_pref = false;
  std::vector<std::pair<int32_t, NSTerm>> added_pref;
  // PodTopologySpreadArgs (podtopologyspread/plugin.go:104-131): defaultingType System (the v1 default,
  // defaults.go:225-229) uses systemDefaultConstraints (plugin.go:46-57); List uses defaultConstraints
  bool pts_system_defaulted = true;
  std::vector<Spread> pts_defaults;
  int device = 0;
  int loop_timing_stride = 1;  // time every k-th persistent-loop launch with HIP events (0: none)
  int timing_stride = 0;  // >0: time every k-th k_filter_score launch with HIP events (bench.py)
  bool persistent_loop = true;  // runs of node-local pods go through k_sched_loop (one launch per run)
  bool resident_loop = true;    // ksg_schedule_one of a node-local pod: a k_sched_loop launch that stays resident
                                // between calls, fed through a host-pinned pod ring ("residentLoop")
  bool agg_loop = true;         // runs of PTS/IPA pods go through k_agg_loop (with persistent_loop)
  int agg_debug = 0;            // AggView::debug (diagnostic)
  // resident loops: relay the doorbell through device memory from this many workgroups on (one PCIe poller instead
  // of G; round 6, profiles/r06d_resident_ab.txt: C2's 40 workgroups 19.8 -> 14.8 us per call, DTS's 20 27.0 -> 25.3)
  int ring_relay_min = 2;
  int first_chunk = 32;         // pods in a pipelined batch's first chunk (the host work before the first launch)
  int loop_wave_map = 0;        // k_sched_loop role-to-wave placement (kWaveMap in kernels.hip)
  bool resident_ahead = true;   // resident loops: the next pod's phase 1 ahead of its doorbell (LoopView, AggView bit 7)
  int debug_give_up_at = -1;    // diagnostic: the persistent loops give up at this pod of a run
  int loop_wg = 0;              // k_sched_loop workgroups (0: min(node units, CUs, 128))
  int loop_unit = 128;          // k_sched_loop nodes per workgroup unit: 128 (when it fits) or 256 ("loopUnit")
  // sharded: the loop's per-pod exchange device-to-device (granules over xGMI).  Default on for RCCL
  // ranks (one process per GPU); in-process groups (localGroup, one device) only when asked: their
  // loops must share the device's queues, and residency of all of them at once is not guaranteed
  int dev_exchange = -1;        // -1 default, 0 off, 1 on
  bool loop_stamps = false;     // diagnostic: per-phase s_memrealtime stamps of k_sched_loop (stderr)
  // node-sharded evaluation: this context evaluates the snapshot-order block range of `rank`
  // out of `world`; the per-pod exchanges run over RCCL (nccl_id) or in-process (local_group)
  int world = 1, rank = 0;
  std::string nccl_id, local_group;
  // a transport was configured: run the node-sharded pipeline even at worldSize 1 (tests it alone)
  bool sharded() const { return world > 1 || !nccl_id.empty() || !local_group.empty(); }
  Config();
};
bool decode_config(const char* p, size_t n, Config* c, std::string* err);
// SignPod's text for profile k (Engine::sign interns it); false: a nil signature (framework.go:884-924)
bool sign_text(const Config& k, const PodSpec& p, const PodResources& fit, std::string* out);
bool valid_ns_term(const NSTerm& t);

// ===================================================================================
// Cluster: host shadow + interning
// ===================================================================================
struct Interner {
  std::unordered_map<std::string, int32_t> ids;
  std::vector<std::string> strs;
  int32_t get(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    int32_t id = (int32_t)strs.size();
    ids.emplace(s, id);
    strs.push_back(s);
    return id;
  }
  int32_t find(const std::string& s) const {
    auto it = ids.find(s);
    return it == ids.end() ? -1 : it->second;
  }
};

struct LabelKey {
  Interner values;      // local value ids
  int32_t slot = -1;    // materialised HBM column, -1 if none
};

struct BoundPod {  // a pod in the cache (added bound or assumed)
  std::string uid, node;
  PodResources res;
  std::vector<uint32_t> port_ids;
  bool with_affinity = false;  // podWithAffinity (framework/types.go:386-389)
  int32_t slot = -1;           // pod-table slot (PTS/IPA aggregation)
  // DefaultPreemption (victim order, PDB matching, nominated-node eligibility)
  std::string name;
  int32_t priority = 0;
  bool has_start = false, preempt_terminating = false, req_anti = false;
  int64_t start_ns = 0;
};

struct NodeRec {
  NodeSpec spec;
  std::vector<std::pair<int32_t, int32_t>> labels;  // (key id, local value id)
  std::vector<uint32_t> taint_ids;
  std::vector<uint32_t> image_ids;  // sorted unique image name ids on the node
  int64_t alloc_cpu = 0, alloc_mem = 0, alloc_eph = 0, alloc_pods = 0;
  std::map<int32_t, int64_t> scalar_alloc;
  // NodeInfo.Requested / NonZeroRequested / Pods / UsedPorts
  int64_t req_cpu = 0, req_mem = 0, req_eph = 0, nz_cpu = 0, nz_mem = 0;
  int32_t num_pods = 0;
  std::map<int32_t, int64_t> scalar_req;
  std::set<uint32_t> ports;
  std::vector<std::string> pods;  // uids in NodeInfo.Pods order
  // false: a ghost NodeInfo (cache.go:442-446, 672-689) -- pods arrived before their node, or the
  // node was removed while pods remained; it holds their requests but is skipped by snapshots
  bool real = true;
  bool pre_dirty = true;  // k_preempt_seg: the node's pod segment must be rebuilt (Engine::preempt)
  // the shadow changed since the device columns were last written (a re-layout by gather keeps a
  // node's device columns only if it is not stale, Cluster::relayout_gather)
  bool stale = true;
  int32_t laid_ix = -1;     // the node's index in the device layout of epoch laid_epoch
  uint64_t laid_epoch = 0;
};

struct TaintRec { std::string key, value, effect; };
struct PortRec { std::string ip, proto; int32_t port; };
struct ImageState { int64_t size = 0; std::set<std::string> nodes; };

// device mirror buffers
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

class Cluster {
 public:
  explicit Cluster(const Config& cfg);
  ~Cluster();
  Config cfg;
  std::string err;

  // informer-fed cache events
  int upsert_namespace(const NamespaceSpec& ns);
  // Service / ReplicationController / ReplicaSet / StatefulSet listers (podtopologyspread/plugin.go:145-150)
  int upsert_object(SelectorObj&& o);
  int remove_object(int kind, const std::string& ns, const std::string& name);
  // helper.DefaultSelector (plugins/helper/spread.go:37-95) as a LabelSel: the merged Service / RC
  // selector maps in `match`, the RS / SS requirements in `exprs`; false when it is Empty()
  bool default_selector(const PodSpec& p, LabelSel* out);
  std::map<std::string, std::map<std::string, LabelSel>> services;  // namespace -> name -> selector
  std::map<std::pair<std::string, std::string>, LabelSel> owners[3];  // OBJ_RC / RS / SS by (ns, name)
  int add_node(NodeSpec&& n);
  int update_node(NodeSpec&& n);
  int remove_node(const std::string& name);
  // device_done: the HBM mirror already holds the pod (device-side AssumePod)
  // slot: the pod-table slot reserved for an assumed pod at compile time (-1: allocate one)
  // res: the pod's PodInfo.CalculateResource when the caller already has it (a compiled pod)
  int add_pod(const PodSpec& p, const std::string& uid_override = "", bool device_done = false, int32_t slot = -1,
              const std::string* node_override = nullptr, const PodResources* res = nullptr);
  int remove_pod(const std::string& uid);
  int32_t pods_with_affinity = 0;
  // DefaultPreemption's device-resident pod segments (Engine::preempt): nodes whose pods changed since
  // the segments were last built, and what decides whether the cached importance order still holds
  std::vector<std::string> pre_dirty_nodes;
  int64_t req_anti_pods = 0;              // pods with required anti-affinity terms
  int64_t nostart_pods = 0;               // pods without status.startTime (GetPodStartTime's clock)
  int64_t max_start_ns = INT64_MIN;       // latest startTime ever seen (never lowered)
  uint64_t layout_epoch() const { return laid_epoch_; }
  void mark_pre_dirty(NodeRec& r) {
    if (!r.pre_dirty) {
      r.pre_dirty = true;
      pre_dirty_nodes.push_back(r.spec.name);
    }
  }

  // UpdateSnapshot (cache.go:190-296): the snapshot's nodeInfoList order, rebuilt from
  // nodeTree.list only when a node new to the snapshot appears or one is gone; called at the start
  // of every scheduling cycle (and by the node listing)
  const std::vector<std::string>& order();
  int32_t index_of(const std::string& node) const;
  NodeRec* node(const std::string& name);
  // every value of label key `key` is on one snapshot node at most (kubernetes.io/hostname): its
  // per-domain counts are per-node counts (k_agg_loop keeps them with the node's owner)
  bool key_unique(int32_t key);

  // interning used by the compiler
  Interner label_keys;
  std::vector<LabelKey> keys;
  Interner taint_ix;
  std::vector<TaintRec> taints;
  Interner image_ix;
  std::map<std::string, ImageState> image_states;
  Interner port_ix;
  std::vector<PortRec> ports;
  Interner scalar_ix;  // extended / scalar resource columns
  std::map<std::string, NamespaceSpec> namespaces;
  std::unordered_map<std::string, BoundPod> pods;

  int32_t key_id(const std::string& k);
  Interner ns_ix;  // namespace names
  int32_t ns_id(const std::string& ns) { return ns_ix.get(ns); }
  // sorted (key id << 32 | value id) set of a label map; values are interned
  std::vector<unsigned long long> label_set(const StrMap& labels);
  void pod_table_precompile(const PodSpec& p);  // PodSpec::pt_pre (ksg_pod_compile; else at first use)
  // metav1.LabelSelectorAsSelector into an int32 program appended to *pool; false on a parse error
  // prevalidated_match: s.match is a labels.Set turned into a selector without validation
  bool compile_lsel(const LabelSel& s, const StrMap* merge_labels, std::vector<int32_t>* pool, int32_t* off,
                    bool prevalidated_match = false);

  // ---- pod table: every bound/assumed pod as (node, namespace, flags, labels) + its affinity terms
  std::vector<int32_t> pt_node, pt_ns;
  std::vector<uint32_t> pt_flags, pt_lbl_off, pt_lbl_cnt;
  std::vector<unsigned long long> pt_pool;
  std::vector<int32_t> pt_free;
  std::vector<std::vector<int32_t>> pt_terms;  // slot -> term indices
  std::vector<DTerm> tt;
  std::vector<int32_t> tt_pool, tt_free;
  std::map<int32_t, int32_t> exanti_keys, score_keys_req, score_keys_pref;  // key id -> live term count
  bool pods_dirty = true;
  // reserve a slot for `p` (node index -1 until placed); its terms go live with the slot
  int32_t pod_table_put(const PodSpec& p, int32_t node_index);
  void pod_table_drop(int32_t slot);
  // the term-pool words the last pod_table_put appended (the resident k_agg_loop's RingEntry)
  int32_t last_tpool_off = 0, last_tpool_cnt = 0;
  // slot s's pod-table entry as a RingEntry (+ labels, term-pool words, terms) into out; its size, or 0
  // when it does not fit in cap bytes or in the device arrays as they are (the table must go up again)
  size_t ring_entry(int32_t s, uint8_t* out, size_t cap) const;
  // lazy: skip the upload (keeping pods_dirty) when the device copy has room for every slot -- the
  // device-side AssumePod only writes pod_node[slot] -- and no pod of the call reads the table
  int upload_pod_table(bool lazy = false);
  // pod-table slots a pipelined batch may still take after its first launch (Engine::run_batch): the
  // device's pod_node column keeps room for them, since the loops' assumes write pod_node[slot]
  int32_t pt_headroom = 0;
  std::vector<double> log_tab;  // go math.Log(k), k < log_n
  int32_t scalar_slot(const std::string& n);  // -1 if too many distinct scalars
  uint32_t port_id(std::string ip, std::string proto, int32_t port);

  // ---- HBM mirror
  MirrorView view;
  hipStream_t stream = nullptr;
  bool layout_dirty = true;
  bool defer_relayout = false;  // ensure_label_slot only marks layout_dirty (pods in flight)
  bool mirror_suspect = false;  // device columns may hold assumes the cache lacks: rebuild all of them
  std::vector<uint32_t> node_toff_, node_ioff_;  // taint / image CSR offsets as laid out on the device
  int upload_node_static(int32_t i);  // queue an in-place node update (flushed by ensure_mirror)
  int flush_node_updates();
  std::vector<int32_t> static_dirty_;
  std::vector<uint8_t> static_queued_;
  DevBuf upd_dev_;
  int ensure_mirror(bool pods_needed = true);  // (re)build device arrays if dirty
  bool mirror_pending();  // would ensure_mirror(false) touch the device (the resident loop must stop first)
  // the next batch's AssumePods may add up to `extra` host-port ids to one node (widens the stride)
  void reserve_ports(int32_t extra);
  int32_t ports_hw_ = 0;    // largest UsedPorts set of any node so far
  int32_t ports_need_ = 0;  // port row stride the device layout must have
  // diff the device mirror (dynamic + static node columns, pod table) against the host shadow;
  // sync: run ensure_mirror first (what the next cycle does)
  int compare_mirror(bool sync, int32_t* ndiff, int32_t* first);
  int ensure_label_slot(int32_t key);        // materialise a label column
  int upload_node_dynamic(int32_t idx);      // queue one node's Requested/ports (flushed by ensure_mirror)
  int flush_node_dynamic();
  std::vector<int32_t> dyn_dirty_;
  std::vector<uint8_t> dyn_queued_;
  DevBuf dyn_dev_;
  int64_t next_start = 0;                    // Scheduler.nextStartNodeIndex
  // ksg_generation: cache mutations applied (node add / update / remove, pod add / remove -- assumes and
  // forgets included) and rebuilds of the snapshot's node list (its order may have changed)
  uint64_t events = 0, list_gen = 0;
  double taint_ids_per_node = 0, img_ids_per_node = 0;  // CSR densities (algorithmic-bytes model)
  int64_t taint_max_per_node = 0;                        // bounds k_sched_loop's raw-score granules
  int64_t alloc_bound = 0;                               // max cpu/memory allocatable seen (INT64_MAX: a negative one)

 private:
  std::vector<std::string> zones_;
  std::map<std::string, std::vector<std::string>> tree_;
  std::unordered_map<std::string, std::unique_ptr<NodeRec>> nodes_;
  std::vector<std::string> order_;  // snapshot.nodeInfoList (names)
  std::unordered_map<std::string, int32_t> index_;
  // snapshot.nodeInfoMap's names, and the events since the last UpdateSnapshot that can make it
  // rebuild the list: names added (maybe new to the map) and names removed (maybe still in it)
  std::unordered_set<std::string> snap_names_, snap_new_, snap_gone_;
  int32_t tree_nodes_ = 0;  // nodeTree.numNodes
  uint64_t node_gen_ = 1;   // bumped by every node event (key_unique's cache)
  std::unordered_map<int32_t, std::pair<uint64_t, bool>> uniq_cache_;
  int32_t slots_used_ = 0, slots_cap_ = 0;
  std::vector<DevBuf> bufs_;
  DevBuf pt_dev_[9];  // pod table / term table device arrays (own lifetime, grown geometrically)
  int grow(DevBuf& b, size_t bytes);

  void tree_add(const NodeSpec& n);
  void tree_remove(const NodeSpec& n);
  void set_node(NodeRec& r, NodeSpec&& n);  // NodeInfo.SetNode + image states
  void intern_node(NodeRec& r);
  void add_images(const NodeSpec& n);
  void remove_images(const NodeSpec& n);
  void apply_pod(NodeRec& r, const BoundPod& bp, int sign);
  void* dalloc(size_t bytes);
  void free_all();
  int upload_label_column(int32_t key);
  // node add / remove / zone move: move every unchanged node's device columns to its new index
  // (one gather per column block) instead of rebuilding the mirror; false if the layout must be
  // rebuilt (capacity grown, first layout)
  int relayout_gather(bool* done);
  uint64_t laid_epoch_ = 0;              // the device layout's epoch (NodeRec::laid_epoch)
  int32_t laid_slots_ = 0;               // label slots laid out
  size_t taint_cap_ = 0, img_cap_ = 0;   // device CSR id capacities
  DevBuf gather_dev_;                    // relayout_gather scratch
 public:
  uint64_t relayouts_full = 0, relayouts_gather = 0;  // diagnostics
};

// ===================================================================================
// Engine: pod compilation + kernel batches
// ===================================================================================
struct CompiledPod {
  std::vector<uint8_t> blob;  // PodDesc + payload, 16-byte multiple
  PodResources res;
  std::vector<uint32_t> port_ids;
  int32_t num_all = 0;        // nodes in the evaluation list
  int32_t subset_first = -1;  // for nextStart bookkeeping
  bool prefilter_reject = false;
  int32_t prefilter_code = 0, prefilter_plugin = 255;
  bool error = false;         // PreScore/Score error -> status Error, no launch
  uint32_t score_mask = 0;
  int32_t slot = -1;          // pod-table slot reserved for the assume
  bool prefilter_error = false;  // a PreFilter returned Error (PodTopologySpread selector)
  bool ipa_own_req = false;   // the pod has required (anti-)affinity terms (IPA PreFilter Skip rule)
  bool ipa_parse_error = false;  // IPA PreFilter: NewPodInfo failed -> UnschedulableAndUnresolvable
  bool topo_score_error = false; // PTS/IPA PreScore Error
  int32_t arena_words = 0;
  bool agg_ok = false;        // fits k_agg_loop's histogram placement
  int32_t own_terms = 0;      // the pod's own affinity terms (k_agg_loop's term-list bound)
  int32_t sig = -1;           // OpportunisticBatching: the interned SignPod signature (-1: nil)
};
struct Blob;
class Comm;

class Engine {
 public:
  explicit Engine(Cluster* c);
  ~Engine();
  Cluster* c;
  std::unordered_map<int32_t, PodSpec> queue;  // handle -> compiled-for-API pod (find / insert / erase only)
  std::unordered_map<int32_t, std::string> assumed;  // handle -> uid
  // the nominator (ksg_add_nominated_pod): pod uid -> (nominated node name, spec.priority)
  std::unordered_map<std::string, std::pair<std::string, int32_t>> nominated;
  // KSG_ENOTSUP (+ err) when a pod of the call would see another pod's nomination of equal or higher priority on a
  // snapshot node (RunFilterPluginsWithNominatedPods, not run here)
  int check_nominations(const std::vector<const PodSpec*>& pods);
  int32_t next_handle = 1;

  enum Mode { CYCLE, FILTER_ONE, SCORE_ONE };
  // compile `p` for the current cluster; rot_start from Cluster::next_start
  int compile(const PodSpec& p, Mode mode, int plugin, bool assume, bool eval, CompiledPod* out,
              const uint8_t* node_list = nullptr);
  double cprof_[8] = {};  // loopStamps: compile time per section (us), reported with the host line
  std::chrono::steady_clock::time_point api_t0_{};  // loopStamps: ksg_schedule_batch entry
  double reserve_us_ = 0;
  double mirror_us_ = 0;    // loopStamps: ensure_mirror before the batch's first launch (us)
  double c0_us_[3] = {};    // loopStamps: chunk 0's plan + scalar check, program vectors, compile (us)
  int compile_topology(const PodSpec& p, Mode mode, int plugin, int32_t N, Blob* B, PodDesc* D, uint32_t* fmask,
                       uint32_t* smask, CompiledPod* out);
  // run a batch of cycles (device-resident, sequential semantics)
  int run_batch(const std::vector<const PodSpec*>& pods, const std::vector<int32_t>& handles, bool assume,
                ksg_result* results, ksg_eval_out* eval);
  // run_batch, and for an in-process rank group whose persistent loop gave up (its ranks' loops could not all
  // be resident at once: HIP gives no control over which hardware queue a stream lands on), the pods from the
  // failed chunk on once more over the all-reduce path
  int run_batch_api(const std::vector<const PodSpec*>& pods, const std::vector<int32_t>& handles, bool assume,
                    ksg_result* results, ksg_eval_out* eval);
  int fault_first_ = -1;        // the first pod loop_fault left unscheduled (-1: none), for run_batch_api
  bool force_allreduce_ = false;  // run_batch_api's retry: no device exchange
  uint64_t loop_retries_ = 0;   // batches run_batch_api re-ran over the all-reduce path
  uint64_t loop_give_ups_ = 0;  // batches whose persistent loop gave up (forced ones included)
  int run_plugin(const PodSpec& p, Mode mode, int plugin, const uint8_t* nodes, int32_t* code, uint8_t* codes,
                 uint32_t* reasons, int64_t* raw, int64_t* norm);
  // DefaultPreemption's PostFilter for a pod that failed its cycle (preempt.cpp)
  int preempt(const PodSpec& p, const char* args_json, size_t args_len, ksg_preempt_result* res, std::string* detail);
  // The resident single-pod loop: ksg_schedule_one of a node-local pod through a
  // k_sched_loop launch that stays resident between calls; *handled false: the caller takes the launch path
  int schedule_resident(const PodSpec& p, int32_t handle, ksg_result* res, bool* handled);
  int resident_stop();  // end the resident launch: every other user of the device or the mirror calls it first

  // measurement: average k_filter_score duration (sampled with events when cfg.timing_stride > 0,
  // else the batch's kernel time / launches) and its algorithmic bytes per launch
  double algo_bytes(const PodDesc& d) const;
  double agg_bytes(const PodDesc& d) const;  // the pod-table pass of an aggregating pod
  double last_kernel_ms = 0, last_bytes = 0;
  int32_t last_launches = 0;
  int32_t last_kernel = 0;  // 0: k_filter_score figures; 1: k_sched_loop (per-pod time in the loop)
  int cu_count = 0;
  // workgroups of each persistent loop a CU holds at once (loop_occupancy: [0] k_sched_loop 128-node
  // unit, [1] 256-node unit, [2] k_agg_loop, [3] node-sharded k_agg_loop); a loop's whole grid -- all
  // ranks' grids for in-process groups, which share the device -- must fit in cu_count * that
  int loop_occ[4] = {0, 0, 0, 0};
  bool loop_ok(const CompiledPod& p) const;
  bool loop_bounds_ok(const CompiledPod& p) const;  // the loops' granule payload bounds
  bool agg_loop_ok(const CompiledPod& p) const;
  // node-sharded evaluation (cfg.world > 1): this rank's block range + the exchange transport
  std::unique_ptr<Comm> comm;
  int32_t next_slot_ = -1;  // compile(): a pod-table slot reserved by run_batch's pipeline
  hipStream_t cstream = nullptr;    // run_batch's copy stream (pipelined chunks' H2D / D2H)
  std::vector<hipEvent_t> pev;      // its per-chunk staged / finished events
  // nextStartNodeIndex advances by a data-dependent count (percentageOfNodesToScore < 100, or
  // numNodesToFind = 1 without score plugins): it is kept on the device across a batch
  bool rotdev() const;
  // OpportunisticBatching (framework/runtime/batch.go:31-242): the profile signs pods
  // (the gate is on and PodTopologySpread has no default constraints, plugin.go:92-102)
  bool ob_acting() const;
  int32_t sign(const PodSpec& p, const PodResources& fit);  // SignPod, interned; -1: nil
  int ob_sequence(CompiledPod& cp, const PodSpec& p, int64_t now);  // the cycle's count, clock, hint permission
  int ob_sync(hipStream_t s);      // device state allocated; node indices remapped after a list rebuild
  void ob_invalidate();            // after a device fault: no hint from a state the fault may have torn
  int64_t ob_now();                // time.Now() of one scheduling cycle (ksg_set_clock, else the wall clock)
  int64_t ob_clock_ = 0;
  int64_t ob_clock_step_ = 0;      // ksg_debug_clock_step: the fixed clock advances by this per cycle
  bool nom_batch_ = false;         // this batch holds a pod with status.nominatedNodeName (rotdev: its outcome
                                   // moves nextStartNodeIndex on the device)
  int64_t ob_cycle_ = 0;           // SchedulingCycle(): one per scheduling cycle of this context
  int32_t ob_prev_sig_ = -1;       // the previous cycle's signature (-1: nil, or no previous cycle)
  uint64_t ob_list_gen_ = 0;       // the node-list generation the device state's indices refer to
  std::vector<std::string> ob_order_;  // the snapshot order of that generation (for the remap)
  std::unordered_map<std::string, int32_t> ob_sigs_;
  uint64_t ob_hinted_ = 0;         // pods placed by a hint (diagnostic)
  int32_t shard_blk0 = 0, shard_nblk = -1;
  void shard_range(int32_t n, int32_t* blk0, int32_t* nblk) const;

 private:
  // per-batch device scratch
  DevBuf d_descs, d_status, d_fmask, d_blk, d_fixed, d_raw, d_out, d_total;
  DevBuf d_ob, d_ob_heap, d_ob_map;      // OpportunisticBatching: ObState, ObEnt[cap], the remap
  DevBuf d_meta;                         // owns the three views below (ensure_scratch)
  DevBuf d_off, d_stats, d_results;      // views: program offsets + sizes, PodStats, DevResult
  DevBuf d_arena;  // PTS/IPA histograms; kept all-zero between pods (k_select re-zeroes what it used)
  DevBuf d_xa, d_xp, d_xb, d_xs;  // node-sharded exchange vectors, one set per pod of the batch
  DevBuf d_evg;             // node-sharded evaluation output, gathered over the ranks
  DevBuf d_gran, d_fail, d_stamps;  // k_sched_loop: exchange granules (local), give-up flag, stamps
  uint64_t assume_seq_ = 0;  // assumed pods' cache uids: "<uid>#a<n>", n counted per context
  DevBuf d_grp;  // in-process groups, the leader's: every rank's loop launch arguments (group_launch)
  // one rank's part of an in-process group's loop dispatch (Comm::group_launch): its arguments, its timing events
  struct GroupReq {
    LoopGroupArg la;
    AggGroupArg aa;
    hipEvent_t t0, t1;
  };
  int group_launch(GroupReq* req, bool agg, int nwg, int unit);
  std::vector<unsigned long long*> gran_all;  // every rank's granule array as mapped here ([rank] = d_gran)
  uint32_t gran_tag = 0;
  DevBuf d_agran, d_region;  // k_agg_loop: exchange granules, per-pod shared regions (fixed size once set up)
  std::vector<unsigned long long*> agran_all, region_all;  // every rank's, as mapped here (node-sharded)
  DevBuf d_aggpeers;  // node-sharded k_agg_loop: the device copy of agran_all + region_all
  DevBuf d_astamps;          // k_agg_loop diagnostic stamps
  DevBuf d_relay;            // the resident k_agg_loop's relayed doorbell and staging (AggView::relay)
  DevBuf d_aspill;           // k_agg_loop: workgroup pod / term lists past the LDS ones (AggView::spill)
  DevBuf d_pre;              // k_preempt: per-node records, victims, per-node results, victim flags
  // k_preempt_seg: every node's pods as an importance-ordered segment (host copy + identities)
  DevBuf d_seg, d_segcnt, d_psout, d_pdb, d_pick, d_contrib_buf, d_wide;
  DevBuf d_vsc;  // preemption: the pods' requests of the preemptor's extended resources + the per-node scratch
  std::vector<PRec> h_seg;
  std::vector<int32_t> h_segcnt;
  std::vector<std::vector<const BoundPod*>> seg_pods;
  uint64_t seg_epoch = ~0ull;
  std::vector<uint8_t> seg_flags;  // per node: bit 0 more than kSegCap pods, bit 1 a pod with > 2 host ports
  int32_t seg_n = -1, seg_overflow = 0, seg_many_ports = 0;
  void seg_build(int32_t i, NodeRec& r);
  int seg_refresh();
  int gran_setup();
  int agg_setup();
  int next_gran_tag(uint32_t* tag);
  std::vector<hipEvent_t> lev;  // k_sched_loop timing events (pairs)
  std::vector<hipEvent_t> cev;  // run_batch pipeline: one event per chunk (results landed)
  int run_sharded(const std::vector<CompiledPod>& cp, const BatchView& bv, int first, int last, int* launches,
                  double* bytes, int* timed);
  void* h_pinned = nullptr;
  size_t h_pinned_bytes = 0;
  // k_agg_loop's template cache: the slots (kAggTc per workgroup) and the per-pod plan (TcWord), pinned + device
  DevBuf d_tcache, d_tcw;
  uint32_t* h_tcw = nullptr;
  size_t h_tcw_n = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> tev;  // sampled k_filter_score timing events (pairs)
  int ensure(DevBuf& b, size_t bytes);
  int ensure_scratch(size_t desc_bytes, int pods, bool eval, int32_t arena_words);
  BatchView bview(int pods);
  PodRing* ring_ = nullptr;       // the resident loop's pod ring (host-pinned, device-mapped)
  PodRing* ring_dev_ = nullptr;   // its device address
  bool res_running_ = false;
  int res_q_ = 0, res_gs_ = 0, res_unit_ = 0;  // pods posted to the running launch; its geometry
  std::vector<uint8_t> res_prev_blob_, res_prev_entry_;  // k_agg_loop ring: the program / entry posted last
  long res_posts_[12] = {};  // k_agg_loop ring posts: same, RING_TERMS, staged (+ ring_terms_patch's why) (loopStamps)
  int res_kind_ = 0;              // the running launch: 1 k_sched_loop, 2 k_agg_loop (pod-table pods)
  int64_t res_terms_ = 0;         // k_agg_loop: own affinity terms of the pods posted (its spill rows' budget)
  std::chrono::steady_clock::time_point res_last_{};  // the last result the host took
  double res_prof_[5] = {};       // loopStamps: compile / post / device / settle us, calls
};

}  // namespace ksg
