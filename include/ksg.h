/*
 * ksg.h -- C ABI of the MI355X-native kube-scheduler node-evaluation path.
 *
 * This is the drop-in boundary for the per-pod hot path of kube-scheduler:
 *   PreFilter -> Filter -> PreScore -> Score -> NormalizeScore -> weight/sum -> host selection
 * as driven by Scheduler.schedulePod (pkg/scheduler/schedule_one.go:564-618),
 * findNodesThatFitPod (schedule_one.go:622-712), findNodesThatPassFilters (:771-854),
 * prioritizeNodes (:937-1048) and the nodeScoreHeap pop (:1050-1098), followed by
 * Scheduler.assume (:1102-1137) -> Cache.AssumePod (backend/cache/cache.go:397).
 *
 * Objects cross the boundary as the Kubernetes JSON encoding of v1.Node / v1.Pod /
 * v1.Namespace (what `json.Marshal` of the client-go object produces), so the Go side
 * of a cgo shim needs no hand-written marshalling of the scheduler types.  Everything
 * else is plain pointers + sizes; no torch / HIP types appear in any signature.
 *
 * Error convention (mirrors fwk.Status, staging/src/k8s.io/kube-scheduler/framework/
 * interface.go:43-80,130-135): functions return 0 (KSG_OK) on success and a negative
 * KSG_E* value on failure; ksg_last_error() returns the message.  A scheduling
 * outcome (Unschedulable, UnschedulableAndUnresolvable, plugin Error) is not an ABI
 * failure: it is reported in ksg_result.status with the fwk.Code numbering.
 *
 * Threading: one context per scheduling goroutine, not thread-safe -- exactly as
 * ScheduleOne is serialised (schedule_one.go:65-66, scheduler.go:538).
 */
#ifndef KSG_H_
#define KSG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSG_ABI_VERSION 2 /* 2: ksg_eval_out.normalized_scores */

/* ---- return codes of the ABI functions ------------------------------------------ */
#define KSG_OK 0
#define KSG_EINVAL (-1)   /* malformed JSON / object / argument */
#define KSG_ENOTFOUND (-2) /* unknown node / pod / handle */
#define KSG_EEXIST (-3)   /* object already present */
#define KSG_EDEVICE (-4)  /* HIP / RCCL failure */
#define KSG_ENOTSUP (-5)  /* feature outside the supported parity contract */
#define KSG_ENOMEM (-6)

/* ---- fwk.Code (interface.go:46-99) ----------------------------------------------- */
#define KSG_CODE_SUCCESS 0
#define KSG_CODE_ERROR 1
#define KSG_CODE_UNSCHEDULABLE 2
#define KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE 3
#define KSG_CODE_WAIT 4
#define KSG_CODE_SKIP 5
#define KSG_CODE_PENDING 6

/* ---- in-tree plugins on the hot path (names.go); ids index every per-plugin array ---
 * Filter order = pkg/scheduler/apis/config/testing/defaults/defaults.go:84-101
 * (volume/DRA/NodeDeclaredFeatures plugins Skip for the pods of the parity contract).
 * Score order  = defaults.go:119-143. */
#define KSG_PLUGIN_NODE_UNSCHEDULABLE 0
#define KSG_PLUGIN_NODE_NAME 1
#define KSG_PLUGIN_TAINT_TOLERATION 2
#define KSG_PLUGIN_NODE_AFFINITY 3
#define KSG_PLUGIN_NODE_PORTS 4
#define KSG_PLUGIN_NODE_RESOURCES_FIT 5
#define KSG_PLUGIN_POD_TOPOLOGY_SPREAD 6
#define KSG_PLUGIN_INTER_POD_AFFINITY 7
#define KSG_PLUGIN_BALANCED_ALLOCATION 8
#define KSG_PLUGIN_IMAGE_LOCALITY 9
#define KSG_NUM_PLUGINS 10
#define KSG_PLUGIN_NONE 255

/* ---- failure reason bits (one bit per distinct upstream reason string) ------------- */
#define KSG_R_UNSCHEDULABLE (1u << 0)        /* "node(s) were unschedulable" */
#define KSG_R_NODE_NAME (1u << 1)            /* "node(s) didn't match the requested node name" */
#define KSG_R_TAINT (1u << 2)                /* "node(s) had untolerated taint(s)" */
#define KSG_R_NODE_AFFINITY_POD (1u << 3)    /* "node(s) didn't match Pod's node affinity/selector" */
#define KSG_R_NODE_AFFINITY_ENFORCED (1u << 4)/* "node(s) didn't match scheduler-enforced node affinity" */
#define KSG_R_NODE_PORTS (1u << 5)           /* "node(s) didn't have free ports for the requested pod ports" */
#define KSG_R_TOO_MANY_PODS (1u << 6)        /* "Too many pods" */
#define KSG_R_INSUFFICIENT_CPU (1u << 7)     /* "Insufficient cpu" */
#define KSG_R_INSUFFICIENT_MEMORY (1u << 8)  /* "Insufficient memory" */
#define KSG_R_INSUFFICIENT_EPHEMERAL (1u << 9)/* "Insufficient ephemeral-storage" */
#define KSG_R_INSUFFICIENT_SCALAR (1u << 10) /* "Insufficient <extended resource>" (any) */
#define KSG_R_PTS_MISSING_LABEL (1u << 11)   /* "...topology spread constraints (missing required label)" */
#define KSG_R_PTS_SKEW (1u << 12)            /* "node(s) didn't match pod topology spread constraints" */
#define KSG_R_IPA_AFFINITY (1u << 13)        /* "node(s) didn't match pod affinity rules" */
#define KSG_R_IPA_ANTI_AFFINITY (1u << 14)   /* "node(s) didn't match pod anti-affinity rules" */
#define KSG_R_IPA_EXISTING_ANTI (1u << 15)   /* "node(s) didn't satisfy existing pods anti-affinity rules" */
#define KSG_R_PREFILTER (1u << 16)           /* node rejected by a PreFilter status / PreFilterResult */

typedef struct ksg_ctx ksg_ctx;

/* ScheduleResult (schedule_one.go:613-617) + the FitError/Error outcome. */
typedef struct ksg_result {
  int32_t status;          /* KSG_CODE_SUCCESS, or the code of the FitError/Error */
  int32_t node_index;      /* snapshot index of SuggestedHost, -1 if none */
  int32_t evaluated_nodes; /* ScheduleResult.EvaluatedNodes */
  int32_t feasible_nodes;  /* ScheduleResult.FeasibleNodes */
  int64_t total_score;     /* TotalScore of the chosen node (0 if F <= 1) */
} ksg_result;

/* Full per-node view of one cycle, used by parity tests, diagnosis rebuilding
 * (Diagnosis.NodeToStatus, framework/types.go:1082-1180; NodePluginScores,
 * interface.go:284-295) and the plugin-level shim.  All arrays are
 * caller-owned, sized for ksg_num_nodes() (and KSG_NUM_PLUGINS x num_nodes for
 * plugin_scores / normalized_scores), indexed by snapshot index; any may be NULL.
 * normalized_scores is what a ScorePlugin's Score + NormalizeScore hand RunScorePlugins
 * (framework.go:1351-1423): in [0, 100] for every plugin in score_plugin_mask;
 * plugin_scores is that value times the profile weight (framework.go:1434-1446), and
 * total_scores their sum -- NodePluginScores.TotalScore. */
typedef struct ksg_eval_out {
  int32_t prefilter_code;    /* non-success PreFilter status code (0 if PreFilter passed) */
  int32_t prefilter_plugin;  /* plugin that produced it, KSG_PLUGIN_NONE otherwise */
  uint8_t *node_code;        /* [N] fwk.Code of the node's Filter status (0 = feasible) */
  uint8_t *node_plugin;      /* [N] first failing Filter plugin, KSG_PLUGIN_NONE if feasible */
  uint32_t *node_reasons;    /* [N] KSG_R_* bits of that status */
  uint32_t score_plugin_mask;/* out: bit p set if score plugin p ran (not skipped) */
  int64_t *plugin_scores;    /* [KSG_NUM_PLUGINS][N] weighted normalised score (feasible nodes) */
  int64_t *total_scores;     /* [N] TotalScore (feasible nodes; 0 elsewhere) */
  int64_t *normalized_scores;/* [KSG_NUM_PLUGINS][N] normalised score before the weight (ABI 2) */
} ksg_eval_out;

/* ---- context ------------------------------------------------------------------------
 * config_json mirrors the KubeSchedulerConfiguration subset that shapes this path
 * (staging/src/k8s.io/kube-scheduler/config/v1/types.go:44-160, defaults.go):
 *   {"percentageOfNodesToScore": 100,
 *    "scoreWeights": {"TaintToleration":3, ...},           (default_plugins.go:35-50)
 *    "disabledPlugins": ["ImageLocality", ...],
 *    "nodeResourcesFit": {"scoringStrategy": {"type": "LeastAllocated",
 *                         "resources": [{"name":"cpu","weight":1}, ...],
 *                         "requestedToCapacityRatio": {"shape": [...]}},
 *                         "ignoredResources": [], "ignoredResourceGroups": []},
 *    "balancedAllocation": {"resources": [...]},
 *    "interPodAffinity": {"hardPodAffinityWeight": 1, "ignorePreferredTermsOfExistingPods": false},
 *    "nodeAffinity": {"addedAffinity": <v1.NodeAffinity>},
 *    "podTopologySpread": {"defaultingType": "System" | "List",     (PodTopologySpreadArgs)
 *                          "defaultConstraints": [<v1.TopologySpreadConstraint without labelSelector>]},
 *    "device": 0, "distributed": {"worldSize": 1, "rank": 0, "ncclId": "<hex>"}}
 * Absent keys take the upstream defaults.  Returns NULL on failure (ksg_create_error()). */
ksg_ctx *ksg_create(const char *config_json, size_t len);
const char *ksg_create_error(void);
void ksg_destroy(ksg_ctx *ctx);
const char *ksg_last_error(const ksg_ctx *ctx);

/* ---- cluster-state mirror: replaces the Cache event methods that feed the snapshot
 * (backend/cache/cache.go:515-695, eventhandlers.go:51-412).  Snapshot node order is
 * the nodeTree zone round-robin order (node_tree.go:119-143). */
int ksg_upsert_namespace(ksg_ctx *ctx, const char *ns_json, size_t len);
/* The listers PodTopologySpread's default constraints read (podtopologyspread/plugin.go:145-150,
 * helper.DefaultSelector in plugins/helper/spread.go:37-95): a v1 Service or ReplicationController,
 * or an apps/v1 ReplicaSet or StatefulSet, as JSON (kind, metadata.namespace/name, spec.selector).
 * Upsert replaces the object of that kind, namespace and name; remove takes the kind name
 * ("Service", "ReplicationController", "ReplicaSet", "StatefulSet").  A pod without constraints of
 * its own then gets the profile's default constraints (System: kubernetes.io/hostname maxSkew 3 and
 * topology.kubernetes.io/zone maxSkew 5, ScheduleAnyway) with the merged selector of the objects that
 * select it (common.go:59-75). */
int ksg_upsert_object(ksg_ctx *ctx, const char *obj_json, size_t len);
int ksg_remove_object(ksg_ctx *ctx, const char *kind, const char *ns, const char *name);
int ksg_add_node(ksg_ctx *ctx, const char *node_json, size_t len);
int ksg_update_node(ksg_ctx *ctx, const char *node_json, size_t len);
int ksg_remove_node(ksg_ctx *ctx, const char *name);
int ksg_add_pod(ksg_ctx *ctx, const char *pod_json, size_t len); /* bound: spec.nodeName set */
int ksg_remove_pod(ksg_ctx *ctx, const char *uid);
int ksg_num_nodes(const ksg_ctx *ctx);
/* name of the node at snapshot index `index`; returns its length or a KSG_E* code */
int ksg_node_name(const ksg_ctx *ctx, int32_t index, char *buf, size_t cap);

/* ---- pods to schedule: compiled once, like PodInfo creation (framework/types.go:1183).
 * KSG_ENOTSUP: the pod needs a plugin outside the device path -- a PersistentVolumeClaim, generic
 * ephemeral, CSI-migratable in-tree (GCE PD, AWS EBS, Cinder, Azure Disk/File, vSphere, Portworx), RBD
 * or iSCSI volume (VolumeBinding, VolumeZone, NodeVolumeLimits, VolumeRestrictions) or
 * spec.resourceClaims (DynamicResources), or a declared node feature (NodeDeclaredFeatures: a container
 * restartPolicyRules action RestartAllContainers, or hostNetwork with hostUsers false).  The context is
 * unaffected; such pods stay with the caller's own scheduling path. */
int ksg_pod_compile(ksg_ctx *ctx, const char *pod_json, size_t len, int32_t *handle);
int ksg_pod_release(ksg_ctx *ctx, int32_t handle);

/* ---- scheduling cycles -------------------------------------------------------------- */
#define KSG_FLAG_ASSUME 1u /* on success, AssumePod the pod onto the chosen node */

/* One cycle; `eval` may be NULL.  Replaces schedulePod for one pod. */
int ksg_schedule_one(ksg_ctx *ctx, int32_t handle, uint32_t flags, ksg_result *result,
                     ksg_eval_out *eval);
/* n cycles in queue order with sequential semantics: pod i sees the assumes of pods
 * 0..i-1 (KSG_FLAG_ASSUME).  The whole batch runs device-resident. */
int ksg_schedule_batch(ksg_ctx *ctx, const int32_t *handles, int32_t n, uint32_t flags,
                       ksg_result *results);
/* Cache.ForgetPod (cache.go:412) of an assumed pod -- unreserveAndForget (schedule_one.go:358) */
int ksg_forget(ksg_ctx *ctx, int32_t handle);

/* ---- the scheduling queue's nominator (backend/queue/nominator.go) -------------------
 * Pods nominated to a node and waiting for it (PostFilter's NominatingInfo, status.nominatedNodeName).
 * ksg_add_nominated_pod: PodNominator.AddNominatedPod / UpdateNominatedPod of pod_json -- its uid is nominated
 * to its status.nominatedNodeName with its spec.priority, replacing an earlier nomination of the uid (none: the
 * uid is forgotten).  ksg_delete_nominated_pod: DeleteNominatedPodIfExists (also done by every assume of the uid
 * through this context, schedule_one.go:1131-1134).  A pod's own nomination is evaluateNominatedNode (the pod
 * tries that node alone first).  OTHER pods' nominations change a pod's Filter: RunFilterPluginsWithNominatedPods
 * (framework.go:1211-1294) adds every pod of equal or higher priority nominated to a node before filtering it,
 * which this library does not run -- ksg_schedule_one / ksg_schedule_batch / ksg_preempt return KSG_ENOTSUP,
 * scheduling nothing, when a pod of the call has such a nomination on a snapshot node besides its own. */
int ksg_add_nominated_pod(ksg_ctx *ctx, const char *pod_json, size_t len);
int ksg_delete_nominated_pod(ksg_ctx *ctx, const char *uid);

/* ---- OpportunisticBatching (framework/runtime/batch.go:31-242) ----------------------
 * With featureGates.OpportunisticBatching on (the default) and a profile whose PodTopologySpread has no
 * default constraints (disabled, or {"defaultingType": "List", "defaultConstraints": []}), pods get a
 * SignPod signature (framework.go:884-924); a signed pod whose previous cycle in this context was a pod of
 * the same signature that left a sorted node list less than 500 ms ago (maxBatchAge) is placed on that
 * list's next node when the last chosen node rejects it and the hinted node passes every filter
 * (GetNodeHint, evaluateNominatedNode: schedule_one.go:650-668,718-752) -- ksg_result.evaluated_nodes 1,
 * feasible_nodes 1, no scores; else it runs the full cycle and stores its own list (StoreScheduleResults).
 * Every pod of a ksg_schedule_one / ksg_schedule_batch call is one scheduling cycle (SchedulingCycle()),
 * and each cycle reads the clock when it starts (batch.go:202): ksg_set_clock(ctx, now_ns) makes it now_ns (a
 * caller's time.Now(), nanoseconds), 0 the wall clock (CLOCK_MONOTONIC); ksg_debug_clock_step(ctx, step_ns)
 * advances that fixed clock by step_ns per cycle (a test's clock that moves inside one call).  A node-sharded
 * context refuses such a profile at ksg_create.  ksg_debug_batching: pods placed by a hint so far, and the
 * cycles counted. */
int ksg_set_clock(ksg_ctx *ctx, int64_t now_ns);
int ksg_debug_clock_step(ksg_ctx *ctx, int64_t step_ns);
int ksg_debug_batching(const ksg_ctx *ctx, uint64_t *hinted, uint64_t *cycles);

/* ---- plugin-granular entry points ---------------------------------------------------
 * The FilterPlugin contract of one plugin over every snapshot node: its PreFilter
 * (interface.go:513-532) then Filter (interface.go:542-567) per node.  *prefilter_code
 * gets the PreFilter status (KSG_CODE_SKIP: the Filter did not run; codes are all 0).
 * codes[N] / reasons[N] receive each node's Filter status. */
int ksg_run_filter_plugin(ksg_ctx *ctx, int32_t handle, int32_t plugin, int32_t *prefilter_code,
                          uint8_t *codes, uint32_t *reasons);
/* The ScorePlugin + ScoreExtensions contract of one plugin: PreScore (interface.go:598-606)
 * over the node list, Score per listed node (:619-628) into raw[N], NormalizeScore
 * (:609-614) over the list into normalized[N] (unweighted).  The list is the snapshot nodes
 * with nodes[i] != 0 (nodes == NULL: every node) -- the feasible list prioritizeNodes would
 * pass; unlisted entries stay 0.  *status_code gets the PreScore status (KSG_CODE_SKIP: not
 * scored) or a Score error. */
int ksg_run_score_plugin(ksg_ctx *ctx, int32_t handle, int32_t plugin, const uint8_t *nodes,
                         int32_t *status_code, int64_t *raw, int64_t *normalized);

/* ---- DefaultPreemption PostFilter ------------------------------------------
 * Replaces Evaluator.Preempt (framework/preemption/preemption.go:103-170) for a pod whose cycle
 * ended in a FitError: PodEligibleToPreemptOthers (default_preemption.go:364-388), findCandidates
 * (preemption.go:174-196), DryRunPreemption -- SelectVictimsOnNode (default_preemption.go:252-354)
 * per node, on the device -- and SelectCandidate / pickOneNodeForPreemption (preemption.go:262-397).
 * The call only selects: deleting the victims and setting status.nominatedNodeName (executor.go)
 * stay with the caller, whose informer events later remove the victims (ksg_remove_pod).
 * args_json (NULL: defaults):
 *   {"offset": <int>,        GetOffsetAndNumCandidates' random offset (rand.Int31n upstream), taken
 *                            modulo the number of potential nodes
 *    "minCandidateNodesPercentage": 10, "minCandidateNodesAbsolute": 100,   (DefaultPreemptionArgs)
 *    "now": <unix ns>,       GetPodStartTime's clock for pods without status.startTime (utils.go:52-58;
 *                            absent: the wall clock, time.Now() as upstream)
 *    "allNodes": false,      true: every snapshot node is a potential node (DryRunPreemption over
 *                            the node list, as the reference's unit tests call it)
 *    "listCandidates": false, true: detail lists every candidate (else "candidates" is empty)
 *    "pdbs": [<policy/v1 PodDisruptionBudget JSON>, ...]}
 * Potential nodes are taken in snapshot order (the reference iterates a map there) and checked with
 * Parallelizer parallelism 1 semantics; victims of equal priority and start time keep NodeInfo.Pods
 * order; candidates tied on every criterion resolve to the earliest in candidate-list order.
 * The device re-evaluates a victim's removal for NodeResourcesFit (every requested resource, extended
 * ones included), NodePorts and the pod's PodTopologySpread / InterPodAffinity counts (RemovePod /
 * AddPod extensions, filtering.go:157-212 / interpodaffinity/filtering.go:75-85), on both device paths
 * (the resident pod segments, and host-staged records for nodes of more than 128 pods, more than two
 * host ports per pod, more than 8 budgets, or a "now" earlier than a bound pod's start time).
 * Any number of spread constraints, affinity terms and existing-anti-affinity keys the pod compiler
 * accepts is tracked (up to 8 of each kind in registers, more in a per-node device workspace).
 * detail (may be NULL) receives NUL-terminated JSON: {"offset", "numCandidates",
 * "potential", "message", "candidates": [{"node", "numPDBViolations", "victims": [uid...]}] (listCandidates),
 * "selected": <node|null>, "victims": [uid...]}; *detail_len gets its length (KSG_ENOMEM if cap is
 * too small; the result is still filled). */
#define KSG_PREEMPT_OK 0            /* a node was nominated */
#define KSG_PREEMPT_NOT_ELIGIBLE 1  /* PodEligibleToPreemptOthers said no (PreemptionPolicy, terminating victims) */
#define KSG_PREEMPT_NO_CANDIDATES 2 /* "preemption is not helpful for scheduling" */
typedef struct ksg_preempt_result {
  int32_t status;             /* KSG_CODE_SUCCESS (a node was nominated) or KSG_CODE_UNSCHEDULABLE */
  int32_t reason;             /* KSG_PREEMPT_* */
  int32_t node_index;         /* snapshot index of the nominated node, -1 if none */
  int32_t num_potential;      /* nodes findCandidates passed to DryRunPreemption */
  int32_t num_candidates;     /* candidates DryRunPreemption returned */
  int32_t num_victims;        /* victims on the nominated node */
  int64_t num_pdb_violations; /* Victims.NumPDBViolations of the nominated node */
} ksg_preempt_result;
int ksg_preempt(ksg_ctx *ctx, int32_t handle, const char *args_json, size_t args_len, ksg_preempt_result *result,
                char *detail, size_t detail_cap, size_t *detail_len);

/* ---- node-sharded evaluation ---------------------------------------------
 * A context created with {"distributed": {"worldSize": W, "rank": r, "ncclId": "<hex>"}}
 * holds the whole cluster mirror (every rank is fed the same informer events) and evaluates
 * the nodes of its contiguous range of the snapshot order; per pod, RCCL all-reduces carry the
 * feasible counts, the NormalizeScore maxima/minima (framework.go:1409-1423) and every rank's
 * best (TotalScore, heap pre-order key, node) -- the argmax of selectHost (schedule_one.go:
 * 1054-1085) -- so every rank returns the identical ScheduleResult and applies the identical
 * AssumePod.  ksg_create is collective across the W ranks (ncclCommInitRank).  With
 * "localGroup": "<name>" instead of ncclId, W contexts in ONE process on one device form the
 * group (each driven by its own thread); used to test the sharded path on one GPU.
 * ksg_comm_unique_id writes ncclGetUniqueId as 256 hex characters + NUL (rank 0 calls it and
 * hands it to the other ranks) and returns the length. */
int ksg_comm_unique_id(char *buf, size_t cap);
/* first snapshot index and count of the nodes this rank evaluates */
int ksg_shard_range(const ksg_ctx *ctx, int32_t *first_node, int32_t *num_nodes);

/* Measurement of the last batch (bench.py): *kernel 0 -> the average k_filter_score duration
 * (HIP events on the dispatch packets) and its algorithmic bytes per launch; *kernel 1 -> most
 * pods ran in the persistent k_sched_loop: its duration per pod and algorithmic bytes per pod;
 * *kernel 2 -> the same for k_agg_loop (pods with PodTopologySpread / InterPodAffinity counts).
 * *launches: the k_filter_score launches, or the pods the dominant loop kernel ran. */
int ksg_last_batch_kernel_stats(const ksg_ctx *ctx, double *avg_kernel_ms,
                                double *bytes_per_launch, int32_t *launches, int32_t *kernel);

/* Recovery diagnostic: diffs the device mirror -- every node's Requested, NonZeroRequested, pod
 * count, allocatable, unschedulable flag and host ports, and the pod table's node index per slot --
 * against the host cache shadow it is uploaded from (the NodeInfo fields of framework/types.go:
 * 172-220 that AssumePod changes, cache.go:365-380).  sync != 0 first does what the next scheduling
 * cycle does (re-upload a mirror marked stale, e.g. after a persistent-loop give-up returned
 * KSG_EDEVICE).  *ndiff: differing nodes + pod-table slots, -1 if no mirror is laid out for the
 * current snapshot; *first: the first differing snapshot index (n + slot for a pod-table slot), -1. */
int ksg_debug_compare_mirror(ksg_ctx *ctx, int32_t sync, int32_t *ndiff, int32_t *first);

/* Mirror-ingestion diagnostic: how many times the HBM mirror was rebuilt from the cache (*full) and
 * how many node adds / removes / zone moves were applied by moving the unchanged nodes' columns on
 * the device instead (*gather; UpdateSnapshot's list rebuild, cache.go:273-283). */
int ksg_debug_relayouts(const ksg_ctx *ctx, uint64_t *full, uint64_t *gather);

/* Persistent-loop health: *give_ups counts the batches whose persistent loop gave up (an exchange granule
 * never arrived within 10 s, or a forced debugLoopGiveUpAt), *retries the batches an in-process node-sharded
 * group then re-ran over the all-reduce path (every rank having given up at the same pod).
 * Both stay 0 in a healthy run; the tests assert it. */
int ksg_debug_loop_stats(const ksg_ctx *ctx, uint64_t *give_ups, uint64_t *retries);

/* Parity diagnostic (no device needed): fills out[k] = math.Log(float64(k)) for 0 <= k < n with
 * the table PodTopologySpread's score kernel reads (topologyNormalizingWeight, podtopologyspread/
 * scoring.go:287-299: log(size + 2)).  Returns n. */
int ksg_debug_log_table(double *out, int32_t n);

/* The plugin-level shim's consistency check: *events counts the cache mutations the
 * context has applied (node add / update / remove, pod add / remove, and the assumes and forgets of its
 * scheduling calls), *list_gen the rebuilds of the snapshot's node list (UpdateSnapshot's
 * updateNodeInfoSnapshotList, backend/cache/cache.go:223-290: the index order may have changed).  A
 * binding that counts the events it forwarded detects a mirror that missed one; list_gen tells it when
 * to re-resolve node names to snapshot indices (ksg_node_name). */
int ksg_generation(const ksg_ctx *ctx, uint64_t *list_gen, uint64_t *events);

/* Measurement helper: ksg_schedule_one(ctx, handles[k], flags, &results[k], NULL) for k = 0..n-1, one call
 * after the other from native code, as a binding's scheduling goroutine issues them; *us_per_call is the
 * mean wall time of one call (the per-pod API's latency without an interpreter's call overhead).  Stops at
 * the first call that fails and returns its code. */
int ksg_debug_schedule_calls(ksg_ctx *ctx, const int32_t *handles, int32_t n, uint32_t flags, ksg_result *results,
                             double *us_per_call);

/* The requests the library derives from one v1.Pod (no context, no device): out[0..4] are
 * CalculateResource's Requested MilliCPU / Memory / EphemeralStorage and Non0CPU / Non0Mem
 * (pkg/scheduler/framework/types.go:1035-1076, with the in-place resize status resources of
 * component-helpers/resource/helpers.go:193-260,299-304), out[5..7] Fit's PreFilter request
 * (noderesources/fit.go:317-325, spec only).  Returns 8, or KSG_EINVAL. */
int ksg_debug_pod_resources(const char *pod_json, size_t len, int64_t *out, int32_t cap);

/* OpportunisticBatching's SignPod (framework/runtime/framework.go:884-924) of one v1.Pod under one profile
 * (config_json as for ksg_create; no context, no device): the signature text -- one signer key per fragment
 * the profile's plugins contribute, equal texts for equal json.Marshal bytes of the reference's fragment
 * map -- into out (NUL-terminated, *out_len its length).  Returns 1 (signed), 0 (nil: a plugin refused, e.g.
 * InterPodAffinity for a pod with affinity terms, PodTopologySpread with constraints or defaults), or
 * KSG_EINVAL (bad JSON, or cap too small). */
int ksg_debug_pod_signature(const char *config_json, size_t config_len, const char *pod_json, size_t pod_len, char *out,
                            size_t cap, size_t *out_len);

/* Parity diagnostics of the node-sharded exchange (no device needed), so host-side protocol tests drive the
 * layout the kernels use rather than a copy of it.  ksg_debug_exchange_layout fills out[0..20] with
 * kMaxShards, the all-reduce word indices XA_CNT, XA_BELOW, XA_NONIGN, XA_MAX_TAINT, XA_MAX_NA, XA_MAX_IPA,
 * XA_NMIN_IPA, XA_END, XA_PROC, XA_WORDS, XB_KEY, XB_NODE, XB_WORDS, XP_MAX_PTS, XP_NMIN_PTS, XP_WORDS,
 * XS_CNT, XS_BELOW, XS_WORDS and kPreBits (returns 21, KSG_EINVAL if cap is smaller).  ksg_debug_pack_best is
 * the (TotalScore, heap pre-order) key every exchange B carries (selectHost, schedule_one.go:1005-1085).
 * ksg_debug_gran_a packs a persistent loop's exchange-A granule payload (which 0: {below | count}, which 1:
 * {max raw NodeAffinity + 1 | max raw TaintToleration + 1}, 0 when count is 0); _decode inverts both. */
int ksg_debug_exchange_layout(int32_t *out, int32_t cap);
uint64_t ksg_debug_pack_best(int64_t total, uint32_t pos);
uint64_t ksg_debug_gran_a(int32_t which, uint32_t count, uint32_t below, int64_t max_taint, int64_t max_na);
int ksg_debug_gran_a_decode(uint64_t g0, uint64_t g1, uint32_t *count, uint32_t *below, int64_t *taint_p1,
                            int64_t *na_p1);

#ifdef __cplusplus
}
#endif
#endif /* KSG_H_ */
