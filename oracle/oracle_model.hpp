// oracle_model.hpp -- PARITY ORACLE (test infrastructure, never shipped, never measured).
//
// Object model of the Kubernetes API subset read by kube-scheduler's node-evaluation
// path, decoded from the objects' JSON encoding, plus the helper semantics the
// plugins call (labels.Selector, nodeaffinity, tolerations, resource requests).
// Every function names the reference file:line it restates.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "minijson.hpp"

namespace oracle {

using Labels = std::map<std::string, std::string>;
// v1.ResourceList with every quantity held as Quantity.MilliValue() (exact for
// quantities with at most milli precision, which covers every scheduler input we use).
using ResList = std::map<std::string, int64_t>;

// ---- resource.Quantity -------------------------------------------------------------
// staging/src/k8s.io/apimachinery/pkg/api/resource/quantity.go (ParseQuantity,
// MilliValue/Value round up = ceil for the non-negative values requests carry).
bool parse_quantity_milli(const std::string& s, int64_t* milli);
// (ceil for m >= 0 without the m + 999 overflow at the int64 edge; truncation toward zero below 0)
inline int64_t milli_to_value(int64_t m) { return m >= 0 ? m / 1000 + (m % 1000 ? 1 : 0) : m / 1000; }

// ---- labels.Selector -----------------------------------------------------------------
enum class Op { In, NotIn, Exists, DoesNotExist, Gt, Lt, Equals };
struct Requirement {  // labels.Requirement, apimachinery/pkg/labels/selector.go:150-170
  std::string key;
  Op op;
  std::vector<std::string> vals;
};
struct Selector {  // labels.Selector: internalSelector (reqs) or nothingSelector
  bool nothing = false;
  std::vector<Requirement> reqs;
  bool empty() const { return !nothing && reqs.empty(); }  // selector.go:102,406
};
bool requirement_matches(const Requirement& r, const Labels& ls);  // selector.go:247-294
bool selector_matches(const Selector& s, const Labels& ls);        // selector.go:419-426
// labels.NewRequirement validation (selector.go:185-226); false on any error
bool new_requirement(const std::string& key, Op op, const std::vector<std::string>& vals,
                     Requirement* out);
bool go_parse_int64(const std::string& s, int64_t* v);  // strconv.ParseInt(s, 10, 64)

// metav1.LabelSelector as decoded (nil vs {} matters: helpers.go:36-42)
struct LabelSelectorSpec {
  bool present = false;
  std::vector<std::pair<std::string, std::string>> matchLabels;
  struct Expr { std::string key, op; std::vector<std::string> values; };
  std::vector<Expr> matchExpressions;
};
// metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:36-71)
bool label_selector_as_selector(const LabelSelectorSpec& ls, Selector* out);
LabelSelectorSpec decode_label_selector(const mj::Value* v);  // nullptr -> nil

// ---- v1 objects ----------------------------------------------------------------------
struct NSRequirement { std::string key, op; std::vector<std::string> values; };
struct NodeSelectorTerm { std::vector<NSRequirement> matchExpressions, matchFields; };
struct PreferredSchedulingTerm { int32_t weight = 0; NodeSelectorTerm preference; };
struct PodAffinityTermSpec {
  LabelSelectorSpec labelSelector;
  std::vector<std::string> namespaces;
  LabelSelectorSpec namespaceSelector;
  std::string topologyKey;
};
struct WeightedPodAffinityTermSpec { int32_t weight = 0; PodAffinityTermSpec term; };
struct Toleration { std::string key, op, value, effect; };
struct Taint { std::string key, value, effect; };
struct ContainerPort { int32_t containerPort = 0, hostPort = 0; std::string hostIP, protocol; };
struct Container {
  std::string name, image;
  ResList requests;
  std::vector<ContainerPort> ports;
  bool restartAlways = false;  // initContainer restartPolicy: Always (sidecar)
};
struct TopologySpreadConstraint {
  int32_t maxSkew = 0;
  std::string topologyKey, whenUnsatisfiable;
  LabelSelectorSpec labelSelector;
  bool hasMinDomains = false;
  int32_t minDomains = 0;
  std::string nodeAffinityPolicy, nodeTaintsPolicy;  // "" = nil
  std::vector<std::string> matchLabelKeys;
};
struct NodeImage { std::vector<std::string> names; int64_t sizeBytes = 0; };

struct Node {
  std::string name;
  Labels labels;
  bool unschedulable = false;
  std::vector<Taint> taints;
  ResList allocatable;
  std::vector<NodeImage> images;
};

struct Pod {
  std::string name, ns, uid;
  Labels labels;
  bool terminating = false;  // metadata.deletionTimestamp != nil
  std::string nodeName;
  bool hasNodeSelector = false;  // spec.nodeSelector != nil
  Labels nodeSelector;
  // spec.affinity.nodeAffinity
  bool hasRequiredNA = false;  // requiredDuringScheduling... != nil
  std::vector<NodeSelectorTerm> requiredNA;
  bool hasPreferredNA = false;  // preferredDuringScheduling... != nil
  std::vector<PreferredSchedulingTerm> preferredNA;
  // spec.affinity.podAffinity / podAntiAffinity
  bool hasPodAffinity = false, hasPodAntiAffinity = false;
  std::vector<PodAffinityTermSpec> affReq, antiReq;
  std::vector<WeightedPodAffinityTermSpec> affPref, antiPref;
  std::vector<Toleration> tolerations;
  std::vector<Container> containers, initContainers;
  bool hasOverhead = false;
  ResList overhead;
  ResList podRequests;  // spec.resources.requests (pod-level resources)
  // status (InPlacePodVerticalScaling): v1.ContainerStatus name / resources (nil?) .requests /
  // allocatedResources, in list order; status.resources (nil?) .requests; status.allocatedResources;
  // status.conditions' (type, reason) in order
  struct ContainerStatus { std::string name; bool hasResources = false; ResList requests, allocated; };
  std::vector<ContainerStatus> containerStatuses, initContainerStatuses;
  bool hasStatusResources = false;
  ResList statusRequests, statusAllocated;
  std::vector<std::pair<std::string, std::string>> conditions;
  std::vector<TopologySpreadConstraint> tsc;
  std::vector<std::string> imageVolumes;  // volumes[].image.reference
  // DefaultPreemption
  int32_t priority = 0;           // corev1helpers.PodPriority: spec.priority, 0 when nil
  bool hasStartTime = false;      // status.startTime != nil
  int64_t startTimeNs = 0;
  std::string preemptionPolicy;   // spec.preemptionPolicy
  std::string nominatedNodeName;  // status.nominatedNodeName
  bool terminatingByPreemption = false;  // preemption.PodTerminatingByPreemption (preemption/util.go:23-35)
  // metav1.GetControllerOfNoCopy (apimachinery/pkg/apis/meta/v1/controller_ref.go:48-56)
  bool hasController = false;
  std::string ownerAPIVersion, ownerKind, ownerName;
  // SignPod fragments (framework/runtime/framework.go:884-924 over the plugins' SignPod methods and the
  // signers of staging/src/k8s.io/kube-scheduler/framework/signers.go), each a canonical text of the value
  // json.Marshal would encode: two pods' fragments are equal iff the reference's encodings are.  The
  // resources fragment depends on the profile's request options and is formed at signing time.
  struct SignFragments {
    std::string schedulerName;  // v1.Pod.Spec.SchedulerName
    std::string tolerations;    // TolerationsSigner: sorted by (key, value), stable
    std::string labels;         // v1.Pod.Labels (InterPodAffinity)
    std::string hostPorts;      // HostPortsSigner: sorted distinct non-zero host ports
    std::string nodeAffinity;   // NodeAffinitySigner
    std::string nodeSelector;   // v1.Pod.Spec.NodeSelector
    std::string images;         // ImageLocality: sorted distinct normalized image names
    std::string volumes;        // VolumesSigner: sorted non-ConfigMap / non-Secret volume sources
    bool hasClaims = false;     // spec.resourceClaims (DynamicResources refuses to sign)
  } sign;
  // NodeDeclaredFeatures: the pod needs a declared node feature (InferForPodScheduling non-empty:
  // restartPolicyRules with RestartAllContainers, or hostNetwork with hostUsers false)
  bool needsNodeFeatures = false;
};

struct Namespace { std::string name; Labels labels; };

// v1.Service / v1.ReplicationController (spec.selector map[string]string, nil-able) and apps/v1
// ReplicaSet / StatefulSet (spec.selector *metav1.LabelSelector): what helper.DefaultSelector lists
struct SelectorObject {
  std::string kind, ns, name;
  bool hasMap = false;  // Service / RC: selector != nil
  Labels map;
  LabelSelectorSpec sel;  // RS / StatefulSet
};
bool decode_selector_object(const mj::Value& v, SelectorObject* out, std::string* err);
TopologySpreadConstraint decode_tsc(const mj::Value& c);

bool decode_node(const mj::Value& v, Node* out, std::string* err);
bool decode_pod(const mj::Value& v, Pod* out, std::string* err);
void sign_fragments(const mj::Value& v, Pod* out);  // Pod::sign, Pod::needsNodeFeatures
bool decode_namespace(const mj::Value& v, Namespace* out, std::string* err);

// ---- scheduler-side derived types ------------------------------------------------------
// fwk.AffinityTerm (kube-scheduler/framework/types.go:380-396)
struct AffinityTerm {
  std::set<std::string> namespaces;
  Selector selector;
  std::string topologyKey;
  Selector nsSelector;
  bool matches(const Pod& p, const Labels* nsLabels) const;
};
struct WeightedAffinityTerm { AffinityTerm term; int32_t weight = 0; };

struct Resource {  // framework.Resource (framework/types.go:1231-1240)
  int64_t milliCPU = 0, memory = 0, ephemeral = 0;
  int64_t allowedPods = 0;
  std::map<std::string, int64_t> scalar;
};
struct PodResource { Resource res; int64_t non0CPU = 0, non0Mem = 0; };

// framework.PodInfo (framework/types.go:960-1076, NewPodInfo :1183-1226)
struct PodInfo {
  Pod pod;
  std::vector<AffinityTerm> reqAff, reqAnti;
  std::vector<WeightedAffinityTerm> prefAff, prefAnti;
  bool parseError = false;
  PodResource calc;
  // podWithAffinity / podWithRequiredAntiAffinity (framework/types.go:386-395)
  bool withAffinity() const { return pod.hasPodAffinity || pod.hasPodAntiAffinity; }
  bool withRequiredAnti() const { return pod.hasPodAntiAffinity && !pod.antiReq.empty(); }
};
bool new_pod_info(const Pod& p, PodInfo* out);

bool is_scalar_resource_name(const std::string& n);  // scheduler/util/utils.go:200-203
// resource.PodRequests (component-helpers/resource/helpers.go:151-291), as used by
// the scheduler: nonMissing != nullptr applies NonMissingContainerRequests.
// resource.PodRequests (helpers.go:151-291); useStatus: PodResourcesOptions.UseStatusResources (with
// InPlacePodLevelResourcesVerticalScalingEnabled, both on by default)
ResList pod_requests(const Pod& p, const ResList* nonMissing, bool useStatus, bool skipPodLevel = false);
bool pod_level_requests_set(const Pod& p);  // helpers.go:108-124
PodResource calculate_resource(const Pod& p);  // framework/types.go:1035-1076

// tolerations (api/core/v1/toleration.go:52-77; component-helpers helpers.go:64-88)
extern bool g_taint_compare_ops;  // set per call from the context's feature gates
bool tolerates(const Toleration& t, const Taint& taint);
bool tolerations_tolerate(const std::vector<Toleration>& ts, const Taint& taint);
bool find_untolerated_noschedule(const std::vector<Taint>& taints, const std::vector<Toleration>& ts);

// nodeaffinity.RequiredNodeAffinity (component-helpers/.../nodeaffinity.go:300-333)
struct ParsedNodeSelectorTerm {
  bool hasLabels = false;
  Selector labels;
  bool hasFields = false;
  std::vector<std::pair<bool, std::pair<std::string, std::string>>> fields;  // (equal?, (key, value))
  bool parseErr = false;
  bool match(const Node& n) const;  // nodeaffinity.go:190-201
};
ParsedNodeSelectorTerm new_node_selector_term(const NodeSelectorTerm& t);  // :170-188
struct RequiredNodeAffinity {
  bool hasLabelSelector = false;
  Selector labelSelector;
  bool hasNodeSelector = false;
  std::vector<ParsedNodeSelectorTerm> terms;  // LazyErrorNodeSelector (non-empty terms)
  bool match(const Node& n) const;
};
RequiredNodeAffinity get_required_node_affinity(const Pod& p);
struct PreferredTerms { std::vector<std::pair<int32_t, ParsedNodeSelectorTerm>> terms; };
bool new_preferred_terms(const std::vector<PreferredSchedulingTerm>& in, PreferredTerms* out);
int64_t preferred_score(const PreferredTerms& t, const Node& n);
// node-level addedAffinity (NodeAffinityArgs)
bool new_node_selector(const std::vector<NodeSelectorTerm>& terms, std::vector<ParsedNodeSelectorTerm>* out);

std::string get_zone_key(const Node& n);  // component-helpers/node/topology/helpers.go:31-58
std::string normalized_image_name(const std::string& name);  // image_locality.go:154-159

}  // namespace oracle
