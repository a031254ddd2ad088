// cluster.cpp -- host cache shadow and the HBM mirror of the snapshot.
//
// Mirrors backend/cache/cache.go (AddNode/UpdateNode/RemoveNode :630-695, AddPod/RemovePod
// :515-597, ghost nodes :442-446,666-689, image states :712-759), NodeInfo.update
// (framework/types.go:445-468), the nodeTree zone round-robin order (node_tree.go:52-143) and
// UpdateSnapshot's list rule (cache.go:190-296, 318-358).  Node add/remove re-lays the mirror
// out; node updates are rewritten in place; pod events touch one node.
#include <atomic>
#include <algorithm>
#include <cstring>

#include "host.hpp"

namespace ksg {
hipError_t launch_node_update(const MirrorView& m, const NodeUpdate* u, const uint32_t* ids, const LabelEntry* lbl, const ScalarEntry* sc,
                              int count, hipStream_t s);
hipError_t launch_node_dyn(const MirrorView& m, const NodeDyn* d, const uint32_t* port_pool, const ScalarEntry* sc,
                           int count, hipStream_t s);

static const char* zone_key(const NodeSpec& n, std::string* out) {  // node/topology/helpers.go:31-58
  auto get = [&](const char* a, const char* b) -> std::string {
    for (auto& kv : n.labels)
      if (kv.first == a) return kv.second;
    for (auto& kv : n.labels)
      if (kv.first == b) return kv.second;
    return "";
  };
  std::string zone = get("failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone");
  std::string region = get("failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region");
  if (region.empty() && zone.empty()) out->clear();
  else *out = region + std::string(":\0:", 3) + zone;
  return out->c_str();
}

Cluster::Cluster(const Config& c) : cfg(c) {
  std::memset(&view, 0, sizeof(view));
  if (hipSetDevice(cfg.device) != hipSuccess || hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
    err = "cannot open HIP device " + std::to_string(cfg.device);
}

Cluster::~Cluster() {
  free_all();
  for (auto& b : pt_dev_)
    if (b.p) (void)hipFree(b.p);
  if (upd_dev_.p) (void)hipFree(upd_dev_.p);
  if (dyn_dev_.p) (void)hipFree(dyn_dev_.p);
  if (gather_dev_.p) (void)hipFree(gather_dev_.p);  // (LeakSanitizer over the host-stub build, tests/asan)
  if (stream) (void)hipStreamDestroy(stream);
}

void* Cluster::dalloc(size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  bufs_.push_back({p, bytes});
  return p;
}
void Cluster::free_all() {
  for (auto& b : bufs_) (void)hipFree(b.p);
  bufs_.clear();
}

int32_t Cluster::key_id(const std::string& k) {
  int32_t id = label_keys.get(k);
  if ((size_t)id >= keys.size()) keys.resize(id + 1);
  return id;
}
int32_t Cluster::scalar_slot(const std::string& n) {
  int32_t id = scalar_ix.find(n);
  if (id >= 0) return id;
  layout_dirty = true;  // a new column must exist on the device (the layout widens scalar_cols as needed)
  return scalar_ix.get(n);
}
uint32_t Cluster::port_id(std::string ip, std::string proto, int32_t port) {  // HostPortInfo.sanitize
  if (ip.empty()) ip = "0.0.0.0";
  if (proto.empty()) proto = "TCP";
  std::string k = ip + "/" + proto + "/" + std::to_string(port);
  int32_t id = port_ix.find(k);
  if (id >= 0) return (uint32_t)id;
  id = port_ix.get(k);
  ports.push_back({ip, proto, port});
  return (uint32_t)id;
}

// ---- nodeTree ---------------------------------------------------------------------------------
void Cluster::tree_add(const NodeSpec& n) {  // node_tree.go:51-67
  std::string z;
  zone_key(n, &z);
  auto it = tree_.find(z);
  if (it == tree_.end()) {
    zones_.push_back(z);
    tree_[z] = {n.name};
  } else if (std::find(it->second.begin(), it->second.end(), n.name) == it->second.end()) {
    it->second.push_back(n.name);
  } else {
    return;  // already in the zone: not added again
  }
  ++tree_nodes_;
}
void Cluster::tree_remove(const NodeSpec& n) {  // node_tree.go:70-99
  std::string z;
  zone_key(n, &z);
  auto it = tree_.find(z);
  if (it == tree_.end()) return;
  auto& v = it->second;
  auto jt = std::find(v.begin(), v.end(), n.name);
  if (jt == v.end()) return;
  v.erase(jt);
  if (v.empty()) {
    tree_.erase(it);
    zones_.erase(std::find(zones_.begin(), zones_.end(), z));
  }
  --tree_nodes_;
}

// UpdateSnapshot's list rule (cache.go:223-290): nodeInfoList is re-created from nodeTree.list
// only when a node changed since the last snapshot is new to the snapshot's map
// (updateAllLists, :228-234), or when the map holds more names than the tree (deleted nodes,
// :270-273).  Any other change -- a node moving to another zone included -- keeps every node at
// its list position (the list holds pointers into the map, updated in place, :257-259).
const std::vector<std::string>& Cluster::order() {
  bool rebuild = false;
  // (an unordered_set's clear() zeroes its whole bucket array, ~1 MB after a 100k-node load: once
  // per pod that was the largest host cost of a 100k-node batch, so it runs only when there was
  // something to take, and a large set gives its buckets back)
  if (!snap_new_.empty()) {
    for (auto& nm : snap_new_) {
      auto it = nodes_.find(nm);
      if (it != nodes_.end() && it->second->real && snap_names_.insert(nm).second) rebuild = true;
    }
    if (snap_new_.bucket_count() > 1024) std::unordered_set<std::string>().swap(snap_new_);
    else snap_new_.clear();
  }
  if (!snap_gone_.empty()) {  // removeDeletedNodesFromSnapshot (cache.go:361-372)
    for (auto& nm : snap_gone_) {
      auto it = nodes_.find(nm);
      if ((it == nodes_.end() || !it->second->real) && snap_names_.erase(nm)) rebuild = true;
    }
    if (snap_gone_.bucket_count() > 1024) std::unordered_set<std::string>().swap(snap_gone_);
    else snap_gone_.clear();
  }
  if (rebuild) {  // updateNodeInfoSnapshotList(updateAll=true) over nodeTree.list (node_tree.go:119-143)
    ++node_gen_;
    ++list_gen;
    order_.clear();
    size_t longest = 0;
    for (auto& z : zones_) longest = std::max(longest, tree_[z].size());
    for (size_t k = 0; k < longest; ++k)
      for (auto& z : zones_) {
        auto& v = tree_[z];
        if (k < v.size()) order_.push_back(v[k]);
      }
    index_.clear();
    index_.reserve(order_.size() * 2);
    for (size_t i = 0; i < order_.size(); ++i) index_.emplace(order_[i], (int32_t)i);
    layout_dirty = true;
  }
  return order_;
}
int32_t Cluster::index_of(const std::string& n) const {
  auto it = index_.find(n);
  return it == index_.end() ? -1 : it->second;
}
NodeRec* Cluster::node(const std::string& name) {
  auto it = nodes_.find(name);
  return it == nodes_.end() ? nullptr : it->second.get();
}
bool Cluster::key_unique(int32_t key) {
  auto it = uniq_cache_.find(key);
  if (it != uniq_cache_.end() && it->second.first == node_gen_) return it->second.second;
  std::vector<uint8_t> seen(keys[key].values.strs.size(), 0);
  bool ok = true;
  for (auto& nm : order_) {
    const NodeRec* r = node(nm);
    if (!r) continue;
    for (auto& kv : r->labels)
      if (kv.first == key) {
        ok = seen[(size_t)kv.second]++ == 0;
        break;
      }
    if (!ok) break;
  }
  uniq_cache_[key] = {node_gen_, ok};
  return ok;
}

// ---- cache events -------------------------------------------------------------------------------
int Cluster::upsert_namespace(const NamespaceSpec& ns) {
  namespaces[ns.name] = ns;
  return KSG_OK;
}

// ---- the selecting objects of PodTopologySpread's default constraints ---------------------------
int Cluster::upsert_object(SelectorObj&& o) {
  if (o.kind == OBJ_SERVICE) services[o.ns][o.name] = std::move(o.sel);
  else owners[o.kind - 1][{o.ns, o.name}] = std::move(o.sel);
  return KSG_OK;
}
int Cluster::remove_object(int kind, const std::string& ns, const std::string& name) {
  if (kind == OBJ_SERVICE) {
    auto it = services.find(ns);
    if (it == services.end() || !it->second.erase(name)) return KSG_ENOTFOUND;
    if (it->second.empty()) services.erase(it);
    return KSG_OK;
  }
  if (kind < OBJ_RC || kind > OBJ_SS) return KSG_EINVAL;
  return owners[kind - 1].erase({ns, name}) ? KSG_OK : KSG_ENOTFOUND;
}

// helper.DefaultSelector (plugins/helper/spread.go:37-95).  Services of the pod's namespace whose
// (non-nil) selector matches the pod's labels merge their selector maps (GetPodServices :98-119); the
// controller owner then merges an RC's map (:67-71) or appends an RS / StatefulSet selector's
// requirements (:72-87; a nil or unparsable LabelSelector adds nothing).  Matching is an AND of
// requirements, so their order (sorted by key upstream) does not matter.
bool Cluster::default_selector(const PodSpec& p, LabelSel* out) {
  std::map<std::string, std::string> set;  // labels.Set; labels.Merge lets the later map win
  auto sit = services.find(p.ns);
  if (sit != services.end())
    for (auto& kv : sit->second) {
      const LabelSel& s = kv.second;
      if (!s.present) continue;  // nil selector: matches nothing (:109-112)
      bool m = true;             // labels.Set(selector).AsSelectorPreValidated().Matches(pod labels)
      for (auto& r : s.match) {
        auto it = std::lower_bound(p.labels.begin(), p.labels.end(), std::make_pair(r.first, std::string()));
        m = m && it != p.labels.end() && it->first == r.first && it->second == r.second;
      }
      if (m)
        for (auto& r : s.match) set[r.first] = r.second;
    }
  out->present = true;
  out->exprs.clear();
  if (p.has_controller) {
    // schema.ParseGroupVersion (runtime/schema/group_version.go:211-227); an error keeps the services' selector
    std::string group, version;
    const std::string& gv = p.owner_api;
    const size_t slashes = (size_t)std::count(gv.begin(), gv.end(), '/');
    bool ok = true;
    if (gv.empty() || gv == "/") {
    } else if (slashes == 0) {
      version = gv;
    } else if (slashes == 1) {
      group = gv.substr(0, gv.find('/'));
      version = gv.substr(gv.find('/') + 1);
    } else {
      ok = false;
    }
    int kind = -1;
    if (ok && group.empty() && version == "v1" && p.owner_kind == "ReplicationController") kind = OBJ_RC;
    if (ok && group == "apps" && version == "v1" && p.owner_kind == "ReplicaSet") kind = OBJ_RS;
    if (ok && group == "apps" && version == "v1" && p.owner_kind == "StatefulSet") kind = OBJ_SS;
    if (kind >= 0) {
      auto it = owners[kind - 1].find({p.ns, p.owner_name});  // listers are namespaced by the pod's namespace
      if (it != owners[kind - 1].end()) {
        const LabelSel& s = it->second;
        if (kind == OBJ_RC) {
          for (auto& r : s.match) set[r.first] = r.second;
        } else if (s.present) {
          std::vector<int32_t> scratch;
          int32_t off;
          if (compile_lsel(s, nullptr, &scratch, &off)) {  // metav1.LabelSelectorAsSelector without error
            for (auto& r : s.match) out->exprs.push_back({r.first, "In", {r.second}});
            for (auto& e : s.exprs) out->exprs.push_back(e);
          }
        }
      }
    }
  }
  out->match.assign(set.begin(), set.end());
  return !(out->match.empty() && out->exprs.empty());  // selector.Empty() (common.go:65-67)
}

void Cluster::add_images(const NodeSpec& n) {
  for (auto& im : n.images)
    for (auto& name : im.names) {
      auto it = image_states.find(name);
      if (it == image_states.end()) {
        ImageState st;
        st.size = im.size;  // first registration wins (cache.go:717-722)
        st.nodes.insert(n.name);
        image_states.emplace(name, std::move(st));
      } else {
        it->second.nodes.insert(n.name);
      }
      image_ix.get(name);
    }
}
void Cluster::remove_images(const NodeSpec& n) {
  for (auto& im : n.images)
    for (auto& name : im.names) {
      auto it = image_states.find(name);
      if (it == image_states.end()) continue;
      it->second.nodes.erase(n.name);
      if (it->second.nodes.empty()) image_states.erase(it);
    }
}

void Cluster::intern_node(NodeRec& r) {
  r.stale = true;
  r.labels.clear();
  for (auto& kv : r.spec.labels) {
    int32_t k = key_id(kv.first);
    r.labels.push_back({k, keys[k].values.get(kv.second)});
  }
  r.taint_ids.clear();
  for (auto& t : r.spec.taints) {
    std::string key = t[0] + '\x1f' + t[1] + '\x1f' + t[2];
    int32_t id = taint_ix.find(key);
    if (id < 0) {
      id = taint_ix.get(key);
      taints.push_back({t[0], t[1], t[2]});
    }
    r.taint_ids.push_back((uint32_t)id);
  }
  r.image_ids.clear();
  for (auto& im : r.spec.images)
    for (auto& name : im.names) r.image_ids.push_back((uint32_t)image_ix.get(name));
  std::sort(r.image_ids.begin(), r.image_ids.end());
  r.image_ids.erase(std::unique(r.image_ids.begin(), r.image_ids.end()), r.image_ids.end());
  // NewResource(node.Status.Allocatable) (framework/types.go:1263-1291)
  r.alloc_cpu = r.alloc_mem = r.alloc_eph = r.alloc_pods = 0;
  r.scalar_alloc.clear();
  for (auto& a : r.spec.alloc) {
    if (a.name == "cpu") r.alloc_cpu += a.milli;
    else if (a.name == "memory") r.alloc_mem += milli_ceil(a.milli);
    else if (a.name == "pods") r.alloc_pods += milli_ceil(a.milli);
    else if (a.name == "ephemeral-storage") r.alloc_eph += milli_ceil(a.milli);
    else if (scalar_resource(a.name)) {
      int32_t s = scalar_slot(a.name);
      if (s >= 0) r.scalar_alloc[s] += milli_ceil(a.milli);
    }
  }
  // magnitude bound of cpu/memory allocatable ever seen (eval_node_fast's FP64 division domain)
  for (int64_t v : {r.alloc_cpu, r.alloc_mem}) alloc_bound = std::max(alloc_bound, v < 0 ? INT64_MAX : v);
}

void Cluster::set_node(NodeRec& r, NodeSpec&& n) {  // addNodeImageStates + NodeInfo.SetNode
  add_images(n);
  r.spec = std::move(n);
  r.real = true;
  intern_node(r);
}

// Cache.AddNode (cache.go:630-646).  A node the cache already holds as a ghost (pods that arrived
// first, or a removed node whose pods remain) gets its Node object back, keeping those pods.
// An AddNode for a node the cache holds with its Node object is taken as UpdateNode: upstream
// would append the name to a second zone list if the zone changed (nodeTree.addNode does not
// look in other zones), which the informer never asks for.
int Cluster::add_node(NodeSpec&& n) {
  ++node_gen_;
  auto it = nodes_.find(n.name);
  if (it != nodes_.end() && it->second->real) return update_node(std::move(n));
  ++events;
  NodeRec* r;
  if (it == nodes_.end()) {
    auto rec = std::make_unique<NodeRec>();
    r = rec.get();
    nodes_[n.name] = std::move(rec);
  } else {
    r = it->second.get();
  }
  const std::string name = n.name;
  tree_add(n);
  set_node(*r, std::move(n));
  snap_new_.insert(name);
  snap_gone_.erase(name);
  layout_dirty = true;  // the row appears (or returns with the ghost's pods)
  // a ghost's pods join the pod table's node index at the next ensure_mirror
  return KSG_OK;
}

// Cache.UpdateNode (cache.go:648-664): nodeTree.updateNode moves the node between zone lists, but
// the snapshot list keeps its position until the next rebuild (order()), so the mirror row is
// rewritten in place whenever its taint / image CSR ranges keep their sizes.
int Cluster::update_node(NodeSpec&& n) {
  ++node_gen_;
  auto it = nodes_.find(n.name);
  if (it == nodes_.end() || !it->second->real) return add_node(std::move(n));
  ++events;
  NodeRec& r = *it->second;
  remove_images(r.spec);
  std::string z0, z1;
  zone_key(r.spec, &z0);
  zone_key(n, &z1);
  if (z0 != z1) {  // node_tree.go:102-115
    tree_remove(r.spec);
    tree_add(n);
  }
  const size_t nt0 = r.taint_ids.size(), ni0 = r.image_ids.size();
  set_node(r, std::move(n));
  if (!layout_dirty && r.taint_ids.size() == nt0 && r.image_ids.size() == ni0)
    return upload_node_static(index_of(r.spec.name));
  layout_dirty = true;
  return KSG_OK;
}

// Cache.RemoveNode (cache.go:672-695): the node leaves the tree and the image states; while pods
// remain on it, it stays in the cache as a ghost with their requests (their delete events may
// still be on the way), skipped by snapshots and by the pod table's aggregation.
int Cluster::remove_node(const std::string& name) {
  ++node_gen_;
  auto it = nodes_.find(name);
  if (it == nodes_.end() || !it->second->real) { err = "node " + name + " is not found"; return KSG_ENOTFOUND; }
  ++events;
  NodeRec& r = *it->second;
  remove_images(r.spec);
  tree_remove(r.spec);
  r.real = false;
  for (auto& uid : r.pods) {  // leave the aggregation (not in any snapshot list any more)
    auto pt = pods.find(uid);
    if (pt != pods.end() && pt->second.slot >= 0) pt_node[pt->second.slot] = -1;
  }
  pods_dirty = true;
  if (r.pods.empty()) nodes_.erase(it);  // removeNodeInfoFromList
  snap_gone_.insert(name);
  snap_new_.erase(name);
  layout_dirty = true;
  return KSG_OK;
}

void Cluster::apply_pod(NodeRec& r, const BoundPod& bp, int sign) {  // NodeInfo.update
  r.stale = true;
  r.req_cpu += sign * bp.res.cpu;
  r.req_mem += sign * bp.res.mem;
  r.req_eph += sign * bp.res.eph;
  r.nz_cpu += sign * bp.res.nz_cpu;
  r.nz_mem += sign * bp.res.nz_mem;
  r.num_pods += sign;
  for (auto& s : bp.res.scalar) {
    int32_t slot = scalar_slot(s.first);
    if (slot >= 0) r.scalar_req[slot] += sign * s.second;
  }
  for (uint32_t p : bp.port_ids) {  // HostPortInfo.Add/Remove: set semantics (types.go:555-587)
    if (sign > 0) r.ports.insert(p);
    else r.ports.erase(p);
    ports_hw_ = std::max(ports_hw_, (int32_t)r.ports.size());
  }
}

// Cache.addPod (cache.go:437-466).  node_override: the node an assumed pod was placed on (the spec
// itself is left unbound).  A pod whose node the cache does not hold creates a ghost NodeInfo.
int Cluster::add_pod(const PodSpec& p, const std::string& uid_override, bool device_done, int32_t slot,
                     const std::string* node_override, const PodResources* res) {
  const std::string uid = uid_override.empty() ? p.uid : uid_override;
  const std::string& node_name = node_override ? *node_override : p.node_name;
  if (node_name.empty()) { err = "pod is not bound"; return KSG_EINVAL; }
  if (pods.count(uid)) { err = "pod " + uid + " exists"; return KSG_EEXIST; }
  ++events;
  NodeRec* r = node(node_name);
  if (!r) {
    auto rec = std::make_unique<NodeRec>();
    rec->spec.name = node_name;
    rec->real = false;
    r = rec.get();
    nodes_[node_name] = std::move(rec);
  }
  BoundPod bp;
  bp.uid = uid;
  bp.node = node_name;
  bp.res = res ? *res : calc_resources(p);
  bp.with_affinity = p.has_pod_affinity || p.has_pod_anti;
  bp.name = p.name;
  bp.priority = p.priority;
  bp.has_start = p.has_start;
  bp.start_ns = p.start_ns;
  bp.preempt_terminating = p.preempt_terminating;
  bp.req_anti = !p.anti_req.empty();
  req_anti_pods += bp.req_anti ? 1 : 0;
  if (p.has_start) max_start_ns = std::max(max_start_ns, p.start_ns);
  else ++nostart_pods;
  mark_pre_dirty(*r);
  pods_with_affinity += bp.with_affinity ? 1 : 0;
  auto take = [&](const Container& c) {
    for (auto& hp : c.ports)
      if (hp.port > 0) bp.port_ids.push_back(port_id(hp.ip, hp.proto, hp.port));
  };
  for (auto& c : p.init_containers)
    if (c.sidecar) take(c);
  for (auto& c : p.containers) take(c);
  apply_pod(*r, bp, +1);
  r->pods.push_back(uid);
  // pod_table_put may materialise label columns (and relayout the mirror), so the node index is
  // taken afterwards; while the layout is dirty it is re-derived by the next ensure_mirror
  bp.slot = slot >= 0 ? slot : pod_table_put(p, -1);
  const int32_t ix = r->real ? index_of(node_name) : -1;
  pt_node[bp.slot] = layout_dirty ? -1 : ix;
  pods.emplace(uid, std::move(bp));
  if (!layout_dirty && !device_done) return upload_node_dynamic(ix);
  return KSG_OK;
}

// Cache.removePod (cache.go:480-513): a ghost node goes once its last pod has gone
int Cluster::remove_pod(const std::string& uid) {
  auto it = pods.find(uid);
  if (it == pods.end()) { err = "unknown pod " + uid; return KSG_ENOTFOUND; }
  ++events;
  NodeRec* r = node(it->second.node);
  pods_with_affinity -= it->second.with_affinity ? 1 : 0;
  req_anti_pods -= it->second.req_anti ? 1 : 0;
  nostart_pods -= it->second.has_start ? 0 : 1;
  if (r) mark_pre_dirty(*r);
  pod_table_drop(it->second.slot);
  int32_t ix = -1;
  if (r) {
    apply_pod(*r, it->second, -1);
    auto& v = r->pods;
    auto jt = std::find(v.begin(), v.end(), uid);
    if (jt != v.end()) {  // removeFromSlice: swap with last (framework/types.go:397-420)
      *jt = v.back();
      v.pop_back();
    }
    if (r->real) ix = index_of(r->spec.name);
    else if (v.empty()) nodes_.erase(it->second.node);
  }
  pods.erase(it);
  if (!layout_dirty) return upload_node_dynamic(ix);
  return KSG_OK;
}

// ---- HBM mirror -----------------------------------------------------------------------------------
#define HIPCHK(x)                                            \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      err = std::string(#x) + ": " + hipGetErrorString(e_); \
      return KSG_EDEVICE;                                    \
    }                                                        \
  } while (0)

// HostPortInfo has no size limit (kube-scheduler/framework/types.go:553-642): the device's port row
// stride follows the largest UsedPorts set, plus what the next batch's AssumePods can add (`extra`
// ids, Engine::run_batch), and a wider stride is a full re-layout.
void Cluster::reserve_ports(int32_t extra) {
  ports_need_ = std::max(ports_need_, ports_hw_ + extra);
  if (view.ports && ports_need_ > view.port_slots) layout_dirty = true;
}

// The device work ensure_mirror(false) would do (re-layout, queued node updates, a pod-table upload the
// lazy rule does not skip): the resident loop holds node cores in LDS and the mirror's addresses in its
// arguments, so it stops before any of it (Engine::schedule_resident).
bool Cluster::mirror_pending() {
  order();
  if (view.ports && std::max(ports_need_, ports_hw_) > view.port_slots) return true;
  if (layout_dirty || !static_dirty_.empty() || !dyn_dirty_.empty()) return true;
  if (pods_dirty && pt_dev_[0].p && pt_dev_[0].bytes >= pt_node.size() * 4 + 4) return false;
  return pods_dirty || (int32_t)log_tab.size() < (int32_t)order_.size() + 4;
}

int Cluster::ensure_mirror(bool pods_needed) {
  order();
  ports_need_ = std::max(ports_need_, ports_hw_);  // pod events since the last cycle
  if (view.ports && ports_need_ > view.port_slots) layout_dirty = true;
  if (!layout_dirty) {
    int rc = flush_node_updates();
    if (!rc) rc = flush_node_dynamic();
    return rc ? rc : upload_pod_table(!pods_needed);
  }
  if (!defer_relayout && !mirror_suspect) {  // node adds / removes / zone moves: move the unchanged nodes' columns
    bool done = false;
    const int rc = relayout_gather(&done);
    if (rc || done) return rc;
  }
  static_dirty_.clear();  // the re-layout below uploads every node
  static_queued_.assign(order_.size(), 0);  // every queued flag, listed or not (the re-layout uploads all)
  dyn_queued_.assign(order_.size(), 0);
  dyn_dirty_.clear();
  HIPCHK(hipStreamSynchronize(stream));
  free_all();
  const int32_t n = (int32_t)order_.size();
  const int32_t cap = ((n + kBlock - 1) / kBlock) * kBlock + kBlock;
  // keep the label slot assignment; grow slot capacity geometrically
  int32_t used = 0;
  for (auto& k : keys) used += k.slot >= 0;
  slots_used_ = used;
  slots_cap_ = std::max(8, slots_used_ * 2);
  std::memset(&view, 0, sizeof(view));
  view.n = n;
  view.cap = cap;
  auto a64 = [&]() { return (int64_t*)dalloc((size_t)cap * 8); };
  view.alloc_cpu = a64();
  view.alloc_mem = a64();
  view.alloc_eph = a64();
  view.alloc_pods = (int32_t*)dalloc((size_t)cap * 4);
  view.flags = (uint32_t*)dalloc((size_t)cap * 4);
  const int32_t sc = std::max<int32_t>(kMaxScalar, (((int32_t)scalar_ix.strs.size() + 7) / 8) * 8);
  view.scalar_cols = sc;
  view.scalar_alloc = (int64_t*)dalloc((size_t)cap * 8 * sc);
  view.req_cpu = a64();
  view.req_mem = a64();
  view.req_eph = a64();
  view.nz_cpu = a64();
  view.nz_mem = a64();
  view.num_pods = (int32_t*)dalloc((size_t)cap * 4);
  view.scalar_req = (int64_t*)dalloc((size_t)cap * 8 * sc);
  view.taint_off = (uint32_t*)dalloc((size_t)(cap + 1) * 4);
  view.img_off = (uint32_t*)dalloc((size_t)(cap + 1) * 4);
  view.labels = (int32_t*)dalloc((size_t)cap * 4 * slots_cap_);
  view.label_num = (int64_t*)dalloc((size_t)cap * 8 * slots_cap_);
  view.label_num_ok = (uint8_t*)dalloc((size_t)cap * slots_cap_);
  for (int32_t i = 0; i < n; ++i) ports_hw_ = std::max(ports_hw_, (int32_t)nodes_[order_[(size_t)i]]->ports.size());
  ports_need_ = std::max(ports_need_, ports_hw_);
  const int32_t ps = std::max<int32_t>(kPortSlots, ((ports_need_ + ports_need_ / 2 + 7) / 8) * 8);
  view.port_slots = ps;
  view.ports = (uint32_t*)dalloc((size_t)cap * 4 * ps);

  std::vector<int64_t> acpu(cap, 0), amem(cap, 0), aeph(cap, 0), rcpu(cap, 0), rmem(cap, 0), reph(cap, 0),
      zcpu(cap, 0), zmem(cap, 0);
  std::vector<int32_t> apods(cap, 0), npods(cap, 0);
  std::vector<uint32_t> flags(cap, 0), toff(cap + 1, 0), ioff(cap + 1, 0), tids, iids;
  int64_t taint_max = 0;
  std::vector<int64_t> salloc((size_t)cap * sc, 0), sreq((size_t)cap * sc, 0);
  std::vector<uint32_t> ports((size_t)cap * ps, 0xffffffffu);
  for (int32_t i = 0; i < n; ++i) {
    const NodeRec& r = *nodes_[order_[i]];
    acpu[i] = r.alloc_cpu;
    amem[i] = r.alloc_mem;
    aeph[i] = r.alloc_eph;
    apods[i] = (int32_t)r.alloc_pods;
    flags[i] = r.spec.unschedulable ? 1u : 0u;
    rcpu[i] = r.req_cpu;
    rmem[i] = r.req_mem;
    reph[i] = r.req_eph;
    zcpu[i] = r.nz_cpu;
    zmem[i] = r.nz_mem;
    npods[i] = r.num_pods;
    for (auto& kv : r.scalar_alloc) salloc[(size_t)kv.first * cap + i] = kv.second;
    for (auto& kv : r.scalar_req) sreq[(size_t)kv.first * cap + i] = kv.second;
    toff[i] = (uint32_t)tids.size();
    tids.insert(tids.end(), r.taint_ids.begin(), r.taint_ids.end());
    taint_max = std::max<int64_t>(taint_max, (int64_t)r.taint_ids.size());
    ioff[i] = (uint32_t)iids.size();
    iids.insert(iids.end(), r.image_ids.begin(), r.image_ids.end());
    int q = 0;
    for (uint32_t p : r.ports) ports[(size_t)i * ps + q++] = p;
  }
  for (int32_t i = n; i <= cap; ++i) {
    toff[i] = (uint32_t)tids.size();
    ioff[i] = (uint32_t)iids.size();
  }
  node_toff_ = toff;  // CSR ranges of every node (upload_node_static rewrites a node's ids in place)
  node_ioff_ = ioff;
  taint_ids_per_node = n ? (double)tids.size() / n : 0.0;
  taint_max_per_node = taint_max;
  img_ids_per_node = n ? (double)iids.size() / n : 0.0;
  taint_cap_ = tids.size() + tids.size() / 2 + 1024;  // room for nodes added by relayout_gather
  img_cap_ = iids.size() + iids.size() / 2 + 1024;
  view.taint_ids = (uint32_t*)dalloc(taint_cap_ * 4);
  view.img_ids = (uint32_t*)dalloc(img_cap_ * 4);
  auto up = [&](const void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(const_cast<void*>(dst), src, bytes, hipMemcpyHostToDevice, stream);
  };
  HIPCHK(up(view.alloc_cpu, acpu.data(), (size_t)cap * 8));
  HIPCHK(up(view.alloc_mem, amem.data(), (size_t)cap * 8));
  HIPCHK(up(view.alloc_eph, aeph.data(), (size_t)cap * 8));
  HIPCHK(up(view.alloc_pods, apods.data(), (size_t)cap * 4));
  HIPCHK(up(view.flags, flags.data(), (size_t)cap * 4));
  HIPCHK(up(view.scalar_alloc, salloc.data(), salloc.size() * 8));
  HIPCHK(up(view.req_cpu, rcpu.data(), (size_t)cap * 8));
  HIPCHK(up(view.req_mem, rmem.data(), (size_t)cap * 8));
  HIPCHK(up(view.req_eph, reph.data(), (size_t)cap * 8));
  HIPCHK(up(view.nz_cpu, zcpu.data(), (size_t)cap * 8));
  HIPCHK(up(view.nz_mem, zmem.data(), (size_t)cap * 8));
  HIPCHK(up(view.num_pods, npods.data(), (size_t)cap * 4));
  HIPCHK(up(view.scalar_req, sreq.data(), sreq.size() * 8));
  HIPCHK(up(view.taint_off, toff.data(), toff.size() * 4));
  HIPCHK(up(view.img_off, ioff.data(), ioff.size() * 4));
  if (!tids.empty()) HIPCHK(up(view.taint_ids, tids.data(), tids.size() * 4));
  if (!iids.empty()) HIPCHK(up(view.img_ids, iids.data(), iids.size() * 4));
  HIPCHK(up(view.ports, ports.data(), ports.size() * 4));
  HIPCHK(hipStreamSynchronize(stream));
  layout_dirty = false;
  for (int32_t k = 0; k < (int32_t)keys.size(); ++k)
    if (keys[k].slot >= 0) {
      int rc = upload_label_column(k);
      if (rc) return rc;
    }
  ++laid_epoch_;
  for (int32_t i = 0; i < n; ++i) {
    NodeRec& r = *nodes_[order_[(size_t)i]];
    r.stale = false;
    r.laid_ix = i;
    r.laid_epoch = laid_epoch_;
  }
  laid_slots_ = slots_used_;
  mirror_suspect = false;
  ++relayouts_full;
  // snapshot indices moved: re-derive every pod's node index in the pod table
  for (auto& kv : pods)  // (pods on ghost nodes stay out of the aggregation)
    if (kv.second.slot >= 0) {
      const NodeRec* r = node(kv.second.node);
      pt_node[kv.second.slot] = r && r->real ? index_of(kv.second.node) : -1;
    }
  pods_dirty = true;
  return upload_pod_table();
}

hipError_t launch_gather_rows(uint8_t* dst, const uint8_t* src, const int32_t* idx, int n, int cap, int rows, int esz,
                              hipStream_t s);
hipError_t launch_gather_csr(uint32_t* dst, const uint32_t* src, const int32_t* idx, const uint32_t* old_off,
                             const uint32_t* new_off, int n, hipStream_t s);

// Cache.AddNode / RemoveNode / a zone move between two cycles: UpdateSnapshot rebuilds the list
// (cache.go:273-283) and snapshot indices shift.  Every node whose shadow did not change keeps its
// device columns: one gather per column block moves them to the new index; new and changed nodes go
// up as NodeUpdate / NodeDyn records.  The capacities (cap, label slots, CSR ids) must still fit.
int Cluster::relayout_gather(bool* done) {
  *done = false;
  const int32_t n = (int32_t)order_.size();
  const int32_t cap = view.cap;
  if (!view.req_cpu || laid_epoch_ == 0 || n == 0 || n + 1 > cap || slots_used_ > slots_cap_ ||
      (int32_t)scalar_ix.strs.size() > view.scalar_cols)
    return KSG_OK;
  std::vector<NodeRec*> recs((size_t)n);
  for (int32_t i = 0; i < n; ++i) recs[(size_t)i] = nodes_[order_[(size_t)i]].get();
  std::vector<int32_t> src((size_t)n, -1);
  std::vector<uint32_t> toff((size_t)cap + 1, 0), ioff((size_t)cap + 1, 0);
  size_t nt = 0, ni = 0;
  int64_t taint_max = 0;
  int32_t fresh = 0;
  for (int32_t i = 0; i < n; ++i) {
    const NodeRec& r = *recs[(size_t)i];
    if ((int32_t)r.ports.size() > view.port_slots) return KSG_OK;  // the full path widens the stride
    src[(size_t)i] = (r.laid_epoch == laid_epoch_ && !r.stale) ? r.laid_ix : -1;
    fresh += src[(size_t)i] < 0;
    toff[(size_t)i] = (uint32_t)nt;
    ioff[(size_t)i] = (uint32_t)ni;
    nt += r.taint_ids.size();
    ni += r.image_ids.size();
    taint_max = std::max<int64_t>(taint_max, (int64_t)r.taint_ids.size());
  }
  for (int32_t i = n; i <= cap; ++i) {
    toff[(size_t)i] = (uint32_t)nt;
    ioff[(size_t)i] = (uint32_t)ni;
  }
  if (nt > taint_cap_ || ni > img_cap_) return KSG_OK;
  if (fresh * 2 > n) return KSG_OK;  // mostly new columns: the full path is as cheap
  // device scratch: the index map, the new CSR offsets, one column block
  // (the widest block: the scalar columns, the label columns, or the host-port rows, which a batch of
  // host-port pods widens by one slot per pod, Cluster::reserve_ports)
  const size_t blk = (size_t)cap * std::max<size_t>(8 * (size_t)std::max(view.scalar_cols, std::max(slots_used_, 1)),
                                                    4 * (size_t)std::max(view.port_slots, 1));
  const size_t o_src = 0, o_toff = ((size_t)n * 4 + 255) & ~size_t(255),
               o_ioff = o_toff + (((size_t)(cap + 1) * 4 + 255) & ~size_t(255)),
               o_blk = o_ioff + (((size_t)(cap + 1) * 4 + 255) & ~size_t(255));
  const size_t o_ids = o_blk + blk, need = o_ids + std::max(taint_cap_, img_cap_) * 4 + 256;
  if (gather_dev_.bytes < need) {
    if (gather_dev_.p) (void)hipFree(gather_dev_.p);
    gather_dev_.p = nullptr;
    gather_dev_.bytes = 0;
    HIPCHK(hipMalloc(&gather_dev_.p, need));
    gather_dev_.bytes = need;
  }
  uint8_t* g = (uint8_t*)gather_dev_.p;
  const int32_t* d_src = (const int32_t*)(g + o_src);
  HIPCHK(hipMemcpyAsync(g + o_src, src.data(), (size_t)n * 4, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(g + o_toff, toff.data(), toff.size() * 4, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(g + o_ioff, ioff.data(), ioff.size() * 4, hipMemcpyHostToDevice, stream));
  auto col = [&](const void* p, int rows, int esz) -> int {  // gather into the scratch block, copy back
    if (rows <= 0) return KSG_OK;
    HIPCHK(launch_gather_rows(g + o_blk, (const uint8_t*)p, d_src, n, cap, rows, esz, stream));
    HIPCHK(hipMemcpyAsync(const_cast<void*>(p), g + o_blk, (size_t)rows * cap * (esz > 8 ? esz : esz), hipMemcpyDeviceToDevice,
                          stream));
    return KSG_OK;
  };
  int rc;
  for (const void* p : {(const void*)view.alloc_cpu, (const void*)view.alloc_mem, (const void*)view.alloc_eph,
                        (const void*)view.req_cpu, (const void*)view.req_mem, (const void*)view.req_eph,
                        (const void*)view.nz_cpu, (const void*)view.nz_mem})
    if ((rc = col(p, 1, 8))) return rc;
  for (const void* p : {(const void*)view.alloc_pods, (const void*)view.num_pods, (const void*)view.flags})
    if ((rc = col(p, 1, 4))) return rc;
  if ((rc = col(view.scalar_alloc, view.scalar_cols, 8)) || (rc = col(view.scalar_req, view.scalar_cols, 8)) ||
      (rc = col(view.ports, 1, 4 * view.port_slots)) || (rc = col(view.labels, laid_slots_, 4)) ||
      (rc = col(view.label_num, laid_slots_, 8)) || (rc = col(view.label_num_ok, laid_slots_, 1)))
    return rc;
  // CSR ids, then the new offsets
  HIPCHK(launch_gather_csr((uint32_t*)(g + o_ids), view.taint_ids, d_src, view.taint_off, (const uint32_t*)(g + o_toff), n,
                           stream));
  HIPCHK(hipMemcpyAsync(const_cast<uint32_t*>(view.taint_ids), g + o_ids, std::max<size_t>(nt, 1) * 4,
                        hipMemcpyDeviceToDevice, stream));
  HIPCHK(launch_gather_csr((uint32_t*)(g + o_ids), view.img_ids, d_src, view.img_off, (const uint32_t*)(g + o_ioff), n,
                           stream));
  HIPCHK(hipMemcpyAsync(const_cast<uint32_t*>(view.img_ids), g + o_ids, std::max<size_t>(ni, 1) * 4,
                        hipMemcpyDeviceToDevice, stream));
  HIPCHK(hipMemcpyAsync(const_cast<uint32_t*>(view.taint_off), g + o_toff, toff.size() * 4, hipMemcpyDeviceToDevice, stream));
  HIPCHK(hipMemcpyAsync(const_cast<uint32_t*>(view.img_off), g + o_ioff, ioff.size() * 4, hipMemcpyDeviceToDevice, stream));
  view.n = n;
  node_toff_ = toff;
  node_ioff_ = ioff;
  taint_ids_per_node = (double)nt / n;
  taint_max_per_node = taint_max;
  img_ids_per_node = (double)ni / n;
  layout_dirty = false;
  // label columns materialised since the last layout: whole columns from the shadow
  for (int32_t k = 0; k < (int32_t)keys.size(); ++k)
    if (keys[k].slot >= laid_slots_ && (rc = upload_label_column(k))) return rc;
  // new and changed nodes: their static and dynamic columns as records
  static_queued_.assign((size_t)n, 0);
  dyn_queued_.assign((size_t)n, 0);
  static_dirty_.clear();
  dyn_dirty_.clear();
  for (int32_t i = 0; i < n; ++i)
    if (src[(size_t)i] < 0) {
      static_queued_[(size_t)i] = dyn_queued_[(size_t)i] = 1;
      static_dirty_.push_back(i);
      dyn_dirty_.push_back(i);
    }
  if ((rc = flush_node_updates()) || (rc = flush_node_dynamic())) return rc;
  ++laid_epoch_;
  for (int32_t i = 0; i < n; ++i) {
    recs[(size_t)i]->stale = false;
    recs[(size_t)i]->laid_ix = i;
    recs[(size_t)i]->laid_epoch = laid_epoch_;
  }
  laid_slots_ = slots_used_;
  ++relayouts_gather;
  for (auto& kv : pods)  // snapshot indices moved: every pod's node index in the pod table
    if (kv.second.slot >= 0) {
      const NodeRec* r = node(kv.second.node);
      pt_node[kv.second.slot] = r && r->real ? index_of(kv.second.node) : -1;
    }
  pods_dirty = true;
  *done = true;
  return upload_pod_table();
}

int Cluster::upload_label_column(int32_t key) {
  const int32_t slot = keys[key].slot;
  const int32_t cap = view.cap;
  std::vector<int32_t> col(cap, -1);
  std::vector<int64_t> num(cap, 0);
  std::vector<uint8_t> ok(cap, 0);
  // numeric value per local value id (labels.Requirement Gt/Lt parse, selector.go:265-289)
  auto& vals = keys[key].values.strs;
  std::vector<int64_t> vnum(vals.size(), 0);
  std::vector<uint8_t> vok(vals.size(), 0);
  for (size_t v = 0; v < vals.size(); ++v) vok[v] = parse_go_int(vals[v], &vnum[v]) ? 1 : 0;
  for (int32_t i = 0; i < view.n; ++i) {
    const NodeRec& r = *nodes_[order_[i]];
    for (auto& kv : r.labels)
      if (kv.first == key) {
        col[i] = kv.second;
        num[i] = vnum[kv.second];
        ok[i] = vok[kv.second];
      }
  }
  const size_t off = (size_t)slot * cap;
  HIPCHK(hipMemcpyAsync(const_cast<int32_t*>(view.labels) + off, col.data(), (size_t)cap * 4, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(const_cast<int64_t*>(view.label_num) + off, num.data(), (size_t)cap * 8, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(const_cast<uint8_t*>(view.label_num_ok) + off, ok.data(), (size_t)cap, hipMemcpyHostToDevice, stream));
  HIPCHK(hipStreamSynchronize(stream));
  return KSG_OK;
}

int Cluster::ensure_label_slot(int32_t key) {
  if (keys[key].slot >= 0) return KSG_OK;
  keys[key].slot = slots_used_++;
  if (layout_dirty || slots_used_ > slots_cap_) {
    layout_dirty = true;  // regrow on the next ensure_mirror
    // (deferred while a pipelined batch has pods in flight: the shadow lacks their assumes until
    // the batch drains and mirrors them, engine.cpp run_batch)
    return defer_relayout ? KSG_OK : ensure_mirror();
  }
  return upload_label_column(key);
}

// The node's static columns (NodeInfo.node: allocatable, unschedulable, taints, images, the
// materialised label columns) at snapshot position i are rewritten in place: the node is queued
// and the queue goes to the device in one H2D + one k_node_update launch at the next cycle's
// ensure_mirror -- the device-side counterpart of UpdateSnapshot's generation diff
// (backend/cache/cache.go:223-265).
int Cluster::upload_node_static(int32_t i) {
  if (i < 0 || layout_dirty || (size_t)i + 1 >= node_toff_.size()) {
    layout_dirty = true;
    return KSG_OK;
  }
  if (static_queued_.size() < (size_t)view.n) static_queued_.resize((size_t)view.n, 0);
  if (!static_queued_[i]) {
    static_queued_[i] = 1;
    static_dirty_.push_back(i);
  }
  return KSG_OK;
}

int Cluster::flush_node_updates() {
  if (static_dirty_.empty()) return KSG_OK;
  const size_t cnt = static_dirty_.size();
  std::vector<NodeUpdate> rec(cnt);
  std::vector<uint32_t> ids;
  std::vector<LabelEntry> lbl;
  std::vector<ScalarEntry> scv;
  std::vector<int64_t> vnum;
  for (size_t q = 0; q < cnt; ++q) {
    const int32_t i = static_dirty_[q];
    static_queued_[i] = 0;
    NodeRec& r = *nodes_[order_[i]];
    NodeUpdate& u = rec[q];
    std::memset(&u, 0, sizeof(u));
    u.node = i;
    u.alloc_cpu = r.alloc_cpu;
    u.alloc_mem = r.alloc_mem;
    u.alloc_eph = r.alloc_eph;
    u.alloc_pods = (int32_t)r.alloc_pods;
    u.flags = r.spec.unschedulable ? 1u : 0u;
    u.sc_off = (uint32_t)scv.size();
    for (auto& kv : r.scalar_alloc) scv.push_back({kv.first, 0, kv.second});
    u.sc_cnt = (uint32_t)(scv.size() - u.sc_off);
    u.taint_off = node_toff_[i];
    u.img_off = node_ioff_[i];
    u.n_taint = (int32_t)r.taint_ids.size();
    u.n_img = (int32_t)r.image_ids.size();
    u.id_off = (uint32_t)ids.size();
    ids.insert(ids.end(), r.taint_ids.begin(), r.taint_ids.end());
    ids.insert(ids.end(), r.image_ids.begin(), r.image_ids.end());
    u.lbl_off = (uint32_t)lbl.size();
    for (int32_t k = 0; k < (int32_t)keys.size(); ++k) {  // labels.Requirement Gt/Lt parse (selector.go:265-289)
      if (keys[k].slot < 0) continue;
      LabelEntry e{keys[k].slot, -1, 0, 0, 0};
      for (auto& kv : r.labels)
        if (kv.first == k) e.value = kv.second;
      if (e.value >= 0) e.ok = parse_go_int(keys[k].values.strs[e.value], &e.num) ? 1 : 0;
      if (!e.ok) e.num = 0;
      lbl.push_back(e);
    }
    u.lbl_cnt = (int32_t)(lbl.size() - u.lbl_off);
    r.stale = false;  // (a queued node's dynamic columns are flushed right after, in ensure_mirror)
  }
  static_dirty_.clear();
  const size_t b0 = cnt * sizeof(NodeUpdate), b1 = std::max<size_t>(ids.size(), 1) * 4,
               b2 = std::max<size_t>(lbl.size(), 1) * sizeof(LabelEntry),
               b3 = std::max<size_t>(scv.size(), 1) * sizeof(ScalarEntry);
  const size_t o1 = (b0 + 15) & ~size_t(15), o2 = (o1 + b1 + 15) & ~size_t(15), o3 = (o2 + b2 + 15) & ~size_t(15),
               total = o3 + b3;
  if (upd_dev_.bytes < total) {
    if (upd_dev_.p) (void)hipFree(upd_dev_.p);
    upd_dev_.p = nullptr;
    HIPCHK(hipMalloc(&upd_dev_.p, total * 2));
    upd_dev_.bytes = total * 2;
  }
  std::vector<uint8_t> host(total, 0);
  std::memcpy(host.data(), rec.data(), b0);
  if (!ids.empty()) std::memcpy(host.data() + o1, ids.data(), ids.size() * 4);
  if (!lbl.empty()) std::memcpy(host.data() + o2, lbl.data(), lbl.size() * sizeof(LabelEntry));
  if (!scv.empty()) std::memcpy(host.data() + o3, scv.data(), scv.size() * sizeof(ScalarEntry));
  uint8_t* d = (uint8_t*)upd_dev_.p;
  HIPCHK(hipMemcpyAsync(d, host.data(), total, hipMemcpyHostToDevice, stream));
  HIPCHK(launch_node_update(view, (const NodeUpdate*)d, (const uint32_t*)(d + o1), (const LabelEntry*)(d + o2),
                            (const ScalarEntry*)(d + o3), (int)cnt, stream));
  HIPCHK(hipStreamSynchronize(stream));  // the host staging vector dies here
  return KSG_OK;
}

// A node's dynamic columns (NodeInfo.Requested / NonZeroRequested / len(Pods) / UsedPorts) after a
// pod event are queued like the static ones and go up at the next cycle as one H2D of NodeDyn
// records + one k_node_dyn launch (a cache fed thousands of pod events between cycles pays one
// copy, not ~25 per event).
int Cluster::upload_node_dynamic(int32_t i) {
  if (i < 0 || layout_dirty) return KSG_OK;
  if (dyn_queued_.size() < (size_t)view.n) dyn_queued_.resize((size_t)view.n, 0);
  if (!dyn_queued_[i]) {
    dyn_queued_[i] = 1;
    dyn_dirty_.push_back(i);
  }
  return KSG_OK;
}

int Cluster::flush_node_dynamic() {
  if (dyn_dirty_.empty()) return KSG_OK;
  const size_t cnt = dyn_dirty_.size();
  std::vector<NodeDyn> rec(cnt);
  std::vector<uint32_t> pool;  // UsedPorts ids
  std::vector<ScalarEntry> scv;  // scalar requests
  for (size_t q = 0; q < cnt; ++q) {
    const int32_t i = dyn_dirty_[q];
    dyn_queued_[i] = 0;
    NodeRec& r = *nodes_[order_[i]];
    NodeDyn& d = rec[q];
    std::memset(&d, 0, sizeof(d));
    d.node = i;
    d.num_pods = r.num_pods;
    d.req_cpu = r.req_cpu;
    d.req_mem = r.req_mem;
    d.req_eph = r.req_eph;
    d.nz_cpu = r.nz_cpu;
    d.nz_mem = r.nz_mem;
    d.sc_off = (uint32_t)scv.size();
    for (auto& kv : r.scalar_req)
      if (kv.second) scv.push_back({kv.first, 0, kv.second});
    d.sc_cnt = (uint32_t)(scv.size() - d.sc_off);
    d.port_off = (uint32_t)pool.size();
    d.port_cnt = (uint32_t)r.ports.size();  // <= view.port_slots: ensure_mirror re-lays out first otherwise
    pool.insert(pool.end(), r.ports.begin(), r.ports.end());
    r.stale = false;
  }
  dyn_dirty_.clear();
  const size_t rec_bytes = cnt * sizeof(NodeDyn), o_sc = (rec_bytes + pool.size() * 4 + 15) & ~size_t(15),
               bytes = o_sc + std::max<size_t>(scv.size(), 1) * sizeof(ScalarEntry);
  if (dyn_dev_.bytes < bytes) {
    if (dyn_dev_.p) (void)hipFree(dyn_dev_.p);
    dyn_dev_.p = nullptr;
    dyn_dev_.bytes = 0;
    HIPCHK(hipMalloc(&dyn_dev_.p, bytes * 2));
    dyn_dev_.bytes = bytes * 2;
  }
  HIPCHK(hipMemcpyAsync(dyn_dev_.p, rec.data(), rec_bytes, hipMemcpyHostToDevice, stream));
  if (!pool.empty())
    HIPCHK(hipMemcpyAsync((uint8_t*)dyn_dev_.p + rec_bytes, pool.data(), pool.size() * 4, hipMemcpyHostToDevice, stream));
  if (!scv.empty())
    HIPCHK(hipMemcpyAsync((uint8_t*)dyn_dev_.p + o_sc, scv.data(), scv.size() * sizeof(ScalarEntry), hipMemcpyHostToDevice,
                          stream));
  HIPCHK(launch_node_dyn(view, (const NodeDyn*)dyn_dev_.p, (const uint32_t*)((uint8_t*)dyn_dev_.p + rec_bytes),
                         (const ScalarEntry*)((uint8_t*)dyn_dev_.p + o_sc), (int)cnt, stream));
  HIPCHK(hipStreamSynchronize(stream));  // the host records die here
  return KSG_OK;
}


// Parity diagnostic (ksg_debug_compare_mirror): the device mirror's node columns and pod table
// against the host shadow they are uploaded from.  A difference means a device-side AssumePod the
// cache does not hold (or the reverse) -- what a loop give-up leaves until the mirror is rebuilt.
int Cluster::compare_mirror(bool sync, int32_t* ndiff, int32_t* first) {
  order();
  if (sync) {
    const int rc = ensure_mirror();
    if (rc) return rc;
  }
  *ndiff = 0;
  *first = -1;
  const int32_t n = view.n;
  if (!view.req_cpu || n != (int32_t)order_.size()) {  // no mirror laid out for this order: nothing to compare
    *ndiff = -1;
    return KSG_OK;
  }
  HIPCHK(hipStreamSynchronize(stream));
  std::vector<int64_t> rc_((size_t)n), rm((size_t)n), re((size_t)n), zc((size_t)n), zm((size_t)n), ac((size_t)n), am((size_t)n);
  std::vector<int32_t> np((size_t)n), ap((size_t)n);
  const int32_t ps = view.port_slots;
  std::vector<uint32_t> fl((size_t)n), pt((size_t)n * ps);
  auto down = [&](void* dst, const void* src, size_t bytes) -> int {
    if (!bytes) return KSG_OK;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return KSG_OK;
  };
  int rc;
  if ((rc = down(rc_.data(), view.req_cpu, (size_t)n * 8)) || (rc = down(rm.data(), view.req_mem, (size_t)n * 8)) ||
      (rc = down(re.data(), view.req_eph, (size_t)n * 8)) || (rc = down(zc.data(), view.nz_cpu, (size_t)n * 8)) ||
      (rc = down(zm.data(), view.nz_mem, (size_t)n * 8)) || (rc = down(ac.data(), view.alloc_cpu, (size_t)n * 8)) ||
      (rc = down(am.data(), view.alloc_mem, (size_t)n * 8)) || (rc = down(np.data(), view.num_pods, (size_t)n * 4)) ||
      (rc = down(ap.data(), view.alloc_pods, (size_t)n * 4)) || (rc = down(fl.data(), view.flags, (size_t)n * 4)) ||
      (rc = down(pt.data(), view.ports, (size_t)n * ps * 4)))
    return rc;
  auto bad = [&](int32_t where) {
    if (*first < 0) *first = where;
    ++*ndiff;
  };
  for (int32_t i = 0; i < n; ++i) {
    const NodeRec* r = node(order_[(size_t)i]);
    if (!r) {
      bad(i);
      continue;
    }
    std::set<uint32_t> dp;
    for (int k = 0; k < ps; ++k)
      if (pt[(size_t)i * ps + k] != 0xffffffffu) dp.insert(pt[(size_t)i * ps + k]);
    if (rc_[i] != r->req_cpu || rm[i] != r->req_mem || re[i] != r->req_eph || zc[i] != r->nz_cpu || zm[i] != r->nz_mem ||
        np[i] != r->num_pods || ac[i] != r->alloc_cpu || am[i] != r->alloc_mem || ap[i] != (int32_t)r->alloc_pods ||
        (fl[i] & 1u) != (r->spec.unschedulable ? 1u : 0u) || dp != r->ports)
      bad(i);
  }
  if (!pods_dirty && view.pods_hw > 0) {  // the pod table as uploaded: every slot's node
    std::vector<int32_t> pn((size_t)view.pods_hw);
    if ((rc = down(pn.data(), view.pod_node, (size_t)view.pods_hw * 4))) return rc;
    for (int32_t sl = 0; sl < view.pods_hw && (size_t)sl < pt_node.size(); ++sl)
      if (pn[(size_t)sl] != pt_node[(size_t)sl]) bad(n + sl);
  }
  return KSG_OK;
}

}  // namespace ksg
