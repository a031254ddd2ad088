"""Builders for the Kubernetes JSON objects that cross the ksg.h boundary.

They play the role of the reference's test wrappers (pkg/scheduler/testing/wrappers.go:
st.MakeNode().Capacity(...).Label(...), st.MakePod().Req(...).Node(...)) so that fixtures
and synthetic clusters read like the reference's own tests.  Output is plain dicts in
the v1.Node / v1.Pod / v1.Namespace JSON schema.
"""
import copy


def _res(d):
    return {k: str(v) for k, v in d.items()} if d else {}


class NodeW:
    """st.MakeNode() (pkg/scheduler/testing/wrappers.go)."""

    def __init__(self, name):
        self.o = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name}, "spec": {}, "status": {}}

    def label(self, k, v):
        self.o["metadata"].setdefault("labels", {})[k] = v
        return self

    def labels(self, d):
        for k, v in d.items():
            self.label(k, v)
        return self

    def capacity(self, res):  # status.allocatable (the scheduler only reads allocatable)
        self.o["status"]["allocatable"] = _res(res)
        self.o["status"]["capacity"] = _res(res)
        return self

    def taints(self, taints):
        self.o["spec"]["taints"] = [dict(t) for t in taints]
        return self

    def unschedulable(self, v=True):
        self.o["spec"]["unschedulable"] = v
        return self

    def images(self, imgs):
        """imgs: {name: size} or [(names, size)]"""
        if isinstance(imgs, dict):
            imgs = [([n], s) for n, s in imgs.items()]
        self.o["status"]["images"] = [{"names": list(n), "sizeBytes": int(s)} for n, s in imgs]
        return self

    def obj(self):
        return copy.deepcopy(self.o)


class PodW:
    """st.MakePod() (pkg/scheduler/testing/wrappers.go)."""

    def __init__(self, name="p", namespace="default", uid=None):
        self.o = {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": namespace, "uid": uid or f"{namespace}-{name}"},
            "spec": {"containers": []},
        }

    def uid(self, u):
        self.o["metadata"]["uid"] = u
        return self

    def label(self, k, v):
        self.o["metadata"].setdefault("labels", {})[k] = v
        return self

    def labels(self, d):
        for k, v in d.items():
            self.label(k, v)
        return self

    def node(self, n):
        self.o["spec"]["nodeName"] = n
        return self

    def terminating(self):
        self.o["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
        return self

    def container(self, image="", requests=None, ports=None, name=None):
        c = {"name": name or f"c{len(self.o['spec']['containers'])}", "image": image}
        if requests is not None:
            c["resources"] = {"requests": _res(requests)}
        if ports:
            c["ports"] = [dict(p) for p in ports]
        self.o["spec"]["containers"].append(c)
        return self

    def req(self, requests):  # st.MakePod().Req(...): one container per call
        return self.container(requests=requests)

    def init_req(self, requests, sidecar=False):
        c = {"name": f"i{len(self.o['spec'].get('initContainers', []))}", "image": "",
             "resources": {"requests": _res(requests)}}
        if sidecar:
            c["restartPolicy"] = "Always"
        self.o["spec"].setdefault("initContainers", []).append(c)
        return self

    def overhead(self, res):
        self.o["spec"]["overhead"] = _res(res)
        return self

    def pod_requests(self, res):
        self.o["spec"]["resources"] = {"requests": _res(res)}
        return self

    def host_port(self, port, ip="", proto="TCP"):
        p = {"containerPort": port, "hostPort": port, "protocol": proto}
        if ip:
            p["hostIP"] = ip
        if not self.o["spec"]["containers"]:
            self.container()
        self.o["spec"]["containers"][-1].setdefault("ports", []).append(p)
        return self

    def node_selector(self, d):
        self.o["spec"]["nodeSelector"] = dict(d)
        return self

    def tolerations(self, ts):
        self.o["spec"]["tolerations"] = [dict(t) for t in ts]
        return self

    def _aff(self):
        return self.o["spec"].setdefault("affinity", {})

    def node_affinity_required(self, terms):
        """terms: list of {"matchExpressions": [...], "matchFields": [...]}"""
        na = self._aff().setdefault("nodeAffinity", {})
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
        return self

    def node_affinity_in(self, key, values):
        return self.node_affinity_required([{"matchExpressions": [{"key": key, "operator": "In", "values": list(values)}]}])

    def node_affinity_preferred(self, terms):
        """terms: list of (weight, {"matchExpressions": [...]})"""
        na = self._aff().setdefault("nodeAffinity", {})
        na["preferredDuringSchedulingIgnoredDuringExecution"] = [{"weight": w, "preference": t} for w, t in terms]
        return self

    def _pat(self, sel, topo, namespaces=None, ns_selector=None):
        t = {"labelSelector": sel, "topologyKey": topo}
        if namespaces is not None:
            t["namespaces"] = list(namespaces)
        if ns_selector is not None:
            t["namespaceSelector"] = ns_selector
        return t

    def pod_affinity(self, topo, sel, namespaces=None, ns_selector=None, anti=False):
        key = "podAntiAffinity" if anti else "podAffinity"
        pa = self._aff().setdefault(key, {})
        pa.setdefault("requiredDuringSchedulingIgnoredDuringExecution", []).append(
            self._pat(sel, topo, namespaces, ns_selector))
        return self

    def pod_affinity_preferred(self, weight, topo, sel, namespaces=None, ns_selector=None, anti=False):
        key = "podAntiAffinity" if anti else "podAffinity"
        pa = self._aff().setdefault(key, {})
        pa.setdefault("preferredDuringSchedulingIgnoredDuringExecution", []).append(
            {"weight": weight, "podAffinityTerm": self._pat(sel, topo, namespaces, ns_selector)})
        return self

    def spread(self, max_skew, topo, when, sel, min_domains=None, node_affinity_policy=None,
               node_taints_policy=None, match_label_keys=None):
        c = {"maxSkew": max_skew, "topologyKey": topo, "whenUnsatisfiable": when, "labelSelector": sel}
        if min_domains is not None:
            c["minDomains"] = min_domains
        if node_affinity_policy:
            c["nodeAffinityPolicy"] = node_affinity_policy
        if node_taints_policy:
            c["nodeTaintsPolicy"] = node_taints_policy
        if match_label_keys:
            c["matchLabelKeys"] = list(match_label_keys)
        self.o["spec"].setdefault("topologySpreadConstraints", []).append(c)
        return self

    def image_volume(self, ref):
        self.o["spec"].setdefault("volumes", []).append({"name": f"v{len(self.o['spec'].get('volumes', []))}",
                                                           "image": {"reference": ref}})
        return self

    def obj(self):
        return copy.deepcopy(self.o)


def make_namespace(name, labels=None):
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name, "labels": dict(labels or {})}}


def match_labels(**kv):
    return {"matchLabels": dict(kv)}


def expr(key, op, values=None):
    e = {"key": key, "operator": op}
    if values is not None:
        e["values"] = list(values)
    return e
