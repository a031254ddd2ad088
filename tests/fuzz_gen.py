"""Seeded random clusters + pod streams for product-vs-oracle parity (node-local plugins).

Covers the features the device path implements: resources (incl. init/sidecar containers,
overhead, pod-level requests, extended resources), unschedulable nodes, taints/tolerations of
every effect, nodeSelector, required/preferred node affinity (all operators, matchFields ->
PreFilterResult subsets), host ports (incl. 0.0.0.0 wildcards), images, nodeName, and the
profile knobs (scoring strategies, resource lists, added affinity, weights, disabled plugins).
"""
import random

from ksg.objects import NodeW, PodW, expr, make_namespace

ZONES = ["zone-a", "zone-b", "zone-c"]
TAINT_KEYS = ["dedicated", "gpu", "spot"]
IMAGES = [("registry.example/app:v1", 300 * 1000 * 1000), ("registry.example/db", 900 * 1000 * 1000),
          ("docker.io/library/nginx:1.25", 60 * 1000 * 1000), ("registry.example/big:2", 1500 * 1000 * 1000)]


def rand_node(rng, i, extended=True):
    name = f"n{i:05d}"
    cpu = rng.choice(["2", "4", "8", "16", "3500m"])
    mem = rng.choice(["4Gi", "8Gi", "16Gi", "32Gi", "12000Mi"])
    cap = {"cpu": cpu, "memory": mem, "pods": str(rng.choice([3, 10, 110]))}
    if rng.random() < 0.3:
        cap["ephemeral-storage"] = rng.choice(["10Gi", "100Gi"])
    if extended and rng.random() < 0.3:
        cap["example.com/gpu"] = str(rng.randint(0, 4))
    w = NodeW(name).capacity(cap).label("kubernetes.io/hostname", name)
    if rng.random() < 0.9:
        w.label("topology.kubernetes.io/zone", rng.choice(ZONES))
    if rng.random() < 0.5:
        w.label("disk", rng.choice(["ssd", "hdd"]))
    if rng.random() < 0.6:
        w.label("gen", str(rng.randint(1, 6)))
    if rng.random() < 0.07:
        w.unschedulable()
    taints = []
    for _ in range(rng.choice([0, 0, 0, 1, 2])):
        taints.append({"key": rng.choice(TAINT_KEYS), "value": rng.choice(["", "x", "y"]),
                       "effect": rng.choice(["NoSchedule", "PreferNoSchedule", "PreferNoSchedule", "NoExecute"])})
    if taints:
        w.taints(taints)
    imgs = rng.sample(IMAGES, rng.randint(0, 2))
    if imgs:
        w.images({n: s for n, s in imgs})
    return w.obj()


def rand_requests(rng):
    r = {}
    if rng.random() < 0.8:
        r["cpu"] = rng.choice(["100m", "250m", "500m", "1", "1500m", "3"])
    if rng.random() < 0.8:
        r["memory"] = rng.choice(["128Mi", "500Mi", "1Gi", "3Gi", "7Gi"])
    if rng.random() < 0.1:
        r["ephemeral-storage"] = "1Gi"
    if rng.random() < 0.1:
        r["example.com/gpu"] = str(rng.randint(1, 2))
    return r


def rand_tolerations(rng):
    out = []
    for _ in range(rng.choice([0, 0, 1, 2])):
        op = rng.choice(["Equal", "Exists"])
        t = {"key": rng.choice(TAINT_KEYS + [""]) if op == "Exists" else rng.choice(TAINT_KEYS), "operator": op}
        if op == "Equal":
            t["value"] = rng.choice(["", "x", "y"])
        eff = rng.choice(["", "NoSchedule", "PreferNoSchedule", "NoExecute"])
        if eff:
            t["effect"] = eff
        out.append(t)
    return out


def rand_expr(rng, names):
    k = rng.random()
    if k < 0.3:
        return expr("topology.kubernetes.io/zone", rng.choice(["In", "NotIn"]), rng.sample(ZONES, rng.randint(1, 2)))
    if k < 0.5:
        return expr("disk", rng.choice(["Exists", "DoesNotExist"]))
    if k < 0.7:
        return expr("gen", rng.choice(["Gt", "Lt"]), [str(rng.randint(1, 5))])
    if k < 0.8:
        return expr("kubernetes.io/hostname", "In", rng.sample(names, min(3, len(names))))
    return expr("disk", "In", [rng.choice(["ssd", "hdd", "nvme"])])


APPS = ["web", "db", "cache", "batch"]
NAMESPACES = [("default", {"team": "a"}), ("prod", {"team": "a", "env": "prod"}), ("dev", {"team": "b"})]
TOPO_KEYS = ["topology.kubernetes.io/zone", "kubernetes.io/hostname", "disk"]


def rand_label_selector(rng):
    r = rng.random()
    if r < 0.1:
        return None  # nil selector
    if r < 0.15:
        return {}  # everything
    if r < 0.6:
        return {"matchLabels": {"app": rng.choice(APPS)}}
    if r < 0.8:
        return {"matchExpressions": [{"key": "app", "operator": rng.choice(["In", "NotIn"]),
                                      "values": rng.sample(APPS, rng.randint(1, 2))}]}
    return {"matchExpressions": [{"key": rng.choice(["tier", "app"]), "operator": rng.choice(["Exists", "DoesNotExist"])}]}


def rand_pa_term(rng):
    t = {"topologyKey": rng.choice(TOPO_KEYS)}
    sel = rand_label_selector(rng)
    if sel is not None:
        t["labelSelector"] = sel
    r = rng.random()
    if r < 0.2:
        t["namespaces"] = rng.sample([n for n, _ in NAMESPACES], rng.randint(1, 2))
    elif r < 0.35:
        t["namespaceSelector"] = rng.choice([{}, {"matchLabels": {"team": "a"}}, {"matchLabels": {"env": "prod"}}])
    return t


def add_topology(rng, p, allow_required=True):
    """Pod (anti-)affinity terms and topology spread constraints."""
    spec = p.o["spec"]
    if rng.random() < 0.3:
        aff = spec.setdefault("affinity", {})
        for kind in ("podAffinity", "podAntiAffinity"):
            if rng.random() < 0.5:
                continue
            a = aff.setdefault(kind, {})
            if allow_required and rng.random() < 0.5:
                a["requiredDuringSchedulingIgnoredDuringExecution"] = [rand_pa_term(rng) for _ in range(rng.randint(1, 2))]
            if rng.random() < 0.6:
                a["preferredDuringSchedulingIgnoredDuringExecution"] = [
                    {"weight": rng.randint(1, 100), "podAffinityTerm": rand_pa_term(rng)} for _ in range(rng.randint(1, 2))]
    if rng.random() < 0.3:
        for _ in range(rng.randint(1, 2)):
            c = {"maxSkew": rng.randint(1, 3), "topologyKey": rng.choice(TOPO_KEYS),
                 "whenUnsatisfiable": rng.choice(["DoNotSchedule", "ScheduleAnyway"])}
            sel = rand_label_selector(rng)
            if sel is not None:
                c["labelSelector"] = sel
            if rng.random() < 0.2:
                c["minDomains"] = rng.randint(1, 4)
                c["whenUnsatisfiable"] = "DoNotSchedule"
            if rng.random() < 0.2:
                c["nodeTaintsPolicy"] = rng.choice(["Honor", "Ignore"])
            if rng.random() < 0.2:
                c["nodeAffinityPolicy"] = rng.choice(["Honor", "Ignore"])
            if rng.random() < 0.15:
                c["matchLabelKeys"] = ["tier"]
            spec.setdefault("topologySpreadConstraints", []).append(c)


def rand_pod(rng, k, names, ns=None, topology=True):
    ns = ns or rng.choice([n for n, _ in NAMESPACES])
    p = PodW(f"p{k}", ns)
    p.label("app", rng.choice(APPS))
    if rng.random() < 0.5:
        p.label("tier", rng.choice(["fe", "be"]))
    if rng.random() < 0.05:
        p.terminating()
    for _ in range(rng.choice([1, 1, 2])):
        ports = None
        if rng.random() < 0.12:
            ports = [{"containerPort": 8080, "hostPort": rng.choice([80, 443, 8080]),
                      "protocol": rng.choice(["TCP", "UDP"]), **({"hostIP": "10.0.0.1"} if rng.random() < 0.3 else {})}]
        img = rng.choice([n for n, _ in IMAGES] + ["registry.example/other:1", ""])
        p.container(image=img, requests=rand_requests(rng), ports=ports)
    if rng.random() < 0.1:
        p.init_req(rand_requests(rng), sidecar=rng.random() < 0.5)
    if rng.random() < 0.05:
        p.overhead({"cpu": "50m", "memory": "64Mi"})
    tol = rand_tolerations(rng)
    if tol:
        p.tolerations(tol)
    if rng.random() < 0.15:
        p.node_selector({"topology.kubernetes.io/zone": rng.choice(ZONES)})
    r = rng.random()
    if r < 0.2:
        terms = [{"matchExpressions": [rand_expr(rng, names) for _ in range(rng.randint(1, 2))]}
                 for _ in range(rng.randint(1, 2))]
        p.node_affinity_required(terms)
    elif r < 0.25 and names:
        p.node_affinity_required([{"matchFields": [
            {"key": "metadata.name", "operator": "In", "values": rng.sample(names, min(len(names), rng.randint(1, 4)))}]}])
    if rng.random() < 0.25:
        p.node_affinity_preferred([(rng.randint(1, 100), {"matchExpressions": [rand_expr(rng, names)]})
                                   for _ in range(rng.randint(1, 3))])
    if rng.random() < 0.02 and names:
        p.o["spec"]["nodeName"] = rng.choice(names + ["missing-node"])
    if topology:
        add_topology(rng, p)
    return p.obj()


CONFIGS = [
    {},
    {"nodeResourcesFit": {"scoringStrategy": {"type": "MostAllocated"}}},
    {"nodeResourcesFit": {"scoringStrategy": {
        "type": "RequestedToCapacityRatio",
        "resources": [{"name": "cpu", "weight": 2}, {"name": "memory", "weight": 1}, {"name": "example.com/gpu", "weight": 3}],
        "requestedToCapacityRatio": {"shape": [{"utilization": 0, "score": 10}, {"utilization": 60, "score": 3},
                                               {"utilization": 100, "score": 0}]}}}},
    {"nodeResourcesFit": {"scoringStrategy": {"type": "LeastAllocated", "resources": [
        {"name": "cpu", "weight": 1}, {"name": "memory", "weight": 2}, {"name": "example.com/gpu", "weight": 5}]}},
     "balancedAllocation": {"resources": [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1},
                                          {"name": "example.com/gpu", "weight": 1}]}},
    {"nodeAffinity": {"addedAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": "gen", "operator": "Lt", "values": ["6"]}]}]},
        "preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 7, "preference": {"matchExpressions": [{"key": "disk", "operator": "In", "values": ["ssd"]}]}}]}}},
    {"disabledPlugins": ["ImageLocality", "NodeResourcesBalancedAllocation"], "scoreWeights": {"TaintToleration": "1"}},
    {"interPodAffinity": {"hardPodAffinityWeight": 5}},
    {"interPodAffinity": {"ignorePreferredTermsOfExistingPods": True, "hardPodAffinityWeight": 0}},
]


def rand_cluster(seed, n_nodes, n_existing, cfg_index=None, topology=True):
    rng = random.Random(seed)
    cfg = CONFIGS[cfg_index if cfg_index is not None else rng.randrange(len(CONFIGS))]
    nodes = [rand_node(rng, i) for i in range(n_nodes)]
    names = [n["metadata"]["name"] for n in nodes]
    existing = []
    for k in range(n_existing):
        p = rand_pod(rng, 100000 + k, names, topology=topology)
        p["spec"].get("affinity", {}).pop("nodeAffinity", None)
        p["spec"]["nodeName"] = rng.choice(names)
        existing.append(p)
    return rng, cfg, nodes, existing, names


def add_resize_status(rng, pod):
    """In-place resize state on a bound pod (InPlacePodVerticalScaling, GA): container statuses whose
    resources / allocatedResources differ from the spec, sometimes for an init or sidecar container of
    the same name, a pod-level request with status.resources, and a PodResizePending (Deferred /
    Infeasible) or PodResizeInProgress condition (component-helpers resource/helpers.go:193-320)."""
    spec, st = pod["spec"], pod.setdefault("status", {})

    def some():
        r = {}
        if rng.random() < 0.8:
            r["cpu"] = rng.choice(["50m", "200m", "750m", "2", "4"])
        if rng.random() < 0.7:
            r["memory"] = rng.choice(["64Mi", "300Mi", "2Gi", "6Gi"])
        if rng.random() < 0.1:
            r["ephemeral-storage"] = rng.choice(["512Mi", "2Gi"])
        return r

    for key, skey in (("containers", "containerStatuses"), ("initContainers", "initContainerStatuses")):
        for c in spec.get(key, []):
            if rng.random() < 0.6:
                cs = {"name": c["name"]}
                if rng.random() < 0.85:
                    cs["resources"] = {"requests": some()} if rng.random() < 0.9 else {}
                if rng.random() < 0.5:
                    cs["allocatedResources"] = some()
                st.setdefault(skey, []).append(cs)
    if rng.random() < 0.15:
        spec["resources"] = {"requests": some()}
        if rng.random() < 0.7:
            st["resources"] = {"requests": some()}
            if rng.random() < 0.5:
                st["allocatedResources"] = some()
    r = rng.random()
    if r < 0.25:
        st.setdefault("conditions", []).append({"type": "PodResizePending", "status": "True",
                                                "reason": rng.choice(["Deferred", "Infeasible"])})
    elif r < 0.35:
        st.setdefault("conditions", []).append({"type": "PodResizeInProgress", "status": "True"})
    return pod


def namespaces():
    return [make_namespace(n, l) for n, l in NAMESPACES]


# ---- PodTopologySpread default constraints: the selecting objects (helper.DefaultSelector) ------------
OWNER_KINDS = [("apps/v1", "ReplicaSet"), ("apps/v1", "StatefulSet"), ("v1", "ReplicationController"),
               ("extensions/v1beta1", "ReplicaSet"), ("apps/v1/x", "ReplicaSet")]


def rand_objects(rng, n=8):
    """Services / RCs / RSs / StatefulSets over the APPS labels, in the fuzz namespaces."""
    out = []
    for k in range(n):
        kind = rng.choice(["Service", "Service", "ReplicationController", "ReplicaSet", "StatefulSet"])
        ns = rng.choice([n for n, _ in NAMESPACES])
        o = {"apiVersion": "apps/v1" if kind in ("ReplicaSet", "StatefulSet") else "v1", "kind": kind,
             "metadata": {"name": f"{kind.lower()}-{k % 3}", "namespace": ns}, "spec": {}}
        if kind in ("Service", "ReplicationController"):
            r = rng.random()
            if r < 0.1:
                pass  # nil selector
            elif r < 0.15:
                o["spec"]["selector"] = {}
            else:
                sel = {"app": rng.choice(APPS)}
                if rng.random() < 0.3:
                    sel["tier"] = rng.choice(["fe", "be"])
                o["spec"]["selector"] = sel
        else:
            sel = rand_label_selector(rng)
            if sel is not None:
                o["spec"]["selector"] = sel
        out.append(o)
    last = {}  # one object per (kind, namespace, name): a later one replaces it, as an upsert does
    for o in out:
        last[(o["kind"], o["metadata"]["namespace"], o["metadata"]["name"])] = o
    return list(last.values())


def add_owner(rng, p):
    """A controller ownerReference naming one of rand_objects' names (which may not exist)."""
    if rng.random() < 0.7:
        api, kind = rng.choice(OWNER_KINDS)
        p["metadata"]["ownerReferences"] = [{"apiVersion": api, "kind": kind, "name": f"{kind.lower()}-{rng.randint(0, 2)}",
                                             "controller": rng.random() < 0.9}]
    return p


PTS_DEFAULT_CONFIGS = [
    {},  # System defaulting: hostname maxSkew 3 + zone maxSkew 5, ScheduleAnyway
    {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": [
        {"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule"},
        {"maxSkew": 2, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "ScheduleAnyway"}]}},
    {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": [
        {"maxSkew": 2, "topologyKey": "disk", "whenUnsatisfiable": "ScheduleAnyway", "nodeTaintsPolicy": "Honor"},
        {"maxSkew": 3, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "DoNotSchedule",
         "minDomains": 2}]}},
    {"podTopologySpread": {"defaultingType": "List"}},
]
