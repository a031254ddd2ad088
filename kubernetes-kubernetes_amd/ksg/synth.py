"""Seeded synthetic clusters shaped like the reference's scheduler_perf workloads.

SchedulingBasic (test/integration/scheduler_perf/misc/performance-config.yaml:57-63):
  nodes from templates/node-default.yaml -- allocatable cpu 4, memory 32Gi, pods 110,
  label kubernetes.io/hostname (node_util.go:99-111);
  pods from templates/pod-default.yaml -- one container, requests cpu 100m / memory 500Mi,
  image registry.k8s.io/pause:3.10.2, containerPort 80 without a hostPort.
`hetero=True` is SURVEY.md §8(d)'s heterogeneous variant (mixed capacities, pre-load, images)
that makes scores untied so placement parity is exercised on distinct maxima too.
"""
import random

from .objects import NodeW, PodW

PAUSE = "registry.k8s.io/pause:3.10.2"
GI = 1024 ** 3


def node_default(name):
    return (NodeW(name).capacity({"cpu": "4", "memory": "32Gi", "pods": "110"})
            .label("kubernetes.io/hostname", name).obj())


def pod_default(name, ns="default", node=None):
    p = PodW(name, ns).container(image=PAUSE, requests={"cpu": "100m", "memory": "500Mi"},
                                 ports=[{"containerPort": 80}])
    if node:
        p.node(node)
    return p.obj()


def scheduling_basic(n_nodes, n_init, n_pods, hetero=False, seed=0x5EED):
    """-> (nodes, init_pods (bound), measured pods), all as v1 JSON dicts."""
    rng = random.Random(seed)
    nodes = []
    images = [(f"registry.example/img-{k}:v1", rng.randint(10, 2000) * 1000 * 1000) for k in range(16)]
    for i in range(n_nodes):
        name = f"node-{i:06d}"
        if not hetero:
            nodes.append(node_default(name))
            continue
        cpu = rng.choice([4, 8, 16, 32, 64])
        mem = rng.choice([16, 32, 64, 128, 256])
        w = (NodeW(name).capacity({"cpu": str(cpu), "memory": f"{mem}Gi", "pods": "110"})
             .label("kubernetes.io/hostname", name).label("topology.kubernetes.io/zone", f"zone-{i % 10}"))
        imgs = rng.sample(images, rng.randint(0, 3))
        if imgs:
            w.images({n: s for n, s in imgs})
        nodes.append(w.obj())
    init = []
    names = [n["metadata"]["name"] for n in nodes]
    for k in range(n_init):
        if hetero:
            node = rng.choice(names)
            p = PodW(f"init-{k}", "default").container(
                image=PAUSE, requests={"cpu": f"{rng.randint(1, 8) * 250}m", "memory": f"{rng.randint(1, 16) * 256}Mi"})
            init.append(p.node(node).obj())
        else:
            init.append(pod_default(f"init-{k}", node=names[k % len(names)]))
    pods = []
    for k in range(n_pods):
        if hetero:
            p = PodW(f"pod-{k}", "default").container(
                image=rng.choice([PAUSE] + [n for n, _ in images]),
                requests={"cpu": f"{rng.randint(1, 10) * 100}m", "memory": f"{rng.randint(1, 20) * 100}Mi"})
            pods.append(p.obj())
        else:
            pods.append(pod_default(f"pod-{k}"))
    return nodes, init, pods


def _pause_pod(name, ns, labels):
    p = PodW(name, ns).labels(labels).container(image=PAUSE, requests={"cpu": "100m", "memory": "500Mi"},
                                                ports=[{"containerPort": 80}])
    return p


def pod_with_pod_affinity(name, ns):
    """templates/pod-with-pod-affinity.yaml: required affinity to color=blue in the zone."""
    p = _pause_pod(name, ns, {"color": "blue"})
    p.o["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
        "labelSelector": {"matchLabels": {"color": "blue"}}, "topologyKey": "topology.kubernetes.io/zone",
        "namespaces": ["sched-1", "sched-0"]}]}}
    return p.obj()


def pod_with_topology_spreading(name, ns):
    """templates/pod-with-topology-spreading.yaml: zone spread, maxSkew 5, DoNotSchedule."""
    p = _pause_pod(name, ns, {"color": "blue"})
    p.o["spec"]["topologySpreadConstraints"] = [{
        "maxSkew": 5, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule",
        "labelSelector": {"matchLabels": {"color": "blue"}}}]
    return p.obj()


def pod_with_preferred_pod_anti_affinity(name, ns):
    """templates/pod-with-preferred-pod-anti-affinity.yaml: soft hostname anti-affinity, weight 1."""
    p = _pause_pod(name, ns, {"color": "yellow"})
    p.o["spec"]["affinity"] = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [{
        "weight": 1, "podAffinityTerm": {"labelSelector": {"matchLabels": {"color": "yellow"}},
                                         "topologyKey": "kubernetes.io/hostname",
                                         "namespaces": ["sched-1", "sched-0"]}}]}}
    return p.obj()


def scheduling_pod_affinity(n_nodes, n_init, n_pods, seed=0x5EED):
    """BASELINE C3 / SchedulingPodAffinity (affinity/performance-config.yaml:96-139): every node in
    zone1; init pods (sched-0) and measured pods (sched-1) from pod-with-pod-affinity."""
    nodes = [NodeW(f"node-{i:06d}").capacity({"cpu": "4", "memory": "32Gi", "pods": "110"})
             .label("kubernetes.io/hostname", f"node-{i:06d}").label("topology.kubernetes.io/zone", "zone1").obj()
             for i in range(n_nodes)]
    names = [n["metadata"]["name"] for n in nodes]
    init = []
    for k in range(n_init):
        p = pod_with_pod_affinity(f"init-{k}", "sched-0")
        p["spec"]["nodeName"] = names[k % n_nodes]
        init.append(p)
    pods = [pod_with_pod_affinity(f"pod-{k}", "sched-1") for k in range(n_pods)]
    return nodes, init, pods


def pod_with_node_inclusion_policy(name, ns):
    """templates/pod-with-node-inclusion-policy.yaml: hostname spread, maxSkew 1, DoNotSchedule,
    nodeAffinityPolicy / nodeTaintsPolicy Honor, selector foo=bar."""
    p = _pause_pod(name, ns, {"foo": "bar"})
    p.o["spec"]["topologySpreadConstraints"] = [{
        "maxSkew": 1, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "DoNotSchedule",
        "nodeAffinityPolicy": "Honor", "nodeTaintsPolicy": "Honor", "labelSelector": {"matchLabels": {"foo": "bar"}}}]
    return p.obj()


def scheduling_c3(n_nodes, n_init, n_pods, taint_every=5, seed=0x5EED):
    """BASELINE C3 (configs[2]): SchedulingPodAffinity + NodeAffinity + taints.

    Nodes: node-default in zone1 (affinity/performance-config.yaml:96-139, labelNodePrepareStrategy
    zone1); every `taint_every`-th one is node-with-taint (foo:NoSchedule) -- 1000 of 5000, as in
    SchedulingWithNodeInclusionPolicy (topology_spreading/performance-config.yaml:149-180).
    Init pods: pod-with-pod-affinity in sched-0, bound round-robin to the untainted nodes (the
    pods tolerate no taint).  Measured stream, in turn: pod-with-pod-affinity (sched-1),
    pod-with-node-affinity (zone In [zone1, zone2], affinity/performance-config.yaml:222-259),
    pod-with-node-inclusion-policy (hostname spread honouring affinity and taints)."""
    nodes, plain = [], []
    for i in range(n_nodes):
        name = f"node-{i:06d}"
        w = (NodeW(name).capacity({"cpu": "4", "memory": "32Gi", "pods": "110"})
             .label("kubernetes.io/hostname", name).label("topology.kubernetes.io/zone", "zone1"))
        if i % taint_every == taint_every - 1:
            w.taints([{"key": "foo", "effect": "NoSchedule"}])
        else:
            plain.append(name)
        nodes.append(w.obj())
    init = []
    for k in range(n_init):
        p = pod_with_pod_affinity(f"init-{k}", "sched-0")
        p["spec"]["nodeName"] = plain[k % len(plain)]
        init.append(p)
    pods = []
    for k in range(n_pods):
        kind = k % 3
        if kind == 0:
            pods.append(pod_with_pod_affinity(f"pod-{k}", "sched-1"))
        elif kind == 1:
            pods.append(pod_with_node_affinity(f"pod-{k}", "sched-1", ["zone1", "zone2"]))
        else:
            pods.append(pod_with_node_inclusion_policy(f"pod-{k}", "sched-1"))
    return nodes, init, pods


def topology_spreading(n_nodes, n_init, n_pods, preferred_anti=False, seed=0x5EED):
    """BASELINE C4 / TopologySpreading (topology_spreading/performance-config.yaml:20-59): zones
    moon-1/2/3 round-robin, init pod-default pods, measured pod-with-topology-spreading (or, with
    preferred_anti, pod-with-preferred-pod-anti-affinity)."""
    nodes = [NodeW(f"node-{i:06d}").capacity({"cpu": "4", "memory": "32Gi", "pods": "110"})
             .label("kubernetes.io/hostname", f"node-{i:06d}")
             .label("topology.kubernetes.io/zone", f"moon-{i % 3 + 1}").obj() for i in range(n_nodes)]
    names = [n["metadata"]["name"] for n in nodes]
    init = [pod_default(f"init-{k}", ns="sched-0", node=names[k % n_nodes]) for k in range(n_init)]
    make = pod_with_preferred_pod_anti_affinity if preferred_anti else pod_with_topology_spreading
    pods = [make(f"pod-{k}", "sched-1") for k in range(n_pods)]
    return nodes, init, pods


def pod_with_node_affinity(name, ns, zones):
    """templates/pod-with-node-affinity.yaml: required zone In [...]"""
    p = _pause_pod(name, ns, {"color": "green"})
    p.o["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [
            {"key": "topology.kubernetes.io/zone", "operator": "In", "values": zones}]}]}}}
    return p.obj()


def pod_with_required_anti_affinity(name, ns):
    """templates/pod-with-pod-anti-affinity.yaml: required hostname anti-affinity to itself."""
    p = _pause_pod(name, ns, {"color": "red"})
    p.o["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
        "labelSelector": {"matchLabels": {"color": "red"}}, "topologyKey": "kubernetes.io/hostname",
        "namespaces": ["sched-1", "sched-0"]}]}}
    return p.obj()


def mixed_cluster(n_nodes, n_init, n_pods, zones=10, seed=0x5EED):
    """BASELINE C5: n_nodes heterogeneous nodes in `zones` zones round-robin, 1 %
    tainted NoSchedule, pre-loaded with n_init bound pod-default / affinity-seed pods; the measured
    stream draws 50 % pod-default, 10 % each node-affinity, required pod-affinity, required
    hostname anti-affinity, preferred hostname anti-affinity, zone spread (fixed proportions,
    seeded order)."""
    rng = random.Random(seed)
    nodes = []
    for i in range(n_nodes):
        name = f"node-{i:06d}"
        w = (NodeW(name).capacity({"cpu": str(rng.choice([8, 16, 32, 64])),
                                   "memory": f"{rng.choice([32, 64, 128, 256])}Gi", "pods": "110"})
             .label("kubernetes.io/hostname", name).label("topology.kubernetes.io/zone", f"zone-{i % zones}"))
        if i % 100 == 37:
            w.taints([{"key": "dedicated", "value": "infra", "effect": "NoSchedule"}])
        nodes.append(w.obj())
    names = [n["metadata"]["name"] for n in nodes]
    init = []
    for k in range(n_init):
        node = names[rng.randrange(n_nodes)]
        if k % 10 == 0:  # seeds for the required pod-affinity pods (color=blue in some zones)
            p = _pause_pod(f"init-{k}", "sched-0", {"color": "blue"}).obj()
            p["spec"]["nodeName"] = node
            init.append(p)
        else:
            init.append(pod_default(f"init-{k}", ns="sched-0", node=node))
    kinds = ["default"] * 5 + ["node-affinity", "pod-affinity", "anti-affinity", "preferred-anti", "spread"]
    pods = []
    for k in range(n_pods):
        kind = kinds[rng.randrange(len(kinds))]
        nm = f"pod-{k}"
        if kind == "default":
            pods.append(pod_default(nm, ns="sched-1"))
        elif kind == "node-affinity":
            pods.append(pod_with_node_affinity(nm, "sched-1", [f"zone-{z}" for z in rng.sample(range(zones), 2)]))
        elif kind == "pod-affinity":
            pods.append(pod_with_pod_affinity(nm, "sched-1"))
        elif kind == "anti-affinity":
            pods.append(pod_with_required_anti_affinity(nm, "sched-1"))
        elif kind == "preferred-anti":
            pods.append(pod_with_preferred_pod_anti_affinity(nm, "sched-1"))
        else:
            pods.append(pod_with_topology_spreading(nm, "sched-1"))
    return nodes, init, pods


def pod_with_label(name, ns):
    """templates/pod-with-label.yaml: label app=scheduler-perf, one pause container without requests."""
    return PodW(name, ns).labels({"app": "scheduler-perf"}).container(image="registry.k8s.io/pause:3.10.1").obj()


def default_topology_spreading(n_nodes, n_init, n_pods, seed=0x5EED):
    """scheduler_perf DefaultTopologySpreading (topology_spreading/performance-config.yaml:102-147):
    node-default nodes labelled topology.kubernetes.io/zone moon-1/2/3 round-robin, one Service
    (templates/service.yaml, selector app=scheduler-perf) in service-ns, init pod-default pods, then
    measured pod-with-label pods in service-ns -- they have no constraints of their own, so every one
    is scored by PodTopologySpread's system default constraints (hostname maxSkew 3, zone maxSkew 5)
    with the Service's selector.  -> (nodes, init pods (bound), measured pods, objects)."""
    nodes, init, _ = topology_spreading(n_nodes, n_init, 0, seed=seed)
    for p in init:
        p["metadata"]["namespace"] = "default"
    service = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "service-0", "namespace": "service-ns"},
               "spec": {"selector": {"app": "scheduler-perf"}, "ports": [{"protocol": "TCP", "port": 80,
                                                                            "targetPort": 8000}]}}
    pods = [pod_with_label(f"pod-{k}", "service-ns") for k in range(n_pods)]
    return nodes, init, pods, [service]


PAUSE_310_1 = "registry.k8s.io/pause:3.10.1"  # the batching templates' image


def batching(n_nodes, n_pods, kind="hostport"):
    """scheduler_perf's OpportunisticBatching workloads (test/integration/scheduler_perf/batching/
    performance-config.yaml): node-default nodes and one pod template that fits once per node --
    HostPortConflict: templates/pod-hostport-80.yaml (100m / 100Mi, hostPort 80); ResourceSaturation:
    templates/pod-saturation.yaml (3 cpu / 1Gi on 4-cpu nodes).  Run them with the no-topology profile
    (batching/scheduler-config-no-topology.yaml: PodTopologySpread List defaulting, no default constraints).
    -> (nodes, pods)."""
    nodes = [node_default(f"node-{i:06d}") for i in range(n_nodes)]
    pods = []
    for k in range(n_pods):
        if kind == "hostport":
            p = PodW(f"pod-hostport-80-{k}", "default").container(
                image=PAUSE_310_1, requests={"cpu": "100m", "memory": "100Mi"},
                ports=[{"containerPort": 80, "hostPort": 80}])
        elif kind == "saturation":
            p = PodW(f"pod-saturation-{k}", "default").container(image=PAUSE_310_1,
                                                                 requests={"cpu": "3", "memory": "1Gi"})
        else:
            raise ValueError(kind)
        pods.append(p.obj())
    return nodes, pods
