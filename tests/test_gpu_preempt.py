"""DefaultPreemption on the device (k_preempt through ksg_preempt) against the CPU oracle's restatement
of default_preemption.go / preemption.go.

Bar: the identical PostFilter outcome -- reason, nominated node, every DryRunPreemption candidate with
its victims (in order) and NumPDBViolations, the selected node's victims -- over random clusters with
mixed priorities, start times (some pods without one: the caller's clock), PodDisruptionBudgets, host
ports, extended resources, pod counts, and every potential-node / offset / numCandidates regime.
"""
import random

import pytest

from oracle_binding import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from ksg.native import Scheduler
    return Scheduler


ZONES = ["z1", "z2", "z3"]


def mk_node(i, rng):
    alloc = {"cpu": f"{rng.choice([1000, 2000, 4000])}m", "memory": str(rng.choice([2, 4, 8]) * 1024 ** 3),
             "pods": str(rng.choice([4, 6, 110]))}
    if rng.random() < 0.3:
        alloc["example.com/gpu"] = str(rng.choice([1, 2, 4]))
    n = {"apiVersion": "v1", "kind": "Node",
         "metadata": {"name": f"n{i:04d}", "labels": {"kubernetes.io/hostname": f"n{i:04d}",
                                                      "topology.kubernetes.io/zone": rng.choice(ZONES)}},
         "spec": {}, "status": {"allocatable": alloc, "capacity": alloc}}
    if rng.random() < 0.1:
        n["spec"]["taints"] = [{"key": "dedicated", "value": "x", "effect": "NoSchedule"}]
    if rng.random() < 0.05:
        n["spec"]["unschedulable"] = True
    return n


def mk_pod(name, rng, node=None, prio=None, big=False):
    req = {"cpu": f"{rng.choice([100, 250, 500, 900]) * (3 if big else 1)}m",
           "memory": str(rng.choice([128, 512, 1024]) * (3 if big else 1) * 1024 ** 2)}
    if rng.random() < (0.3 if big else 0.15):
        req["example.com/gpu"] = "1"
    c = {"name": "c", "image": "img", "resources": {"requests": req}}
    if rng.random() < 0.15:
        c["ports"] = [{"containerPort": 80, "hostPort": rng.choice([8080, 8081]), "protocol": "TCP"}]
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": rng.choice(["default", "team"]), "uid": name,
                      "labels": {"app": rng.choice(["a", "b", "c"])}},
         "spec": {"containers": [c], "priority": prio if prio is not None else rng.choice([-100, 0, 0, 100, 500])},
         "status": {}}
    if rng.random() < 0.7:
        p["status"]["startTime"] = f"2024-01-01T00:{rng.randrange(60):02d}:{rng.randrange(60):02d}Z"
    if rng.random() < 0.1:
        p["spec"]["tolerations"] = [{"key": "dedicated", "operator": "Exists", "effect": "NoSchedule"}]
    if node:
        p["spec"]["nodeName"] = node
    return p


def pdbs(rng):
    out = []
    for k in range(rng.randrange(0, 4)):
        sel = rng.choice([{"matchLabels": {"app": rng.choice(["a", "b"])}},
                          {"matchExpressions": [{"key": "app", "operator": "In", "values": ["a", "c"]}]},
                          {}])
        out.append({"metadata": {"namespace": rng.choice(["default", "team"])}, "spec": {"selector": sel},
                    "status": {"disruptionsAllowed": rng.randrange(0, 3),
                               "disruptedPods": {f"e{rng.randrange(40)}": "2024-01-01T00:00:00Z"}}})
    return out


def build(make, nodes, existing):
    b = make({})
    b.upsert_namespace({"metadata": {"name": "default"}})
    b.upsert_namespace({"metadata": {"name": "team"}})
    for n in nodes:
        b.add_node(n)
    for p in existing:
        b.add_pod(p)
    return b


def cluster(seed, n_nodes, per_node):
    rng = random.Random(seed)
    nodes = [mk_node(i, rng) for i in range(n_nodes)]
    existing = []
    for i, n in enumerate(nodes):
        for k in range(rng.randrange(per_node + 1)):
            existing.append(mk_pod(f"e{i}-{k}", rng, node=n["metadata"]["name"]))
    return rng, nodes, existing


def compare(dev, orc, pod, args):
    """Both device paths (the device-resident pod segments, and host-staged records via the
    debugHostStaged diagnostic), each with both dry-run stores (registers, and the per-node workspace
    via debugWideDryRun), against the oracle."""
    args = dict(args, listCandidates=True)
    r2, d2 = orc.preempt(orc.compile(pod), args)
    for extra in ({}, {"debugHostStaged": True}, {"debugWideDryRun": True},
                  {"debugHostStaged": True, "debugWideDryRun": True}):
        r1, d1 = dev.preempt(dev.compile(pod), dict(args, **extra))
        assert r1.as_tuple() == r2.as_tuple(), (extra, r1.as_tuple(), r2.as_tuple(), d1, d2)
        assert d1 == d2, extra
    return r1, d1


@pytest.mark.parametrize("seed", range(6))
def test_preempt_matches_oracle_random(native, seed):
    rng, nodes, existing = cluster(seed, 60 + 40 * seed, 6)
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(12):
        pod = mk_pod(f"pre{q}", rng, prio=rng.choice([100, 500, 1000]), big=True)
        args = {"offset": rng.randrange(1000), "now": 1704067200 * 10 ** 9 + rng.randrange(3600) * 10 ** 9,
                "pdbs": pdbs(rng), "allNodes": rng.random() < 0.3,
                "minCandidateNodesPercentage": rng.choice([0, 10, 40, 100]),
                "minCandidateNodesAbsolute": rng.choice([1, 3, 100])}
        if args["minCandidateNodesPercentage"] == 0 and args["minCandidateNodesAbsolute"] == 0:
            args["minCandidateNodesAbsolute"] = 1
        r, d = compare(dev, orc, pod, args)
        found += r.status == 0
        if r.status == 0 and q % 3 == 0:  # actuate: the victims go, the pod binds; the next query sees it
            for uid in d["victims"]:
                dev.remove_pod(uid)
                orc.remove_pod(uid)
            p2 = dict(pod, spec=dict(pod["spec"], nodeName=d["selected"]))
            dev.add_pod(p2)
            orc.add_pod(p2)
    assert found > 0  # the streams do exercise a nomination


@pytest.mark.parametrize("seed", range(2))
def test_preempt_without_now(native, seed):
    """Calls that omit "now": product and oracle each read the wall clock once per call (GetPodStartTime's
    time.Now()).  Every pod here has status.startTime, so the clock is never decisive and the outcomes
    (candidates, victims, their order by start time) must agree exactly."""
    rng, nodes, existing = cluster(70 + seed, 120, 6)
    for k, p in enumerate(existing):
        p["status"]["startTime"] = f"2024-01-01T{k % 24:02d}:{rng.randrange(60):02d}:{rng.randrange(60):02d}Z"
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(10):
        pod = mk_pod(f"pre{q}", rng, prio=rng.choice([100, 500, 1000]), big=True)
        r, _ = compare(dev, orc, pod, {"offset": rng.randrange(1000), "pdbs": pdbs(rng)})
        found += r.status == 0
    assert found > 0


def test_preempt_policy_never_and_terminating_victims(native):
    rng, nodes, existing = cluster(11, 40, 5)
    # a victim on the nominated node terminating by preemption blocks a new preemption
    victim = mk_pod("vt", rng, node=nodes[0]["metadata"]["name"], prio=-100)
    victim["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
    victim["status"]["conditions"] = [{"type": "DisruptionTarget", "status": "True", "reason": "PreemptionByScheduler"}]
    existing.append(victim)
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    pod = mk_pod("pre", rng, prio=1000, big=True)
    pod["status"]["nominatedNodeName"] = nodes[0]["metadata"]["name"]
    r, _ = compare(dev, orc, pod, {})
    never = mk_pod("never", rng, prio=1000, big=True)
    never["spec"]["preemptionPolicy"] = "Never"
    r, _ = compare(dev, orc, never, {})
    assert r.reason == 1


def test_preempt_large_cluster(native):
    """5000 nodes, ~40k bound pods, full nodes: the PreemptionBasic shape (scheduler_perf
    misc/performance-config.yaml) at the C2 node count."""
    rng = random.Random(5)
    nodes = []
    for i in range(5000):
        alloc = {"cpu": "4000m", "memory": str(16 * 1024 ** 3), "pods": "110"}
        nodes.append({"apiVersion": "v1", "kind": "Node",
                      "metadata": {"name": f"n{i:05d}", "labels": {"topology.kubernetes.io/zone": ZONES[i % 3]}},
                      "spec": {}, "status": {"allocatable": alloc, "capacity": alloc}})
    existing = []
    for i in range(5000):
        for k in range(8):
            existing.append({"apiVersion": "v1", "kind": "Pod",
                             "metadata": {"name": f"low-{i}-{k}", "namespace": "default", "uid": f"low-{i}-{k}",
                                          "labels": {"app": "low"}},
                             "spec": {"nodeName": f"n{i:05d}", "priority": rng.choice([0, 10]),
                                      "containers": [{"name": "c", "image": "i", "resources": {"requests": {
                                          "cpu": "500m", "memory": str(2 * 1024 ** 3)}}}]},
                             "status": {"startTime": f"2024-01-01T00:00:{rng.randrange(60):02d}Z"}})
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    for q in range(3):
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"hi{q}", "namespace": "default", "uid": f"hi{q}"},
               "spec": {"priority": 1000, "containers": [{"name": "c", "image": "i", "resources": {"requests": {
                   "cpu": "1200m", "memory": str(3 * 1024 ** 3)}}}]}, "status": {}}
        r, d = compare(dev, orc, pod, {"offset": 1234 + q, "pdbs": [
            {"metadata": {"namespace": "default"}, "spec": {"selector": {"matchLabels": {"app": "low"}}},
             "status": {"disruptionsAllowed": 2}}]})
        assert r.status == 0 and r.num_potential == 5000 and r.num_candidates >= 100


def spread_cluster(seed, n_nodes):
    """Pods labelled app=a/b in one namespace over zoned, hostname-labelled nodes; preemptors spread by
    zone and hostname (DoNotSchedule), so their victims move the spread counts."""
    rng = random.Random(seed)
    nodes = [mk_node(i, rng) for i in range(n_nodes)]
    existing = []
    for i, n in enumerate(nodes):
        for k in range(rng.randrange(6)):
            p = mk_pod(f"e{i}-{k}", rng, node=n["metadata"]["name"])
            p["metadata"]["namespace"] = "default"
            p["metadata"]["labels"] = {"app": rng.choice(["a", "b"])}
            existing.append(p)
    return rng, nodes, existing


@pytest.mark.parametrize("seed", range(4))
def test_preempt_spread_victims_match_oracle(native, seed):
    """Victims that move the preemptor's PodTopologySpread counts (PreemptTopo): both device paths (the
    resident segments and the host-staged records) against the oracle's literal RemovePod / AddPod +
    criticalPaths; some preemptors request an extended resource too."""
    rng, nodes, existing = spread_cluster(100 + seed, 40 + 30 * seed)
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(10):
        pod = mk_pod(f"pre{q}", rng, prio=rng.choice([500, 1000]), big=True)
        pod["metadata"]["namespace"] = "default"
        pod["metadata"]["labels"] = {"app": rng.choice(["a", "b"])}
        keys = rng.sample(["topology.kubernetes.io/zone", "kubernetes.io/hostname"], rng.choice([1, 2]))
        pod["spec"]["topologySpreadConstraints"] = [
            {"maxSkew": rng.choice([1, 2]), "topologyKey": k, "whenUnsatisfiable": "DoNotSchedule",
             "labelSelector": {"matchLabels": {"app": rng.choice(["a", "b"])}}} for k in keys]
        # a clock past every start time keeps the device-resident segments in use
        args = {"offset": rng.randrange(1000), "allNodes": rng.random() < 0.3, "listCandidates": True,
                "now": 1704153600 * 10 ** 9,
                "minCandidateNodesPercentage": rng.choice([10, 100]), "minCandidateNodesAbsolute": rng.choice([1, 100])}
        r1, _ = compare(dev, orc, pod, args)
        found += r1.status == 0
    assert found > 0


def affinity_cluster(seed, n_nodes):
    """Existing pods with required anti-affinity terms (hostname / zone) against app labels, and
    preemptors with required pod affinity / anti-affinity terms: victims move InterPodAffinity's
    existingAntiAffinityCounts, affinityCounts and antiAffinityCounts."""
    rng = random.Random(seed)
    nodes = [mk_node(i, rng) for i in range(n_nodes)]
    existing = []
    for i, n in enumerate(nodes):
        for k in range(rng.randrange(6)):
            p = mk_pod(f"e{i}-{k}", rng, node=n["metadata"]["name"])
            p["metadata"]["namespace"] = "default"
            p["metadata"]["labels"] = {"app": rng.choice(["a", "b", "c"])}
            p["spec"]["containers"][0]["resources"]["requests"].pop("example.com/gpu", None)
            if rng.random() < 0.15:
                p["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"labelSelector": {"matchLabels": {"app": rng.choice(["a", "b"])}},
                     "topologyKey": rng.choice(["kubernetes.io/hostname", "topology.kubernetes.io/zone"])}]}}
            existing.append(p)
    return rng, nodes, existing


@pytest.mark.parametrize("seed", range(4))
def test_preempt_affinity_victims_match_oracle(native, seed):
    """Victims that move the preemptor's InterPodAffinity counts: the device-resident path (PreemptTopo's
    InterPodAffinity deltas, k_preempt_terms, the affinity totals of a self-matching preemptor) against the
    oracle's literal RemovePod / AddPod, on both device paths; some preemptors request an extended resource."""
    rng, nodes, existing = affinity_cluster(200 + seed, 40 + 30 * seed)
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = declined = 0
    for q in range(12):
        pod = mk_pod(f"pre{q}", rng, prio=rng.choice([500, 1000]), big=True)
        pod["metadata"]["namespace"] = "default"
        pod["metadata"]["labels"] = {"app": rng.choice(["a", "b", "c"])}
        kind = rng.choice(["none", "affinity", "anti"])
        if kind != "none":
            key = "podAffinity" if kind == "affinity" else "podAntiAffinity"
            pod["spec"]["affinity"] = {key: {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": rng.choice(["a", "b", "c"])}},
                 "topologyKey": rng.choice(["kubernetes.io/hostname", "topology.kubernetes.io/zone"])}]}}
        args = {"offset": rng.randrange(1000), "allNodes": rng.random() < 0.3, "listCandidates": True,
                "now": 1704153600 * 10 ** 9,
                "minCandidateNodesPercentage": rng.choice([10, 100]), "minCandidateNodesAbsolute": rng.choice([1, 100])}
        r1, _ = compare(dev, orc, pod, args)
        found += r1.status == 0
    assert found > 0


@pytest.mark.parametrize("seed", range(4))
def test_preempt_self_affinity_victims_match_oracle(native, seed):
    """A preemptor that matches its own required affinity terms (filtering.go:404-415): removing victims
    that are the only pods its terms count empties affinityCounts, and the "first pod of a series" rule
    then admits the node.  The matching pods sit on few nodes; the device's per-term totals plus the
    victims' deltas against the oracle's literal RemovePod / AddPod."""
    rng, nodes, existing = affinity_cluster(300 + seed, 30 + 20 * seed)
    # "rare": the pods of one or two nodes only -- removing them as victims can empty affinityCounts
    hosts = rng.sample(sorted({p["spec"]["nodeName"] for p in existing}), 2)
    for p in existing:
        if p["spec"]["nodeName"] == hosts[0] or (p["spec"]["nodeName"] == hosts[1] and rng.random() < 0.3):
            p["metadata"]["labels"] = {"app": "rare"}
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(12):
        # "solo": no existing pod matches (the map is empty from the start)
        app = rng.choice(["rare", "rare", "rare", "a", "solo"])
        pod = mk_pod(f"self{q}", rng, prio=1000, big=True)
        pod["metadata"]["namespace"] = "default"
        pod["metadata"]["labels"] = {"app": app}
        pod["spec"]["containers"][0]["resources"]["requests"].pop("example.com/gpu", None)
        pod["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": app}},
             "topologyKey": rng.choice(["kubernetes.io/hostname", "topology.kubernetes.io/zone"])}]}}
        args = {"offset": rng.randrange(1000), "allNodes": rng.random() < 0.5, "listCandidates": True,
                "now": 1704153600 * 10 ** 9, "minCandidateNodesPercentage": 100, "minCandidateNodesAbsolute": 100}
        r1, _ = compare(dev, orc, pod, args)
        found += r1.status == 0
    assert found > 0


@pytest.mark.parametrize("seed", range(3))
def test_preempt_many_extended_resources(native, seed):
    """Preemptors requesting 1 to 7 extended resources (no fixed limit: the dry run keeps each node's Requested
    of them in a per-node scratch row), victims holding some of them, on both device paths against the
    oracle; with spread constraints on some preemptors, so the topology tracking runs beside them."""
    rng = random.Random(400 + seed)
    res = [f"vendor.example/r{k}" for k in range(7)]
    nodes = []
    for i in range(60 + 20 * seed):
        n = mk_node(i, rng)
        for r in rng.sample(res, rng.randrange(2, 8)):
            n["status"]["allocatable"][r] = str(rng.choice([2, 4, 8]))
        nodes.append(n)
    existing = []
    for i, n in enumerate(nodes):
        for k in range(rng.randrange(6)):
            p = mk_pod(f"e{i}-{k}", rng, node=n["metadata"]["name"])
            p["metadata"]["namespace"] = "default"
            reqs = p["spec"]["containers"][0]["resources"]["requests"]
            for r in rng.sample(res, rng.randrange(0, 4)):
                if r in n["status"]["allocatable"]:
                    reqs[r] = str(rng.choice([1, 2]))
            existing.append(p)
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(12):
        pod = mk_pod(f"x{q}", rng, prio=rng.choice([500, 1000]))
        pod["metadata"]["namespace"] = "default"
        reqs = pod["spec"]["containers"][0]["resources"]["requests"]
        for r in rng.sample(res, rng.randrange(1, 8)):
            reqs[r] = str(rng.choice([1, 2, 3]))
        if q % 3 == 1:
            pod["spec"]["topologySpreadConstraints"] = [
                {"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule",
                 "labelSelector": {"matchLabels": {"app": rng.choice(["a", "b"])}}}]
        args = {"offset": rng.randrange(1000), "now": 1704153600 * 10 ** 9, "allNodes": rng.random() < 0.3,
                "minCandidateNodesPercentage": 100, "minCandidateNodesAbsolute": 100}
        r, _ = compare(dev, orc, pod, args)
        found += r.status == 0
    assert found > 0


def many_keys_cluster(seed, n_nodes):
    """Nodes labelled with 14 topology keys: 7 coarse ones (2-3 values, many nodes per domain) and 7 fine
    ones (a value per pair of nodes); existing pods carry required anti-affinity terms over many distinct
    keys, so the preemptor's existing-anti keys exceed the register store."""
    rng = random.Random(seed)
    coarse = [f"topo.example/c{k}" for k in range(7)]
    fine = [f"topo.example/f{k}" for k in range(7)]
    nodes = []
    for i in range(n_nodes):
        n = mk_node(i, rng)
        for k, key in enumerate(coarse):
            n["metadata"]["labels"][key] = f"v{rng.randrange(2 + k % 2)}"
        for k, key in enumerate(fine):
            n["metadata"]["labels"][key] = f"p{(i + k) // 2}"
        nodes.append(n)
    existing = []
    for i, n in enumerate(nodes):
        for k in range(rng.randrange(6)):
            p = mk_pod(f"e{i}-{k}", rng, node=n["metadata"]["name"])
            p["metadata"]["namespace"] = "default"
            p["metadata"]["labels"] = {"app": rng.choice(["a", "b", "c"]), "tier": rng.choice(["x", "y"])}
            p["spec"]["containers"][0]["resources"]["requests"].pop("example.com/gpu", None)
            if rng.random() < 0.25:
                p["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"labelSelector": {"matchLabels": {"app": "d"}}, "topologyKey": rng.choice(fine)}]}}
            existing.append(p)
    return rng, nodes, existing, coarse, fine


@pytest.mark.parametrize("seed", range(4))
def test_preempt_beyond_register_store(native, seed):
    """Preemptors with more than kPreemptCons (8) DoNotSchedule constraints, required affinity terms,
    required anti-affinity terms or existing-anti keys: the workspace-resident dry run (PreemptWide) on both
    device paths against the oracle's literal RemovePod / AddPod -- no limit below the pod compiler's own
    (kMaxCons spread constraints, kMaxPodTerms terms per kind)."""
    rng, nodes, existing, coarse, fine = many_keys_cluster(500 + seed, 40 + 20 * seed)
    keys = coarse + fine
    dev, orc = build(native, nodes, existing), build(oracle, nodes, existing)
    found = 0
    for q in range(12):
        pod = mk_pod(f"w{q}", rng, prio=rng.choice([500, 1000]), big=True)
        pod["metadata"]["namespace"] = "default"
        # app=d: the existing pods' anti-affinity terms match it (existing-anti keys, up to 7 fine ones)
        pod["metadata"]["labels"] = {"app": rng.choice(["a", "b", "d"]), "tier": rng.choice(["x", "y"])}
        pod["spec"]["containers"][0]["resources"]["requests"].pop("example.com/gpu", None)
        kind = q % 3
        if kind == 0:  # 9-14 DoNotSchedule constraints, one per key
            pod["spec"]["topologySpreadConstraints"] = [
                {"maxSkew": rng.choice([1, 2, 4, 8]), "topologyKey": k, "whenUnsatisfiable": "DoNotSchedule",
                 "labelSelector": {"matchLabels": {rng.choice(["app", "tier"]): rng.choice(["a", "b", "x"])}}}
                for k in rng.sample(keys, rng.randrange(9, 15))]
        elif kind == 1:  # 9-12 required anti-affinity terms (fine keys mostly: victims can clear a domain)
            pod["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": rng.choice(["a", "b", "c"])}}, "topologyKey": k}
                for k in fine + rng.sample(coarse, rng.randrange(2, 6))]}}
        else:  # 9-11 required affinity terms the preemptor itself matches, plus anti terms on fine keys
            pod["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"tier": pod["metadata"]["labels"]["tier"]}}, "topologyKey": k}
                for k in coarse + rng.sample(fine, rng.randrange(2, 5))]},
                "podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"labelSelector": {"matchLabels": {"app": "c"}}, "topologyKey": k} for k in rng.sample(fine, 3)]}}
        args = {"offset": rng.randrange(1000), "allNodes": rng.random() < 0.5, "now": 1704153600 * 10 ** 9,
                "minCandidateNodesPercentage": 100, "minCandidateNodesAbsolute": 100}
        r, _ = compare(dev, orc, pod, args)
        found += r.status == 0
    assert found > 0
