"""The nominator boundary (include/ksg.h ksg_add_nominated_pod) as one scripted scenario, run on
any backend with the ksg ABI (tests/test_nominator_oracle.py: the oracle against the expected outcomes;
tests/test_gpu_nominated.py: the device against the oracle).  addGENominatedPods (framework.go:1265-1294) adds the
pods nominated to a node whose priority is >= the scheduling pod's and whose uid differs; a call where that would
happen on a snapshot node is refused (KSG_ENOTSUP) before anything is scheduled.  An assume of a nominated pod ends
its nomination (schedule_one.go:1131-1134); so does ksg_delete_nominated_pod, or re-adding it without a node."""
from ksg.abi import KSG_ENOTSUP, KsgError


def node(name, cpu="4"):
    return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name}},
            "status": {"allocatable": {"cpu": cpu, "memory": "8Gi", "pods": "20"},
                       "capacity": {"cpu": cpu, "memory": "8Gi", "pods": "20"}}}


def pod(name, prio=0, cpu="500m", nominated=None):
    p = {"metadata": {"name": name, "namespace": "default", "uid": name},
         "spec": {"priority": prio, "containers": [{"name": "c", "image": "i",
                                                     "resources": {"requests": {"cpu": cpu}}}]},
         "status": {}}
    if nominated:
        p["status"]["nominatedNodeName"] = nominated
    return p


def _try(fn):
    """('ok', value) or ('refused', None) for KSG_ENOTSUP; other errors propagate."""
    try:
        return ("ok", fn())
    except KsgError as e:
        if f"rc={KSG_ENOTSUP}" in str(e):
            return ("refused", None)
        raise


def run(b):
    """The scenario on backend b (a fresh context); returns the outcome log."""
    b.upsert_namespace({"metadata": {"name": "default"}})
    for k in range(4):
        b.add_node(node(f"n{k}"))
    log = []

    def one(p, tag):
        out = _try(lambda: b.schedule_one(b.compile(p), assume=True)[0].as_tuple())
        log.append((tag,) + out)

    one(pod("a0"), "no nominations")
    b.add_nominated_pod(pod("hi", prio=100, nominated="n1"))
    one(pod("low"), "lower priority pod, a priority-100 nomination on n1: refused")
    one(pod("eq", prio=100), "equal priority: refused")
    one(pod("top", prio=200), "higher priority pod: the nomination is not added")
    one(pod("hi", prio=100), "the nominated pod itself (own uid)")   # assumed: its nomination ends
    one(pod("low2"), "after the nominated pod was assumed")
    b.add_nominated_pod(pod("ghost", prio=100, nominated="no-such-node"))
    one(pod("low3"), "nominated to a node outside the snapshot")
    b.add_nominated_pod(pod("x", prio=50, nominated="n2"))
    one(pod("p40", prio=40), "priority-50 nomination on n2: refused")
    b.add_nominated_pod(pod("x", prio=50))  # re-added without a node: forgotten
    one(pod("p40b", prio=40), "re-added without a node")
    b.add_nominated_pod(pod("y", prio=10, nominated="n3"))
    hs = [b.compile(pod(f"bt{k}", prio=20 if k else 5)) for k in range(3)]
    log.append(("batch with one pod under a nomination: refused whole",)
               + _try(lambda: [r.as_tuple() for r in b.schedule_batch(hs, assume=True)]))
    b.delete_nominated_pod("y")
    log.append(("batch after the nomination was deleted",)
               + _try(lambda: [r.as_tuple() for r in b.schedule_batch(hs, assume=True)]))
    b.add_nominated_pod(pod("z", prio=1000, nominated="n0"))
    log.append(("preemption under a nomination: refused",)
               + _try(lambda: b.preempt(b.compile(pod("pp", prio=500)), {"offset": 0})[0].as_tuple()))
    return log
