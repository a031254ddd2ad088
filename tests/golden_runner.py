"""Runs the golden fixtures (tests/golden/*.json) against any ksg.h backend."""
import ctypes as C
import glob
import json
import os

from ksg.abi import KsgError

HERE = os.path.dirname(os.path.abspath(__file__))


# fixtures that are not ksg.h cycles: the OpportunisticBatch state machine (tests/test_batching_oracle.py)
NOT_CYCLES = {"batch_basic", "signatures"}


def load_cases():
    out = []
    for path in sorted(glob.glob(os.path.join(HERE, "golden", "*.json"))):
        group = os.path.splitext(os.path.basename(path))[0]
        if group in NOT_CYCLES:
            continue
        with open(path) as f:
            for i, c in enumerate(json.load(f)["cases"]):
                out.append((f"{group}[{i}] {c['name']}", c))
    return out


def case_nodes(case):
    """The case's nodes; `nodes_gen` expands {"count": n, "template": node} with "{i}" in the
    template's name replaced by 0..n-1 (large all-identical clusters stay small on disk)."""
    nodes = list(case["nodes"])
    g = case.get("nodes_gen")
    if g:
        t = json.dumps(g["template"])
        nodes += [json.loads(t.replace("{i}", str(i))) for i in range(g["count"])]
    return nodes


def build(make_backend, case):
    b = make_backend(case.get("config") or {})
    for ns in case.get("namespaces", []):
        b.upsert_namespace(ns)
    for o in case.get("objects", []):  # Services / RCs / RSs / StatefulSets (PodTopologySpread defaults)
        b.upsert_object(o)
    for n in case_nodes(case):
        b.add_node(n)
    for p in case.get("existing", []):
        b.add_pod(p)
    return b


def run_case(make_backend, case):
    """Returns a list of mismatch strings (empty == parity)."""
    if case["kind"] == "config_error":
        try:
            make_backend(case["config"])
        except KsgError:
            return []
        return ["config accepted but the reference rejects it"]
    if case["kind"] == "config_ok":
        try:
            make_backend(case["config"]).close()
        except KsgError as ex:
            return [f"config rejected but the reference accepts it: {ex}"]
        return []
    if case["kind"] == "pod_resources":
        return run_pod_resources_case(make_backend, case)
    b = build(make_backend, case)
    if case["kind"] == "events":
        errs = run_events_case(b, case)
        b.close()
        return errs
    names = b.node_names()
    if case["kind"] == "sequence":
        errs = run_sequence_case(b, case, names)
        b.close()
        return errs
    if case["kind"] == "preempt":
        errs = run_preempt_case(b, case, names)
        b.close()
        return errs
    h = b.compile(case["pod"])
    want_names = [n["metadata"]["name"] for n in case_nodes(case)]
    errs = []
    e = case["expect"]
    if case["kind"] == "score":
        scored = case.get("scored")
        idx = [names.index(n) for n in scored] if scored is not None else None
        st, raw, nrm = b.run_score_plugin(h, case["plugin"], idx)
        if st != e["status"]:
            errs.append(f"status {st} != {e['status']}")
        if e["status"] in (0,):
            got = nrm if "normalized" in e else raw
            want = e.get("normalized", e.get("raw"))
            by = dict(zip(names, got))
            gl = [by[n] for n in (scored if scored is not None else want_names)]
            if gl != want:
                errs.append(f"scores {gl} != {want}")
    elif case["kind"] == "filter":
        pc, codes, reasons = b.run_filter_plugin(h, case["plugin"])
        if pc != e["prefilter"]:
            errs.append(f"prefilter {pc} != {e['prefilter']}")
        if e["prefilter"] == 0:
            byc = dict(zip(names, codes))
            gl = [byc[n] for n in want_names]
            if gl != e["codes"]:
                errs.append(f"codes {gl} != {e['codes']}")
            if "reasons" in e:
                byr = dict(zip(names, reasons))
                gr = [byr[n] for n in want_names]
                if gr != e["reasons"]:
                    errs.append(f"reasons {gr} != {e['reasons']}")
    elif case["kind"] == "cycle":
        errs += run_cycle_case(b, case, names)
    b.close()
    return errs


def run_cycle_case(b, case, names):
    errs = []
    e = case["expect"]
    r, ev = b.schedule_one(b.compile(case["pod"]), assume=False, evaluate=True)
    if "node" in e:
        got = names[r.node_index] if r.node_index >= 0 else None
        if got != e["node"]:
            errs.append(f"node {got} != {e['node']}")
    if "status" in e and r.status != e["status"]:
        errs.append(f"status {r.status} != {e['status']}")
    if "totals" in e:
        by = dict(zip(names, ev["total_scores"]))
        for n, v in e["totals"].items():
            if by[n] != v:
                errs.append(f"total[{n}] {by[n]} != {v}")
    if "feasible" in e and r.feasible_nodes != e["feasible"]:
        errs.append(f"feasible {r.feasible_nodes} != {e['feasible']}")
    if "evaluated" in e and r.evaluated_nodes != e["evaluated"]:
        errs.append(f"evaluated {r.evaluated_nodes} != {e['evaluated']}")
    if "node_in" in e:  # the reference test accepts any of these hosts (random tie-break upstream)
        got = names[r.node_index] if r.node_index >= 0 else None
        if got not in e["node_in"]:
            errs.append(f"node {got} not in {e['node_in']}")
    if "plugin_scores" in e:  # NodePluginScores.Scores: weighted normalised score per plugin and node
        from ksg.abi import PLUGIN_ID
        for plugin, want in e["plugin_scores"].items():
            row = ev["plugin_scores"][PLUGIN_ID[plugin]]
            by = dict(zip(names, row))
            for n, v in want.items():
                if by[n] != v:
                    errs.append(f"{plugin}[{n}] {by[n]} != {v}")
            if not (ev["score_plugin_mask"] >> PLUGIN_ID[plugin]) & 1:
                errs.append(f"{plugin} did not score (skipped)")
    if "node_status" in e:  # Diagnosis.NodeToStatus: (code, plugin, reason bits) per node
        from ksg.abi import PLUGIN_ID
        for n, (code, plugin, reasons) in e["node_status"].items():
            i = names.index(n)
            got = (ev["node_code"][i], ev["node_plugin"][i], ev["node_reasons"][i])
            want = (code, PLUGIN_ID[plugin] if plugin else 255, reasons)
            if got != want:
                errs.append(f"status[{n}] {got} != {want}")
    return errs


def run_preempt_case(b, case, names):
    """DefaultPreemption PostFilter: the DryRunPreemption candidates (victims and NumPDBViolations, compared
    as sets, as the reference test sorts them), the selected node, PodEligibleToPreemptOthers."""
    from ksg.abi import KSG_ENOTSUP
    errs = []
    e = case["expect"]
    try:
        r, d = b.preempt(b.compile(case["pod"]), dict(case.get("args") or {}, listCandidates=True))
    except KsgError as ex:
        if case.get("device") == "ENOTSUP" and getattr(b, "prefix", "") == "ksg_" and f"rc={KSG_ENOTSUP}" in str(ex):
            return []
        return [f"preempt failed: {ex}"]
    if case.get("device") == "ENOTSUP" and getattr(b, "prefix", "") == "ksg_":
        errs.append("device path was expected to decline this case (KSG_ENOTSUP)")
    if "candidates" in e:
        got = {c["node"]: {"victims": sorted(c["victims"]), "numPDBViolations": c["numPDBViolations"]}
               for c in d["candidates"]}
        if got != e["candidates"]:
            errs.append(f"candidates {got} != {e['candidates']}")
    if "selected_in" in e and d.get("selected") not in e["selected_in"]:
        errs.append(f"selected {d.get('selected')} not in {e['selected_in']}")
    if "reason" in e and r.reason != e["reason"]:
        errs.append(f"reason {r.reason} != {e['reason']}")
    return errs


def run_sequence_case(b, case, names):
    """Scheduling cycles of the same pod without assume (findNodesThatFitPod called repeatedly,
    schedule_one_test.go:4472-4485); step i's expectations hold after cycle i."""
    errs = []
    for i, e in enumerate(case["expect"]["steps"]):
        r, _ = b.schedule_one(b.compile(case["pod"]), assume=False)
        got = names[r.node_index] if r.node_index >= 0 else None
        if "node" in e and got != e["node"]:
            errs.append(f"step {i}: node {got} != {e['node']}")
        if "feasible" in e and r.feasible_nodes != e["feasible"]:
            errs.append(f"step {i}: feasible {r.feasible_nodes} != {e['feasible']}")
        if "evaluated" in e and r.evaluated_nodes != e["evaluated"]:
            errs.append(f"step {i}: evaluated {r.evaluated_nodes} != {e['evaluated']}")
    return errs


def run_events_case(b, case):
    """Cache events (informer / assume feed) with UpdateSnapshot steps: each "snapshot" op takes a
    snapshot (the node listing does, as a scheduling cycle would) and checks its node order."""
    errs = []
    for i, op in enumerate(case["ops"]):
        kind = op["op"]
        if kind == "snapshot":
            got = b.node_names()
            if "want" in op and got != op["want"]:
                errs.append(f"op {i}: snapshot {got} != {op['want']}")
            continue
        try:
            if kind == "add_node":
                b.add_node(op["node"])
            elif kind == "update_node":
                b.update_node(op["node"])
            elif kind == "remove_node":
                b.remove_node(op["name"])
            elif kind == "add_pod":
                b.add_pod(op["pod"])
            elif kind == "remove_pod":
                b.remove_pod(op["uid"])
            else:
                errs.append(f"op {i}: unknown op {kind}")
                continue
            if op.get("error"):
                errs.append(f"op {i}: {kind} succeeded, the reference returns an error")
        except KsgError as e:
            if not op.get("error"):
                errs.append(f"op {i}: {kind} failed: {e}")
    return errs


RES_KEYS = ("cpu", "memory", "ephemeral-storage")


def debug_pod_resources(lib, prefix, pod):
    """<prefix>debug_pod_resources: CalculateResource [cpu, memory, eph, non0 cpu, non0 mem] + Fit's request."""
    f = getattr(lib, prefix + "debug_pod_resources")
    f.restype = C.c_int
    f.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int64), C.c_int32]
    b = json.dumps(pod).encode()
    out = (C.c_int64 * 8)()
    rc = f(b, len(b), out, 8)
    if rc != 8:
        raise KsgError(f"{prefix}debug_pod_resources: rc={rc}")
    return list(out)


def pod_resources_mismatches(v, case):
    """The decoded requests of a pod_resources case against its want (see make_fixtures_i.py's views)."""
    w = case["want"]
    if case["view"] in ("calc", "status"):
        got = dict(zip(RES_KEYS + ("non0_cpu", "non0_mem"), v[:5]))
    else:
        got = dict(zip(RES_KEYS, v[5:8]))
    return [f"{k} {got[k]} != {w[k]}" for k in w if got[k] != w[k]]


def _qty(key, v):
    return f"{v}m" if key == "cpu" else str(v)


def run_pod_resources_case(make_backend, case):
    """The requests a pod amounts to, decoded and then as the evaluation sees them:
    calc / status -- the pod bound to a node: a probe pod asking for allocatable - want of one resource
    fits (NodeResourcesFit), one asking for one unit more does not, so the node's Requested column (the
    device mirror, for the device backend) is exactly want; spec -- the pod itself to schedule: it fits
    a node whose allocatable is want and not one with one unit less (Fit's PreFilter request)."""
    b = make_backend({})
    errs = pod_resources_mismatches(debug_pod_resources(b.lib, b.prefix, case["pod"]), case)
    w = case["want"]
    big = {"cpu": 10 ** 9, "memory": 2 ** 50, "ephemeral-storage": 2 ** 50}

    def node(name, alloc):
        return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name}},
                "status": {"allocatable": dict({k: _qty(k, alloc[k]) for k in RES_KEYS}, pods="110")}}

    def probe(key, amount):
        return {"metadata": {"name": f"probe-{key}-{amount}", "namespace": "default", "uid": f"probe-{key}-{amount}"},
                "spec": {"containers": [{"name": "p", "resources": {"requests": {key: _qty(key, amount)}}}]}}

    if case["view"] in ("calc", "status"):
        alloc = {k: w[k] + {"cpu": 1000, "memory": 2 ** 30, "ephemeral-storage": 2 ** 30}[k] for k in RES_KEYS}
        b.add_node(node("n0", alloc))
        bound = json.loads(json.dumps(case["pod"]))
        bound["spec"]["nodeName"] = "n0"
        b.add_pod(bound)
        for k in RES_KEYS:
            for extra, want_code in ((0, 0), (1, 2)):
                h = b.compile(probe(k, alloc[k] - w[k] + extra))
                _, codes, _ = b.run_filter_plugin(h, "NodeResourcesFit")
                b.release(h)
                if (codes[0] == 0) != (want_code == 0):  # a failure is 2, or 3 past the allocatable itself
                    errs.append(f"bound: probe {k} +{extra} code {codes[0]} (Requested {k} != {w[k]})")
    else:
        nodes = [("fit", {k: w[k] for k in RES_KEYS})]
        nodes += [(f"short-{k}", dict(big, **{k: w[k] - 1})) for k in RES_KEYS if w[k] > 0]
        for name, alloc in nodes:
            b.add_node(node(name, {k: (alloc[k] if k in alloc else big[k]) for k in RES_KEYS}))
        names = b.node_names()
        h = b.compile(case["pod"])
        _, codes, _ = b.run_filter_plugin(h, "NodeResourcesFit")
        b.release(h)
        by = dict(zip(names, codes))
        for name, _ in nodes:
            want_code = 0 if name == "fit" else 2
            if (by[name] == 0) != (want_code == 0):
                errs.append(f"Fit request: node {name} code {by[name]} != {want_code}")
    b.close()
    return errs
