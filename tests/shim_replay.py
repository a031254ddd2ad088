"""The plugin-level hook of INTEGRATION.md, replayed: kube-scheduler's framework driving one `Shim`
instance per plugin over one library evaluation (`ksg_eval_out`), step by step as the Go code does.

Go cannot run here, so this restates the framework side the shim plugs into -- the parts whose
contract the shim must satisfy -- and the `Shim` methods of INTEGRATION.md's Go sample one for one:

* `RunPreFilterPlugins`      framework/runtime/framework.go:934-995 (Skip, Unschedulable continues,
                             UnschedulableAndUnresolvable stops, PreFilterResult merge)
* `findNodesThatFitPod`      schedule_one.go:622-712 (PreFilterResult subset, nextStartNodeIndex :686-687)
* `findNodesThatPassFilters` schedule_one.go:771-854 (rotated order, RunFilterPlugins first failure wins,
                             framework.go:1105-1138)
* `schedulePod`              schedule_one.go:564-618 (FitError, the one-feasible-node shortcut)
* `RunPreScorePlugins`       framework.go:1300-1333 (Skip removes the plugin from scoring, :1324-1327)
* `RunScorePlugins`          framework.go:1351-1458 (Score, NormalizeScore, the [0, 100] check :1439-1443,
                             weights and TotalScore :1428-1452)
* `selectHost`               schedule_one.go:1054-1085 with Go's container/heap Init + Pop

The percentageOfNodesToScore cut is not replayed (profiles that sample use the
algorithm-level hook), so the profile must score every node.
Only tests/ use this module.
"""
from ksg.abi import (ERROR, NUM_PLUGINS, PLUGIN_ID, SKIP, SUCCESS, UNSCHEDULABLE,
                     UNSCHEDULABLE_AND_UNRESOLVABLE)

R_PREFILTER = 1 << 16  # KSG_R_PREFILTER

# Extension-point order of the default profile (apis/config/v1/default_plugins.go:35-50): every point
# lists the plugins in the same order, which is the KSG_PLUGIN_* numbering.
PREFILTER_ORDER = [PLUGIN_ID[n] for n in ("NodeAffinity", "NodePorts", "NodeResourcesFit", "PodTopologySpread",
                                          "InterPodAffinity")]
FILTER_ORDER = list(range(8))  # NodeUnschedulable .. InterPodAffinity
SCORE_ORDER = [PLUGIN_ID[n] for n in ("TaintToleration", "NodeAffinity", "NodeResourcesFit", "PodTopologySpread",
                                      "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality")]
DEFAULT_WEIGHTS = {"TaintToleration": 3, "NodeAffinity": 2, "NodeResourcesFit": 1, "PodTopologySpread": 2,
                   "InterPodAffinity": 2, "NodeResourcesBalancedAllocation": 1, "ImageLocality": 1}


def profile_weights(cfg):
    """The framework's scorePluginWeight map for a ksg_create config (scoreWeights over the defaults)."""
    w = dict(DEFAULT_WEIGHTS)
    for k, v in (cfg.get("scoreWeights") or {}).items():
        w[k] = int(v)
    return {PLUGIN_ID[k]: v for k, v in w.items()}


def enabled_plugins(cfg):
    off = {PLUGIN_ID[n] for n in cfg.get("disabledPlugins", [])}
    return [p for p in range(NUM_PLUGINS) if p not in off]


class CycleEval:
    """INTEGRATION.md's cycleEval: the library's one evaluation of the pod, shared by every shim instance."""

    def __init__(self, ev):
        self.code, self.plugin, self.reasons = ev["node_code"], ev["node_plugin"], ev["node_reasons"]
        self.scores = ev["normalized_scores"]  # [plugin][index], before the weight
        self.score_mask = ev["score_plugin_mask"]
        self.pre_code, self.pre_plugin = ev["prefilter_code"], ev["prefilter_plugin"]
        n = len(self.code)
        # NodeAffinity's PreFilterResult (node_affinity.go:148-199): the nodes it did not exclude
        excluded = [i for i in range(n) if self.reasons[i] & R_PREFILTER and self.code[i] == UNSCHEDULABLE_AND_UNRESOLVABLE]
        self.pre_result = None if not excluded or self.pre_code else [i for i in range(n) if i not in set(excluded)]


class Shim:
    """INTEGRATION.md's `Shim`: one instance per plugin name, answering from the shared CycleEval."""

    def __init__(self, pid):
        self.id = pid

    def pre_filter(self, ce):  # -> (PreFilterResult node indices or None, status code)
        if ce.pre_code and ce.pre_plugin == self.id:
            return None, ce.pre_code
        if self.id == PLUGIN_ID["NodeAffinity"] and ce.pre_result is not None:
            return ce.pre_result, SUCCESS
        return None, SUCCESS

    def filter(self, ce, i):
        if ce.code[i] == 0 or ce.plugin[i] != self.id:
            return SUCCESS  # this plugin passes the node; the first failing one reports it
        return ce.code[i]

    def pre_score(self, ce):
        return SUCCESS if ce.score_mask >> self.id & 1 else SKIP

    def score(self, ce, i):
        return ce.scores[self.id][i]

    def normalize_score(self, ce, scores):
        return SUCCESS  # NormalizeScore ran on the device; Score already returned its output


# ---- Go's container/heap with nodeScoreHeap.Less (schedule_one.go:1082-1085, Randomizer 0) ----
def _less(h, i, j):
    return h[i][0] > h[j][0]


def _down(h, i0, n):
    i = i0
    while True:
        j1 = 2 * i + 1
        if j1 >= n:
            break
        j = j1
        if j1 + 1 < n and _less(h, j1 + 1, j1):
            j = j1 + 1
        if not _less(h, j, i):
            break
        h[i], h[j] = h[j], h[i]
        i = j


def heap_init_pop(entries):
    """heap.Init then heap.Pop over [(TotalScore, node)] in feasible order -> the popped node."""
    h = list(entries)
    n = len(h)
    for i in range(n // 2 - 1, -1, -1):
        _down(h, i, n)
    h[0], h[n - 1] = h[n - 1], h[0]
    _down(h, 0, n - 1)
    return h[n - 1][1]


class Framework:
    """One profile's frameworkImpl + the Scheduler fields schedulePod reads (nextStartNodeIndex)."""

    def __init__(self, cfg):
        self.enabled = set(enabled_plugins(cfg))
        self.weights = profile_weights(cfg)
        self.shims = {p: Shim(p) for p in range(NUM_PLUGINS)}
        self.next_start = 0

    def schedule_pod(self, ev, n):
        """-> (status, node index, EvaluatedNodes, FeasibleNodes, TotalScore of the chosen node)."""
        ce = CycleEval(ev)
        # RunPreFilterPlugins
        result, ret = None, SUCCESS
        for p in PREFILTER_ORDER:
            if p not in self.enabled:
                continue
            r, s = self.shims[p].pre_filter(ce)
            if s == UNSCHEDULABLE_AND_UNRESOLVABLE:
                return (UNSCHEDULABLE, -1, 0, 0, 0)
            if s == UNSCHEDULABLE:
                ret = s
                continue
            if s != SUCCESS:
                return (ERROR, -1, 0, 0, 0)
            if r is not None:
                result = set(r) if result is None else result & set(r)
                if not result:
                    return (UNSCHEDULABLE, -1, 0, 0, 0)
        if ret != SUCCESS:
            return (UNSCHEDULABLE, -1, 0, 0, 0)  # FitError with the PreFilter status on every node
        # findNodesThatFitPod: the PreFilterResult's nodes (snapshot order), or all of them
        nodes = list(range(n)) if result is None else sorted(result)
        # findNodesThatPassFilters (every node: percentageOfNodesToScore 100)
        feasible, failed = [], 0
        for i in range(len(nodes)):
            node = nodes[(self.next_start + i) % len(nodes)]
            st = SUCCESS
            for p in FILTER_ORDER:  # RunFilterPlugins: the first non-success status wins
                if p in self.enabled:
                    st = self.shims[p].filter(ce, node)
                    if st != SUCCESS:
                        break
            if st == SUCCESS:
                feasible.append(node)
            elif st in (UNSCHEDULABLE, UNSCHEDULABLE_AND_UNRESOLVABLE):
                failed += 1
            else:
                return (ERROR, -1, 0, 0, 0)
        self.next_start = (self.next_start + len(feasible) + failed) % n
        if not feasible:
            return (UNSCHEDULABLE, -1, failed, 0, 0)
        if len(feasible) == 1:
            return (SUCCESS, feasible[0], 1 + failed, 1, 0)
        # prioritizeNodes: RunPreScorePlugins, then RunScorePlugins over the non-skipped plugins
        scored = [p for p in SCORE_ORDER if p in self.enabled and self.shims[p].pre_score(ce) != SKIP]
        totals = [0] * len(feasible)
        for p in scored:
            lst = [self.shims[p].score(ce, node) for node in feasible]
            if self.shims[p].normalize_score(ce, lst) != SUCCESS:
                return (ERROR, -1, 0, 0, 0)
            for k, s in enumerate(lst):
                if s > 100 or s < 0:  # framework.go:1439-1443
                    return (ERROR, -1, 0, 0, 0)
                totals[k] += s * self.weights[p]
        if not scored and not any(p in self.enabled for p in SCORE_ORDER):
            totals = [1] * len(feasible)  # no score plugins (schedule_one.go:948-957)
        node = heap_init_pop(list(zip(totals, feasible)))
        return (SUCCESS, node, len(feasible) + failed, len(feasible), totals[feasible.index(node)])
