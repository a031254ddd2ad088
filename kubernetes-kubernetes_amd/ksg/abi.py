"""ctypes view of include/ksg.h, shared by the product binding and the test harness.

`Backend(lib, prefix)` wraps a shared library exporting the ksg.h entry points under
`prefix` ("ksg_" for the MI355X product library).  The parity oracle exports the same
shapes under "ksgo_"; only tests/ (and bench.py's cpu_baseline leg) construct a
Backend over it.
"""
import ctypes as C
import json

KSG_OK = 0
KSG_EINVAL, KSG_ENOTFOUND, KSG_EEXIST, KSG_EDEVICE, KSG_ENOTSUP, KSG_ENOMEM = -1, -2, -3, -4, -5, -6

# fwk.Code (staging/src/k8s.io/kube-scheduler/framework/interface.go:46-99)
SUCCESS, ERROR, UNSCHEDULABLE, UNSCHEDULABLE_AND_UNRESOLVABLE, WAIT, SKIP, PENDING = range(7)

PLUGINS = [
    "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
    "NodeResourcesFit", "PodTopologySpread", "InterPodAffinity",
    "NodeResourcesBalancedAllocation", "ImageLocality",
]
NUM_PLUGINS = len(PLUGINS)
PLUGIN_NONE = 255
PLUGIN_ID = {n: i for i, n in enumerate(PLUGINS)}

REASONS = [
    "node(s) were unschedulable",
    "node(s) didn't match the requested node name",
    "node(s) had untolerated taint(s)",
    "node(s) didn't match Pod's node affinity/selector",
    "node(s) didn't match scheduler-enforced node affinity",
    "node(s) didn't have free ports for the requested pod ports",
    "Too many pods",
    "Insufficient cpu",
    "Insufficient memory",
    "Insufficient ephemeral-storage",
    "Insufficient <extended resource>",
    "node(s) didn't match pod topology spread constraints (missing required label)",
    "node(s) didn't match pod topology spread constraints",
    "node(s) didn't match pod affinity rules",
    "node(s) didn't match pod anti-affinity rules",
    "node(s) didn't satisfy existing pods anti-affinity rules",
    "PreFilter",
]

FLAG_ASSUME = 1


class Result(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("node_index", C.c_int32),
        ("evaluated_nodes", C.c_int32),
        ("feasible_nodes", C.c_int32),
        ("total_score", C.c_int64),
    ]

    def as_tuple(self):
        return (self.status, self.node_index, self.evaluated_nodes, self.feasible_nodes, self.total_score)


PREEMPT_OK, PREEMPT_NOT_ELIGIBLE, PREEMPT_NO_CANDIDATES = 0, 1, 2


class PreemptResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("reason", C.c_int32),
        ("node_index", C.c_int32),
        ("num_potential", C.c_int32),
        ("num_candidates", C.c_int32),
        ("num_victims", C.c_int32),
        ("num_pdb_violations", C.c_int64),
    ]

    def as_tuple(self):
        return (self.status, self.reason, self.node_index, self.num_potential, self.num_candidates,
                self.num_victims, self.num_pdb_violations)


class EvalOut(C.Structure):
    _fields_ = [
        ("prefilter_code", C.c_int32),
        ("prefilter_plugin", C.c_int32),
        ("node_code", C.POINTER(C.c_uint8)),
        ("node_plugin", C.POINTER(C.c_uint8)),
        ("node_reasons", C.POINTER(C.c_uint32)),
        ("score_plugin_mask", C.c_uint32),
        ("plugin_scores", C.POINTER(C.c_int64)),
        ("total_scores", C.POINTER(C.c_int64)),
        ("normalized_scores", C.POINTER(C.c_int64)),
    ]


def _sig(lib, prefix):
    f = {}

    def d(name, res, *args):
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = list(args)
        f[name] = fn

    vp, cp, sz, i32, u32 = C.c_void_p, C.c_char_p, C.c_size_t, C.c_int32, C.c_uint32
    d("create", vp, cp, sz)
    d("create_error", cp)
    d("destroy", None, vp)
    d("last_error", cp, vp)
    d("upsert_namespace", C.c_int, vp, cp, sz)
    d("upsert_object", C.c_int, vp, cp, sz)
    d("remove_object", C.c_int, vp, cp, cp, cp)
    d("add_node", C.c_int, vp, cp, sz)
    d("update_node", C.c_int, vp, cp, sz)
    d("remove_node", C.c_int, vp, cp)
    d("add_pod", C.c_int, vp, cp, sz)
    d("remove_pod", C.c_int, vp, cp)
    d("num_nodes", C.c_int, vp)
    d("node_name", C.c_int, vp, i32, C.c_char_p, sz)
    d("pod_compile", C.c_int, vp, cp, sz, C.POINTER(i32))
    d("pod_release", C.c_int, vp, i32)
    d("schedule_one", C.c_int, vp, i32, u32, C.POINTER(Result), C.POINTER(EvalOut))
    d("schedule_batch", C.c_int, vp, C.POINTER(i32), i32, u32, C.POINTER(Result))
    d("forget", C.c_int, vp, i32)
    d("add_nominated_pod", C.c_int, vp, cp, sz)
    d("delete_nominated_pod", C.c_int, vp, cp)
    d("run_filter_plugin", C.c_int, vp, i32, i32, C.POINTER(i32), C.POINTER(C.c_uint8), C.POINTER(C.c_uint32))
    d("run_score_plugin", C.c_int, vp, i32, i32, C.POINTER(C.c_uint8), C.POINTER(i32), C.POINTER(C.c_int64),
      C.POINTER(C.c_int64))
    d("preempt", C.c_int, vp, i32, cp, sz, C.POINTER(PreemptResult), C.c_char_p, sz, C.POINTER(sz))
    d("set_clock", C.c_int, vp, C.c_int64)
    d("debug_clock_step", C.c_int, vp, C.c_int64)
    return f


class KsgError(RuntimeError):
    pass


def _js(obj):
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj)
    if isinstance(obj, str):
        return obj.encode()
    return json.dumps(obj, separators=(",", ":")).encode()


class Backend:
    """One scheduler context (one kube-scheduler profile + its cache mirror)."""

    def __init__(self, lib, prefix, config=None):
        self.lib = lib
        self.prefix = prefix
        self.f = _sig(lib, prefix)
        cfg = _js(config or {})
        self.ctx = self.f["create"](cfg, len(cfg))
        if not self.ctx:
            raise KsgError(f"{prefix}create failed: {self.f['create_error']().decode()}")
        self._names = None

    def close(self):
        if self.ctx:
            self.f["destroy"](self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self):
        """The context's last error text (ksg_last_error); after a recovered loop give-up, its detail."""
        return self.f["last_error"](self.ctx).decode(errors="replace")

    def _chk(self, rc, what):
        if rc < 0:
            raise KsgError(f"{what}: rc={rc}: {self.f['last_error'](self.ctx).decode(errors='replace')}")
        return rc

    # ---- cluster state -----------------------------------------------------------------
    def upsert_namespace(self, ns):
        b = _js(ns)
        self._chk(self.f["upsert_namespace"](self.ctx, b, len(b)), "upsert_namespace")

    def upsert_object(self, obj):
        """A Service / ReplicationController / ReplicaSet / StatefulSet (PodTopologySpread defaults)."""
        b = _js(obj)
        self._chk(self.f["upsert_object"](self.ctx, b, len(b)), "upsert_object")

    def remove_object(self, kind, namespace, name):
        self._chk(self.f["remove_object"](self.ctx, kind.encode(), (namespace or "").encode(), name.encode()),
                  "remove_object")

    def add_node(self, node):
        b = _js(node)
        self._names = None
        self._chk(self.f["add_node"](self.ctx, b, len(b)), "add_node")

    def update_node(self, node):
        b = _js(node)
        self._names = None
        self._chk(self.f["update_node"](self.ctx, b, len(b)), "update_node")

    def remove_node(self, name):
        self._names = None
        self._chk(self.f["remove_node"](self.ctx, name.encode()), "remove_node")

    def add_pod(self, pod):
        b = _js(pod)
        self._chk(self.f["add_pod"](self.ctx, b, len(b)), "add_pod")

    def remove_pod(self, uid):
        self._chk(self.f["remove_pod"](self.ctx, uid.encode()), "remove_pod")

    def num_nodes(self):
        return self._chk(self.f["num_nodes"](self.ctx), "num_nodes")

    def node_names(self):
        if self._names is None:
            out = []
            buf = C.create_string_buffer(512)
            for i in range(self.num_nodes()):
                self._chk(self.f["node_name"](self.ctx, i, buf, 512), "node_name")
                out.append(buf.value.decode())
            self._names = out
        return self._names

    # ---- pods --------------------------------------------------------------------------
    def compile(self, pod):
        b = _js(pod)
        h = C.c_int32()
        self._chk(self.f["pod_compile"](self.ctx, b, len(b), C.byref(h)), "pod_compile")
        return h.value

    def release(self, handle):
        self._chk(self.f["pod_release"](self.ctx, handle), "pod_release")

    def schedule_one(self, handle, assume=True, evaluate=False):
        """Returns (Result, eval dict or None)."""
        r = Result()
        ev = None
        evp = None
        if evaluate:
            n = self.num_nodes()
            code = (C.c_uint8 * n)()
            plug = (C.c_uint8 * n)()
            reas = (C.c_uint32 * n)()
            ps = (C.c_int64 * (n * NUM_PLUGINS))()
            tot = (C.c_int64 * n)()
            nrm = (C.c_int64 * (n * NUM_PLUGINS))()
            ev = EvalOut(0, 0, code, plug, reas, 0, ps, tot, nrm)
            evp = C.byref(ev)
        self._chk(self.f["schedule_one"](self.ctx, handle, FLAG_ASSUME if assume else 0, C.byref(r), evp), "schedule_one")
        if not evaluate:
            return r, None
        n = self.num_nodes()
        out = {
            "prefilter_code": ev.prefilter_code,
            "prefilter_plugin": ev.prefilter_plugin,
            "node_code": [ev.node_code[i] for i in range(n)],
            "node_plugin": [ev.node_plugin[i] for i in range(n)],
            "node_reasons": [ev.node_reasons[i] for i in range(n)],
            "score_plugin_mask": ev.score_plugin_mask,
            "plugin_scores": [[ev.plugin_scores[p * n + i] for i in range(n)] for p in range(NUM_PLUGINS)],
            "total_scores": [ev.total_scores[i] for i in range(n)],
            "normalized_scores": [[ev.normalized_scores[p * n + i] for i in range(n)] for p in range(NUM_PLUGINS)],
        }
        return r, out

    def schedule_batch(self, handles, assume=True):
        n = len(handles)
        hs = (C.c_int32 * n)(*handles)
        rs = (Result * n)()
        self._chk(self.f["schedule_batch"](self.ctx, hs, n, FLAG_ASSUME if assume else 0, rs), "schedule_batch")
        return [rs[i] for i in range(n)]

    @staticmethod
    def batch_arrays(handles):
        """(c_int32 handle array, Result array) for schedule_batch_into: built once, outside a timed loop."""
        n = len(handles)
        return (C.c_int32 * n)(*handles), (Result * n)()

    def schedule_batch_into(self, hs, rs, assume=True):
        """ksg_schedule_batch over a prebuilt handle array into a prebuilt Result array (the shape a
        cgo caller uses: no per-pod Python objects)."""
        self._chk(self.f["schedule_batch"](self.ctx, hs, len(hs), FLAG_ASSUME if assume else 0, rs), "schedule_batch")
        return rs

    def forget(self, handle):
        self._chk(self.f["forget"](self.ctx, handle), "forget")

    def add_nominated_pod(self, pod):
        """The nominator's AddNominatedPod / UpdateNominatedPod: pod's uid is nominated to its
        status.nominatedNodeName (none: forgotten)."""
        b = _js(pod)
        self._chk(self.f["add_nominated_pod"](self.ctx, b, len(b)), "add_nominated_pod")

    def delete_nominated_pod(self, uid):
        self._chk(self.f["delete_nominated_pod"](self.ctx, uid.encode()), "delete_nominated_pod")

    def run_filter_plugin(self, handle, plugin):
        """PreFilter + Filter of one plugin on every node -> (prefilter_code, codes, reasons)."""
        pid = PLUGIN_ID[plugin] if isinstance(plugin, str) else plugin
        n = self.num_nodes()
        pc = C.c_int32()
        codes = (C.c_uint8 * max(n, 1))()
        reas = (C.c_uint32 * max(n, 1))()
        self._chk(self.f["run_filter_plugin"](self.ctx, handle, pid, C.byref(pc), codes, reas), "run_filter_plugin")
        return pc.value, list(codes[:n]), list(reas[:n])

    def run_score_plugin(self, handle, plugin, nodes=None):
        """PreScore + Score + NormalizeScore of one plugin over a node list (default: every
        node; else an iterable of snapshot indices) -> (status, raw, normalized)."""
        pid = PLUGIN_ID[plugin] if isinstance(plugin, str) else plugin
        n = self.num_nodes()
        st = C.c_int32()
        raw = (C.c_int64 * max(n, 1))()
        nrm = (C.c_int64 * max(n, 1))()
        mask = None
        if nodes is not None:
            mask = (C.c_uint8 * max(n, 1))()
            for i in nodes:
                mask[i] = 1
        self._chk(self.f["run_score_plugin"](self.ctx, handle, pid, mask, C.byref(st), raw, nrm), "run_score_plugin")
        return st.value, list(raw[:n]), list(nrm[:n])

    def set_clock(self, now_ns):
        """time.Now() of the next scheduling calls, ns (OpportunisticBatching's maxBatchAge); 0: the wall clock."""
        self._chk(self.f["set_clock"](self.ctx, int(now_ns)), "set_clock")

    def clock_step(self, step_ns):
        """The fixed clock advances by step_ns per scheduling cycle (ksg_debug_clock_step)."""
        self._chk(self.f["debug_clock_step"](self.ctx, int(step_ns)), "debug_clock_step")

    def preempt(self, handle, args=None, detail_cap=1 << 20):
        """DefaultPreemption PostFilter for a compiled pod: (PreemptResult, detail dict)."""
        a = _js(args or {})
        r = PreemptResult()
        buf = C.create_string_buffer(detail_cap)
        dl = C.c_size_t(0)
        self._chk(self.f["preempt"](self.ctx, handle, a, len(a), C.byref(r), buf, detail_cap, C.byref(dl)), "preempt")
        return r, json.loads(buf.value.decode())
