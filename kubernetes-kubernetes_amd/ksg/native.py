"""Loader for the product library lib/libksg.so (HIP kernels for gfx950 + the C ABI).

There is deliberately no fallback: if the library is missing, fails to load, or no HIP
device is visible, `Scheduler(...)` raises.  The parity oracle lives in oracle/ and is
never reachable from here.
"""
import ctypes as C
import os

from .abi import Backend, KsgError

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("KSG_LIB") or os.path.join(PKG, "lib", "libksg.so")  # KSG_LIB: the diagnostic build
HEADER = os.path.join(os.path.dirname(PKG), "include", "ksg.h")

_lib = None


def load():
    """dlopen libksg.so (raises KsgError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise KsgError(f"{LIB} not built: run `make -C {PKG}` or __graft_entry__.build()")
        lib = C.CDLL(LIB)
        lib.ksg_last_batch_kernel_stats.restype = C.c_int
        lib.ksg_last_batch_kernel_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                    C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.ksg_comm_unique_id.restype = C.c_int
        lib.ksg_comm_unique_id.argtypes = [C.c_char_p, C.c_size_t]
        lib.ksg_create_error.restype = C.c_char_p
        lib.ksg_shard_range.restype = C.c_int
        lib.ksg_shard_range.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.ksg_debug_relayouts.restype = C.c_int
        lib.ksg_debug_relayouts.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        lib.ksg_generation.restype = C.c_int
        lib.ksg_generation.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        lib.ksg_debug_compare_mirror.restype = C.c_int
        lib.ksg_debug_compare_mirror.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.ksg_debug_batching.restype = C.c_int
        lib.ksg_debug_batching.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        lib.ksg_debug_loop_stats.restype = C.c_int
        lib.ksg_debug_loop_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        from .abi import Result
        lib.ksg_debug_schedule_calls.restype = C.c_int
        lib.ksg_debug_schedule_calls.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.c_uint32,
                                                 C.POINTER(Result), C.POINTER(C.c_double)]
        _lib = lib
    return _lib


class Scheduler(Backend):
    """One kube-scheduler profile + cache mirror resident in HBM (ksg_create)."""

    def __init__(self, config=None):
        super().__init__(load(), "ksg_", config)

    def kernel_stats(self):
        """(avg ms, algorithmic bytes, launches, kernel name) of the last batch: per k_filter_score
        launch, or per pod inside a persistent loop (k_sched_loop, k_agg_loop) when most pods ran there
        (launches: the pods that loop ran)."""
        ms, by, n, k = C.c_double(), C.c_double(), C.c_int32(), C.c_int32()
        self._chk(self.lib.ksg_last_batch_kernel_stats(self.ctx, C.byref(ms), C.byref(by), C.byref(n), C.byref(k)),
                  "kernel_stats")
        return ms.value, by.value, n.value, {1: "k_sched_loop", 2: "k_agg_loop"}.get(k.value, "k_filter_score")

    def compare_mirror(self, sync=False):
        """(differing nodes + pod-table slots, first difference) between the device mirror and the
        host cache shadow (ksg_debug_compare_mirror); sync: rebuild a stale mirror first."""
        nd, first = C.c_int32(), C.c_int32()
        self._chk(self.lib.ksg_debug_compare_mirror(self.ctx, 1 if sync else 0, C.byref(nd), C.byref(first)),
                  "compare_mirror")
        return nd.value, first.value

    def generation(self):
        """(node-list rebuilds, cache mutations applied) -- ksg_generation, the plugin shim's consistency check."""
        lg, ev = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.ksg_generation(self.ctx, C.byref(lg), C.byref(ev)), "generation")
        return lg.value, ev.value

    def batching(self):
        """(pods placed by an OpportunisticBatching hint, scheduling cycles counted) -- ksg_debug_batching."""
        h, c = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.ksg_debug_batching(self.ctx, C.byref(h), C.byref(c)), "batching")
        return h.value, c.value

    def loop_stats(self):
        """(batches whose persistent loop gave up, batches an in-process group re-ran over the all-reduce
        path) so far (ksg_debug_loop_stats)."""
        g, r = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.ksg_debug_loop_stats(self.ctx, C.byref(g), C.byref(r)), "loop_stats")
        return g.value, r.value

    def relayouts(self):
        """(full mirror rebuilds, gather re-layouts) so far (ksg_debug_relayouts)."""
        f, g = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.ksg_debug_relayouts(self.ctx, C.byref(f), C.byref(g)), "relayouts")
        return f.value, g.value

    def schedule_calls(self, handles, assume=True):
        """ksg_schedule_one for each handle, back to back from native code (ksg_debug_schedule_calls):
        (results, mean wall µs per call)."""
        from .abi import FLAG_ASSUME, Result
        n = len(handles)
        hs = (C.c_int32 * n)(*handles)
        rs = (Result * n)()
        us = C.c_double()
        self._chk(self.lib.ksg_debug_schedule_calls(self.ctx, hs, n, FLAG_ASSUME if assume else 0, rs, C.byref(us)),
                  "schedule_calls")
        return [rs[i] for i in range(n)], us.value

    def shard_range(self):
        """(first snapshot index, node count) this rank evaluates (node-sharded contexts)."""
        a, n = C.c_int32(), C.c_int32()
        self._chk(self.lib.ksg_shard_range(self.ctx, C.byref(a), C.byref(n)), "shard_range")
        return a.value, n.value


def comm_unique_id():
    """ncclGetUniqueId as hex (rank 0 creates it; every rank passes it as distributed.ncclId)."""
    lib = load()
    buf = C.create_string_buffer(512)
    rc = lib.ksg_comm_unique_id(buf, 512)
    if rc < 0:
        raise KsgError(f"ksg_comm_unique_id: rc={rc}: {lib.ksg_create_error().decode(errors='replace')}")
    return buf.value.decode()
