"""Throughput of the MI355X node-evaluation path on scheduler_perf SchedulingBasic (BASELINE C2).

Workload (BASELINE.json configs[1]): 5000 node-default nodes, 1000 bound init pods, then the
measured pod-default pods scheduled one cycle at a time (each assume lands before the next
pod), percentageOfNodesToScore=100, default plugins.  A "step" is one ksg_schedule_batch over
`--batch` pods; the default 10 steps x 1000 pods are the config's 10000 measured pods.
Warmup pods are scheduled and then forgotten (Cache.ForgetPod) so the timed region starts
from the config's initial state.  Pod objects are decoded into the queue (ksg_pod_compile)
before timing, as the informer would have delivered them; the timed region covers PreFilter/
PreScore compilation, the H2D descriptor copy, both kernels per pod, the D2H results and the
host-side assume bookkeeping.

Multi-GPU (--gpus N under torch.distributed.run), DESIGN.md §6.  Default `--mode sharded`: ONE
scheduler whose snapshot is sharded by node across the N GPUs -- every rank holds the mirror,
evaluates its contiguous node range, and per pod two (three with PodTopologySpread scoring) RCCL
all-reduces over xGMI carry the feasible counts, NormalizeScore maxima and the packed
(TotalScore, heap pre-order key, node) argmax; every rank applies the same AssumePod.  With
`--node-scaling weak` (default for c2-c4) the cluster grows with N (nodes x N, per-GPU work
fixed); `strong` keeps the cluster fixed (default for c5, the 100k-node config).  `--mode
replicas` instead runs N independent schedulers (own cluster, own pod stream, no collective).

The CPU baseline is the parity oracle (oracle/, a C++ restatement of the reference) timed on a
bounded sample of the same pod stream from the same initial state: its Filter/Score loops over
nodes on 16 host threads (the reference's default parallelism), and on one thread beside it.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, "HBM")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c2", choices=list(WORKLOADS),
                    help="c2 SchedulingBasic (the metric's config); c1 SchedulingBasic 500 nodes (BASELINE's CPU-reference "
                         "config: run with --steps 1 --batch 1000); c3 SchedulingPodAffinity + NodeAffinity + "
                         "taints; c4 TopologySpreading; c4-anti PreferredPodAntiAffinity; c5 100k-node mixed "
                         "cluster; c2-hetero / c3-pa variants")
    ap.add_argument("--nodes", type=int, default=None, help="cluster nodes at N=1 (default: the config's)")
    ap.add_argument("--init-pods", type=int, default=None, help="bound pods at N=1 (default: the config's)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the oracle check of the timed stream's placements (the cpu_baseline sample)")
    ap.add_argument("--mode", default="sharded", choices=["sharded", "replicas"], help="multi-GPU mode (N>1)")
    ap.add_argument("--shard-single", action="store_true",
                    help="run the node-sharded pipeline (RCCL transport) even at N=1 -- a check of that path")
    ap.add_argument("--node-scaling", default=None, choices=["weak", "strong"],
                    help="sharded mode: grow the cluster with N (weak) or keep it fixed (strong)")
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--pct", type=int, default=100,
                    help="percentageOfNodesToScore (100: the parity contract; 0: upstream's adaptive default)")
    ap.add_argument("--timing-stride", type=int, default=8, help="time every k-th filter kernel with HIP events")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the oracle CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-device-exchange", action="store_true",
                    help="sharded: the per-pod RCCL all-reduce path for every pod (default: the loop's device exchange)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the multi-core CPU baseline (the reference's default parallelism is 16)")
    ap.add_argument("--extra-config", default=None,
                    help="JSON merged into the scheduler config (diagnostics / A-B runs, e.g. '{\"loopUnit\": 256}')")
    ap.add_argument("--no-sub", action="store_true",
                    help="no sub-records: the default N=1 SchedulingBasic line also carries the 100k-node C5 "
                         "record (BASELINE configs[4], the metric's second size) measured by a child bench.py")
    ap.add_argument("--sub-steps", type=int, default=50,
                    help="steps (of --batch pods) of the C5 sub-record: 50 x 1000 = BASELINE configs[4]'s 50000 pods")
    ap.add_argument("--traffic", default=None,
                    help="PMC-derived HBM bytes per k_filter_score launch (from a separate rocprofv3 --pmc run)")
    return ap.parse_args()


# workload -> (name, default nodes, default init pods, BASELINE configs index)
# kernel_stats() of every batch this process ran (warm-up and timed): KSG_LOOP_PODS_OUT=<file> writes the pods
# each persistent-loop kernel ran, so a PMC pass's bytes over all of a kernel's dispatches divide by the pods they
# covered (scripts/prof_summary.py)
LOOP_PODS = []


def write_loop_pods():
    path = os.environ.get("KSG_LOOP_PODS_OUT")
    if path:
        tot = {}
        for _, _, n, k in LOOP_PODS:
            tot[k] = tot.get(k, 0) + n
        json.dump(tot, open(path, "w"))


WORKLOADS = {
    "c1": ("SchedulingBasic", 500, 500, 0),
    "c2": ("SchedulingBasic", 5000, 1000, 1),
    "c2-hetero": ("SchedulingBasic (heterogeneous nodes)", 5000, 1000, None),
    "c3": ("SchedulingPodAffinity + NodeAffinity + taints (1 in 5 nodes foo:NoSchedule; pod-affinity / "
           "node-affinity / node-inclusion-policy spread pods in turn)", 5000, 5000, 2),
    "c3-pa": ("SchedulingPodAffinity", 5000, 5000, None),
    "c4": ("TopologySpreading", 15000, 15000, 3),
    "c4-anti": ("PreferredPodAntiAffinity", 15000, 15000, 3),
    "c5": ("Mixed 100k-node cluster (50% default, 10% each node-affinity / pod-affinity / anti-affinity / "
           "preferred anti-affinity / zone spread)", 100000, 10000, 4),
    "dts": ("DefaultTopologySpreading (pods selected by a Service: PodTopologySpread system default "
            "constraints)", 5000, 5000, None),
    # scheduler_perf batching/performance-config.yaml (OpportunisticBatching, no-topology profile)
    "hostport": ("HostPortConflict (OpportunisticBatching; one hostPort-80 pod per node)", 20000, 0, None),
    "saturation": ("ResourceSaturation (OpportunisticBatching; one 3-cpu pod per 4-cpu node)", 20000, 0, None),
}

# batching/scheduler-config-no-topology.yaml: PodTopologySpread List defaulting without default constraints,
# the profile in which OpportunisticBatching acts
BATCH_CLOCK_NS = 10 ** 15
PROFILES = {"hostport": {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}},
            "saturation": {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cpus():
    """CPUs this process may actually run on: its affinity mask, capped by a cgroup v2 CPU quota (the
    GPU box gives a job a 16-CPU share of a host whose os.cpu_count() is much larger)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return n


def cpu_topology():
    """What the CPU baseline's threads run on: affinity CPUs, the distinct physical cores among them (SMT
    siblings share one), and the cgroup v2 CPU quota (in CPUs) if any."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": len(cpus), "physical_cores": len(cores), "cgroup_cpu_quota": quota}


def cpu_baseline(nodes, init, pods, budget_s, threads=1, pct=100, objects=(), extra=None, profile=None, warm=()):
    """Oracle (C++ restatement of the reference), same pods from the same state.  threads > 1: its
    Filter / Score loops over nodes on a pool of that many threads (the reference's
    Parallelizer.Until with parallelism 16), results identical to the sequential oracle
    (tests/test_oracle_parallel.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_binding import oracle
    cfg = dict(profile or {})
    if threads > 1:
        cfg["cpuThreads"] = threads
    if threads > 1 and extra:  # pool knobs (oracle.cpp: cpuSpinUs, cpuParallelWeights)
        cfg.update(extra)
    if pct != 100:  # the cut filter pass runs sequentially in the oracle (its Score loop stays parallel)
        cfg["percentageOfNodesToScore"] = pct
    o = oracle(cfg)
    if profile:  # the batching workloads: one fixed clock, as the device's (no 500 ms expiry mid-run)
        o.set_clock(BATCH_CLOCK_NS)
    for ob in objects:
        o.upsert_object(ob)
    for n in nodes:
        o.add_node(n)
    for p in init:
        o.add_pod(p)
    # the device's warm-up, replayed (scheduled, then forgotten) where it leaves state behind: the
    # rotation (percentageOfNodesToScore < 100) and OpportunisticBatching's cycle and stored list
    wh = [o.compile(p) for p in warm]
    if wh:
        o.schedule_batch(wh, assume=True)
        for h in wh:
            try:
                o.forget(h)
            except Exception:
                pass
    hs = [o.compile(p) for p in pods]
    done = 0
    results = []
    t0 = time.perf_counter()
    chunk = 50
    while done < len(hs) and time.perf_counter() - t0 < budget_s:
        results += [r.as_tuple() for r in o.schedule_batch(hs[done:done + chunk], assume=True)]
        done += min(chunk, len(hs) - done)
    dt = time.perf_counter() - t0
    # where the cycle's time went (oracle.cpp ksgo_debug_profile): the serial share bounds the scaling
    import ctypes
    from oracle_binding import load
    pr = (ctypes.c_double * 10)()
    load().ksgo_debug_profile(ctypes.c_void_p(o.ctx), pr, 10)
    cyc = max(pr[8], 1.0)
    names = ["prefilter", "filter_pass", "prescore", "score_pass_normalize", "weights", "select_host", "cycle",
             "assume", "cycles", "snapshot_update"]
    breakdown = {k: round(pr[i] / cyc, 1) for i, k in enumerate(names) if k != "cycles"}
    o.close()
    cpu_baseline.breakdown = breakdown  # us per pod of the last call, by cycle section
    return done / dt, done, dt, results


def sub_record(a):
    """The metric's 100k-node size (BASELINE configs[4], C5: the mixed 100k-node cluster on one GPU) measured
    by a child bench.py after this one's scheduler is gone: its pods/s, roofline, CPU baseline and parity."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--steps", str(a.sub_steps),
           "--warmup", "1", "--batch", str(a.batch), "--cpu-seconds", str(min(a.cpu_seconds, 6.0)), "--no-sub"]
    if a.no_cpu_baseline:
        cmd.append("--no-cpu-baseline")
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, timeout=900, text=True)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        sub = json.loads(line)
    except Exception as e:  # reported, never a silent omission
        return {"error": f"C5 sub-record failed: {e!r}"}
    keep = ("metric", "value", "unit", "node_evals_per_s", "steps", "warmup", "ms_per_step", "config", "placed",
            "roofline", "kernel_us_per_step", "cpu_baseline", "parity")
    return {k: sub.get(k) for k in keep}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from ksg.native import Scheduler, comm_unique_id
    from ksg import synth

    c5 = a.workload == "c5"
    sharded = (world > 1 and a.mode == "sharded") or a.shard_single
    if sharded and a.pct != 100:
        sys.exit("--pct != 100 runs unsharded only (use --mode replicas for N > 1)")
    scaling = a.node_scaling or ("strong" if c5 else "weak")
    grow = world if (sharded and scaling == "weak") else 1
    wname, d_nodes, d_init, cfg_ix = WORKLOADS[a.workload]
    n_nodes = (a.nodes or d_nodes) * grow
    n_init = (a.init_pods if a.init_pods is not None else d_init) * grow
    n_meas = a.steps * a.batch
    n_warm = max(a.warmup, 1 if sharded else 0) * a.batch
    objects = []
    if a.workload in ("c1", "c2", "c2-hetero"):
        nodes, init, pods = synth.scheduling_basic(n_nodes, n_init, n_warm + n_meas, hetero=a.workload == "c2-hetero")
    elif a.workload == "c3":
        nodes, init, pods = synth.scheduling_c3(n_nodes, n_init, n_warm + n_meas)
    elif a.workload == "c3-pa":
        nodes, init, pods = synth.scheduling_pod_affinity(n_nodes, n_init, n_warm + n_meas)
    elif c5:
        nodes, init, pods = synth.mixed_cluster(n_nodes, n_init, n_warm + n_meas)
    elif a.workload == "dts":
        nodes, init, pods, objects = synth.default_topology_spreading(n_nodes, n_init, n_warm + n_meas)
    elif a.workload in PROFILES:
        nodes, pods = synth.batching(n_nodes, n_warm + n_meas, a.workload)
        init = []
    else:
        nodes, init, pods = synth.topology_spreading(n_nodes, n_init, n_warm + n_meas,
                                                     preferred_anti=a.workload == "c4-anti")
    if not sharded:
        for k, p in enumerate(pods):  # distinct uids per rank (independent replicas)
            p["metadata"]["uid"] = f"r{rank}-{k}"

    def build(dev_exchange):
        """Scheduler with the cluster loaded, warm-up batches run (then forgotten, so the timed run
        starts from the config state); None if the warm-up failed on this rank."""
        cfg = dict(PROFILES.get(a.workload, {}), device=local, kernelTimingStride=a.timing_stride,
                   percentageOfNodesToScore=a.pct)
        if a.extra_config:
            cfg.update(json.loads(a.extra_config))
        if sharded:  # one scheduler, nodes sharded over the ranks; the RCCL id comes from rank 0
            obj = [comm_unique_id() if rank == 0 else None]
            if dist is not None:
                dist.broadcast_object_list(obj, src=0)
            cfg["distributed"] = {"worldSize": world, "rank": rank, "ncclId": obj[0]}
            cfg["deviceExchange"] = dev_exchange
        s = Scheduler(cfg)
        if a.workload in PROFILES:  # OpportunisticBatching's maxBatchAge clock: fixed, so oracle and device agree
            s.set_clock(BATCH_CLOCK_NS)
        for ob in objects:
            s.upsert_object(ob)
        for n in nodes:
            s.add_node(n)
        for p in init:
            s.add_pod(p)
        handles = [s.compile(p) for p in pods]
        if dist is not None:  # the ranks' hosts loaded the cluster at their own pace: start together
            dist.barrier()
        try:
            for w in range(max(a.warmup, 1 if sharded else 0)):
                s.schedule_batch(handles[w * a.batch:(w + 1) * a.batch], assume=True)
                LOOP_PODS.append(s.kernel_stats())
            for h in handles[:max(a.warmup, 1 if sharded else 0) * a.batch]:
                try:
                    s.forget(h)
                except Exception:
                    pass
        except Exception as e:  # sharded device exchange unavailable here: reported, then the all-reduce path
            print(f"rank {rank}: warm-up with deviceExchange={dev_exchange} failed: {e}", file=sys.stderr, flush=True)
            s.close()
            return None, None
        return s, handles

    dev_exchange = sharded and not a.no_device_exchange
    s, handles = build(dev_exchange)
    if sharded and dist is not None:  # every rank keeps the exchange mode only if every rank's warm-up passed
        ok = torch.tensor([1 if s is not None else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and s is not None:
            s.close()
            s = None
    if s is None:
        dev_exchange = False
        s, handles = build(False)
    n_warm = max(a.warmup, 1 if sharded else 0) * a.batch
    warm, meas = handles[:n_warm], handles[n_warm:]

    # the per-step handle / result arrays are built before timing, as a cgo caller holds them
    arrays = [s.batch_arrays(meas[st * a.batch:(st + 1) * a.batch]) for st in range(a.steps)]
    placed = 0
    kstats = []
    barrier()
    t0 = time.perf_counter()
    for st in range(a.steps):
        s.schedule_batch_into(*arrays[st], assume=True)
        kstats.append(s.kernel_stats())
    barrier()
    dt = time.perf_counter() - t0
    LOOP_PODS.extend(kstats)
    write_loop_pods()
    for _, rs in arrays:  # ksg_result: int32 status first, 24-byte records
        placed += int((np.frombuffer(rs, dtype=np.int32).reshape(len(rs), -1)[:, 0] == 0).sum())
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        pl = torch.tensor([placed], dtype=torch.int64, device="cuda")
        dist.all_reduce(pl)
        placed = int(pl.item())

    total_pods = n_meas * (1 if sharded else world)  # sharded: one scheduler, every rank sees every pod
    if sharded:
        placed //= world
    pods_s = total_pods / dt
    evals_s = pods_s * n_nodes
    kms = sum(k[0] for k in kstats) / len(kstats)
    kbytes = sum(k[1] for k in kstats) / len(kstats)
    kname = max(set(k[3] for k in kstats), key=lambda nm: sum(1 for k in kstats if k[3] == nm))
    achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    traffic = None
    tpath = a.traffic or os.path.join(ROOT, "profiles", f"traffic_{kname}_{a.workload}.json")
    if not os.path.exists(tpath):
        tpath = os.path.join(ROOT, "profiles", f"traffic_{kname}.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("nodes") == n_nodes and world == 1 and tj.get("workload", "c2") == a.workload:
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = None
        warm = pods[:n_warm] if (a.pct != 100 or a.workload in PROFILES) else ()
        if not a.no_cpu_baseline and world == 1:
            # the reference's default parallelism (16 goroutines over nodes), then one thread
            v, done, cdt, ores = cpu_baseline(nodes, init, pods[n_warm:], a.cpu_seconds, threads=a.cpu_threads,
                                              pct=a.pct, objects=objects, profile=PROFILES.get(a.workload), warm=warm)
            bk = cpu_baseline.breakdown
            v1, done1, cdt1, _ = cpu_baseline(nodes, init, pods[n_warm:], a.cpu_seconds / 2, threads=1, pct=a.pct,
                                              objects=objects, profile=PROFILES.get(a.workload), warm=warm)
            bk1 = cpu_baseline.breakdown
            # every CPU the process may use (affinity mask and cgroup quota)
            ncpu = usable_cpus()
            if ncpu == a.cpu_threads:
                va, donea, cdta = v, done, cdt
            else:
                va, donea, cdta, _ = cpu_baseline(nodes, init, pods[n_warm:], a.cpu_seconds / 2, threads=ncpu,
                                                  pct=a.pct, objects=objects, profile=PROFILES.get(a.workload), warm=warm)
            cpu = {"value": round(v, 2), "unit": "pods/s", "cores": a.cpu_threads, "kind": "port",
                   "node_evals_per_s": round(v * n_nodes, 1),
                   "sample": f"first {done} of the {n_meas} measured pods from the same initial state, "
                             f"{cdt:.1f} s, oracle/ C++ restatement, Filter/Score over nodes on "
                             f"{a.cpu_threads} threads ({cpu_model()}, {os.cpu_count()} logical CPUs visible)"
                             + ("; percentageOfNodesToScore < 100: the cut Filter pass is sequential, Score "
                                "on the pool" if a.pct != 100 else ""),
                   "us_per_pod_by_section": bk,
                   "host_cpus": cpu_topology(),
                   "single_thread": {"value": round(v1, 2), "cores": 1,
                                     "sample": f"first {done1} pods, {cdt1:.1f} s, 1 thread",
                                     "us_per_pod_by_section": bk1},
                   "all_cores": {"value": round(va, 2), "cores": ncpu,
                                 "sample": f"first {donea} pods, {cdta:.1f} s, {ncpu} threads = the CPUs this "
                                           f"process may use (affinity mask, cgroup quota)"
                                           + (" -- the same run as the 16-thread value" if ncpu == a.cpu_threads
                                              else "")}}
        parity = None
        if cpu is not None and not a.no_verify:
            # the timed stream's results (ScheduleResult: status, node, evaluated, feasible, total score)
            # against the oracle's over the same pods from the same initial state
            gres = [r.as_tuple() for _, rs in arrays for r in rs][:len(ores)]
            bad = [k for k, (x, y) in enumerate(zip(gres, ores)) if x != y]
            parity = {"checked_pods": len(ores), "mismatches": len(bad), "first_mismatch": bad[0] if bad else None,
                      "against": "oracle/ (same pods, same initial state)"}
            if bad:
                print(f"PARITY FAILURE: {len(bad)} of {len(ores)} timed pods differ from the oracle "
                      f"(first: pod {bad[0]}: {gres[bad[0]]} vs {ores[bad[0]]})", file=sys.stderr, flush=True)
        out = {
            "metric": "pods scheduled/sec + node-evals/sec at 5k/100k nodes, 1/2/4/8 MI355X",
            "value": round(pods_s, 2),
            "unit": "pods/s",
            "node_evals_per_s": round(evals_s, 1),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if (sharded and scaling == "strong") else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (scheduler_perf node-default / pod-default templates, seeded)",
            "config": {"workload": f"{wname} {n_nodes} nodes / {n_init} init pods / "
                                   f"{n_meas} measured pods" + ("" if sharded or world == 1 else " per GPU")
                                   + (f" (BASELINE configs[{cfg_ix}])" if cfg_ix is not None else ""),
                       "nodes": n_nodes, "pods_per_step": a.batch, "percentageOfNodesToScore": a.pct,
                       "plugins": "default",
                       "parallelism": (f"nodes-sharded{world}" if sharded
                                       else f"replicas{world}" if world > 1 else "single"),
                       "exchange": ("device (loop granules stored into every rank's memory over xGMI)"
                                    if dev_exchange else "RCCL all-reduce per pod") if sharded else None},
            "placed": placed,
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "traffic_unit": ("HBM bytes per pod (one pod of a persistent-loop dispatch: PMC FETCH_SIZE "
                                          "+ WRITE_SIZE, separate passes, profiles/traffic_*.json)"
                                          if kname in ("k_sched_loop", "k_agg_loop") else
                                          "HBM bytes per k_filter_score launch (PMC FETCH_SIZE + WRITE_SIZE)"),
                         "avg_kernel_us": round(kms * 1e3, 3),
                         "avg_kernel_us_unit": "per pod" if kname in ("k_sched_loop", "k_agg_loop") else "per launch",
                         "algo_bytes_per_launch": round(kbytes, 1),
                         "algo_bytes_unit": "per pod" if kname in ("k_sched_loop", "k_agg_loop") else "per launch"},
            # the dominant kernel's per-pod (loops) or per-launch time in each timed step: a drift over the
            # steps (C5's fill-front workgroup) shows as max vs min / first vs last
            "kernel_us_per_step": {"kernel": kname, "min": round(min(k[0] for k in kstats) * 1e3, 3),
                                   "max": round(max(k[0] for k in kstats) * 1e3, 3),
                                   "first": round(kstats[0][0] * 1e3, 3), "last": round(kstats[-1][0] * 1e3, 3)},
            "cpu_baseline": cpu,
            "parity": parity,
        }
    s.close()
    if rank == 0:
        if world == 1 and a.workload == "c2" and not a.no_sub and not sharded:
            out["c5_100k"] = sub_record(a)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
