"""Summarise rocprofv3 rocpd databases (gpurun_out/prof/*) into committed text/JSON under profiles/.

  python scripts/prof_summary.py <tag> [nodes] [workload] [pods_per_loop_dispatch]
writes profiles/<tag>_kernel_stats.txt (per-kernel calls / total / average duration, the
`--kernel-trace --stats` summary), profiles/<tag>_pmc.txt (FETCH_SIZE / WRITE_SIZE per kernel),
and profiles/traffic_<kernel>.json (HBM bytes per k_filter_score launch, or per pod of a
k_sched_loop dispatch, for bench.py's roofline.traffic).
"""
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")


def short(name):
    return name.split("(")[0]


def main():
    tag = sys.argv[1]
    nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    workload = sys.argv[3] if len(sys.argv) > 3 else "c2"
    # pods per loop dispatch, on average: from the pods bench.py counted per loop kernel over the profiled run
    # (KSG_LOOP_PODS_OUT, gpurun_out/prof/loop_pods_<pass>.json) when present, else this argument (a 1000-pod
    # batch of one loop kernel runs as 7 chunks: engine.cpp run_batch 32, 160, 485, 194, 78, 31, 20)
    loop_pods = float(sys.argv[4]) if len(sys.argv) > 4 else 1000.0 / 7.0

    def pods_file(sub):
        p = os.path.join(PROF, "loop_pods_" + sub.split("pmc_", 1)[-1] + ".json")
        return json.load(open(p)) if os.path.exists(p) else {}
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    # KSG_PROF_TRACE: the kernel-trace directory under gpurun_out/prof (default "trace")
    c = sqlite3.connect(os.path.join(PROF, os.environ.get("KSG_PROF_TRACE", "trace"), "run_results.db"))
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    tpods = pods_file(os.environ.get("KSG_PROF_TRACE", "trace"))
    lines = [f"# rocprofv3 --kernel-trace --stats -- python3 bench.py (tag {tag})",
             f"{'kernel':60s} {'calls':>8s} {'total_us':>12s} {'avg_us':>9s} {'pct':>6s}"]
    for n, calls, tot, avg, pct in rows:  # top_kernels is in us; kernels.duration is ns
        lines.append(f"{short(n):60s} {calls:8d} {tot:12.1f} {avg:9.3f} {pct:6.2f}")
    # per-dispatch durations of the roofline kernel
    for kn in ("k_filter_score", "k_sched_loop", "k_agg_loop"):
        d = [r[0] for r in c.execute(f"select duration from kernels where name like '%{kn}%'")]
        if d:
            d.sort()
            lines.append(f"{kn} dispatch duration us: median {d[len(d) // 2] / 1e3:.3f} "
                         f"p10 {d[len(d) // 10] / 1e3:.3f} p90 {d[9 * len(d) // 10] / 1e3:.3f}")
            if kn in ("k_sched_loop", "k_agg_loop"):
                lp = tpods[kn] / len(d) if tpods.get(kn) else loop_pods
                lines.append(f"{kn} per pod us (mean dispatch / {lp:.2f} pods per dispatch"
                             + (", the pods bench.py counted" if tpods.get(kn) else "") + f"): "
                             f"{sum(d) / len(d) / 1e3 / lp:.3f}")
    open(os.path.join(out, f"{tag}_kernel_stats.txt"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))

    per = {}
    ppods = {}  # counter -> {kernel: pods its dispatches ran in that pass}
    sfx = os.environ.get("KSG_PROF_PMC_SUFFIX", "")  # e.g. "_c4": gpurun_out/prof/pmc_fetch_c4
    for counter, sub in (("FETCH_SIZE", "pmc_fetch" + sfx), ("WRITE_SIZE", "pmc_write" + sfx)):
        p = os.path.join(PROF, sub, "run_results.db")
        if not os.path.exists(p):
            continue
        ppods[counter] = pods_file(sub)
        cc = sqlite3.connect(p)
        for name, val in cc.execute("select kernel_name, value from counters_collection where counter_name=?",
                                    (counter,)):
            per.setdefault(short(name), {}).setdefault(counter, []).append(val)
    pl = [f"# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), KiB per dispatch (tag {tag})",
          "# gfx950: FETCH_SIZE under-reports wide streaming reads by 2x (MI355X_MICROARCH.md HBM section);",
          "# the access widths here are 4-8 B/lane (uncalibrated) -- both raw and x2 are listed."]
    traffic = {}
    for k, v in sorted(per.items()):
        f = v.get("FETCH_SIZE", [])
        w = v.get("WRITE_SIZE", [])
        fa = sum(f) / len(f) if f else 0.0
        wa = sum(w) / len(w) if w else 0.0
        pl.append(f"{k:60s} dispatches {len(f):6d} FETCH_KiB {fa:10.2f} (x2 {2 * fa:10.2f}) WRITE_KiB {wa:10.2f}")
        for kn, per_unit in (("k_filter_score", 1), ("k_sched_loop", loop_pods), ("k_agg_loop", loop_pods)):
            if k.split("<")[0].endswith(kn):  # (templated kernels: k_sched_loop<2, false>)
                # the pass's bytes over every dispatch of the kernel / the pods those dispatches ran
                pf = ppods.get("FETCH_SIZE", {}).get(kn)
                pw = ppods.get("WRITE_SIZE", {}).get(kn)
                uf = pf / len(f) if pf and f else per_unit
                uw = pw / len(w) if pw and w else per_unit
                traffic[kn] = {"kernel": kn, "nodes": nodes, "workload": workload, "fetch_kib_raw": fa / uf,
                               "write_kib": wa / uw,
                               "bytes_per_launch": round((fa / uf + wa / uw) * 1024.0, 1),
                               "bytes_per_launch_fetch_x2": round((2 * fa / uf + wa / uw) * 1024.0, 1),
                               "note": f"FETCH_SIZE+WRITE_SIZE per {kn} dispatch"
                                       + (f" / {uf:.2f} (fetch pass) and {uw:.2f} (write pass) pods per dispatch"
                                          + (", the pods bench.py counted" if pf and pw else "")
                                          if kn != "k_filter_score" else "")
                                       + ", separate PMC passes (tag " + tag + ")"}
    open(os.path.join(out, f"{tag}_pmc.txt"), "w").write("\n".join(pl) + "\n")
    print("\n".join(pl))
    for kn, t in traffic.items():  # k_agg_loop runs on several workloads: one file per workload
        fn = f"traffic_{kn}_{workload}.json" if kn == "k_agg_loop" else f"traffic_{kn}.json"
        json.dump(t, open(os.path.join(out, fn), "w"), indent=1)

    # shader-counter pass (scripts/gpu.sh sq=<workload>): instruction mix per wave and per pod, clock
    p = os.path.join(PROF, "pmc_sq", "run_results.db")
    if os.path.exists(p):
        cc = sqlite3.connect(p)
        sq = {}
        for name, cn, val in cc.execute("select kernel_name, counter_name, value from counters_collection"):
            if "k_sched_loop" in name:
                sq.setdefault(cn, []).append(val)
        if sq:
            avg = {k: sum(v) / len(v) for k, v in sq.items()}
            waves = avg.get("SQ_WAVES", 1.0) or 1.0
            sl = [f"# rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                  f"GRBM_GUI_ACTIVE GRBM_COUNT, k_sched_loop, per dispatch ({loop_pods:.2f} pods) (tag {tag})"]
            for k in sorted(avg):
                sl.append(f"{k:20s} {avg[k]:16.1f}")
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if k in avg:
                    sl.append(f"{k} per wave per pod: {avg[k] / waves / loop_pods:.1f}")
            open(os.path.join(out, f"{tag}_pmc_sq.txt"), "w").write("\n".join(sl) + "\n")
            print("\n".join(sl))


if __name__ == "__main__":
    main()
