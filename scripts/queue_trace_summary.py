"""Summarise a rocprofv3 --kernel-trace CSV of scripts/group_probe.py: every persistent-loop dispatch
(k_sched_loop / k_agg_loop) with its host thread, hardware queue, stream and start/end time (ms from the
first dispatch), and per queue the streams and threads that used it.
    python scripts/queue_trace_summary.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
ms = lambda t: (int(t) - t0) / 1e6  # noqa: E731
use = defaultdict(lambda: defaultdict(int))
for r in rows:
    use[r["Queue_Id"]][(r["Stream_Id"], r["Thread_Id"])] += 1
print(f"{len(rows)} dispatches; queue -> {{(stream, thread): dispatches}}")
for q in sorted(use, key=int):
    print(f"  queue {q}: {dict(use[q])}")
print("persistent-loop dispatches (sorted by start):")
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    k = r["Kernel_Name"]
    if "k_sched_loop" in k or "k_agg_loop" in k:
        print(f"  {ms(r['Start_Timestamp']):10.3f} .. {ms(r['End_Timestamp']):10.3f} ms  queue {r['Queue_Id']:>3} "
              f"stream {r['Stream_Id']:>3} thread {r['Thread_Id']} grid {r['Grid_Size_X']} {k[:40]}")
