"""GPU busy time vs wall time over the last part of a rocprofv3 kernel trace (bench.py run).

  python tools/trace_gaps.py <trace dir> [fraction of the trace to keep, default 0.5]

Reads <dir>/run_kernel_trace.csv (and run_memory_copy_trace.csv if present), keeps the last
fraction of the dispatches by start time (the timed epochs), and prints: wall span, the union of
busy intervals, the idle share, the largest gaps and the kernels with the most total time.
"""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    if not os.path.exists(path):
        return []
    rows = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Operation") or r.get("Kind") or "copy"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return rows


def main():
    d = sys.argv[1]
    keep = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    ev = load(os.path.join(d, "run_kernel_trace.csv")) + \
        load(os.path.join(d, "run_memory_copy_trace.csv"))
    ev.sort()
    ev = ev[int(len(ev) * (1 - keep)):]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    busy, cur_s, cur_e = 0, ev[0][0], ev[0][1]
    gaps = []
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    print(f"dispatches {len(ev)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  "
          f"idle {100 * (1 - busy / span):.1f} %")
    gaps.sort(reverse=True)
    print("largest gaps (us, next kernel):")
    for g, n in gaps[:12]:
        print(f"  {g / 1e3:9.1f}  {n[:90]}")
    tot = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        tot[n][0] += e - s
        tot[n][1] += 1
    print("kernels by total time:")
    for n, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"  {t / 1e6:8.2f} ms {c:6d}  {100 * t / busy:5.1f} %  {n[:90]}")


if __name__ == "__main__":
    main()
