"""Per-kernel SQ summary of the aggregation kernels from one rocprofv3 --pmc pass over
tools/agg_bench.py (tools/gpu_job.sh streampmc).

  python tools/stream_pmc.py <counter_collection.csv>

Per kernel name (averaged over its dispatches): duration, VALU instructions per wave, VALU busy
(SQ_ACTIVE_INST_VALU x 4 cycles over GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), wave-cycles waiting on
anything (SQ_WAIT_ANY / SQ_WAVE_CYCLES), and vector memory instructions per wave.
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    dur = defaultdict(dict)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        d = r["Dispatch_Id"]
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[name].add(d)
        dur[name][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for name, c in per.items():
        k = len(n[name])
        g = lambda key: c.get(key, 0.0) / k          # noqa: E731  per dispatch
        cyc = g("GRBM_GUI_ACTIVE") / 8
        waves = max(g("SQ_WAVES"), 1.0)
        us = sum(dur[name].values()) / k
        print(f"{name[:60]:60s} dispatches {k:3d}  {us:8.2f} us  "
              f"VALU/wave {g('SQ_INSTS_VALU') / waves:7.1f}  "
              f"VALU busy {4 * g('SQ_ACTIVE_INST_VALU') / max(cyc * 1024, 1):.3f}  "
              f"wait_any {g('SQ_WAIT_ANY') / max(g('SQ_WAVE_CYCLES'), 1):.3f}  "
              f"vmem rd/wr per wave {g('SQ_INSTS_VMEM_RD') / waves:.1f} / "
              f"{g('SQ_INSTS_VMEM_WR') / waves:.1f}  clock {cyc / us / 1e3:.2f} GHz")


if __name__ == "__main__":
    main()
