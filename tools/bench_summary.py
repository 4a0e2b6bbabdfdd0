"""Print the headline numbers and per-kernel TFLOP/s of a bench.py JSON line (debug helper)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"] or {}
a = d["aggregation"] or {}
print(f"value {d['value']} {d['unit']}  ms/step {d['ms_per_step']}  mfma_eff {d['mfma_efficiency_whole_step']}")
print(f"roofline {r.get('kernel')} {r.get('achieved')} TF/s frac {r.get('frac')}  all GEMMs "
      f"{(r.get('all_gemms') or {}).get('achieved')}")
print(f"aggregation {a.get('avg_launch_us')} us {a.get('achieved')} GB/s frac {a.get('frac')}")
for k, v in sorted((r.get("per_kernel") or {}).items()):
    print(f"  {k:20s} {v['avg_ms']:8.4f} ms {v['tflops']:7.1f} TF/s")
