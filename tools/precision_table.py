"""Precision census of a GPU test run (the split-bf16 GEMMs' error against each bound).

  python tools/precision_table.py <dir> [tag ...]

Reads <dir>/flips_<tag>.jsonl (tests/_flips.py: teacher-forced rel-L2 `tf` and decision flips
against fp64, GPU and CPU fp32), <dir>/tol_<tag>.jsonl (per-tensor teacher-forced rel-L2 of the
VGG tests) and the MEASURED lines of <dir>/pytest_<tag>.txt (trajectory ratios, run with -s), and
prints one table per tag: the largest measured value of each check beside the bound the tests
hold (tests/_flips.py TF_TOL / FLIP_C / FLIP_FLOOR, tests/test_gpu_vgg*.py TF_TOL,
tests/test_gpu_configs.py GAP_C / DRIFT_C, tests/test_gpu_parity.py trajectory factors).
"""
import json
import os
import re
import sys


def jl(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [json.loads(x) for x in f if x.strip()]


def main():
    d = sys.argv[1]
    tags = sys.argv[2:] or [""]
    for tag in tags:
        sfx = f"_{tag}" if tag else ""
        print(f"== {tag or 'default'}")
        fl = jl(os.path.join(d, f"flips{sfx}.jsonl"))
        if fl:
            tf = max(r["tf"] for r in fl)
            fg = sum(sum(r["flips_gpu"].values()) for r in fl)
            fc = sum(sum(r["flips_cpu32"].values()) for r in fl)
            worst = max(sum(r["flips_gpu"].values()) - 3 * sum(r["flips_cpu32"].values())
                        for r in fl)
            print(f"  PN1 teacher-forced rel-L2 (max over {len(fl)} checks): {tf:.3e}")
            print(f"  decision flips vs fp64, summed: GPU {fg}, CPU fp32 {fc}; "
                  f"max(GPU - 3 CPU) per check {worst}")
        tl = jl(os.path.join(d, f"tol{sfx}.jsonl"))
        for r in tl:
            w = r.get("worst", {})
            if w:
                k = max(w, key=w.get)
                print(f"  {r['test'][:90]:90s} worst tensor {k} {w[k]:.3e}")
        pt = os.path.join(d, f"pytest{sfx}.txt")
        if os.path.exists(pt):
            with open(pt) as f:
                for line in f:
                    m = re.search(r"MEASURED (\{.*\})", line)
                    if m:
                        print("  MEASURED", m.group(1)[:200])


if __name__ == "__main__":
    main()
