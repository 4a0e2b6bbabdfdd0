"""SURVEY 8(c) ratios of the weight / bias gradients against the number of workers summed
(tests/test_gpu_survey_chunk.py MEASURED records, FLSIM_TOL_LOG census): one row per tensor, one
column per worker count, for each build's census file.

  python tools/survey_k_table.py profiles/r06/survey_k/tol_*.jsonl
"""
import json
import sys


def main():
    for path in sys.argv[1:]:
        rows, ratio = {}, {}
        for line in open(path):
            r = json.loads(line)
            if r.get("kind") == "pn1_chunk_wgrad":
                nw = r["workers"]
                for k, g in r["rel_gpu"].items():
                    rows.setdefault(k, {})[nw] = (g, r["rel_cpu32"][k])
            elif str(r.get("kind", "")).startswith("pn1_chunk_wgrad_nw"):
                ratio[int(r["kind"].rsplit("nw", 1)[1])] = r["survey"]
        ks = sorted({nw for v in rows.values() for nw in v})
        print(f"== {path}: SURVEY 8(c) ratio ||g_gpu - g64|| / (2 ||g_cpu32 - g64|| + 1e-7 ||g64||)"
              f" (<= 1 passes); workers summed: {ks} (128 = one 16,384-sample launch)")
        print(f"{'tensor':16s}" + "".join(f"{nw:>8d}" for nw in ks) +
              "   rel-L2 gpu / cpu32 at the largest")
        for k in rows:
            cells = "".join(f"{ratio.get(nw, {}).get(k, float('nan')):8.2f}" for nw in ks)
            g, c = rows[k][ks[-1]]
            print(f"{k:16s}{cells}   {g:.2e} / {c:.2e}")
        print()


if __name__ == "__main__":
    main()
