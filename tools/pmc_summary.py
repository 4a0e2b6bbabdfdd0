"""Summary of the PMC passes of tools/wgrad_pmc.sh: one row per worker-batched GEMM kernel.

  python tools/pmc_summary.py gpurun_out/pmc_<tag>

Units (MI355X_MICROARCH.md): FETCH_SIZE / WRITE_SIZE in KiB; FETCH_SIZE = TCC_EA0_RDREQ x 64 B and
reports half the bytes of a 16-B-per-lane streaming read (so it is shown raw and x2);
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY in quad-cycles (disjoint: wait + wait_inst + active
~ wave cycles); SQ_VALU_MFMA_BUSY_CYCLES in cycles.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import probe_name  # noqa: E402


def load(d):
    vals = {}
    for path in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = probe_name(r["Kernel_Name"])
                if name is None:
                    continue
                vals.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(
                    float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def main():
    d = sys.argv[1]
    data = load(d)
    rows = []
    for k in sorted(data):
        c = data[k]
        g = c.get
        row = dict(kernel=k)
        if g("FETCH_SIZE") is not None:
            row["fetch_raw_GB"] = round(g("FETCH_SIZE") * 1024 / 1e9, 3)
            row["fetch_x2_GB"] = round(2 * g("FETCH_SIZE") * 1024 / 1e9, 3)
        if g("WRITE_SIZE") is not None:
            row["write_GB"] = round(g("WRITE_SIZE") * 1024 / 1e9, 3)
        if g("TCC_EA0_RDREQ_sum") is not None:
            rq, rq32 = g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_RDREQ_32B_sum") or 0.0
            row["rdreq_M"] = round(rq / 1e6, 2)
            row["rdreq_32B_frac"] = round(rq32 / max(rq, 1), 4)
            row["rdreq_x64_GB"] = round(rq * 64 / 1e9, 3)
            row["rdreq_x128_GB"] = round(rq * 128 / 1e9, 3)
        if g("TCC_HIT_sum") is not None:
            h, m = g("TCC_HIT_sum"), g("TCC_MISS_sum")
            row["l2_hit"] = round(h / max(h + m, 1), 4)
        if g("SQ_WAVE_CYCLES"):
            wc = g("SQ_WAVE_CYCLES")
            row["wait_any"] = round(g("SQ_WAIT_ANY", 0) / wc, 3)
            row["wait_inst_any"] = round(g("SQ_WAIT_INST_ANY", 0) / wc, 3)
            row["active_inst"] = round(g("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("SQ_BUSY_CYCLES"):
            row["mfma_busy_per_sq_busy"] = round(g("SQ_VALU_MFMA_BUSY_CYCLES") /
                                                 g("SQ_BUSY_CYCLES"), 3)
        if g("SQ_INSTS_LDS"):
            row["lds_insts_M"] = round(g("SQ_INSTS_LDS") / 1e6, 2)
        if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_WAIT_INST_LDS") is not None:
            row["lds_bank_conflict_Mcyc"] = round(g("SQ_LDS_BANK_CONFLICT") / 1e6, 2)
            row["wait_inst_lds_Mq"] = round(g("SQ_WAIT_INST_LDS") / 1e6, 2)
        for cn in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_VALU"):
            if g(cn) is not None:
                row[cn.lower()[9:] + "_M"] = round(g(cn) / 1e6, 2)
        if g("GRBM_GUI_ACTIVE") is not None:
            row["grbm_gui_active_M"] = round(g("GRBM_GUI_ACTIVE") / 1e6, 2)
            cyc = g("GRBM_GUI_ACTIVE") / 8          # cycles per XCD = the kernel's cycles
            # utilisations over the chip: 1024 SIMDs (MFMA, VALU issue), 256 CUs (LDS array)
            if g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
                row["mfma_util"] = round(g("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024), 3)
            if g("SQ_LDS_IDX_ACTIVE") is not None:
                row["lds_active_per_cu_cycle"] = round(g("SQ_LDS_IDX_ACTIVE") / (cyc * 256), 3)
            if g("SQ_ACTIVE_INST_VALU") is not None:
                row["valu_active_per_simd"] = round(4 * g("SQ_ACTIVE_INST_VALU") / (cyc * 1024), 3)
        row["raw"] = c
        rows.append(row)
    for r in rows:
        print(json.dumps({k: v for k, v in r.items() if k != "raw"}))
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
