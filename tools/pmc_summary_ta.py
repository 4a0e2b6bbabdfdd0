"""Per-kernel TA / TD / TCP busy and stall fractions from tools/gpu_job.sh's tatd passes.

  python tools/pmc_summary_ta.py gpurun_out/<tag>

Each *_sum counter is summed over its block's instances (one TA, TD and TCP per CU: 256); it is
shown raw and as a fraction of GRBM_GUI_ACTIVE / 8 (cycles per XCD, as pmc_summary.py) x 256.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

NAMES = ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum",
         "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
         "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum"]


def main():
    data = load(sys.argv[1])
    for k in sorted(data):
        c = data[k]
        g = c.get("GRBM_GUI_ACTIVE")
        if not g:
            continue
        denom = g / 8 * 256
        parts = [f"{k:16s} grbm/8 {g / 8 / 1e6:7.2f}M"]
        for n in NAMES:
            if n in c:
                parts.append(f"{n.replace('_sum', '')} {c[n] / denom:.3f}")
        print(" | ".join(parts))


if __name__ == "__main__":
    main()
