"""HBM traffic per launch from the rocprofv3 PMC passes of tools/gpu_profile.sh.

  python tools/pmc_traffic.py <profile dir> [out.json ...]

Reads <dir>/pmc_FETCH_SIZE/run_counter_collection.csv and <dir>/pmc_WRITE_SIZE/...csv, maps the
template kernel names to the probe names bench.py reports, and writes
{kernel: {"bytes_per_launch": B, "fetch": F, "write": W, "launches": n, "source": ...,
"trace_avg_ns": T}} (T = the kernel-trace pass's average duration, when <dir>/trace has it).
Units and corrections follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled.
"""
import csv
import json
import os
import re
import sys

FWD = {(32, 32, 4): 1, (34, 34, 48): 2, (18, 18, 48): 3, (20, 20, 96): 4, (11, 11, 96): 5,
       (13, 13, 192): 6}
DGRAD = {(36, 36, 48): 2, (20, 20, 96): 3, (22, 22, 96): 4, (13, 13, 192): 5, (15, 15, 192): 6,
         (14, 14, 192): 6}


def probe_name(kname):
    if "k_slab_step_seq" in kname:
        return "slab_step_seq"
    m = re.search(r"k_slab_step<(true|false), (true|false)>", kname)
    if m:
        if m.group(1) == "false":
            return "slab_sum"
        return "slab_step" if m.group(2) == "true" else "slab_step_seq"
    if "k_conv1_fwd" in kname:
        return "conv1_fwd"
    m = re.search(r"k_pool_scatter(_nchw)?<(\d+), (\d+), (\d+)", kname)
    if m:
        return f"pool_scatter_{m.group(2)}x{m.group(3)}x{m.group(4)}"
    m = re.search(r"k_agg_stream<(true|false)>", kname)
    if m:
        return "aggregate_adam" if m.group(1) == "true" else "aggregate_adam_seq"
    # linear layers (net_kernels.h linear_fwd / linear_wgrad / linear_dgrad): linear1 runs the
    # 128x128 tiles (fp32 dgrad) or the split-bf16 kernel, linear2 the 64x64 fp32 tiles
    if "RowsKC" in kname or "RowsKM" in kname:
        big = "gemm_x6_kernel" in kname or "gemm_kernel<4, 4, 2, 2" in kname
        if "EpiSlabStore" in kname and "Im2col" not in kname:
            return "linear1_fwd" if big else "linear2_fwd"
        if re.search(r"RowsKM<\d+, \d+, 0, 0>, flsim::RowsKM", kname):
            return "linear1_wgrad" if big else "linear2_wgrad"
        if "EpiDropMask" in kname and "Im2col" not in kname:
            return "linear1_dgrad" if big else "linear2_dgrad"
    m = re.search(r"Im2colKM<(\d+), (\d+), (\d+),", kname)
    if m:
        return f"conv{FWD[tuple(map(int, m.groups()))]}_wgrad"
    m = re.search(r"Im2col(?:KC|Direct)<(\d+), (\d+), (\d+), (\d+),", kname)
    if m:
        ih, iw, ci, pad = map(int, m.groups())
        if pad == 2:
            return f"conv{FWD[(ih, iw, ci)]}_fwd"
        return f"conv{DGRAD[(ih, iw, ci)]}_dgrad"
    return None


# probe name -> the arithmetic of the kernel that ran it: "bf16x6" for gemm_x6_kernel (gemm_x6.h,
# fp32 operands split into three bf16 parts on the bf16 matrix cores), "fp32" otherwise;
# bench.py only borrows a split kernel's traffic from a table tagged bf16x6
maths = {}


def read(path, counter):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = probe_name(r["Kernel_Name"])
            if name is None:
                continue
            maths[name] = ("bf16x6" if "gemm_x6_kernel" in r["Kernel_Name"] or
                           "gemm_dx6_kernel" in r["Kernel_Name"] else "fp32")
            out.setdefault(name, []).append(float(r["Counter_Value"]))
    return out


def main():
    d = sys.argv[1]
    outs = sys.argv[2:] or [os.path.join(d, "traffic.json")]
    fetch = read(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = read(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) & set(write)):
        f = 2 * 1024 * sum(fetch[k]) / len(fetch[k])
        w = 1024 * sum(write[k]) / len(write[k])
        res[k] = dict(bytes_per_launch=int(f + w), fetch=int(f), write=int(w),
                      launches=len(fetch[k]), math=maths.get(k, "fp32"),
                      source=f"rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE, "
                             f"{os.path.basename(os.path.normpath(d))}")
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        tot = {}
        with open(stats) as f:
            for r in csv.DictReader(f):
                name = probe_name(r["Name"])
                if name is None:
                    continue
                c, ns = tot.get(name, (0, 0.0))
                tot[name] = (c + int(r["Calls"]), ns + float(r["TotalDurationNs"]))
        for k, (c, ns) in tot.items():
            if k in res and c:
                res[k]["trace_avg_ns"] = ns / c
    for o in outs:
        os.makedirs(os.path.dirname(os.path.abspath(o)), exist_ok=True)
        with open(o, "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)
    for k, v in res.items():
        print(f"{k:16s} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch  ({v['launches']} launches)")


if __name__ == "__main__":
    main()
