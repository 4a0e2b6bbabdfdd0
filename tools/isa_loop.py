"""Instruction mix of a kernel's hottest basic block (the MFMA main loop) in a clang -S listing.
Usage: python tools/isa_loop.py [--all] <file.s> <symbol-substring> [more substrings...]
--all: every basic block with MFMAs or LDS stores, not only the one with the most MFMAs."""
import re
import sys
from collections import Counter

def blocks(lines, start):
    cur, name = [], "entry"
    for ln in lines[start + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end"):
            break
        if re.match(r"^\.LBB\d+_\d+:", s):
            yield name, cur
            name, cur = s.split(":")[0], []
            continue
        if not s or s.startswith(";") or s.startswith(".") :
            continue
        cur.append(s.split()[0])
    yield name, cur

def classify(op):
    if op.startswith("v_mfma"): return "mfma"
    if op.startswith("ds_read") or op.startswith("ds_load"): return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"): return "ds_write"
    if op.startswith("buffer_load") or op.startswith("global_load"): return "vmem_load"
    if op.startswith("buffer_store") or op.startswith("global_store"): return "vmem_store"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith("s_barrier"): return "barrier"
    if op.startswith("v_mov") or op.startswith("v_pk_mov"): return "v_mov"
    if op.startswith("v_"): return "valu"
    if op.startswith("s_"): return "salu"
    return "other"

def main():
    args = sys.argv[1:]
    every = "--all" in args
    args = [a for a in args if a != "--all"]
    path, subs = args[0], args[1:]
    lines = open(path).read().split("\n")
    for i, ln in enumerate(lines):
        if ln.endswith(":") or ": ;" in ln:
            lab = ln.split(":")[0]
            if lab.startswith("_Z") and all(s in lab for s in subs):
                print(lab[:160])
                if every:
                    for name, ops in blocks(lines, i):
                        c = Counter(classify(o) for o in ops)
                        if c.get("mfma") or c.get("ds_write"):
                            vc = Counter(o for o in ops if classify(o) == "valu")
                            print("  block", name, "instrs", len(ops), dict(c))
                            print("    valu:", vc.most_common(10))
                    continue
                best = max(blocks(lines, i), key=lambda b: sum(1 for o in b[1] if o.startswith("v_mfma")))
                c = Counter(classify(o) for o in best[1])
                print("  block", best[0], "instrs", len(best[1]), dict(c))
                vc = Counter(o for o in best[1] if classify(o) in ("valu", "v_mov"))
                print("  valu ops:", vc.most_common(12))
                sc = Counter(o for o in best[1] if classify(o) == "salu")
                print("  salu ops:", sc.most_common(8))

if __name__ == "__main__":
    main()
