#!/usr/bin/env python3
"""Instruction mix of the largest basic blocks of the kernels in a hipcc
--save-temps .s file (the steady chunks of the temporally blocked marches):
FP64 VALU, DPP moves, buffer loads / stores, scratch (spill) accesses,
waterfall loops (s_and_saveexec), v_readlane (SGPR spill reloads).

    python tools/isa_blocks.py FILE.s [--kernel SUBSTR] [--top N]
"""
import argparse
import collections
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    cur_f, name = None, None
    blocks = collections.defaultdict(list)
    funcs = {}
    for l in open(a.asm):
        m = re.match(r"^(_Z\S+):\s*", l)
        if m and not l.startswith("\t"):
            cur_f = m.group(1)
            name = cur_f + ":entry"
            continue
        m = re.match(r"^(\.LBB(\d+)_\d+):", l)
        if m:
            name = m.group(1)
            funcs.setdefault(m.group(2), cur_f)
            continue
        if l.startswith("\t") and name and not l.strip().startswith((".", ";")):
            blocks[name].append(l.strip().split()[0])
    for fid, fn in sorted(funcs.items(), key=lambda x: int(x[0])):
        if a.kernel not in str(fn):
            continue
        bl = [(n, b) for n, b in blocks.items() if n.startswith(".LBB%s_" % fid)]
        tot = collections.Counter()
        for _, b in bl:
            tot.update(b)
        print(fid, str(fn)[:70], "blocks", len(bl), "saveexec", tot["s_and_saveexec_b64"],
              "scratch", sum(v for k, v in tot.items() if "scratch" in k))
        for n, b in sorted(bl, key=lambda x: -len(x[1]))[:a.top]:
            c = collections.Counter(b)
            fp = sum(c[k] for k in ("v_fma_f64", "v_add_f64", "v_mul_f64", "v_fmac_f64_e32"))
            print("    %-12s %5d fp64 %4d dpp %4d ld %3d st %3d scratch %3d saveexec %3d "
                  "readlane %3d" % (n, len(b), fp, c["v_mov_b32_dpp"], c["buffer_load_dwordx4"],
                                    c["buffer_store_dwordx4"] + c["global_store_dwordx4"],
                                    sum(v for k, v in c.items() if "scratch" in k),
                                    c["s_and_saveexec_b64"], c["v_readlane_b32"]))


if __name__ == "__main__":
    main()
