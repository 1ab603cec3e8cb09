#!/usr/bin/env python3
"""Block / branch map of one rollout kernel's step loop from a gfx950 .s dump
(hipcc --cuda-device-only -S csrc/qt_rollout.hip).  Used to check that the
fast step's common path has no taken branch but the loop back-edge.

  python scripts/loop_blocks.py <file.s> [mangled-name-fragment]
"""

import re
import sys


def main():
    path = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else "ILi2ELi1ELi6ELb0ELb1E"  # yaw-at-rest, linear, K6, no FF, KS
    s = open(path).read()
    name = [m for m in re.findall(r"^(_Z\S*rollout_kernel\S*):", s, re.M) if tag in m][0]
    body = s[s.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    blocks, cur = [], None
    for line in body.splitlines():
        t = line.strip()
        if re.match(r"^\.LBB\S+:", t) or t.startswith("; %bb."):
            cur = {"name": t.split()[0].rstrip(":"), "loop": "Loop" in t, "hdr": "=>This Loop Header" in t,
                   "n": 0, "valu": 0, "salu": 0, "br": []}
            blocks.append(cur)
            continue
        if cur is None or not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        cur["n"] += 1
        cur["valu"] += op.startswith("v_")
        cur["salu"] += op.startswith("s_")
        if op.startswith(("s_cbranch", "s_branch")):
            cur["br"].append(t.split(";")[0].strip())
    for b in blocks:
        if b["loop"] or b["hdr"]:
            mark = "H" if b["hdr"] else " "
            print(f"{mark} {b['name']:14s} n={b['n']:4d} valu={b['valu']:4d} salu={b['salu']:3d} {b['br']}")


if __name__ == "__main__":
    main()
