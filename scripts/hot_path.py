#!/usr/bin/env python3
"""Instruction mix of one rollout kernel's hot step loop, from a gfx950 .s dump
(`make -C lqr-quadcopter-test_amd asm`).  The hot path is followed from the
loop header: fall through, take unconditional branches, and at a conditional
branch continue on the fall-through unless the branch targets an earlier
block (the back edge) or --take lists it.

  python scripts/hot_path.py <file.s> [mangled-name-fragment] [--take LABEL ...]
"""

import collections
import re
import sys


def blocks_of(body):
    out, cur = [], None
    for line in body.splitlines():
        t = line.strip()
        m = re.match(r"^(\.LBB\S+):", t)
        if m or t.startswith("; %bb."):
            cur = {"name": m.group(1) if m else t.split()[1], "hdr": "Loop Header" in t, "ins": []}
            out.append(cur)
            continue
        if cur is None or not t or t.startswith((";", ".")):
            continue
        cur["ins"].append(t.split(";")[0].strip())
    return out


def main():
    args = [a for a in sys.argv[1:] if a != "--outer"]
    take = set()
    if "--take" in args:
        i = args.index("--take")
        take = set(args[i + 1:])
        args = args[:i]
    path = args[0]
    tag = args[1] if len(args) > 1 else "ILi2ELi1ELi6ELb0ELb1E"
    s = open(path).read()
    names = [m for m in re.findall(r"^(_Z\S*rollout_kernel\S*):", s, re.M) if tag in m]
    name = names[0]
    body = s[s.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    bl = blocks_of(body)
    idx = {b["name"]: i for i, b in enumerate(bl)}
    # the step loop: among the innermost loops (block ranges [h, j] closed by
    # a backward branch that contain no other such range), the largest
    spans = []
    for j, b in enumerate(bl):
        for ins in b["ins"]:
            op = ins.split()[0]
            if op.startswith(("s_cbranch", "s_branch")) and ins.split()[1] in idx and idx[ins.split()[1]] <= j:
                spans.append((idx[ins.split()[1]], j))
    inner = [(h, j) for (h, j) in spans
             if not any((h2, j2) != (h, j) and h <= h2 and j2 <= j for (h2, j2) in spans)]
    loops = [(-sum(sum(i.startswith("v_") for i in bl[q]["ins"]) for q in range(h, j + 1)), h) for (h, j) in inner]
    hdrs = [i for i, b in enumerate(bl) if b["hdr"]]
    if "--outer" in sys.argv:
        start = max(hdrs, key=lambda i: len(bl[i]["ins"])) if hdrs else 0
    else:
        start = min(loops)[1] if loops else 0
    i, seen, hot = start, set(), []
    while i not in seen and i < len(bl):
        seen.add(i)
        hot.append(i)
        nxt = i + 1
        for ins in bl[i]["ins"]:
            op = ins.split()[0]
            if op == "s_branch":
                nxt = idx[ins.split()[1]]
                break
            if op.startswith("s_cbranch"):
                tgt = idx[ins.split()[1]]
                if tgt <= start or ins.split()[1] in take:
                    nxt = tgt
                    break
        i = nxt
    mix = collections.Counter()
    n = collections.Counter()
    for i in hot:
        for ins in bl[i]["ins"]:
            op = ins.split()[0]
            cls = "valu" if op.startswith("v_") else ("branch" if op.startswith(("s_cbranch", "s_branch")) else
                                                       ("salu" if op.startswith("s_") else "other"))
            n[cls] += 1
            mix[op] += 1
    print(f"kernel {name[:90]}")
    print("hot path blocks:", " ".join(bl[i]["name"] for i in hot))
    print("counts:", dict(n), "total", sum(n.values()))
    for op, k in mix.most_common():
        print(f"  {k:4d} {op}")


if __name__ == "__main__":
    main()
