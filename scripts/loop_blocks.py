#!/usr/bin/env python3
"""Block / branch map of one rollout kernel's step loop from a gfx950 .s dump
(`make -C lqr-quadcopter-test_amd asm`).  Used to check that the fast step's
common path has no taken branch but the loop back-edge.

  python scripts/loop_blocks.py <file.s> [mangled-name-fragment]
  python scripts/loop_blocks.py <file.s> --table

--table lists, for every yaw-at-rest rollout_kernel instance and every
per-motion loop of rollout_grouped_kernel, the instructions one wave issues
per env step inside the safe horizon (the no-vote loop over its 4 or 2 steps) and
in the voted step that ends each horizon (run_yaw0).
"""

import re
import sys

MOTIONS = {"0": "stationary", "1": "linear", "2": "circular", "3": "sinusoidal", "4": "figure8", "n1": "runtime"}


def blocks_of(s, name):
    body = s[s.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    blocks, cur = [], None
    for line in body.splitlines():
        t = line.strip()
        if re.match(r"^\.LBB\S+:", t) or t.startswith("; %bb."):
            cur = {"name": t.split()[0].rstrip(":"), "loop": "Loop" in t, "hdr": "=>This Loop Header" in t,
                   "inner": "Parent Loop" in t, "n": 0, "valu": 0, "salu": 0, "br": []}
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
    return blocks


def step_loops(blocks):
    """The horizon's two-step body (a self-looping block of > 100 instructions
    whose back edge tests a scalar count) with the voted step after it (the
    next block of > 100 instructions whose branch tests the vote, vcc)."""
    out = []
    big = [b for b in blocks if b["n"] > 100]

    def no_vote(b):
        return any(br.endswith(" " + b["name"]) for br in b["br"]) and not any("vcc" in br for br in b["br"])

    for i, b in enumerate(big):
        if no_vote(b):
            # the voted step: the next big block that ends in the vote (skipping a
            # second no-vote body, run_yaw0's DUAL clamping one)
            is_voted = lambda v: any("vcc" in br for br in v["br"]) and not no_vote(v)  # noqa: E731
            voted = next((v for v in big[i + 1:] if is_voted(v)), None) or \
                next((v for v in reversed(big[:i]) if is_voted(v)), None)
            out.append((b, voted))
    return out


def row(tag, motion, pair, voted):
    """The no-vote loop runs four steps per back edge (two in older builds):
    told apart by its size against the voted step's."""
    v = f"{voted['n']:5d} {voted['valu']:5d} {voted['salu']:5d}" if voted else "    -     -     -"
    k = 4 if voted and pair["n"] > 2.5 * voted["n"] else 2
    print(f"{tag:46s} {motion:11s} {pair['n'] / k:6.1f} {pair['valu'] / k:6.1f} {pair['salu'] / k:5.1f}   {v}")


def table(s):
    print(f"{'kernel':46s} {'motion':11s} {'per no-vote step':>19s}   {'voted step':>17s}")
    print(f"{'':46s} {'':11s} {'instr':>6s} {'VALU':>6s} {'SALU':>5s}   {'instr':>5s} {'VALU':>5s} {'SALU':>5s}")
    for name in re.findall(r"^(_Z\S*rollout_kernel\S*):", s, re.M):
        m = re.search(r"rollout_kernelILi(\d)ELi(n?\d)ELi(\d)ELb(\d)ELb(\d)ELb(\d)E", name)
        if not m or m.group(1) != "2":
            continue
        fl, mo, kc, ff, ks, uni = m.groups()
        for pair, voted in step_loops(blocks_of(s, name)):
            row(f"rollout_kernel<2,{mo.replace('n', '-')},{kc},ff{ff},ks{ks},uni{uni}>", MOTIONS[mo], pair, voted)
    for name in re.findall(r"^(_Z\S*rollout_grouped_kernel\S*):", s, re.M):
        m = re.search(r"rollout_grouped_kernelILi(\d)ELb(\d)ELb(\d)E", name)
        kc, ff, ks = m.groups()
        # the per-motion loops appear in the switch order of rollout_grouped_kernel
        for pair, voted in step_loops(blocks_of(s, name)):
            row(f"rollout_grouped_kernel<{kc},ff{ff},ks{ks}>", "(a motion)", pair, voted)


def main():
    path = sys.argv[1]
    s = open(path).read()
    if len(sys.argv) > 2 and sys.argv[2] == "--table":
        return table(s)
    tag = sys.argv[2] if len(sys.argv) > 2 else "ILi2ELi1ELi6ELb0ELb1E"  # yaw-at-rest, linear, K6, no FF, KS
    name = [m for m in re.findall(r"^(_Z\S*rollout_kernel\S*):", s, re.M) if tag in m][0]
    for b in blocks_of(s, name):
        if b["loop"] or b["hdr"]:
            mark = "H" if b["hdr"] else " "
            print(f"{mark} {b['name']:14s} n={b['n']:4d} valu={b['valu']:4d} salu={b['salu']:3d} {b['br']}")


if __name__ == "__main__":
    main()
