"""Wait states between each MFMA and the first other instruction that touches
its result registers, over every control-flow path of a kernel in a
``hipcc --cuda-device-only -S`` listing (compile-time audit).

    python tools/mfma_hazard.py listing.s [NAME_SUBSTRING] [--min 12]

For every ``v_mfma*`` it walks the basic blocks forward (branch targets and
fall-through, loops included) and counts the issue slots until an
instruction reads or writes any VGPR of the MFMA's destination, except a
following MFMA that takes the same range whole as its accumulator (an
accumulate chain, interlocked by the hardware).  ``s_nop N`` counts N + 1
states, every other instruction one.  It prints the shortest such distance
per MFMA and the instruction reached; a distance below ``--min`` (the 8-pass
XDL requirement of 12 states for D -> VALU / VMEM / LDS access) is flagged.
"""

from __future__ import annotations

import argparse
import json
import re
import sys
from collections import deque

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text: str):
    """VGPRs and AGPRs named in an instruction: {("v", 3), ("a", 17), ...}."""
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update((m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def parse(path: str, want: str):
    s = open(path).read()
    starts = [m for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M) if want in m.group(1)]
    if not starts:
        sys.exit(f"no kernel matching {want}")
    m = starts[0]
    body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
    blocks, order, cur = {}, [], "entry"
    blocks[cur] = []
    order.append(cur)
    for ln in body:
        mm = re.match(r"^(\.LBB\S+):", ln) or re.match(r"^; %(bb\.\d+):", ln)
        if mm:
            cur = mm.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        t = ln.split(";")[0].strip()
        if not t or t.startswith("."):
            continue
        blocks[cur].append(t)
    succ = {}
    for i, b in enumerate(order):
        ins = blocks[b]
        nxt = order[i + 1] if i + 1 < len(order) else None
        out = []
        last = ins[-1] if ins else ""
        for t in ins:
            if t.startswith("s_cbranch") or t.startswith("s_branch"):
                out.append(t.split()[-1])
        if not last.startswith("s_branch") and not last.startswith("s_endpgm") and nxt:
            out.append(nxt)
        succ[b] = out
    return m.group(1), order, blocks, succ


def states(t: str) -> int:
    if t.startswith("s_nop"):
        return int(t.split()[1], 0) + 1
    return 1


def distance(blocks, succ, b, i, stop_at_barrier: bool):
    """Shortest issue-slot distance from MFMA (b, i) to the first instruction
    touching its destination; with stop_at_barrier, paths through an
    s_barrier are not followed (None: every path crosses one)."""
    t = blocks[b][i]
    dtxt = t.split(None, 1)[1].split(",")[0].strip()
    dst = regs(dtxt)
    best = None
    seen = {}
    q = deque([(b, i + 1, 0)])
    while q:
        blk, j, n = q.popleft()
        ins = blocks[blk]
        hit = False
        while j < len(ins):
            u = ins[j]
            if stop_at_barrier and "s_barrier" in u:
                hit = True
                break
            if u.startswith("v_mfma"):
                uo = [x.strip() for x in u.split(None, 1)[1].split(",")]
                if uo[0] == dtxt and uo[-1] == dtxt:  # accumulate chain
                    hit = True
                    break
            if regs(u) & dst:
                if best is None or n < best[0]:
                    best = (n, blk, u)
                hit = True
                break
            n += states(u)
            j += 1
        if hit:
            continue
        for s2 in succ.get(blk, []):
            if s2 in blocks and (s2 not in seen or seen[s2] > n):
                seen[s2] = n
                q.append((s2, 0, n))
    return dtxt, best


def kernels(path: str):
    s = open(path).read()
    return [m.group(1) for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M)
            if "v_mfma" in s[m.end():s.find(".Lfunc_end", m.end())]]


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("listing")
    p.add_argument("kernel", nargs="?", default="",
                   help="name substring; omitted: one summary line per MFMA kernel")
    p.add_argument("--min", type=int, default=12)
    a = p.parse_args()
    names = kernels(a.listing) if not a.kernel else [a.kernel]
    for want in names:
        name, order, blocks, succ = parse(a.listing, want)
        worst, worst_free, nm = None, None, 0
        for b in order:
            for i, t in enumerate(blocks[b]):
                if not t.startswith("v_mfma"):
                    continue
                nm += 1
                dtxt, best = distance(blocks, succ, b, i, False)
                _, free = distance(blocks, succ, b, i, True)
                if best is None:
                    continue
                if a.kernel:
                    flag = "  <-- below %d" % a.min if best[0] < a.min else ""
                    fr = "barrier on every path" if free is None else f"{free[0]} without a barrier"
                    print(f"{b}:{i} {dtxt:10s} {best[0]:4d} states ({fr}) -> {best[1]}: "
                          f"{best[2][:60]}{flag}")
                if worst is None or best[0] < worst[0]:
                    worst = best
                if free is not None and (worst_free is None or free[0] < worst_free[0]):
                    worst_free = free
        if worst is None:
            continue
        print(json.dumps({"kernel": name, "mfma": nm, "min_states": worst[0],
                          "min_states_no_barrier": None if worst_free is None else worst_free[0],
                          "first_reader": worst[2][:60], "ok": worst[0] >= a.min}))


if __name__ == "__main__":
    main()
