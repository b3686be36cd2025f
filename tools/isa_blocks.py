"""Per-basic-block instruction counts of one kernel in a hipcc -S listing
(compile-time aid): scratch (spill) ops, MFMAs, LDS reads/writes, global/buffer
loads, waits, barriers; blocks that end in a backward branch are loops.

    python tools/isa_blocks.py listing.s NAME_SUBSTRING
"""
import re
import sys


def main(path, want):
    s = open(path).read()
    starts = [m for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M)]
    for i, m in enumerate(starts):
        name = m.group(1)
        if want not in name:
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end].split("\n")
        order, stats, pos, branches = [], {}, {}, {}
        blk = "entry"
        order.append(blk)
        stats[blk] = dict(scr=0, mfma=0, dsr=0, dsw=0, vmem=0, wait=0, bar=0, n=0)
        for ln in body:
            mm = re.match(r"(\.LBB\S+):", ln)
            if mm:
                blk = mm.group(1)
                order.append(blk)
                pos[blk] = len(order) - 1
                stats[blk] = dict(scr=0, mfma=0, dsr=0, dsw=0, vmem=0, wait=0, bar=0, n=0)
                continue
            t = ln.strip()
            if not t or t.startswith(";") or t.startswith("."):
                continue
            st = stats[blk]
            st["n"] += 1
            if t.startswith("scratch_") or re.match(r"buffer_(store|load)_dword\S* v\d+, off, s\[0:3\]", t):
                st["scr"] += 1
            elif "v_mfma" in t:
                st["mfma"] += 1
            elif t.startswith("ds_read") or t.startswith("ds_load"):
                st["dsr"] += 1
            elif t.startswith("ds_write") or t.startswith("ds_store"):
                st["dsw"] += 1
            elif t.startswith("buffer_load") or t.startswith("global_load"):
                st["vmem"] += 1
            elif t.startswith("s_waitcnt"):
                st["wait"] += 1
            elif t.startswith("s_barrier"):
                st["bar"] += 1
            mb = re.match(r"s_cbranch_\S+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", t)
            if mb:
                branches.setdefault(blk, []).append(mb.group(1) or mb.group(2))
        print(name)
        for b in order:
            back = [t for t in branches.get(b, []) if t in pos and pos[t] <= order.index(b)]
            st = stats[b]
            flag = " LOOP->" + ",".join(back) if back else ""
            print(f"  {b:14s} n={st['n']:5d} scr={st['scr']:3d} mfma={st['mfma']:3d} dsr={st['dsr']:3d} "
                  f"dsw={st['dsw']:3d} vmem={st['vmem']:3d} wait={st['wait']:3d} bar={st['bar']}{flag}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
