"""Condensed instruction sequence of one basic block of a kernel in a hipcc -S
listing (compile-time aid): runs of the same kind collapse to KIND*count.

    python tools/isa_seq.py listing.s NAME_SUBSTRING BLOCK_LABEL
"""
import re
import sys


def kind(t):
    for k, p in (("MFMA", "v_mfma"), ("DSR", "ds_read"), ("DSW", "ds_write"), ("VMEM", "buffer_load"),
                 ("VMEM", "global_load"), ("BAR", "s_barrier"), ("ST", "buffer_store"),
                 ("ST", "global_store"), ("ATOM", "atomic"), ("SCR", "scratch_")):
        if p in t:
            return k
    if t.startswith("s_waitcnt"):
        return "W(" + t.split(None, 1)[1] + ")"
    if t.startswith("v_"):
        return "V"
    if t.startswith("s_"):
        return "S"
    return "?"


def main(path, want, label):
    s = open(path).read()
    m = [m for m in re.finditer(r"^(_Z\S+):\s*;\s*@", s, re.M) if want in m.group(1)][0]
    body = s[m.end():s.find(".Lfunc_end", m.end())]
    i = body.find("\n" + label + ":")
    blk = body[i + 1:].split("\n")[1:]
    out, prev, cnt = [], None, 0
    for ln in blk:
        t = ln.strip()
        if re.match(r"\.LBB\S+:", t):
            break
        if not t or t.startswith(";") or t.startswith("."):
            continue
        k = kind(t)
        if k == prev:
            cnt += 1
        else:
            if prev:
                out.append(prev + ("*%d" % cnt if cnt > 1 else ""))
            prev, cnt = k, 1
    out.append(prev + ("*%d" % cnt if cnt > 1 else ""))
    print(" ".join(out))


if __name__ == "__main__":
    main(*sys.argv[1:4])
