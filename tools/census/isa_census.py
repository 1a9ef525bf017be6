"""Static ISA census of one kernel in a hipcc -S output: VALU / SALU / LDS / VMEM counts per
basic block and per loop (a block range closed by a backward branch), and an opcode histogram
of the hottest loop.  Compile-only (no GPU).
  python tools/census/isa_census.py /tmp/fks_dev.s SYMBOL_SUBSTRING [--top N]"""
import collections
import re
import sys


def kernel_lines(path, sym):
    out, on = [], False
    for ln in open(path):
        if not on and ln.startswith("_Z") and sym in ln.split(":")[0] and ln.rstrip().endswith(sym_end(ln)):
            on = True
        if on:
            out.append(ln.rstrip("\n"))
            if "s_endpgm" in ln:
                break
    return out


def sym_end(ln):
    return ln.split(";")[0].strip()[-1:]


def blocks(lines):
    cur, name = [], "entry"
    res = []
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            res.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append(s.split(";")[0].strip())
    res.append((name, cur))
    return res


def cls(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    lines = []
    on = False
    for ln in open(path):
        if not on and re.match(r"^_Z\S*" + re.escape(sym) + r"\S*:", ln):
            on = True
        if on:
            lines.append(ln.rstrip("\n"))
            if "s_endpgm" in ln:
                break
    bl = blocks(lines)
    index = {n: i for i, (n, _) in enumerate(bl)}
    loops = []
    for i, (n, ins) in enumerate(bl):
        for s in ins:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", s)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in index and index[tgt] <= i:
                    loops.append((index[tgt], i))
    print(f"kernel lines {len(lines)}, blocks {len(bl)}")
    for lo, hi in sorted(set(loops)):
        c = collections.Counter()
        for n, ins in bl[lo:hi + 1]:
            for s in ins:
                c[cls(s.split()[0])] += 1
        print(f"loop {bl[lo][0]}..{bl[hi][0]} ({hi - lo + 1} blocks): " + ", ".join(f"{k} {v}" for k, v in sorted(c.items())))
    if loops:
        lo, hi = max(set(loops), key=lambda r: sum(len(bl[j][1]) for j in range(r[0], r[1] + 1)))
        h = collections.Counter()
        for n, ins in bl[lo:hi + 1]:
            for s in ins:
                op = s.split()[0]
                if op.startswith("v_") or op.startswith("ds_"):
                    h[op] += 1
        print(f"hottest loop {bl[lo][0]}..{bl[hi][0]}: opcode histogram")
        for op, n in h.most_common(top):
            print(f"  {n:6d} {op}")


if __name__ == "__main__":
    main()
