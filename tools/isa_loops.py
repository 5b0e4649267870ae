"""Loop anatomy of a kernel in a hipcc -S listing: for each basic-block label of the kernel, the
global loads / vmcnt waits / LDS ops / branches in order, and the VALU / SALU counts of each loop
body.  Used to check that prefetches are issued where intended (e.g. not sunk behind their wait).

usage: python tools/isa_loops.py LISTING.s KERNEL_SUBSTRING [--full]
"""
import re
import sys


def kernel_lines(path, sub):
    out, on = [], False
    for line in open(path):
        if not on and re.match(r"^_Z\S*:", line) and sub in line.split(":")[0]:
            on = True
        if on:
            out.append(line.rstrip("\n"))
            if line.startswith(".Lfunc_end"):
                break
    return out


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sub)
    if not lines:
        sys.exit(f"kernel {sub} not found")
    print(lines[0])
    events = []
    for i, l in enumerate(lines):
        s = l.strip()
        if s.startswith(".LBB") or "Loop Header" in s:
            events.append((i, s.split(";")[0] + ("  [loop header]" if "Loop Header" in s else "")))
        elif re.match(r"(global_load|buffer_load|s_waitcnt|s_cbranch|s_branch|ds_bpermute|global_store)", s):
            events.append((i, s))
    for i, s in events:
        print(f"{i:5d}  {s}")
    # loop bodies: from a header label to the last branch back to it
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):.*Loop Header", l)
        if not m:
            continue
        lab = m.group(1)
        ends = [j for j, x in enumerate(lines) if re.search(r"s_(c)?branch\w*\s+" + re.escape(lab) + r"$", x.strip())]
        if not ends:
            continue
        body = lines[i:max(ends) + 1]
        valu = sum(1 for x in body if x.strip().startswith("v_"))
        salu = sum(1 for x in body if x.strip().startswith("s_"))
        print(f"loop {lab}: lines {i}-{max(ends)}  VALU {valu}  SALU {salu}")


if __name__ == "__main__":
    main()
