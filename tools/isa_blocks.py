"""Per-basic-block instruction counts of one kernel in an hipcc -S listing (development aid).

  python3 tools/isa_blocks.py reservoir_amd/csrc/_obj/rsv_segmented.s k2_segmented [--show LABEL]

Prints, for every label of the kernel: VALU (v_*), SALU (s_*), LDS (ds_*), VMEM (global_/buffer_),
the branch that ends the block, and the loop back-edges (a branch to an earlier label).
"""
import re
import sys


def blocks(path, name):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l) or re.match(r"^" + re.escape(name) + r":", l):
            start = i
            break
    if start is None:
        raise SystemExit(f"kernel {name} not found")
    out, cur = [], {"label": lines[start].rstrip(":"), "ins": []}
    for l in lines[start + 1:]:
        if l.startswith("\t.section") or l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            out.append(cur)
            cur = {"label": m.group(1), "ins": []}
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur["ins"].append(s)
    out.append(cur)
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    show = sys.argv[sys.argv.index("--show") + 1] if "--show" in sys.argv else None
    bs = blocks(path, name)
    order = {b["label"]: i for i, b in enumerate(bs)}
    for i, b in enumerate(bs):
        ins = b["ins"]
        v = sum(1 for x in ins if x.startswith("v_"))
        s = sum(1 for x in ins if x.startswith("s_") and not x.startswith("s_waitcnt") and not x.startswith("s_nop"))
        nop = sum(1 for x in ins if x.startswith("s_nop"))
        ds = sum(1 for x in ins if x.startswith("ds_"))
        vm = sum(1 for x in ins if x.startswith("global_") or x.startswith("buffer_"))
        br = [x for x in ins if x.startswith("s_branch") or x.startswith("s_cbranch")]
        back = [x for x in br if x.split()[-1] in order and order[x.split()[-1]] <= i]
        print(f"{b['label']:>12} v={v:4d} s={s:3d} nop={nop:2d} ds={ds:2d} vm={vm:2d}  "
              f"{' '.join(x.split()[0] + ' ' + x.split()[-1] for x in br)}{'  <-- LOOP' if back else ''}")
        if show and b["label"] == show:
            print("\n".join("      " + x for x in ins))


if __name__ == "__main__":
    main()
