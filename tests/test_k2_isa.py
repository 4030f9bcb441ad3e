"""K2's two-deep winner gather (rsv_k2.h, k <= 64) issues each stream's gather by inline asm and
waits for it two streams later with an explicit `s_waitcnt vmcnt(2)`.  The asm output tells the
compiler the register is ready at once, so nothing in the compiler stops it from reading, copying or
reusing that register before the wait -- which would store a wrong key without any other symptom.
This test compiles rsv_segmented.hip to gfx950 ISA (CPU only, ~10 s) and checks, for every asm
gather inside the stream loop of k2_segmented<long> and <int>, that no instruction touches its
destination registers between the gather and the loop's back edge, nor between the loop header and
the wait that covers it."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "reservoir_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _regs(text: str) -> set:
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", text):
        out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"(?<![\w\[:])v(\d+)\b", text):
        out.add(int(m.group(1)))
    return out


def _function(lines, mangled_prefix):
    start = next(i for i, l in enumerate(lines)
                 if l.startswith(mangled_prefix) and l.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def _cfg(fn):
    """Basic blocks (a label starts one, a branch ends one) with their successor blocks."""
    blocks, cur = [], []
    for i, l in enumerate(fn):
        if re.match(r"^\.LBB\d+_\d+:", l) and cur:
            blocks.append(cur)
            cur = []
        cur.append(i)
        if re.search(r"\ts_(?:cbranch_\w+|branch|endpgm)\b", l):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    label_block = {}
    for b, blk in enumerate(blocks):
        m = re.match(r"^(\.LBB\d+_\d+):", fn[blk[0]])
        if m:
            label_block[m.group(1)] = b
    succ = []
    for b, blk in enumerate(blocks):
        last = fn[blk[-1]]
        nxt = []
        m = re.search(r"\ts_(cbranch_\w+|branch) (\.LBB\d+_\d+)", last)
        if m:
            nxt.append(label_block[m.group(2)])
            if m.group(1) != "branch" and b + 1 < len(blocks):
                nxt.append(b + 1)
        elif "s_endpgm" not in last and b + 1 < len(blocks):
            nxt.append(b + 1)
        succ.append(nxt)
    return blocks, succ


def _check(fn):
    """From every asm gather, along every path of the control-flow graph until the wait that covers
    it (the second asm vmcnt(2) on the path -- the first covers the other slot's gather -- or an
    asm vmcnt(0)), no instruction may touch the gather's destination registers: no copy, spill or
    reuse of a register whose load is still in flight."""
    body = [l.split(";")[0] for l in fn]  # drop comments (the asm markers are comments)
    asm = lambda i: i > 0 and "ASMSTART" in fn[i - 1]  # noqa: E731
    gathers = [i for i, l in enumerate(fn) if "global_load_dword" in l and asm(i)]
    assert len(gathers) >= 2, "the two-deep gather's asm was not found"
    blocks, succ = _cfg(fn)
    where = {i: b for b, blk in enumerate(blocks) for i in blk}
    checked_paths = 0
    for g in gathers:
        regs = _regs(re.search(r"global_load_dword(?:x2)?\s+(v\[\d+:\d+\]|v\d+)", fn[g]).group(1))
        b0 = where[g]
        todo, seen = [(b0, blocks[b0].index(g) + 1, 0)], set()
        while todo:
            b, pos, nw = todo.pop()
            if (b, pos, nw) in seen:
                continue
            seen.add((b, pos, nw))
            covered = False
            for j in blocks[b][pos:]:
                if asm(j) and re.search(r"s_waitcnt vmcnt\(0\)", fn[j]):
                    covered = True
                    break
                if asm(j) and re.search(r"s_waitcnt vmcnt\(2\)", fn[j]):
                    nw += 1
                    if nw >= 2:
                        covered = True
                        break
                    continue
                if j == g:
                    covered = True  # back at the gather: its own registers are rewritten by it
                    break
                assert not (_regs(body[j]) & regs), (
                    f"gather into v{sorted(regs)} (line {g}) touched before its wait: {fn[j].strip()}")
            if not covered:
                checked_paths += 1
                todo.extend((s, 0, nw) for s in succ[b])
    assert checked_paths > 0


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("make") is None, reason="hipcc not available")
def test_k2_two_deep_gather_registers(tmp_path):
    out = tmp_path / "rsv_segmented.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                    os.path.join(CSRC, "rsv_segmented.hip"), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    lines = out.read_text().split("\n")
    for key in ("l", "i"):  # KeyT = int64_t, int32_t
        _check(_function(lines, f"_ZN3rsv2k212k2_segmentedI{key}EEvPKT_PKllj"))
