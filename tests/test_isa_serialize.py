"""ISA check of the serialisers' hand-counted wait.

`serialize_run` (csrc/dg_serialize_wave.h) loads the next tile's records into
registers by inline asm, and the member serialiser's pipeline (and the A/B
`serialize_pipe`) load what a later tile needs by LDS-DMA into rings; each
trusts one `s_waitcnt vmcnt(N)` before the loaded words are used.  VMEM operations complete in
issue order, so that wait covers the DMAs only if at least N VMEM operations
were issued after them on every path (or an earlier wait already covered
them).  A compiler change that merges, splits or adds a VMEM operation there
would make the records silently wrong; and nothing may read or write a
register load's destination before the wait covers it.

This test disassembles the built gfx950 code object (CPU only, no GPU), finds
the asm markers (`s_nop 7; s_nop 6` after the DMAs, `s_nop 7; s_nop 4` after
register loads, `s_nop 7; s_nop 5` before each counted wait), builds the control-flow graph of `serialize_wave_kernel`
and `member_serialize_kernel` and walks every path from each DMA group.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("DG_ISA_LIB") or os.path.join(ROOT, "delta-compression_amd", "lib", "libdeltagpu.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

KERNELS = ("serialize_wave_kernel", "member_serialize_kernel")
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<[^>+]+\+0x([0-9a-f]+)>")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def _gfx950_disasm(tmp):
    """Disassembly of the library's gfx950 code objects (one per source)."""
    so = os.path.join(tmp, "lib.so")
    shutil.copy(LIB, so)
    subprocess.run([OBJDUMP, "--offloading", so], cwd=tmp, check=True, capture_output=True)
    text = []
    for f in sorted(os.listdir(tmp)):
        if "gfx950" in f:
            r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", os.path.join(tmp, f)], check=True,
                               capture_output=True, text=True)
            text.append(r.stdout)
    return "\n".join(text)


def _kernel(disasm, name):
    """[(addr, mnemonic, operands)] of the kernel whose mangled name holds `name`."""
    out, on, base = [], False, 0
    for line in disasm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            on = name in m.group(2)
            base = int(m.group(1), 16)
            continue
        if not on:
            continue
        if not line.strip():
            if out:
                break
            continue
        m = INSN.match(line)
        if m:
            out.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return out, base


def _regs(ops):
    r = set()
    for m in VREG.finditer(ops):
        if m.group(1) is not None:
            r.add(int(m.group(1)))
        else:
            r.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return r


def _check_kernel(ins, base, raw_lines):
    # branch targets from the raw lines (the trailing comment carries them)
    target = {}
    for addr, line in raw_lines:
        m = TARGET.search(line)
        if m and ("s_branch" in line or "s_cbranch" in line):
            target[addr] = base + int(m.group(1), 16)
    addr_ix = {a: k for k, (a, _, _) in enumerate(ins)}

    def succ(i):
        a, mn, _ = ins[i]
        if mn == "s_endpgm":
            return []
        if mn.startswith("s_setpc") or mn.startswith("s_swappc"):
            raise AssertionError(f"indirect branch at {a:#x}")
        fall = [i + 1] if i + 1 < len(ins) else []
        if mn == "s_branch":
            return [addr_ix[target[a]]]
        if mn.startswith("s_cbranch"):
            return fall + [addr_ix[target[a]]]
        return fall

    groups = []   # (index after the marker, destination registers: none for LDS-DMA)
    for i in range(1, len(ins) - 1):
        if not (ins[i][1] == "s_nop" and ins[i][2].startswith("7") and ins[i + 1][1] == "s_nop"):
            continue
        if ins[i + 1][2].startswith("6"):     # LDS-DMA group (serialize_pipe, member pipeline)
            assert any(ins[i - k][1].startswith("global_load_lds") for k in range(1, 6) if i - k >= 0), \
                f"{ins[i][0]:#x}: DMA marker without a DMA before it"
            groups.append((i + 2, set()))
        elif ins[i + 1][2].startswith("4"):   # register loads (serialize_run's rec_load4)
            loads = ins[i - 4:i]
            assert all(mn == "global_load_dword" for _, mn, _ in loads), \
                f"{ins[i][0]:#x}: load marker without the four record loads before it"
            dst = set()
            for _, _, ops in loads:
                dst |= _regs(ops.split(",")[0])
            groups.append((i + 2, dst))
    waits = {i + 2 for i in range(len(ins) - 2)
             if ins[i][1] == "s_nop" and ins[i][2].startswith("7") and ins[i + 1][1] == "s_nop"
             and ins[i + 1][2].startswith("5") and ins[i + 2][1] == "s_waitcnt"}
    assert groups, "DMA marker not found"
    assert waits, "wait marker not found"
    checked = 0
    for start, dst in groups:
        assert len(dst) in (0, 4), dst
        # states: (instruction index, VMEM ops issued since the loads (capped),
        # known wave-uniform flags).  The compiler joins if/else arms through
        # a flag SGPR pair (s_mov_b64 s[a:b], -1 / 0 ... s_and_b64 vcc, exec,
        # s[a:b]; s_cbranch_vccz): tracking those constants keeps the walk to
        # the paths the code can take.
        seen, stack, reached = set(), [(start, 0, frozenset())], 0
        while stack:
            i, n, known = stack.pop()
            if (i, n, known) in seen:
                continue
            seen.add((i, n, known))
            a, mn, ops = ins[i]
            kd = dict(known)
            if mn == "s_waitcnt" and "vmcnt" in ops:
                k = int(re.search(r"vmcnt\((\d+)\)", ops).group(1))
                if i in waits:
                    reached += 1
                    assert k <= n, (f"{a:#x}: vmcnt({k}) with only {n} VMEM operations issued after the "
                                    f"record loads on some path: the records may not have landed")
                if k <= n:
                    continue          # the loads have landed on this path
            elif _regs(ops) & dst:
                raise AssertionError(f"{a:#x}: {mn} {ops} touches the record registers {sorted(dst)} "
                                     f"before the wait covers their loads")
            if VMEM.match(mn):
                n = min(n + 1, 64)
            first = ops.split(",")[0].strip() if ops else ""
            nexts = succ(i)
            # exec: full in the uniform code the walk starts in; a wave whose
            # exec may be empty is one inside a divergent region
            if first == "exec" and not mn.startswith("s_cbranch"):
                if mn.startswith("s_or_b64") and "exec, exec" in ops:
                    kd.pop("exec_low", None)              # the region's mask restored
                elif not (mn == "s_mov_b64" and ops.split(",")[1].strip() == "-1"):
                    kd["exec_low"] = 1
            elif mn.endswith("saveexec_b64"):
                kd["exec_low"] = 1
            if mn in ("s_cbranch_execz", "s_cbranch_execnz") and "exec_low" not in kd:
                nexts = [nexts[0]] if mn == "s_cbranch_execz" else [nexts[1]]
            elif mn in ("s_cbranch_vccz", "s_cbranch_vccnz") and "vcc" in kd:
                taken = (kd["vcc"] == 0) == (mn == "s_cbranch_vccz")
                nexts = [nexts[1]] if taken else [nexts[0]]
            elif mn == "s_mov_b64" and re.fullmatch(r"s\[\d+:\d+\]", first) and ops.split(",")[1].strip() in ("0", "-1"):
                kd[first] = int(ops.split(",")[1])
            elif mn == "s_and_b64" and first == "vcc" and "exec" in ops:
                other = [x.strip() for x in ops.split(",")[1:] if x.strip() != "exec"]
                if len(other) == 1 and other[0] in kd:
                    kd["vcc"] = kd[other[0]]   # exec is never empty here (uniform flag)
                else:
                    kd.pop("vcc", None)
            elif first and not mn.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_cmp")):
                # any other write of a tracked register forgets it
                for key in list(kd):
                    if key == first or (key != "vcc" and first.startswith("s[") and key == first):
                        kd.pop(key)
                if first == "vcc" or first.startswith("vcc"):
                    kd.pop("vcc", None)
                if first.startswith("s"):
                    m = re.fullmatch(r"s(\d+)|s\[(\d+):(\d+)\]", first)
                    if m:
                        lo = int(m.group(1) or m.group(2))
                        hi = int(m.group(1) or m.group(3))
                        for key in list(kd):
                            km = re.fullmatch(r"s\[(\d+):(\d+)\]", key)
                            if km and int(km.group(1)) <= hi and lo <= int(km.group(2)):
                                kd.pop(key)
            nk = frozenset(kd.items())
            for j in nexts:
                stack.append((j, n, nk))
        assert reached, "no path from the record loads reaches the wait"
        checked += 1
    return checked


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(OBJDUMP), reason="library or llvm-objdump missing")
@pytest.mark.parametrize("kernel", KERNELS)
def test_serialiser_record_wait_is_counted(kernel):
    with tempfile.TemporaryDirectory() as tmp:
        dis = _gfx950_disasm(tmp)
    ins, base = _kernel(dis, kernel)
    assert ins, f"{kernel} not found in the code object"
    raw = []
    on = False
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            on = kernel in m.group(2)
            continue
        if on:
            m = INSN.match(line)
            if m:
                raw.append((int(m.group(3), 16), line))
            elif not line.strip() and raw:
                break
    assert _check_kernel(ins, base, raw) >= 1


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(OBJDUMP), reason="library or llvm-objdump missing")
def test_checker_rejects_a_short_count_and_a_missing_store():
    """The checker itself: the same instructions with the counted wait raised
    by one, or with one of the tile's stores gone, fail."""
    kernel = "serialize_wave_kernel"
    with tempfile.TemporaryDirectory() as tmp:
        dis = _gfx950_disasm(tmp)
    ins, base = _kernel(dis, kernel)
    raw, on = [], False
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            on = kernel in m.group(2)
            continue
        if on:
            m = INSN.match(line)
            if m:
                raw.append((int(m.group(3), 16), line))
            elif not line.strip() and raw:
                break
    assert _check_kernel(ins, base, raw) >= 1
    # (a) the counted wait one higher than the stores behind the DMAs
    w = next(i + 2 for i in range(len(ins) - 2) if ins[i][1] == "s_nop" and ins[i][2].startswith("7")
             and ins[i + 1][1] == "s_nop" and ins[i + 1][2].startswith("5")
             and re.search(r"vmcnt\(([1-9]\d*)\)", ins[i + 2][2]))
    k = int(re.search(r"vmcnt\((\d+)\)", ins[w][2]).group(1))
    bad = list(ins)
    bad[w] = (ins[w][0], "s_waitcnt", f"vmcnt({k + 1})")
    with pytest.raises(AssertionError, match="may not have landed"):
        _check_kernel(bad, base, raw)
    # (b) one buffer store of the staged flush (the last one before the wait) gone
    j = max(i for i in range(w) if ins[i][1].startswith("buffer_store"))
    bad = list(ins)
    bad[j] = (ins[j][0], "s_nop", "0")
    with pytest.raises(AssertionError, match="may not have landed"):
        _check_kernel(bad, base, raw)


