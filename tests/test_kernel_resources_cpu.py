"""Register budget of the hot kernels (compile-time, no GPU): the one-launch
tower runs two waves per SIMD (256 VGPRs each), and its K loop sits at the
edge of that budget -- a change that makes the compiler spill inside the
loops halves the kernel's speed (round 3: 140 spilled VGPRs, 2911 games/s
against 5270).  hipcc's resource remarks for az_tower16.hip must show the
double-buffered kernels every config runs (128-row Connect-4, 96-row 9x9,
the chess input-row forms in 128- and 64-row tiles)
at no spilled VGPR, the in-place fallbacks at <= 8, and the 192-row in-place
tile 9x9 runs (two accumulator sets of 6 blocks) at <= 24, outside its K
loops.

Round 5's K loop is hand-scheduled assembly (az_kloop_asm.h): its loads
complete asynchronously into registers the compiler only sees as asm
operands, so test_kloop_asm_invariants reads the compiled ISA for what the
schedule relies on -- no compiler wait or spill between the groups, and no
compiler instruction touching a register a group's loads may still be
writing."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "custom-alphazero_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_tower_kernel_register_budget(tmp_path):
    out = subprocess.run(
        [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Rpass-analysis=kernel-resource-usage",
         "-c", os.path.join(CSRC, "az_tower16.hip"), "-o", str(tmp_path / "t.o")],
        capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    spills, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and name:
            spills[name] = int(m.group(1))
    # <tile blocks, wave groups, input-row form (chess), double-buffered>
    t128 = [v for k, v in spills.items() if "tower16_kernelILi8ELi2ELb0ELb1E" in k]
    t96 = [v for k, v in spills.items() if "tower16_kernelILi6ELi2ELb0ELb1E" in k]
    rows = [v for k, v in spills.items() if "tower16_kernelILi8ELi2ELb1ELb1E" in k]
    inplace = [v for k, v in spills.items() if "tower16_kernel" in k and "Lb0EEEv" in k and "ILi12E" not in k]
    t192 = [v for k, v in spills.items() if "tower16_kernelILi12ELi2ELb0ELb0E" in k]
    rows64 = [v for k, v in spills.items() if "tower16_kernelILi4ELi2ELb1ELb1E" in k]
    # round 6: Connect-4's dual launch (128- or 96-row tiles by the live count)
    dual = [v for k, v in spills.items() if "tower16_dual_kernelILi8ELi6ELb1E" in k]
    assert dual and dual[0] == 0, spills
    assert t128 and t96 and rows and rows64 and t192 and len(inplace) == 4, spills
    assert t128[0] == 0 and t96[0] == 0 and rows[0] == 0 and rows64[0] == 0, spills  # the forms every config runs
    assert max(inplace) <= 8, spills  # the in-place fallback (LDS too small for two tiles)
    assert t192[0] <= 24, spills  # test_kloop_asm_invariants: none between the K loop's groups


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_tree_kernels_do_not_spill(tmp_path):
    """the per-game tree kernels' launch bound is their block size
    (128 threads), so the allocator may use what it needs -- no spills."""
    out = subprocess.run(
        [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, "az_tree.hip"), "-o", str(tmp_path / "t.o")],
        capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    spills, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and name:
            spills[name] = int(m.group(1))
    assert any("select_group_kernel" in k for k in spills) and any("expand_kernel" in k for k in spills), spills
    assert all(v == 0 for k, v in spills.items() if "select" in k or "expand" in k or "play_kernel" in k), spills


def _regs(text):
    """VGPR numbers an instruction's operand text names (vN, v[a:b])."""
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        out.add(int(a))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_kloop_asm_invariants(tmp_path):
    s_file = tmp_path / "t.s"
    out = subprocess.run(
        [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
         os.path.join(CSRC, "az_tower16.hip"), "-o", str(s_file)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = s_file.read_text().split("\n")
    starts = [i for i, l in enumerate(lines)
              if re.match(r"^_ZN2az12_GLOBAL__N_1(14tower16_kernel|19tower16_dual_kernel)\S*:", l)]
    assert len(starts) == 10  # 9 tower16_kernel forms + Connect-4's dual launch (round 6)
    groups_seen = 0
    for st in starts:
        en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
        # basic blocks (labels .LBB*), each a list of ("asm", [code]) / ("gap", [code]) pieces, and
        # their successors: the check follows control flow, not the text order the compiler chose
        blocks, names, cur, kind, seg = [], {}, [], "gap", []
        for l in lines[st + 1:en]:
            m = re.match(r"^(\.LBB\S+):", l)
            if m:
                cur.append((kind, seg))
                blocks.append(cur)
                names[m.group(1)] = len(blocks)
                cur, kind, seg = [], "gap", []
                continue
            if ";;#ASMSTART" in l or ";;#ASMEND" in l:
                cur.append((kind, seg))
                seg, kind = [], ("asm" if ";;#ASMSTART" in l else "gap")
                continue
            code = l.split(";")[0].strip()
            if code and not code.startswith("."):
                seg.append(code)
        cur.append((kind, seg))
        blocks.append(cur)
        body = "\n".join("\n".join(x) for b in blocks for _, x in b)
        assert "scratch_" not in body or "Lb0EEEv" in lines[st], lines[st]  # spill-free product forms

        def succ(k):
            codes = [x for kd, sg in blocks[k] if kd == "gap" for x in sg]
            last = codes[-1] if codes else ""
            op = last.split()[0] if last else ""
            if op == "s_endpgm":
                return []
            if op == "s_branch":
                return [names[last.split()[1]]]
            out = [k + 1] if k + 1 < len(blocks) else []
            if op.startswith("s_cbranch"):
                out.append(names[last.split()[1]])
            return out

        def run(k, inflight, check):
            """the block's exit state from its entry state: registers the
            last group's loads may still write (None: drained / none)"""
            for kd, sg in blocks[k]:
                if kd == "asm":
                    loads = [x for x in sg if x.startswith(("ds_read", "buffer_load"))]
                    if any(x.startswith("v_mfma") for x in sg):
                        inflight = set()
                        for x in loads:
                            inflight |= _regs(x.split(",")[0])
                    elif any(x.startswith("s_waitcnt vmcnt(0) lgkmcnt(0)") for x in sg):
                        inflight = None  # the drain
                    elif loads:  # the prologue: its loads are in flight into the first group
                        inflight = set()
                        for x in loads:
                            inflight |= _regs(x.split(",")[0])
                    continue
                if inflight is None:
                    continue
                for x in sg:
                    if check:
                        # a vmcnt wait would drain the weight prefetch (lgkmcnt: the rare
                        # rescale path's own LDS reads, over-waiting the ring reads only)
                        assert not (x.startswith("s_waitcnt") and "vmcnt" in x), (lines[st][:80], x)
                        assert not x.startswith("scratch_"), (lines[st][:80], x)  # a spill inside the K loop
                        assert not (_regs(x) & inflight), (lines[st][:80], x)
            return inflight

        entry = [None] * len(blocks)  # None: not reached, or reached drained
        reached = [False] * len(blocks)
        reached[0] = True
        work = [0]
        while work:  # forward dataflow to a fixpoint (states only grow)
            k = work.pop()
            out = run(k, entry[k], False)
            for n in succ(k):
                new = entry[n] if out is None else (set(out) | (entry[n] or set()))
                if not reached[n] or new != entry[n]:
                    reached[n] = True
                    entry[n] = new
                    work.append(n)
        for k in range(len(blocks)):
            if reached[k]:
                run(k, entry[k], True)
        groups_seen += sum(1 for b in blocks for kd, sg in b if kd == "asm" and any(x.startswith("v_mfma") for x in sg))
    assert groups_seen > 0
