"""The tower's assembly K loop (csrc/gen_kloop_asm.py -> az_kloop_asm.h),
executed symbolically on the host: every variant the kernels instantiate,
run as az_tower16.hip's k_loop_asm sequences it (prologue, the projection's
group, 9 tap groups with their skip masks, drain).

The model: each register holds a label (which k-step's weight fragment, or
which tap / block / chunk / term of the activations) once its load has
landed; buffer loads and LDS reads complete in issue order per counter, and
`s_waitcnt vmcnt(N)` / `lgkmcnt(N)` retire the oldest until N are left.
Every MFMA must read landed registers holding exactly the operands its
accumulator needs at that k-step (t1*B0, t0*b1, t0*B0 per N block), every
accumulator must see each of its k-steps' 6 products once (skipped taps
none), and a load may not land in a register an earlier MFMA of the same
k-step still needed.  A wrong soffset, buffer index, ring slot or wait
count fails here instead of as a wrong forward on the GPU."""
import importlib.util
import os
import re
from collections import Counter, deque

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "custom-alphazero_amd", "csrc")
spec = importlib.util.spec_from_file_location("gen_kloop_asm", os.path.join(CSRC, "gen_kloop_asm.py"))
gen = importlib.util.module_from_spec(spec)
spec.loader.exec_module(gen)
KSTEP = gen.KSTEP
# (B fragment q, A term t) of the six MFMAs of one block and k-step, by N block n:
# n = 0 reads fragments 0 (B0) and 1 (b1), n = 1 fragments 2 and 3
NEEDED = Counter({(0, 1, 0): 1, (1, 0, 0): 1, (0, 0, 0): 1, (2, 1, 1): 1, (3, 0, 1): 1, (2, 0, 1): 1})


class Machine:
    def __init__(self, MBW):
        self.MBW = MBW
        self.reg = {}  # operand name -> label (landed)
        self.vm = deque()  # pending (reg, label)
        self.lgkm = deque()
        self.acc = {}  # (block, n) -> Counter of (kstep, q, t)
        self.seq = {}  # (block, n) -> the (kstep, q, t) sequence in issue order
        self.log = []

    def land(self, q, keep):
        while len(q) > keep:
            r, lab = q.popleft()
            self.reg[r] = lab

    def run(self, text, ctx):
        """ctx: sc/sn k-step bases ('R' or 'M', index), d/n A sources, skip mask."""
        tmp = None
        kstep = None
        for line in text.split("\\n\\t"):
            line = line.strip()
            m = re.match(r"; k-step chunk (\d)", line)
            if m:
                c = int(m.group(1))
                kstep = (ctx["sc"][0], ctx["sc"][1] + c)
                chunk = c
                continue
            ops = re.findall(r"%\[(\w+)\]", line)
            if line.startswith("s_add_u32"):
                base = ctx[ops[1]]
                tmp = (base[0], base[1] + int(line.rsplit(",", 1)[1]) // KSTEP)
            elif line.startswith("buffer_load_dwordx4"):
                dst, _, rsrc, soff = ops
                base = tmp if soff == "tmp" else ctx[soff]
                assert ctx[rsrc] == base[0], line  # the descriptor of the pack the k-step lives in
                off = int(line.rsplit("offset:", 1)[1])
                lab = ("B", base[0], base[1], off // 1024)
                self.pending_write(dst)
                self.vm.append((dst, lab))
            elif line.startswith("ds_read_b128"):
                dst, src = ops
                off = int(line.rsplit("offset:", 1)[1])
                blk = int(src[1:])
                lab = ("A", ctx[src[0]], blk, (off % 256) // 64, off // 256)
                self.pending_write(dst)
                self.lgkm.append((dst, lab))
            elif line.startswith("s_waitcnt"):
                m = re.search(r"vmcnt\((\d+)\)", line)
                if m:
                    self.land(self.vm, int(m.group(1)))
                m = re.search(r"lgkmcnt\((\d+)\)", line)
                if m:
                    self.land(self.lgkm, int(m.group(1)))
            elif line.startswith("v_mfma"):
                cdst, b, a, csrc = ops
                assert cdst == csrc, line
                blk, n = int(cdst[1]), int(cdst[3])
                for r in (b, a):
                    assert r in self.reg and not any(p[0] == r for p in self.vm) and \
                        not any(p[0] == r for p in self.lgkm), (line, r, "read before its load landed")
                bl, al = self.reg[b], self.reg[a]
                assert bl[0] == "B" and (bl[1], bl[2]) == kstep, (line, bl, kstep)
                assert al[0] == "A" and al[1] == ctx["d"] and al[2] == blk and al[3] == chunk, (line, al, ctx["d"], chunk)
                assert not (ctx["skip"] >> blk) & 1, (line, "skipped block computed")
                self.acc.setdefault((ctx["acc"], blk, n), Counter())[(kstep, bl[3], al[4], n)] += 1
                self.seq.setdefault((ctx["acc"], blk, n), []).append((kstep, bl[3], al[4]))
            elif line.startswith("s_nop") or line.startswith(";") or not line:
                pass
            else:
                raise AssertionError(f"unmodelled instruction {line!r}")

    def pending_write(self, dst):
        # the in-order model: a register with an older load still pending
        # would take two writes in flight -- never generated
        assert not any(p[0] == dst for p in self.vm) and not any(p[0] == dst for p in self.lgkm), dst


ORDER = {0: [(0, 1), (1, 0), (0, 0)], 1: [(2, 1), (3, 0), (2, 0)]}  # per N block: t1*B0, t0*b1, t0*B0


def run_loop(MBW, C0, PF, R, skw, ORD=0, LAST_HN=1):
    m = Machine(MBW)
    group = gen.term_group_asm if ORD else gen.group_asm

    def grp(MBW, C0, skc, PF, hn, tp):  # tp: the tap's parity (the residual steps precede tap 0: 1)
        return group(MBW, C0, skc, PF, hn, TP=tp)
    prologue = gen.term_prologue_asm if ORD else gen.prologue_asm
    # prologue: A from the phase's first source, B from its first k-step
    first_src = ("own",) if R else ("tap", 0)
    first_k = ("R", 0) if R else ("M", C0)
    m.run(prologue(MBW, C0, PF, 1 if R else 0), {"sc": first_k, "d": first_src, "skip": 0, "acc": "-",
                                          "rc": first_k[0]})
    if R:
        m.run(grp(MBW, 0, 0, PF, 1, 1), {"sc": ("R", 0), "sn": ("M", 0), "d": ("own",), "n": ("tap", 0),
                                             "skip": 0, "acc": "res", "rc": "R", "rn": "M"})
    for t in range(9):
        mask = (skw >> (2 * t)) & 3
        skc = mask if MBW > 1 else 0
        # the last tap (HN = 1, as k_loop_asm runs it) prefetches its own first
        # k-steps again, the drain waits for them; HN = 0: nothing in flight after it
        nxt = ("tap", t + 1) if t < 8 else ("tap", 8)
        sn = ("M", 4 * (t + 1) + C0) if t < 8 else ("M", 4 * t + C0)
        hn = 1 if t < 8 else LAST_HN
        m.run(grp(MBW, C0, skc, PF, hn, t & 1), {"sc": ("M", 4 * t), "sn": sn, "d": ("tap", t), "n": nxt,
                                             "skip": skc, "acc": "main", "rc": "M", "rn": "M"})
    if LAST_HN == 0:
        assert not m.vm and not m.lgkm, (m.vm, m.lgkm)
    m.land(m.vm, 0)
    m.land(m.lgkm, 0)
    # every accumulator: each k-step's six products exactly once, skipped taps none
    for blk in range(MBW):
        for n in range(2):
            got = m.acc.get(("main", blk, n), Counter())
            want = Counter()
            for t in range(9):
                mask = (skw >> (2 * t)) & 3 if MBW > 1 else 0
                if (mask >> blk) & 1:
                    continue
                for c in range(C0, 4):
                    for (q, tt, nn), k in NEEDED.items():
                        if nn == n:
                            want[(("M", 4 * t + c), q, tt, n)] += k
            assert got == want, (MBW, C0, PF, R, blk, n)
            # the sum order each accumulator must keep (bitwise the compiled loop's)
            seq = m.seq.get(("main", blk, n), [])
            assert [x[1:] for x in seq] == ORDER[n] * (len(seq) // 3), (MBW, C0, PF, R, ORD, blk, n)
            assert [x[0] for x in seq] == sorted(x[0] for x in seq), (MBW, C0, PF, R, ORD, blk, n)
            if R:
                got = m.acc.get(("res", blk, n), Counter())
                want = Counter({(("R", c), q, tt, n): k for c in range(4) for (q, tt, nn), k in NEEDED.items()
                                if nn == n})
                assert got == want, (MBW, C0, PF, R, blk, n, "residual")
                seq = m.seq[("res", blk, n)]
                assert [x[1:] for x in seq] == ORDER[n] * 4 and [x[0] for x in seq] == sorted(x[0] for x in seq)


# the kernels' forms: (blocks per wave, first chunk, prefetch depth, residual steps)
FORMS = [(4, 0, 2, 0), (4, 0, 2, 4), (3, 0, 2, 0), (3, 0, 2, 4), (1, 0, 2, 0), (1, 0, 2, 4), (1, 2, 1, 0),
         (4, 2, 1, 0), (6, 0, 1, 0), (6, 0, 1, 4), (2, 0, 2, 0), (2, 0, 2, 4), (4, 0, 1, 4), (1, 0, 1, 0),
         (2, 0, 3, 0), (2, 0, 3, 4), (1, 0, 3, 0), (2, 2, 1, 0)]
# skip words: none, a slot plan's (two border blocks, 3 taps each), every tap skipping one block
SKIPS = [0, sum(1 << (2 * t) for t in (0, 1, 2)) | sum(2 << (2 * t) for t in (6, 7, 8)),
         sum((1 + (t & 1)) << (2 * t) for t in range(9))]


@pytest.mark.parametrize("MBW,C0,PF,R", FORMS)
@pytest.mark.parametrize("skw", SKIPS)
@pytest.mark.parametrize("ORD", [0, 1])
@pytest.mark.parametrize("LAST_HN", [1, 0])
def test_kloop_schedule_is_exact(MBW, C0, PF, R, skw, ORD, LAST_HN):
    if C0 and R:
        pytest.skip("the stem has no residual steps")
    run_loop(MBW, C0, PF, R, skw if MBW > 1 else 0, ORD, LAST_HN)
