"""Generate az_kloop_asm.h: the tower's K loop as hand-scheduled gfx950
assembly, one inline-asm statement per group of k-steps (a tap's 4 input
channel chunks, or the block's 4 residual k-steps).

Why: compiled from HIP, the K loop (az_tower16.hip k_loop) kept its fp32
accumulators in VGPRs and rotated them through the MFMA destinations (an
MFMA's result written over a dead A operand, copies on every loop
back-edge, s_nop pads for the write-after-read hazards that rotation
creates), and the register allocator needed all 256 VGPRs for ~130 live
values.  Here the accumulators, the A (activation) ring and the B
(weight) double buffer are "+v" operands of one asm statement per group,
so every MFMA accumulates in place (dst = srcC) and nothing is copied
between groups; every LDS read and weight load sits where the schedule
wants it with an exact s_waitcnt before the MFMAs that need it.  (AGPR
accumulators were tried first: any AGPR use makes the compiler split the
unified register file 128/128, and the 128 VGPRs left spilled into AGPRs
around every group.)

The arithmetic is the compiled loop's, MFMA for MFMA: per accumulator the
k-steps in order and per k-step t1*B0, t0*b1, t0*B0 (the two N blocks'
chains interleaved, which does not change any sum), so outputs are bitwise
those of the HIP loop.

Schedule per k-step (chunk c of a tap; the LAG ring of az_tower16.hip):
  * the next k-step's 4 weight fragments by buffer_load (PF = 1);
  * per M block mb: its 6 MFMAs, then one ring read -- after block 0 the
    last block's fragments of THIS chunk (lagged), after block mb >= 1
    block mb-1's fragments of the next chunk (or of the next tap's first
    chunk at ad_next) -- so no read overwrites registers an MFMA issued
    fewer than 6 MFMAs earlier reads (an s_nop 4 where a skipped block
    leaves no MFMA in between);
  * s_waitcnt vmcnt / lgkmcnt counted from the issue order (reads of the
    previous group's tail included).
Run: python gen_kloop_asm.py  (writes az_kloop_asm.h beside it)
"""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "az_kloop_asm.h")
KSTEP = 16384  # bytes of one k-step's packed B fragments (az_tower16.hip load_bk)


def nbufs(PF):
    """B buffers for a prefetch depth: k-step j of tap t lives in buffer
    (4 (t mod 2) + j) mod NB -- so with 8 (PF 3-4) a group's buffers depend on
    its tap's parity TP and the kernels dispatch on it."""
    return 2 if PF == 1 else 4 if PF == 2 else 8


def group_asm(MBW, C0, SKC, PF=1, HASNEXT=1, LAGFIRST=0, LAST_NOP=1, TP=0):
    """Assembly text of one group (chunks C0..3) and its operand names.
    Operands (names used in the text):
      %[aK_T]   ring slot K (block), term T (0: t0, 1: t1)   "+v" az_u4
      %[bJ_Q]   B buffer J (k-step parity), fragment Q      "+v" az_u4
      %[dK]     this group's LDS byte address of block K    "v"
      %[nK]     the next group's address of block K (K < MBW-1)  "v"
      %[voff]   lane offset into the packed fragments       "v"
      %[rc] %[rn]  buffer descriptors of this / the next group  "s" (x4)
      %[sc] %[sn]  soffset of this group's chunk-0 k-step / the next group's first  "s"
      %[tmp]    scratch SGPR                                "=&s"
      %[cK_N]   accumulator of block K, N block N           "+v" az_f4
    """
    lines = []
    emit = lines.append
    chunks = list(range(C0, 4))
    skipped = lambda mb: (SKC >> mb) & 1  # noqa: E731
    # read issue order (block, chunk, where) for lgkmcnt: a read is 2 ds_read_b128
    issued = []
    if not LAGFIRST:
        # previous group's tail: blocks 0..MBW-2 of our first chunk (after its
        # blocks 1..MBW-1); one block: its own, after its MFMAs
        for b in range(max(MBW - 1, 1)):
            issued.append((b, C0))

    def wait_for(block, chunk):
        """lgkmcnt value that guarantees the read of (block, chunk) has landed."""
        for i in range(len(issued) - 1, -1, -1):
            if issued[i] == (block, chunk):
                after = len(issued) - 1 - i
                return 2 * after
        raise AssertionError(f"read of {(block, chunk)} not issued")

    last_mfma_slot = None  # ring slot the most recent MFMA group read
    for ci, c in enumerate(chunks):
        last_chunk = c == 3
        prefetch = c + PF < 4 or HASNEXT
        P = 4 * sum(1 for j in range(c + 1, c + PF + 1) if j <= 3 or HASNEXT)  # weight loads issued after this k-step's
        NB = nbufs(PF)
        bs = (4 * TP + c) % NB  # this k-step's B buffer
        emit(f"; k-step chunk {c}")
        if prefetch:
            # the k-step this one prefetches: chunk k of this group, or (k >= 4)
            # the next group's (k - 4)-th, chunk C0 + k - 4 (sn: its first)
            k = c + PF
            bn = (4 * TP + (k if k < 4 else C0 + k)) % NB
            if k < 4:
                emit(f"s_add_u32 %[tmp], %[sc], {k * KSTEP}")
                src = "%[rc], %[tmp]"
            elif k == 4:
                src = "%[rn], %[sn]"
            else:
                emit(f"s_add_u32 %[tmp], %[sn], {(k - 4) * KSTEP}")
                src = "%[rn], %[tmp]"
            for q in range(4):
                emit(f"buffer_load_dwordx4 %[b{bn}_{q}], %[voff], {src} offen offset:{q * 1024}")
        b_waited = False
        for mb in range(MBW):
            if not skipped(mb):
                # A fragments of (mb, c)
                w = wait_for(mb, c)
                if w is not None:
                    emit(f"s_waitcnt lgkmcnt({min(w, 15)})")
                A = [f"%[a{mb}_0]", f"%[a{mb}_1]"]
                acc0 = f"%[c{mb}_0]"
                acc1 = f"%[c{mb}_1]"
                if not b_waited:
                    emit(f"s_waitcnt vmcnt({P + 3})")
                emit(f"v_mfma_f32_16x16x32_f16 {acc0}, %[b{bs}_0], {A[1]}, {acc0}")
                if not b_waited:
                    emit(f"s_waitcnt vmcnt({P + 1})")
                emit(f"v_mfma_f32_16x16x32_f16 {acc1}, %[b{bs}_2], {A[1]}, {acc1}")
                emit(f"v_mfma_f32_16x16x32_f16 {acc0}, %[b{bs}_1], {A[0]}, {acc0}")
                if not b_waited:
                    emit(f"s_waitcnt vmcnt({P})")
                    b_waited = True
                emit(f"v_mfma_f32_16x16x32_f16 {acc1}, %[b{bs}_3], {A[0]}, {acc1}")
                emit(f"v_mfma_f32_16x16x32_f16 {acc0}, %[b{bs}_0], {A[0]}, {acc0}")
                emit(f"v_mfma_f32_16x16x32_f16 {acc1}, %[b{bs}_2], {A[0]}, {acc1}")
                last_mfma_slot = mb
            # the ring read after block mb
            rd = None
            if mb == 0:
                if not (LAGFIRST and ci == 0) and not skipped(MBW - 1) and MBW > 1:
                    rd = (MBW - 1, c, f"%[d{MBW - 1}]")
            else:
                if not last_chunk:
                    if not skipped(mb - 1):
                        rd = (mb - 1, c + 1, f"%[d{mb - 1}]")
                elif HASNEXT:
                    rd = (mb - 1, C0, f"%[n{mb - 1}]")
            if MBW == 1 and mb == 0:
                # single block: its next fragments right after its own MFMAs
                if not last_chunk:
                    rd = (0, c + 1, "%[d0]")
                elif HASNEXT:
                    rd = (0, C0, "%[n0]")
            if rd is not None:
                blk, ch, addr = rd
                if last_mfma_slot == blk:
                    emit("s_nop 4")  # the MFMAs just issued read this slot
                emit(f"ds_read_b128 %[a{blk}_0], {addr} offset:{64 * ch}")
                emit(f"ds_read_b128 %[a{blk}_1], {addr} offset:{64 * ch + 256}")
                issued.append((blk, ch))
        if not b_waited:
            # every block skipped: the buffer still has to land before it is reused
            emit(f"s_waitcnt vmcnt({P})")
    if LAST_NOP:
        # whatever the compiler puts between two groups (or the epilogue) may
        # read an accumulator or write a fragment register: MFMA -> VALU
        # hazards it cannot see inside the asm, covered here
        emit("s_nop 7")
        emit("s_nop 7")
    return "\\n\\t".join(lines)


def term_group_asm(MBW, C0, SKC, PF=1, HASNEXT=1, TP=0):
    """The same group in term-major order: per k-step all blocks' t1*B0
    products (phase 0), then all blocks' t0*b1 (phase 1), then t0*B0 (phase
    2), so an accumulator's three dependent MFMAs sit 2*MBW instructions
    apart instead of 2 (each accumulator still sums t1*B0, t0*b1, t0*B0 in
    that order: bitwise the block-major sums).  Reads by term: block mb's
    next t1 fragment right after its phase-1 pair (t1 is dead after phase
    0), its next t0 fragment after block mb+1's phase-2 pair (lagged: one
    pair between the last reader and the load), the last block's in the
    next k-step after block 0's phase-0 pair.  Weight fragments load in the
    order 0, 2, 1, 3 (phase 0 needs fragments 0 and 2).  HASNEXT = 0: the
    loop's last group -- no prefetch or reads for a next one, so the drain
    after it waits for nothing."""
    lines = []
    emit = lines.append
    chunks = list(range(C0, 4))
    skipped = lambda mb: (SKC >> mb) & 1  # noqa: E731
    NB = nbufs(PF)
    # reads in flight at group entry (the predecessor's or the prologue's),
    # in issue order: every block's t1 of chunk C0, then t0 of blocks < MBW-1
    issued = [(mb, C0, 1) for mb in range(MBW)] + [(mb, C0, 0) for mb in range(MBW - 1)]

    def wait_a(blk, ch, term):
        for i in range(len(issued) - 1, -1, -1):
            if issued[i] == (blk, ch, term):
                emit(f"s_waitcnt lgkmcnt({min(len(issued) - 1 - i, 15)})")
                return
        raise AssertionError(f"read of {(blk, ch, term)} not issued")

    def read(blk, ch, term, addr):
        emit(f"ds_read_b128 %[a{blk}_{term}], {addr} offset:{64 * ch + 256 * term}")
        issued.append((blk, ch, term))

    for c in chunks:
        last_chunk = c == 3
        bs = (4 * TP + c) % NB
        # weight loads issued after this k-step's: the next PF k-steps' (the next group's only with HASNEXT)
        P = 4 * sum(1 for j in range(c + 1, c + PF + 1) if j <= 3 or HASNEXT)
        emit(f"; k-step chunk {c}")
        k = c + PF
        bn = (4 * TP + (k if k < 4 else C0 + k)) % NB
        src = None
        if k < 4:
            emit(f"s_add_u32 %[tmp], %[sc], {k * KSTEP}")
            src = "%[rc], %[tmp]"
        elif not HASNEXT:
            pass
        elif k == 4:
            src = "%[rn], %[sn]"
        else:
            emit(f"s_add_u32 %[tmp], %[sn], {(k - 4) * KSTEP}")
            src = "%[rn], %[tmp]"
        if src:
            for q in (0, 2, 1, 3):
                emit(f"buffer_load_dwordx4 %[b{bn}_{q}], %[voff], {src} offen offset:{q * 1024}")
        live = [mb for mb in range(MBW) if not skipped(mb)]
        # phase 0: t1 * B0
        emit(f"s_waitcnt vmcnt({P + 2})")  # fragments 0 and 2 of this k-step
        for i, mb in enumerate(live):
            wait_a(mb, c, 1)
            emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_0], %[b{bs}_0], %[a{mb}_1], %[c{mb}_0]")
            emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_1], %[b{bs}_2], %[a{mb}_1], %[c{mb}_1]")
            if i == 0 and not skipped(MBW - 1) and MBW > 1:
                read(MBW - 1, c, 0, f"%[d{MBW - 1}]")  # the last block's t0, lagged from the k-step before
        if MBW == 1:
            read(0, c, 0, "%[d0]")
        if not live and MBW > 1 and not skipped(MBW - 1):
            read(MBW - 1, c, 0, f"%[d{MBW - 1}]")
        # phase 1: t0 * b1; then the block's next t1
        emit(f"s_waitcnt vmcnt({P})")
        for mb in range(MBW):
            if not skipped(mb):
                wait_a(mb, c, 0)
                emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_0], %[b{bs}_1], %[a{mb}_0], %[c{mb}_0]")
                emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_1], %[b{bs}_3], %[a{mb}_0], %[c{mb}_1]")
            if not last_chunk:
                if not skipped(mb):
                    read(mb, c + 1, 1, f"%[d{mb}]")
            elif HASNEXT:
                read(mb, C0, 1, f"%[n{mb}]")
        # phase 2: t0 * B0; then the previous block's next t0
        last_mfma = None
        for mb in range(MBW):
            if not skipped(mb):
                emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_0], %[b{bs}_0], %[a{mb}_0], %[c{mb}_0]")
                emit(f"v_mfma_f32_16x16x32_f16 %[c{mb}_1], %[b{bs}_2], %[a{mb}_0], %[c{mb}_1]")
                last_mfma = mb
            if mb >= 1:
                blk = mb - 1
                if (last_chunk and HASNEXT) or (not last_chunk and not skipped(blk)):
                    if last_mfma == blk:
                        emit("s_nop 4")  # no pair between the slot's last reader and this load
                    read(blk, C0 if last_chunk else c + 1, 0, f"%[n{blk}]" if last_chunk else f"%[d{blk}]")
    emit("s_nop 7")
    emit("s_nop 7")
    return "\\n\\t".join(lines)


def term_prologue_asm(MBW, C0, PF, TP=0):
    """The term-major group's entry state: the first PF k-steps' weights
    (fragments 0, 2, 1, 3), every block's t1 of chunk C0, then the t0 of
    blocks 0..MBW-2."""
    NB = nbufs(PF)
    text = []
    for k in range(PF):
        if k:
            text.append(f"s_add_u32 %[tmp], %[sc], {k * KSTEP}")
        for q in (0, 2, 1, 3):
            text.append(f"buffer_load_dwordx4 %[b{(4 * TP + C0 + k) % NB}_{q}], %[voff], %[rc], "
                        f"{'%[tmp]' if k else '%[sc]'} offen offset:{q * 1024}")
    for blk in range(MBW):
        text.append(f"ds_read_b128 %[a{blk}_1], %[d{blk}] offset:{64 * C0 + 256}")
    for blk in range(MBW - 1):
        text.append(f"ds_read_b128 %[a{blk}_0], %[d{blk}] offset:{64 * C0}")
    return "\\n\\t".join(text)


def prologue_asm(MBW, C0, PF, TP=0):
    """The prologue: the first PF k-steps' B fragments (rc, from soffset sc)
    and the A reads a group's predecessor leaves in flight (blocks 0..MBW-2
    of chunk C0; one block: its own)."""
    NB = nbufs(PF)
    text = []
    for k in range(PF):
        if k:
            text.append(f"s_add_u32 %[tmp], %[sc], {k * KSTEP}")
        for q in range(4):
            text.append(f"buffer_load_dwordx4 %[b{(4 * TP + C0 + k) % NB}_{q}], %[voff], %[rc], "
                        f"{'%[tmp]' if k else '%[sc]'} offen offset:{q * 1024}")
    for blk in range(max(MBW - 1, 1)):
        text.append(f"ds_read_b128 %[a{blk}_0], %[d{blk}] offset:{64 * C0}")
        text.append(f"ds_read_b128 %[a{blk}_1], %[d{blk}] offset:{64 * C0 + 256}")
    return "\\n\\t".join(text)


def operand_list(MBW, NB=2):
    outs = []
    for k in range(MBW):
        for t in range(2):
            outs.append(f'[a{k}_{t}] "+v"(aq[{k}][{t}])')
    for j in range(NB):
        for q in range(4):
            outs.append(f'[b{j}_{q}] "+v"(bq[{j}][{q}])')
    outs.append('[tmp] "=&s"(tmp)')
    for k in range(MBW):
        for n in range(2):
            outs.append(f'[c{k}_{n}] "+v"(acc[{k}][{n}])')
    ins = []
    for k in range(MBW):
        ins.append(f'[d{k}] "v"(ad[{k}])')
    for k in range(MBW):
        ins.append(f'[n{k}] "v"(an[{k}])')
    ins += ['[voff] "v"(voff)', '[rc] "s"(rc)', '[rn] "s"(rn)', '[sc] "s"(sc)', '[sn] "s"(sn)']
    return outs, ins


def main():
    out = []
    out.append("// az_kloop_asm.h -- GENERATED by gen_kloop_asm.py: do not edit.\n"
               "// The tower's K-loop groups as hand-scheduled assembly (see the generator's\n"
               "// docstring); included by az_tower16.hip.\n#pragma once\n\nnamespace az {\nnamespace {\n")
    out.append("typedef int az_rsrc __attribute__((ext_vector_type(4)));\n"
               "// register operands must be vector types (HIP's uint4 is a struct)\n"
               "typedef unsigned az_u4 __attribute__((ext_vector_type(4)));\n"
               "typedef float az_f4 __attribute__((ext_vector_type(4)));\n")
    out.append("// ORD 0: block-major k-steps (group_asm), 1: term-major (term_group_asm)\n"
               "// TP: the tap's parity (selects the B buffers when PF >= 3: nbufs())\n"
               "template <int MBW, int C0, int SKC, int PF, int ORD, int HN = 1, int TP = 0>\nstruct KGroup;\n"
               "template <int MBW, int C0, int PF, int ORD, int TP = 0>\nstruct KPro;\n"
               "template <int MBW, int NB>\nstruct KDrain;\n")
    # the prologue: the first PF k-steps' B fragments and the A reads a
    # group's predecessor leaves in flight (blocks 0..MBW-2 of chunk C0; one
    # block: its own)
    # forms: (C0, PF, ORD, TP); PF 3 (8 buffers) for the 1-2-block waves only
    def forms(MBW):
        f = [(c, p, o, 0) for c, p in ((0, 1), (0, 2), (2, 1)) for o in (0, 1)]
        if MBW <= 2:
            f += [(0, 3, 1, tp) for tp in (0, 1)]
        return f

    for MBW in (1, 2, 3, 4, 6):
        for C0, PF, ORD, TP in forms(MBW):
            NB = nbufs(PF)
            body = (term_prologue_asm if ORD else prologue_asm)(MBW, C0, PF, TP)
            outs = [f'[a{k}_{t}] "+v"(aq[{k}][{t}])' for k in range(MBW) for t in range(2)]
            outs += [f'[b{j}_{q}] "+v"(bq[{j}][{q}])' for j in range(NB) for q in range(4)]
            outs.append('[tmp] "=&s"(tmp)')
            ins = [f'[d{k}] "v"(ad[{k}])' for k in range(MBW)] + ['[voff] "v"(voff)', '[rc] "s"(rc)', '[sc] "s"(sc)']
            out.append(f"template <>\nstruct KPro<{MBW}, {C0}, {PF}, {ORD}, {TP}> {{\n"
                       f"  __device__ __forceinline__ static void run(az_u4 (&aq)[{MBW}][2], az_u4 (&bq)[{NB}][4],\n"
                       f"      const int (&ad)[{MBW}], int voff, az_rsrc rc, int sc) {{\n"
                       f"    int tmp;\n"
                       f"    asm volatile(\"{body}\"\n"
                       f"        : {', '.join(outs)}\n"
                       f"        : {', '.join(ins)}\n"
                       f"        : \"memory\");\n"
                       f"  }}\n}};\n")
        # the drain: the last group's prefetches land before the registers are reused
        for NB in ((2, 4, 8) if MBW <= 2 else (2, 4)):
            outs = [f'"+v"(aq[{k}][{t}])' for k in range(MBW) for t in range(2)]
            outs += [f'"+v"(bq[{j}][{q}])' for j in range(NB) for q in range(4)]
            outs += [f'"+v"(acc[{k}][{n}])' for k in range(MBW) for n in range(2)]
            out.append(f"template <>\nstruct KDrain<{MBW}, {NB}> {{\n"
                       f"  __device__ __forceinline__ static void run(az_f4 (&acc)[{MBW}][2], az_u4 (&aq)[{MBW}][2],\n"
                       f"      az_u4 (&bq)[{NB}][4]) {{\n"
                       f"    asm volatile(\"s_waitcnt vmcnt(0) lgkmcnt(0)\"\n"
                       f"        : {', '.join(outs)}\n"
                       f"        :\n"
                       f"        : \"memory\");\n"
                       f"  }}\n}};\n")
    count = 0
    for MBW in (1, 2, 3, 4, 6):
        for C0, PF, ORD, TP in forms(MBW):
            NB = nbufs(PF)
            for SKC, HN in [(k, h) for k in (0, 1, 2) for h in (1, 0)]:
                if MBW == 1 and SKC:
                    continue
                count += 1
                text = (term_group_asm(MBW, C0, SKC, PF, HN, TP) if ORD else group_asm(MBW, C0, SKC, PF, HN, TP=TP))
                outs, ins = operand_list(MBW, NB)
                out.append(f"template <>\nstruct KGroup<{MBW}, {C0}, {SKC}, {PF}, {ORD}, {HN}, {TP}> {{\n"
                           f"  __device__ __forceinline__ static void run(az_f4 (&acc)[{MBW}][2], az_u4 (&aq)[{MBW}][2], az_u4 (&bq)[{NB}][4],\n"
                           f"      const int (&ad)[{MBW}], const int (&an)[{MBW}], int voff, az_rsrc rc, az_rsrc rn,\n"
                           f"      int sc, int sn) {{\n"
                           f"    int tmp;\n"
                           f"    asm volatile(\"{text}\"\n"
                           f"        : {', '.join(outs)}\n"
                           f"        : {', '.join(ins)}\n"
                           f"        : \"memory\");\n"
                           f"  }}\n}};\n")
    out.append("}  // namespace\n}  // namespace az\n")
    with open(OUT, "w") as fh:
        fh.write("\n".join(out))
    print(f"wrote {OUT}: {count} group variants")


if __name__ == "__main__":
    main()
