#!/usr/bin/env python3
"""Generate approx_counter_amd/csrc/wm_tid_blocks.inc: the inline-asm text blocks of
the count kernel's table-driven inner loop ("~Eq from an LDS table").

    python tools/gen_tid_blocks.py      # rewrites the .inc (committed; the build does not run this)

One block runs NB text bases (NB = 32, 16, 8, 4, 2, 1) of one window through the
Wu-Manber NFA for P interleaved patterns per lane (see wm_count.hip).  The text
is wave-uniform: base j's 2-bit code sits at bits 2j..2j+1 of the SGPR `code`
(bases 16-31 of a 32-base block in `code2`) and, in the N-aware path, its N flag
at bit j of the SGPR `nm`.  Per base:
  SALU   c = code field (4 if N); M0 = ebase + 256*c
  LDS    ds_read_addtid_b32 e  -> e = lane's ~Eq mask for character c
         (a per-wave table of 5 x 64 words built once per wave: no VALU op per
         base for ~Eq; the read is issued three bases ahead)
  VALU   8 ops of NFA + 1.5 of hit accumulation (AND3 over two bases).
The schedule is skewed: step s runs row 0 of base s, row 1 of base s-1 and row 2
of base s-2, three independent dependency chains per wave (in-order issue would
otherwise stall on every one of the 8 dependent ops of a base).  Values rotate
through 4 register slots, so blocks of a multiple of 4 bases end in place.
M0 is compiler-reserved: each block saves and restores it in the same statement.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "approx_counter_amd", "csrc", "wm_tid_blocks.inc")
import sys

AHEAD = 4  # LDS reads in flight ahead of the base being computed
WAIT_PAIR = True  # one s_waitcnt per two bases (the SALU is the CU-shared resource)
NE = AHEAD + 3  # rotating ~Eq registers (base i's is read by rows 0-2 at steps i..i+2)
FIRST_SKIP = 12  # bases of a window's start with no possible occurrence end (k >= 15: k - 3 >= 12)
TABLE_BYTES = 5 * 64 * 4  # one lane word's ~Eq table (5 characters x 64 lanes x u32); word w's at w * this


def m0_setup(j, with_n, eb0):
    """SALU: M0 = ebase + 256 * (code of base j, or 4 for N).  With eb0 the
    wave's table sits at LDS address 0 (one-wave workgroups) and the add goes."""
    word, jj = (("%[code]", "%[code2]", "%[code3]", "%[code4]")[j // 16], j % 16)  # one code word per 16 bases
    lit = (2 << 16) | (2 * jj)
    s = [f"s_bfe_u32 %[t], {word}, {lit:#x}"]
    if with_n:
        s += [f"s_bitcmp1_b32 %[nm], {j}", "s_cselect_b32 %[t], 4, %[t]"]
    if eb0:
        s += ["s_lshl_b32 m0, %[t], 8"]
    else:
        s += ["s_lshl_b32 %[t], %[t], 8", "s_add_u32 m0, %[t], %[eb]"]
    return s


def block(nb, with_n, eb0, skip=0, W=1, init=False):
    """Skewed (software-pipelined) schedule: step s runs row 0 of base s, row 1 of
    base s-1 and row 2 of base s-2 -- three independent dependency chains per wave.
    Row r of base i needs row r of base i-1 and row r-1 of bases i-1 and i, all
    produced at earlier steps.  Values live in 4 rotating slots per (row, D/T);
    slot 3 is the operand register, so blocks of a multiple of 4 bases end in place.
    W = 2: two lane words per wave (2 x P candidates per lane) share each base's SALU
    work; word w reads its own ~Eq table (LDS offset w * 1280 B) and its ops are
    interleaved with the other word's, six dependency chains per wave.
    init: a window's first block reads the NFA's initial state from loop-invariant
    input registers (%[id1], %[is0] ...; d0 = a0 = ~0 is the inline constant -1)
    and only writes the state operands, so no per-window copy of the initial
    state into them precedes it."""

    def pre(w):
        return "" if W == 1 else f"w{w}"

    def D(w, r, i):
        if init and i == -1:
            return "-1" if r == 0 else f"%[id{r}]"
        return f"%[{pre(w)}d{r}]" if i % 4 == 3 else f"%[{pre(w)}D{r}{i % 4}]"

    def T(w, r, i):
        if init and i == -1:
            return f"%[is{r}]"
        return f"%[{pre(w)}s{r}]" if i % 4 == 3 else f"%[{pre(w)}T{r}{i % 4}]"

    def E(w, i):
        return f"%[{pre(w)}e{i % NE}]"

    def X(w, r):
        return f"%[{pre(w)}x{r}]"

    def A(w, r):
        return f"%[{pre(w)}a{r}]"

    def rd(w, i):
        return f"ds_read_addtid_b32 {E(w, i)}" + (f" offset:{w * TABLE_BYTES}" if w else "")

    L = []
    for j in range(min(AHEAD, nb)):
        L += m0_setup(j, with_n, eb0)
        L += ["s_nop 0"] + [rd(w, j) for w in range(W)]
    for st in range(nb + 2):
        rows = [(r, st - r) for r in range(3) if 0 <= st - r < nb]
        if st < nb:
            issued = min(st + AHEAD, nb)
            if not WAIT_PAIR:
                L.append(f"s_waitcnt lgkmcnt({W * (issued - (st + 1))})")
            elif st % 2 == 0:  # bases st and st+1 (reads complete in order)
                L.append(f"s_waitcnt lgkmcnt({W * max(0, issued - min(st + 2, nb))})")
        ahead = st < nb and st + AHEAD < nb
        if ahead:
            L += m0_setup(st + AHEAD, with_n, eb0)
        # phase A: row 0's new D; rows 1-2's x = s_{r-1} & d_{r-1} & t_{r-1}
        for r, i in rows:
            for w in range(W):
                if r == 0:
                    L.append(f"v_or_b32 {D(w, 0, i)}, {T(w, 0, i - 1)}, {E(w, i)}")
                else:
                    L.append(f"v_bitop3_b32 {X(w, r)}, {T(w, r - 1, i - 1)}, {D(w, r - 1, i - 1)}, {T(w, r - 1, i)} "
                             f"bitop3:0x80")
            if r == 0 and ahead:  # one state after the M0 write
                L += [rd(w, st + AHEAD) for w in range(W)]
        # phase B: row 0's shift; rows 1-2's new D = (s_r | ~Eq) & x
        for r, i in rows:
            for w in range(W):
                if r == 0:
                    L.append(f"v_lshrrev_b32 {T(w, 0, i)}, %[P], {D(w, 0, i)}")
                else:
                    L.append(f"v_bitop3_b32 {D(w, r, i)}, {T(w, r, i - 1)}, {E(w, i)}, {X(w, r)} bitop3:0xa8")
        # phase C: rows 1-2's shifts, then the hit accumulators (pairs of bases)
        for r, i in rows:
            if r > 0:
                for w in range(W):
                    L.append(f"v_lshrrev_b32 {T(w, r, i)}, %[P], {D(w, r, i)}")
        for r, i in rows:
            if i < skip:  # a window's first bases: no occurrence can end there (skip <= k - 3)
                continue
            for w in range(W):
                if init and i == skip + 1:  # the accumulator's first AND: from the initial a_r
                    assert skip % 2 == 0 and i < nb
                    if r == 0:
                        L.append(f"v_and_b32 {A(w, r)}, {D(w, r, i - 1)}, {D(w, r, i)}")
                    else:
                        L.append(f"v_bitop3_b32 {A(w, r)}, %[id{r}], {D(w, r, i - 1)}, {D(w, r, i)} bitop3:0x80")
                elif i % 2 == 1:
                    L.append(f"v_bitop3_b32 {A(w, r)}, {A(w, r)}, {D(w, r, i - 1)}, {D(w, r, i)} bitop3:0x80")
                elif i == nb - 1:  # unpaired last base (odd nb)
                    L.append(f"v_and_b32 {A(w, r)}, {A(w, r)}, {D(w, r, i)}")
    if init:
        assert skip > 0 and (nb - 1) % 4 == 3 and nb > skip + 1  # every state operand is written
    if (nb - 1) % 4 != 3:  # final state not in the operand slot
        for w in range(W):
            for r in range(3):
                L.append(f"v_mov_b32 %[{pre(w)}d{r}], {D(w, r, nb - 1)}")
                L.append(f"v_mov_b32 %[{pre(w)}s{r}], {T(w, r, nb - 1)}")
    return L


def body(nb, eb0, skip=0, W=1, init=False):
    """Whole statement text: N-free chunks take the fast path, chunks with an N
    the N-aware one (same registers, so hipcc sees one statement)."""
    L = ["s_mov_b32 %[keep], m0", "s_cmp_lg_u32 %[nm], 0", "s_cbranch_scc1 .Lnpath%="]
    L += block(nb, False, eb0, skip, W, init)
    L += ["s_branch .Lend%=", ".Lnpath%=:"]
    L += block(nb, True, eb0, skip, W, init)
    L += [".Lend%=:", "s_mov_b32 m0, %[keep]"]
    return "\n".join(f'            "{ln}\\n\\t"' for ln in L)


def emit(nb, skip=0, name=None, W=1, init=False):
    extra = [f"code{i}" for i in range(2, (nb + 15) // 16 + 1)]
    code2_in = "".join(f', [{c}] "s"({c})' for c in extra)
    code2_arg = "".join(f", uint32_t {c}" for c in extra)
    pres = [""] if W == 1 else [f"w{w}" for w in range(W)]
    scratch = []
    for p in pres:
        scratch += [f"{p}D{r}{k}" for r in range(3) for k in range(3)] + [f"{p}T{r}{k}" for r in range(3) for k in range(3)]
        scratch += [f"{p}x1", f"{p}x2"] + [f"{p}e{k}" for k in range(NE)]
    decl = ", ".join(scratch)
    outs = ", ".join(f'[{v}] "=&v"({v})' for v in scratch)
    states = []
    for w, p in enumerate(pres):
        sv = "s" if W == 1 else f"s{w}"
        mode = "=&v" if init else "+v"
        states.append(", ".join(f'[{p}{f}] "{mode}"({sv}.{f})' for f in ("d0", "d1", "d2", "s0", "s1", "s2", "a0", "a1", "a2")))
    if W == 1 and not init:  # (the one-word text exactly as before W existed)
        state_ops = """[d0] "+v"(s.d0), [d1] "+v"(s.d1), [d2] "+v"(s.d2), [s0] "+v"(s.s0), [s1] "+v"(s.s1),
              [s2] "+v"(s.s2), [a0] "+v"(s.a0), [a1] "+v"(s.a1), [a2] "+v"(s.a2)"""
        sig = "TidNfa& s"
    else:
        state_ops = ",\n              ".join(states)
        sig = "TidNfa& s" if W == 1 else ", ".join(f"TidNfa& s{w}" for w in range(W))
    init_in = "".join(f', [{v}] "v"(ini.{v[1:]})' for v in ("is0", "is1", "is2", "id1", "id2")) if init else ""
    if init:
        sig += ", const TidInit& ini"
    operands = f"""            : {state_ops},
              {outs},
              [t] "=&s"(t), [keep] "=&s"(keep)
            : [code] "s"(code){code2_in}, [nm] "s"(nm), [eb] "s"(eb), [P] "n"(P){init_in}
            : "memory", "scc");"""
    return f"""template <int P, bool EB0>
__device__ __forceinline__ void {name or f"tid_block{nb}"}({sig}, uint32_t code{code2_arg}, uint32_t nm, uint32_t eb) {{
    uint32_t {decl};
    uint32_t t, keep;
    if constexpr (EB0) {{
        asm volatile(
{body(nb, True, skip, W, init)}
{operands}
    }} else {{
        asm volatile(
{body(nb, False, skip, W, init)}
{operands}
    }}
}}
"""


def main():
    global AHEAD, NE, WAIT_PAIR, OUT
    if "--v6" in sys.argv:  # A/B: one wait per base, 3 reads ahead (build/var only)
        AHEAD, WAIT_PAIR = 3, False
        NE = AHEAD + 3
        OUT = os.path.join(ROOT, "build", "wm_tid_blocks_v6.inc")
    if "--ahead" in sys.argv:  # A/B: N reads ahead (build/var only)
        AHEAD = int(sys.argv[sys.argv.index("--ahead") + 1])
        NE = AHEAD + 3
        OUT = os.path.join(ROOT, "build", f"wm_tid_blocks_a{AHEAD}.inc")
    parts = [
        "// GENERATED by tools/gen_tid_blocks.py -- do not edit.  Inline-asm blocks of the\n"
        "// table-driven count loop (wm_count.hip, DESIGN.md §4).\n"
        "// TidNfa: d* complemented NFA rows, s* = d* >> P, a* AND of the rows over the window.\n"
        "struct TidNfa {\n    uint32_t d0, d1, d2, s0, s1, s2, a0, a1, a2;\n};\n"
        "// The initial state a window's first block reads (d0 = a0 = ~0, a1 = d1, a2 = d2).\n"
        "struct TidInit {\n    uint32_t s0, s1, s2, d1, d2;\n};\n\n"
    ]
    for nb in (32, 16, 8, 4, 2, 1):  # 64-base blocks measured no faster (r01_kernel_log.md)
        parts.append(emit(nb))
    # A window's first 32 bases without the hit accumulation of bases 0-11: an
    # occurrence with <= 2 edits spans >= k - 2 bases, so none ends before base
    # k - 3 (valid for k >= 15; wm_count.hip picks it then).
    parts.append("// tid_block32 for a window's first 32 bases, k >= 15: no hit accumulation over bases 0-11.")
    parts.append(emit(32, skip=FIRST_SKIP, name="tid_block32_first", init=True))
    # Two lane words per wave (AC_WORDS = 2 builds, wm_count.hip): the same blocks over two states.
    parts.append("// Two lane words per wave (AC_WORDS == 2): both words' NFAs, one base's SALU work shared.")
    for nb in (32, 16, 8, 4, 2, 1):
        parts.append(emit(nb, W=2, name=f"tid2_block{nb}"))
    parts.append(emit(32, skip=FIRST_SKIP, name="tid2_block32_first", W=2, init=True))
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
