"""Hand-derived known-answer tests for the GapAssem surface added in round 2: refineClipping
(X-drop, both ends, the "reached clipL" warning), removeConsGaps over a deleted base, and the
writeACE / writeInfo / writeMSA writers.

The reference cannot be built here (gclib is absent), so each expected value below was derived
BY HAND from /root/reference/GapAssem.cpp; the derivation is written next to each case (line
numbers are into GapAssem.cpp).  The CPU tests check the oracle (oracle/gapassem_oracle.c)
against them; the `gpu` tests check the product (gapassem_consensus, the HIP path through the
GapAssem C++ API) against the same literals.

Layouts are PWL1 rows (offset, seq, ofs, clp5, clp3, revcompl), named row0, row1, ...;
minoffset = min offset, length = max(offset + seqlen + sum(ofs)) - minoffset.
Conventions used in the derivations:
  toMSA (:551-591): col = offset - minoffset; per base i: ofs[i] gap columns, then the base;
    bases with i < clipL or i >= seqlen - clipR are clipped (not counted); clipL/clipR are
    clp5/clp3, swapped for revcompl rows.  mincol/maxcol = first/last unclipped base column.
  bestChar (:1048-1069): max count; ties keep the order A,C,G,T,N,- (stable qsort of 6);
    '-'/N at the max defer to the next tied entry.
  refineMSA (:1133-1181): consensus over [mincol, maxcol], gaps as '*' (dropped with
    removeConsGaps, each via removeColumn(col - cols_removed)), then per row refineClipping with
    cpos = offset - minoffset - mincol, removeClipGaps (removeConsGaps only), and a second
    refineClipping(skipDels) if gaps were removed.
"""
import struct

import pytest

from conftest import GA_CLI, GA_ORACLE, run
from test_oracle_kat import read_pwc, write_pwl


def rows_of(pwc_raw, seqlens):
    """(offset, numgaps, clp5, clp3, ofs) per row from a PWC1 result."""
    b = pwc_raw
    length, _, _, _, clen, _ = struct.unpack_from("<6i", b, 4)
    p = 28 + clen + 24 * length
    (n,) = struct.unpack_from("<I", b, p)
    p += 4
    out = []
    for k in range(n):
        off, ng, c5, c3 = struct.unpack_from("<4i", b, p)
        p += 16
        ofs = list(struct.unpack_from(f"<{seqlens[k]}h", b, p))
        p += 2 * seqlens[k]
        out.append((off, ng, c5, c3, ofs))
    return out


def consensus_run(binary, tmp_path, rows, extra=(), writers=False):
    lay = tmp_path / "l.pwl"
    write_pwl(lay, rows)
    args = [binary, lay, tmp_path / "o.pwc", *extra]
    if writers:
        args += ["--ace", tmp_path / "o.ace", "--info", tmp_path / "o.info", "--msa", tmp_path / "o.mfa"]
    rc, out, err = run(args)
    res = read_pwc(tmp_path / "o.pwc") if rc == 0 else None
    return rc, err, res


# ---------------------------------------------------------------- K1: refineClipping, right end
# rows 0,1: offset 0, (ACGT)x6 (24 bases); row2: offset 0, "ACGTACGTAC"+"T"*14, clp3 = 18 (forward:
# clipR = 18, bases 6..23 clipped) -> consensus = (ACGT)x6, mincol 0, maxcol 23.
# refineClipping(row2) (:182-349): clipL = 0, clipR = 18, glen = 24, gclipR = 18, gseq = row2.
#   cp = cpos + glen - gclipR - 1 = 0 + 24 - 18 - 1 = 5, sp = 5: gseq[5] 'C' == cons[5] 'C' (no back walk).
#   score = max = 1, bestpos = 5; forward: cp/sp 6..9 match G,T,A,C -> score 2,3,4,5, bestpos 9;
#   10: T/G -> 2; 11: T/T -> 3; 12: T/A -> 0; 13: T/C -> -3; 14: T/G -> -6; 15: T/T -> -5;
#   16: T/A -> -8; 17: T/C -> -11; 18: T/G -> -14; 19: T/T -> -13; 20: T/A -> -16 = XDROP: stop.
#   bestpos 9 > 5 -> clipR = seqlen - gxpos[9] - 1 = 24 - 9 - 1 = 14 -> clp3 = 14.
K1_ROWS = [(0, "ACGT" * 6, [0] * 24, 0, 0, 0), (0, "ACGT" * 6, [0] * 24, 0, 0, 0),
           (0, "ACGTACGTAC" + "T" * 14, [0] * 24, 0, 18, 0)]
K1_CONS = "ACGT" * 6
K1_ROW2 = (0, 0, 0, 14)

# ---------------------------------------------------------------- K2: refineClipping, left end, reverse row
# rows 0,1: "ACGT"x4; row2: revcompl 1, "TTGAACGT"+"ACGTACGT", clp3 = 8, clp5 = 0 -> clipL = clp3 = 8
# (bases 0..7 clipped), clipR = 0 -> consensus (ACGT)x4, mincol 0, maxcol 15.
# refineClipping(row2): glen 16, gclipL = 8, gclipR = 0; clipR = 0: no right pass.
#   left: cp = cpos + gclipL = 8, sp = 8: 'A' == cons[8] 'A'.  score = 1, bestpos = startpos = 8;
#   backward: 7 T/T 2 (best 7); 6 G/G 3 (6); 5 C/C 4 (5); 4 A/A 5 (4); 3 A/T 2; 2 G/G 3; 1 T/C 0;
#   0 T/A -3; --cp < 0: stop.  bestpos 4 < 8 -> clipL = gxpos[4] = 4 -> clp3 = 4 (clp5 stays 0).
K2_ROWS = [(0, "ACGT" * 4, [0] * 16, 0, 0, 0), (0, "ACGT" * 4, [0] * 16, 0, 0, 0),
           (0, "TTGAACGT" + "ACGTACGT", [0] * 16, 0, 8, 1)]
K2_ROW2 = (0, 0, 0, 4)

# ---------------------------------------------------------------- K3: "reached clipL" warning
# rows 0,1: "AAAAAAAA"; row2: "CCCCCCCC", clp3 = 4 (bases 0..3 unclipped).  Columns 0..3: A:2 C:1 ->
# A; 4..7: A:2 -> A.  Consensus "AAAAAAAA".
# refineClipping(row2): clipR = 4, gclipR = 4, gclipL = 0; cp = sp = 8 - 4 - 1 = 3.
#   back walk while gseq[sp] != cons[cp]: C != A -> clipR 5, sp 2; clipR 6, sp 1; clipR 7, sp 0;
#   clipR 8, sp -1 < gclipL -> GMessage("Warning: reached clipL trying to find an initial match on
#   row2!\n") and return — clipR is a reference to clp3, so clp3 = 8 stays.
K3_ROWS = [(0, "A" * 8, [0] * 8, 0, 0, 0), (0, "A" * 8, [0] * 8, 0, 0, 0), (0, "C" * 8, [0] * 8, 0, 4, 0)]
K3_ERR = b"Warning: reached clipL trying to find an initial match on row2!\n"
K3_ROW2 = (0, 0, 0, 8)

# ---------------------------------------------------------------- K4: removeConsGaps over a deleted base (+ writeInfo)
# row0, row1: "ACGT" ofs [0,0,1,0]   -> A0 C1 -2 G3 T4
# row2:       "ACNGT" ofs [0,0,-1,0,0] (base 2 already deleted: ofs -1 adds no column, the base still
#             counts, :574-581) -> A0 C1 N2 G3 T4
# row3:       "ACGTAC" ofs [0,0,1,0,3,0] -> A0 C1 -2 G3 T4 -5 -6 -7 A8 C9
# length = max(5, 5, 4, 10) = 10.  Counts: col2 N:1 -:3 -> '-'; cols 5,6,7 -:1 -> '-'; the rest
# one base each (A,C,G,T,A,C at 0,1,3,4,8,9).  mincol 0, maxcol 9.
# refineMSA with removeConsGaps: col2 -> removeColumn(2): alpos 2 (:755-779): row0 walk salpos
#   1,2 then 2+1+ofs[2]=4 > 2 at spos 2 -> removeBase(2): ofs[2] 1->0, numgaps 0; row1 the same;
#   row2: 1, 2, 2+1-1 = 2 (not > 2), 2+1+0 = 3 > 2 at spos 3 -> ofs[3] = -1, numgaps -1-1 = -2;
#   row3: spos 2 -> ofs[2] = 0, numgaps 3.  cols_removed 1.
# col5 -> removeColumn(4): rows 0,1,2 walk past their last base (unaffected); row3: 1,2,3,4, then
#   4+1+3 = 8 > 4 at spos 4 -> ofs[4] = 2 (numgaps 2).  col6 -> removeColumn(4): ofs[4] = 1;
#   col7 -> removeColumn(4): ofs[4] = 0 (numgaps 0).  Consensus "ACGTAC", 4 columns removed.
# Per row: clips are 0 (refineClipping returns at once); removeClipGaps zeroes ofs[0] only (i <= 0).
# writeInfo (:1264-1367): ">contig1 4 ACGTAC"; asml = seqoffset + 1 and asmr starts at asml - 1, so
#   base j is compared with consensus[asmr - 1] = one column to its right (the reference's indexing):
#   row0/row1 "ACGT" vs "CGTA": pid 0.00, asmr 5; row2: j0 A/C, j1 C/G, j2 'd' (asmr stays 3),
#   j3 'd', j4 T vs cons[3] 'T' match -> pid 1/3 -> 33.33, alndata "dd" (runs <= 2 print only the
#   letters), asmr 4; row3 "ACGTAC" vs "CGTAC\\0": 0.00, asmr 7.
K4_ROWS = [(0, "ACGT", [0, 0, 1, 0], 0, 0, 0), (0, "ACGT", [0, 0, 1, 0], 0, 0, 0),
           (0, "ACNGT", [0, 0, -1, 0, 0], 0, 0, 0), (0, "ACGTAC", [0, 0, 1, 0, 3, 0], 0, 0, 0)]
K4_CONS = "ACGTAC"
K4_ROWS_OUT = [(0, 0, 0, 0, [0, 0, 0, 0]), (0, 0, 0, 0, [0, 0, 0, 0]), (0, -2, 0, 0, [0, 0, -1, -1, 0]),
               (0, 0, 0, 0, [0, 0, 0, 0, 0, 0])]
K4_COUNTS = [(4, 0, 0, 0, 0, 0), (0, 4, 0, 0, 0, 0), (0, 0, 0, 0, 1, 3), (0, 0, 4, 0, 0, 0), (0, 0, 0, 4, 0, 0),
             (0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 1), (1, 0, 0, 0, 0, 0), (0, 1, 0, 0, 0, 0)]
K4_INFO = (">contig1 4 ACGTAC\n"
           "row0 4 1 2 5 1 4 0.00 \n"
           "row1 4 1 2 5 1 4 0.00 \n"
           "row2 5 1 2 4 1 5 33.33 dd\n"
           "row3 6 1 2 7 1 6 0.00 \n")

# ---------------------------------------------------------------- K5: writeACE / writeInfo / writeMSA, one reverse row
# row0: offset 0, "ACGTACGTAC"                 -> cols 0..9
# row1: offset 2, "GTTACGTA", ofs[2] = 3       -> G2 T3 -4 -5 -6 T7 A8 C9 G10 T11 A12
# row2: offset 1, "CGTAC", revcompl 1, clp5 1  -> clipL = clp3 = 0, clipR = clp5 = 1: C1 G2 T3 A4, the
#        last base (C at col 5) clipped.
# length = max(10, 2+8+3, 1+5) = 13.  Columns: 0 A; 1 C:2; 2 G:3; 3 T:3; 4 A:2 -:1 -> A; 5 C:1 -:1 ->
# C (C before - in the stable order); 6 G:1 -:1 -> G; 7 T:2; 8 A:2; 9 C:2; 10 G; 11 T; 12 A.
# Consensus "ACGTACGTACGTA", mincol 0, maxcol 12 (removeConsGaps off: nothing removed).
# refineClipping(row2): clipR = 1, glen 5, gclipR 1; cpos = 1; cp = 1+5-1-1 = 4, sp = 3: 'A' == cons[4].
#   forward: sp 4 'C' == cons[5] 'C' -> score 2, bestpos 4; sp 5 = glen: stop.
#   clipR = 5 - gxpos[4] - 1 = 0 -> clp5 = 0.
# writeACE (:1200-1262): 2 forward, 1 reverse -> 'U'; consensus in lines of 60; "AF <id> <U|C>
#   <offset - minoffset - mincol + 1>"; per row "RD <id> <seqlen+numgaps> 0 0", the gapped read with
#   '*' (as stored: writeACE runs before writeMSA's finalize), then QA from the clips plus the gaps
#   inside them (ofs[0] for the left side) — all clips 0 here.
# writeInfo: seqoffset 1 / 3 / 2; bases compared one column right (see K4): every pid 0.00; row1's
#   gap run of 3 prints "%d%c%d-" with the 2 aligned bases before it: "2g3-"; row2 (reverse) swaps
#   seql / seqr: 5 1.
# writeMSA (:1039-1046, printMFasta :482-520): finalize() reverse-complements row2's bases (prepSeq
#   :89-101, ofs untouched): CGTAC -> GTACG; each row: `offset` dashes, then the gapped bases.
K5_ROWS = [(0, "ACGTACGTAC", [0] * 10, 0, 0, 0), (2, "GTTACGTA", [0, 0, 3, 0, 0, 0, 0, 0], 0, 0, 0),
           (1, "CGTAC", [0] * 5, 1, 0, 1)]
K5_CONS = "ACGTACGTACGTA"
K5_COUNTS = [(1, 0, 0, 0, 0, 0), (0, 2, 0, 0, 0, 0), (0, 0, 3, 0, 0, 0), (0, 0, 0, 3, 0, 0), (2, 0, 0, 0, 0, 1),
             (0, 1, 0, 0, 0, 1), (0, 0, 1, 0, 0, 1), (0, 0, 0, 2, 0, 0), (2, 0, 0, 0, 0, 0), (0, 2, 0, 0, 0, 0),
             (0, 0, 1, 0, 0, 0), (0, 0, 0, 1, 0, 0), (1, 0, 0, 0, 0, 0)]
K5_ROWS_OUT = [(0, 0, 0, 0, [0] * 10), (2, 3, 0, 0, [0, 0, 3, 0, 0, 0, 0, 0]), (1, 0, 0, 0, [0] * 5)]
K5_ACE = ("CO contig1 13 3 0 U\n"
          "ACGTACGTACGTA\n"
          "\nBQ \n\n"
          "AF row0 U 1\n"
          "AF row1 U 3\n"
          "AF row2 C 2\n"
          "\n"
          "RD row0 10 0 0\n"
          "ACGTACGTAC\n"
          "\nQA 1 10 1 10\nDS \n\n"
          "RD row1 11 0 0\n"
          "GT***TACGTA\n"
          "\nQA 1 11 1 11\nDS \n\n"
          "RD row2 5 0 0\n"
          "CGTAC\n"
          "\nQA 1 5 1 5\nDS \n\n")
K5_INFO = (">contig1 3 ACGTACGTACGTA\n"
           "row0 10 1 2 11 1 10 0.00 \n"
           "row1 8 3 4 14 1 8 0.00 2g3-\n"
           "row2 5 2 3 7 5 1 0.00 \n")
K5_MSA = (">row0\nACGTACGTAC\n"
          ">row1\n--GT---TACGTA\n"
          ">row2\n-GTACG\n")


def _check_k1(res, err):
    assert res["cons"] == K1_CONS and (res["mincol"], res["maxcol"]) == (0, 23)
    assert rows_of(res["raw"], [24, 24, 24])[2][:4] == K1_ROW2
    assert err == b""


def _check_k2(res, err):
    assert res["cons"] == "ACGT" * 4
    assert rows_of(res["raw"], [16, 16, 16])[2][:4] == K2_ROW2
    assert err == b""


def _check_k3(res, err):
    assert res["cons"] == "A" * 8
    assert rows_of(res["raw"], [8, 8, 8])[2][:4] == K3_ROW2
    assert err == K3_ERR


def _check_k4(res, tmp_path):
    assert res["cons"] == K4_CONS and res["removed"] == 4
    assert (res["length"], res["mincol"], res["maxcol"]) == (10, 0, 9)
    assert [tuple(c) for c in res["counts"]] == K4_COUNTS
    assert rows_of(res["raw"], [4, 4, 5, 6]) == K4_ROWS_OUT
    assert open(tmp_path / "o.info").read() == K4_INFO


def _check_k5(res, tmp_path):
    assert res["cons"] == K5_CONS and res["removed"] == 0
    assert (res["length"], res["mincol"], res["maxcol"]) == (13, 0, 12)
    assert [tuple(c) for c in res["counts"]] == K5_COUNTS
    assert rows_of(res["raw"], [10, 8, 5]) == K5_ROWS_OUT
    assert open(tmp_path / "o.ace").read() == K5_ACE
    assert open(tmp_path / "o.info").read() == K5_INFO
    assert open(tmp_path / "o.mfa").read() == K5_MSA


def _all_cases(binary, tmp_path):
    for name, rows, check in (("k1", K1_ROWS, _check_k1), ("k2", K2_ROWS, _check_k2), ("k3", K3_ROWS, _check_k3)):
        d = tmp_path / name
        d.mkdir()
        rc, err, res = consensus_run(binary, d, rows)
        assert rc == 0, err
        check(res, err)
    d = tmp_path / "k4"
    d.mkdir()
    rc, err, res = consensus_run(binary, d, K4_ROWS, extra=["--remove-gaps"], writers=True)
    assert rc == 0 and err == b"", err
    _check_k4(res, d)
    d = tmp_path / "k5"
    d.mkdir()
    rc, err, res = consensus_run(binary, d, K5_ROWS, writers=True)
    assert rc == 0 and err == b"", err
    _check_k5(res, d)


def test_gapassem_kats_oracle(built, tmp_path):
    _all_cases(GA_ORACLE, tmp_path)


@pytest.mark.gpu
def test_gapassem_kats_product(built, tmp_path):
    _all_cases(GA_CLI, tmp_path)
