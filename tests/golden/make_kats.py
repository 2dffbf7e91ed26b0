#!/usr/bin/env python3
"""Writes the hand-derived known-answer tests (KATs) under tests/golden/kat/<name>/.

The reference (gpertea/pwasm pafreport) cannot be built in this image (gclib is absent), so
every expected output below was derived BY HAND from the reference source and is written
here as a literal.  Derivations (line refs into /root/reference/pafreport.cpp):
  kat1_forward  - SURVEY.md §8(a) KAT: S merge-free substitution (:547-573), I event (:579-601),
                  setTContext (:120-128), getRefContext (:721-733), predictImpact S/I (:801-883).
  kat2_reverse  - '-' strand: offset = r_len - r_alnend (:488-490), D/I rloc transforms
                  (:597,615), S kept on the aligned strand then flipped (:634-640),
                  tloc = |tseq| - tloc (:633), revcomp tctx (:631), tdiffs.Reverse (:643),
                  merged S run "GC"/"TA" (:556-560), getRefContext end-of-query quirk (:726-729).
  kat3_status   - homopolymer (:735-748), motif list order (:41,751-763), AA0 quirk for
                  rloc<3 (:829), stop introduced by S (:834-837), "[15]" + abbreviated tctx
                  (:920-934), aa4 containing '.', in-frame deletion scanned to the natural stop,
                  rlabel = qname with 2 FASTA records (:366-379), duplicate q~t warning
                  (:319-333), self alignment skipped (:314-317), '#' comment (:304).
  kat4_fullgenome - -F: rlabel "q:start-end" (:368-372), codon analysis skipped (:259,915)
                  so each line ends with a tab.
  kat6_msa_w    - -w progressive MSA (:382-421, 447-450; GapAssem.cpp:605-753 GSeqAlign(s1,s2) /
                  addAlign / injectGap / addSeq, :1039-1046 + :482-520 writeMSA): query qa aligned
                  to t1, then qb to t2 (another query: qa's GASeq and MSA are dropped, :338-351,
                  rseqs never filled), then qa again to t3, t4, t5 — a fresh MSA, the one written
                  (refMSA = the last query's).  Derivation with qa = AACCGGTTAACC:
                  t3 ":4-tt:8" / 4M2D8M: rgap (CIGAR D, :689-697) qa.setGap(4,2); GSeqAlign(qa,t3)
                    length 14.
                  t4 ":4-ggg:4+a:3" / 4M3D4M1I3M: rseq(qa copy).setGap(4,3); tgap (CIGAR I, :681-688)
                    at tpos 11: t4.setGap(11,1).  addAlign: i=4 d = 2-3 < 0 -> injectGap(qa,4,1) in the
                    MSA: alpos = 0+4+2 = 6; qa.addGap(4,1); t3 walks to spos 6 (salpos 7 > 6) ->
                    t3.addGap(6,1); length 15; t4 added at offset 0.
                  t5 ":10-c:2" / 10M1D2M: rseq.setGap(10,1).  addAlign: i=4 d = 3-0 > 0 ->
                    omsa.injectGap(rseq,4,3): t5.addGap(4,3); i=10 d = 0-1 -> injectGap(qa,10,1):
                    alpos = 0+10+3 = 13; qa.addGap(10,1); t3 walks to spos 12 (its gap at 6 counted)
                    -> t3.addGap(12,1); t4 to spos 12 (gap at 11) -> t4.addGap(12,1); t5 added.
                  Rows (all offset 0, forward; finalize changes nothing): qa gaps {4:3, 10:1},
                  t3 {6:1, 12:1}, t4 {11:1, 12:1}, t5 {4:3}; printMFasta prints '-' per gap.
  kat11_debug_msa - kat6 with -D (:443-446 -> GSeqAlign::print(stderr,'v') GapAssem.cpp:1013-1037 ->
                  printGappedSeq :412-440): ">MSA (4)", a separator of 14 blanks (the "%11s %c " format
                  of " ", ' ': 11 = the longest row name) and 16 'v' (MSA length), then per row the name
                  right-aligned to 11, ' ', '+', ' ', the offset in blanks (all 0) and the gapped row.
  kat13_debug_msa_offsets - -D -w with a self alignment (-D sets verbose: :198-201, :315), a row that
                  starts inside the query (t2, r_alnstart 9) and a '-' row.  Derivation, qa =
                  AACCGGTTAACC:  t1 ":4-tt:8" / 4M2D8M: qa.setGap(4,2), GSeqAlign(qa,t1) length 14.
                  t2 ":3" / 3M at qa 9-12, offset 9: addAlign i=4 d=2 -> omsa.injectGap(rseq,4,2):
                    alpos 4, t2's offset 9 >= 4 so only its offset moves (:733-737) -> 11; addSeq(t2, 11).
                  t3 '-' ":3*ct:8" / 12M on RC = GGTTAACCGGTT, offset 12-12 = 0, tseq GGTcAACCGGTT:
                    i=4 d=2 -> t3.addGap(4,2) (first base at column >= 4).
                  t4 ":8-g:4" / 8M1D4M: rseq.setGap(8,1); i=4 d=2 -> t4.addGap(4,2); i=8 d=-1 ->
                    injectGap(qa,8,1) in refMSA: alpos = 8+2 = 10; qa.addGap(8,1); t1 (no gaps) walks to
                    base 10 -> addGap(10,1); t2's offset 11 >= 10 -> 12; t3 (gap 2 at 4) walks to base 8
                    -> addGap(8,1); length 15; addSeq(t4, 0).
                  print: finalize reverse-complements t3's bases, not its gaps (prepSeq :89-101):
                    AACCGGTTgACC with {4:2, 8:1}; t2 is printed after 12 blanks (offset - minoffset 0),
                    and writeMSA prints those 12 columns as '-'.
  kat14_debug_no_w - -D without -w: verbose messages only (the reference then dereferences the NULL
                  refMSA at :444 — DESIGN.md D7: nothing more is printed here).
  kat12_*       - -v / -c (:217-240): "Max clipping set to 5 bases", "Percentual max clipping set to
                  5%" (iround(100*0.05f) = 5), each before the self-alignment message (:315); without
                  -v neither prints.  -s/-p/-m/-d take a value and are never used (-s's file is never
                  created, :274).  err_clip_*: -c 0 and -c 100% (:220-225), exit 1.
  err_*         - the reference's error messages (format strings copied from the source
                  lines cited in each case), exit code 1, and report lines printed before it.
Each case dir holds: q.fa, in.paf, args.json ({"args": [...], "rc": N}), stdout, stderr.
Run: python3 tests/golden/make_kats.py   (idempotent)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "kat")

CDS = "ATGAAACCCGGGTTTAAACCCGGGTTTTAA"
FA1 = ">cds\n" + CDS + "\n"
G1 = "ATGGCCTGGAAAAAGATCCCTACGGTACTTGCATAA"
FA3 = ">g1 first gene\n" + G1 + "\n>g2\n" + CDS + "\n"

USAGE = (
    "Usage:\n"
    " pafreport <paf_with_cg_cs> -r <refseq.fa> [-s <summary.txt>]\n"
    "    [-o <diff_report.dfa>][-w <outfile.mfa>] [-G|-F|-C|-N]\n"
    "    \n"
    "   <paf_with_cg_cs> is the input PAF file with high quality query sequence(s)\n"
    "      aligned to many target sequences using minimap2 --cs\n"
    "   -r provide the fasta file with query sequence(s) (required)\n"
    "   -o write difference data for each alignment into <diff_report.dfa>\n"
    "   -s write event summary counts into <summary.txt>\n"
    "   -w write MSA as multifasta into <outfile.mfa>\n"
    "   -G gene CDS analysis mode (default for query<100K; assumes -C)\n"
    "   -F full genome alignment mode (default for query>100Kb; assumes -N)\n"
    "   -C perform codon impact analysis\n"
    "   -N skip codon impact analysis\n"
)


def paf(*cols):
    return "\t".join(str(c) for c in cols) + "\n"


K1 = paf("cds", 30, 0, 30, "+", "asm1", 100, 10, 41, 29, 31, 60, "NM:i:2", "AS:i:50", "cg:Z:15M1D15M",
         "cs:Z::4*ga:10-t:15")
K1_OUT = (">asm1:10-41+ coverage:100.00 score=50 edit_distance=2\n"
          "S\t5\t2(K)\tA:G\t5\tATGAgACCCG\tATGAAACCC\t[unknown]\tAA2|K:R\n"
          "I\t16\t6(K)\t:T\t16\tGGTTTtAAACC\tGTTTAAACC\t[unknown]\tpremature stop at AA6\n")

K2 = paf("cds", 30, 0, 30, "-", "asm2", 500, 100, 131, 25, 33, 60, "NM:i:5", "AS:i:40", "cg:Z:9M1I9M2D11M",
         "cs:Z::3*ga:5+g:4*gt*ca:3-aa:11")
K2_OUT = (">asm2:100-131- coverage:100.00 score=40 edit_distance=5\n"
          "I\t12\t4(G)\t:TT\t14\tCCCGGttGTTgc\tCCGGGTTTA\t[unknown]\tframe shift GFKP+:GCLN+\n"
          "S\t15\t5(F)\tTA:GC\t19\ttGTTgcAACCG\tGGTTTAAAC\t[unknown]\tAA5|F:L, AA6|K:Q\n"
          "D\t21\t7(P)\tC:\t23\tcAACCGGGTT\tAACCCGGGT\t[unknown]\tframe shift PGF+:PGF+\n"
          "S\t27\t9(F)\tT:C\t29\tGGGTTcTAA\tGGGTTTTAA\t[unknown]\tsynonymous\n")

K3A = paf("g1", 36, 0, 36, "+", "tA", 1000, 200, 251, 30, 51, 60, "NM:i:19", "AS:i:10",
          "cg:Z:11M1D5M1I7M15D12M", "cs:Z::1*ct:6*ag:2-a:5+t:7-acgtacgtacgtacg:12")
K3 = ("# comment\n" + K3A +
      paf("g1", 36, 0, 36, "+", "g1", 36, 0, 36, 36, 36, 60, "NM:i:0", "AS:i:72", "cg:Z:36M", "cs:Z::36") +
      K3A +
      paf("g2", 30, 0, 30, "+", "tB", 800, 10, 37, 24, 30, 60, "NM:i:3", "AS:i:20", "cg:Z:6M3I21M",
          "cs:Z::6+ccc:21") +
      paf("g2", 30, 10, 25, "+", "tC", 100, 0, 15, 15, 15, 60, "NM:i:0", "AS:i:30", "cg:Z:15M", "cs:Z::15"))
K3_OUT = (">g1--tA:200-251+ coverage:100.00 score=10 edit_distance=19\n"
          "S\t2\t1(M)\tT:C\t2\tAcGGCCT\tATGGCCTGG\tmotif CCTGG\tAA0|M:T\n"
          "S\t9\t3(W)\tG:A\t9\tGCCTGaAAaAA\tCCTGGAAAA\tmotif CCTGG\tAA3|W:.|premature stop at AA3\n"
          "I\t12\t4(K)\t:A\t12\tTGaAAaAAAGA\tGGAAAAAGA\thomopolymer\tframe shift KKIP+:KKDP+\n"
          "D\t17\t6(I)\tT:\t18\tAAAGACCCTA\tAAGATCCCT\tmotif GATC\tframe shift IPTV+:TLRY+\n"
          "I\t25\t9(V)\t:[15]\t25\tCTACG[15]GTACT\tTACGGTACT\tmotif GTAC\tpremature stop at AA17\n"
          ">g2--tB:10-37+ coverage:100.00 score=20 edit_distance=3\n"
          "D\t7\t3(P)\tCCC:\t7\tTGAAAGGGTT\tGAAACCCGG\t[unknown]\tpremature stop at AA9\n"
          ">g2--tC:0-15+ coverage:50.00 score=30 edit_distance=0\n")
K3_ERR = "Warning: alignment g1 to tA already seen, ignoring \n"

K4_OUT = (">cds:0-30--asm1:10-41+ coverage:100.00 score=50 edit_distance=2\n"
          "S\t5\t2(K)\tA:G\t5\tATGAgACCCG\tATGAAACCC\t[unknown]\t\n"
          "I\t16\t6(K)\t:T\t16\tGGTTTtAAACC\tGTTTAAACC\t[unknown]\t\n")


# -w (kat6_msa_w): two queries, qa repeated after qb
QA = "AACCGGTTAACC"
FA6 = ">qa\n" + QA + "\n>qb\nGGGGAAAA\n"
K6 = (paf("qa", 12, 0, 12, "+", "t1", 200, 100, 113, 12, 13, 60, "NM:i:1", "AS:i:10", "cg:Z:6M1D6M", "cs:Z::6-g:6") +
      paf("qb", 8, 0, 8, "+", "t2", 200, 100, 108, 8, 8, 60, "NM:i:0", "AS:i:16", "cg:Z:8M", "cs:Z::8") +
      paf("qa", 12, 0, 12, "+", "t3", 200, 100, 114, 12, 14, 60, "NM:i:2", "AS:i:10", "cg:Z:4M2D8M", "cs:Z::4-tt:8") +
      paf("qa", 12, 0, 12, "+", "t4", 200, 100, 114, 11, 15, 60, "NM:i:4", "AS:i:8", "cg:Z:4M3D4M1I3M",
          "cs:Z::4-ggg:4+a:3") +
      paf("qa", 12, 0, 12, "+", "t5", 200, 100, 113, 12, 13, 60, "NM:i:1", "AS:i:12", "cg:Z:10M1D2M", "cs:Z::10-c:2"))
K6_MSA = (">qa\nAACC---GGTTAA-CC\n"
          ">t3:100-114+\nAACCtt-GGTTAA-CC\n"
          ">t4:100-114+\nAACCgggGGTT-A-CC\n"
          ">t5:100-113+\nAACC---GGTTAAcCC\n")


# kat7_near_start: events at rloc 4..7 (render's fast path since round 4: r_trloc = 3*(aapos-2)
# = 0 or 3, the codon window from the query start, and insertions whose modseq tail starts before
# rloc - 8), forward and reverse.  Derivation (Q = CDS, 0-based):
#  asm7  ':5-gc:25'  I at q 5: tseq = Q[0:5]+gc+Q[5:]; tctx = tseq[0:12] (:120-128); aa = Q[3:6]
#        AAA K, aapos 2 (:893-898); rctx Q[1:10] (:721-733); r_trloc 0, modseq = Q with GC at 5,
#        no stop in ATG AAG CAC CCG GGT TTA AAC CCG GGT TTT -> frame shift aa4 KPGF / maa4 KHPG.
#  asm8  ':6+cc:22'  D at q 6: tctx = tseq[1:11] (evt_len 0); aa = Q[6:9] CCC P, aapos 3; rctx
#        Q[2:11]; r_trloc 3, modseq = Q[3:] cut at 3 len 2 = AAA CGG GTT TAA -> stop at i 9:
#        AA 1+(9+3)/3 = 5.
#  asm9  ':4*ga*ta:24' merged S (:556-560) AA->GT at q 4, evtlen stays 1 so tctx = tseq[0:10];
#        aamods {1}: AAA K -> AGT S, AA 1+4/3 = 2.
#  asm10 ':7-ttt:23' I at q 7: tctx tseq[2:15]; aa Q[6:9] P, aapos 3; rctx Q[3:12]; r_trloc 3,
#        modseq = Q[3:] with TTT at 4 -> AAA CTT TCC GGG TTT AAA CCC GGG TTT TAA: stop at i 27, AA 11.
#  asm11 '-' ':25-ga:5' on RC = revcomp(Q): I at aligned q 25, rloc = 30-25 = 5 (:597), evtbases
#        revcomp(ga) = TC; tctx = tseq[20:31] (tc_end clipped to |tseq|-1) = CGGGTgaTTCA, revcomp
#        TGAAtcACCCG; tloc = 32-25 = 7 (:633); modseq = Q with TC at 5 -> frame shift KPGF / NHPG.
#  asm12 '-' ':21+ggg:6': D of RC[21:24] = GGG -> evtbases CCC, rloc = 30-21-3 = 6 (:615);
#        tctx tseq[16:26] = AACCCTTTCA, revcomp TGAAAGGGTT; tloc 27-21 = 6; modseq = Q[3:] cut at
#        3 len 3 = AAA GGG TTT AAA CCC GGG TTT TAA: stop at i 21, AA 9.
K7 = (paf("cds", 30, 0, 30, "+", "asm7", 100, 10, 42, 30, 32, 60, "NM:i:2", "AS:i:50", "cg:Z:5M2D25M", "cs:Z::5-gc:25")
      + paf("cds", 30, 0, 30, "+", "asm8", 100, 20, 48, 28, 30, 60, "NM:i:2", "AS:i:50", "cg:Z:6M2I22M", "cs:Z::6+cc:22")
      + paf("cds", 30, 0, 30, "+", "asm9", 100, 30, 60, 28, 30, 60, "NM:i:2", "AS:i:50", "cg:Z:30M",
            "cs:Z::4*ga*ta:24")
      + paf("cds", 30, 0, 30, "+", "asm10", 100, 0, 33, 30, 33, 60, "NM:i:3", "AS:i:50", "cg:Z:7M3D23M",
            "cs:Z::7-ttt:23")
      + paf("cds", 30, 0, 30, "-", "asm11", 100, 5, 37, 30, 32, 60, "NM:i:2", "AS:i:50", "cg:Z:25M2D5M",
            "cs:Z::25-ga:5")
      + paf("cds", 30, 0, 30, "-", "asm12", 100, 40, 67, 27, 30, 60, "NM:i:3", "AS:i:40", "cg:Z:21M3I6M",
            "cs:Z::21+ggg:6"))
K7_OUT = (">asm7:10-42+ coverage:100.00 score=50 edit_distance=2\n"
          "I\t6\t2(K)\t:GC\t6\tATGAAgcACCCG\tTGAAACCCG\t[unknown]\tframe shift KPGF+:KHPG+\n"
          ">asm8:20-48+ coverage:100.00 score=50 edit_distance=2\n"
          "D\t7\t3(P)\tCC:\t7\tTGAAACGGGT\tGAAACCCGG\t[unknown]\tpremature stop at AA5\n"
          ">asm9:30-60+ coverage:100.00 score=50 edit_distance=2\n"
          "S\t5\t2(K)\tAA:GT\t5\tATGAgtCCCG\tATGAAACCC\t[unknown]\tAA2|K:S\n"
          ">asm10:0-33+ coverage:100.00 score=50 edit_distance=3\n"
          "I\t8\t3(P)\t:TTT\t8\tGAAACtttCCGGG\tAAACCCGGG\t[unknown]\tpremature stop at AA11\n"
          ">asm11:5-37- coverage:100.00 score=50 edit_distance=2\n"
          "I\t6\t2(K)\t:TC\t8\tTGAAtcACCCG\tTGAAACCCG\t[unknown]\tframe shift KPGF+:NHPG+\n"
          ">asm12:40-67- coverage:100.00 score=40 edit_distance=3\n"
          "D\t7\t3(P)\tCCC:\t7\tTGAAAGGGTT\tGAAACCCGG\t[unknown]\tpremature stop at AA9\n")

# kat8_tctx_walk: four events within 5 target bases of each other, so every target context crosses
# another event (tctx_kernel's op walk, not the query-copy fast form).  asm20 ':10*cg:1-tt:3+aa:2*gc:10'
# tseq = Q[0:10] c G tt TTT AC g Q[20:] (30): S q10 tloc 10, I q12 tloc 12, D q15 tloc 17 (tpos after
# ':3'), S q19 tloc 19 (the D in between: no merge, :556).  tctx (:120-128) = tseq[5:16], [7:19],
# [12:22] (D: evt_len 0), [14:25].  Impacts (:801-883): S q10 r_trloc 6, codon 1 GGG G -> GCG A;
# I q12 r_trloc 9, modseq GGG TT TTTAAA.. -> FKPG / FLNP, no stop; D q15 r_trloc 12, TTT + Q[17:] ->
# KPGF / TRVL; S q19 r_trloc 15, CCC P -> CGC R.
K8 = paf("cds", 30, 0, 30, "+", "asm20", 100, 50, 80, 24, 32, 60, "NM:i:6", "AS:i:30", "cg:Z:12M2D3M2I13M",
         "cs:Z::10*cg:1-tt:3+aa:2*gc:10")
K8_OUT = (">asm20:50-80+ coverage:100.00 score=30 edit_distance=6\n"
          "S\t11\t4(G)\tG:C\t11\tACCCGcGttTT\tCCCGGGTTT\t[unknown]\tAA4|G:A\n"
          "I\t13\t5(F)\t:TT\t13\tCCGcGttTTTAC\tCGGGTTTAA\t[unknown]\tframe shift FKPG+:FLNP+\n"
          "D\t16\t6(K)\tAA:\t18\tttTTTACgCG\tGTTTAAACC\t[unknown]\tframe shift KPGF+:TRVL+\n"
          "S\t20\t7(P)\tC:G\t20\tTTTACgCGGGT\tAAACCCGGG\t[unknown]\tAA7|P:R\n")

# kat9_tctx_walk_reverse: the same pattern on the '-' strand, decoded on RC = revcomp(Q)
# (:361-363): asm21 ':8*tc:2-gg:3+ta:3*ac:10', tseq = RC[0:8] t GG gg GTT AAC a RC[20:] (30).
# Aligned events S q8 t8, I q11 t11, D q14 t16, S q19 t19; tctx = tseq[3:14], [6:18], [11:21],
# [14:25], each reverse-complemented (:631), tloc = 30 - tloc (:633); S flipped after the contexts
# (:634-640): rloc 30-8-1 = 21 and 30-19-1 = 10; I rloc 30-11 = 19 (:597), D 30-14-2 = 14
# (:615); tdiffs reversed (:643).  Impacts on Q: S q10 G->T (GGG G -> GTG V, AA4); D q14 TA,
# r_trloc 9 -> FKPG / LTRV; I q19 CC, r_trloc 15: aa4 ends in TAA = '.', modseq has no stop ->
# frame shift PGF. / PPGF; S q21 G->A (GGG G -> AGG R, AA8).
K9 = paf("cds", 30, 0, 30, "-", "asm21", 100, 60, 90, 24, 32, 60, "NM:i:6", "AS:i:30", "cg:Z:11M2D3M2I14M",
         "cs:Z::8*tc:2-gg:3+ta:3*ac:10")
K9_OUT = (">asm21:60-90- coverage:100.00 score=30 edit_distance=6\n"
          "S\t11\t4(G)\tG:T\t12\tACCCGtGTTAA\tCCCGGGTTT\t[unknown]\tAA4|G:V\n"
          "D\t15\t5(F)\tTA:\t15\tGtGTTAACcc\tGGTTTAAAC\t[unknown]\tframe shift FKPG+:LTRV+\n"
          "I\t20\t7(P)\t:CC\t20\tTTAACccCCaGG\tAAACCCGGG\t[unknown]\tframe shift PGF.+:PPGF+\n"
          "S\t22\t8(G)\tG:A\t23\tCccCCaGGTTT\tACCCGGGTT\t[unknown]\tAA8|G:R\n")

# kat10_general: events outside render's fast path (emit_event's general instantiation).
#  asm30 ':3*ta*ga*ga*tc*ac*ac:21' an S run of 6 (merged, :556-560; evtlen stays 1 so tctx =
#        tseq[0:9]); rctx clipped at the query start (ctxstart -1 -> 0, :724); aamods {1, 2}:
#        AAA K -> TGG W, CCC P -> TAA '.' (:826-837): "AA2|K:W, AA3|P:.|premature stop at AA3".
#  asm31 ':9-acgtacgtac:21' a 10-base insertion: tctx tseq[4:24] (20 <= 22, not abbreviated);
#        r_trloc 6, modseq CCC ACG TAC GTA CGG GTT TAA -> stop at i 18, AA 1+(18+6)/3 = 9.
#  asm32 ':10+ggtttaaacccgg:7' a 13-base deletion: evtbases "[13]" (> MAX_EVLEN, :936-941),
#        tctx tseq[5:15]; r_trloc 6, modseq CCCG + GTTTTAA: GGT G, TTT F, no stop -> GF / GF.
K10 = (paf("cds", 30, 0, 30, "+", "asm30", 100, 0, 30, 24, 30, 60, "NM:i:6", "AS:i:20", "cg:Z:30M",
           "cs:Z::3*ta*ga*ga*tc*ac*ac:21")
       + paf("cds", 30, 0, 30, "+", "asm31", 100, 10, 50, 30, 40, 60, "NM:i:10", "AS:i:20", "cg:Z:9M10D21M",
             "cs:Z::9-acgtacgtac:21")
       + paf("cds", 30, 0, 30, "+", "asm32", 100, 20, 37, 17, 30, 60, "NM:i:13", "AS:i:10", "cg:Z:10M13I7M",
             "cs:Z::10+ggtttaaacccgg:7"))
K10_OUT = (">asm30:0-30+ coverage:100.00 score=20 edit_distance=6\n"
           "S\t4\t2(K)\tAAACCC:TGGTAA\t4\tATGtggtaa\tATGAAACCC\t[unknown]\tAA2|K:W, AA3|P:.|premature stop at AA3\n"
           ">asm31:10-50+ coverage:100.00 score=20 edit_distance=10\n"
           "I\t10\t4(G)\t:ACGTACGTAC\t10\tAACCCacgtacgtacGGGTT\tACCCGGGTT\t[unknown]\tpremature stop at AA9\n"
           ">asm32:20-37+ coverage:100.00 score=10 edit_distance=13\n"
           "D\t11\t4(G)\t[13]:\t11\tACCCGGTTTT\tCCCGGGTTT\t[unknown]\tframe shift GF+:GF+\n")


# kat13_debug_msa_offsets (derivation in the module docstring)
SELF_QA = paf("qa", 12, 0, 12, "+", "qa", 12, 0, 12, 12, 12, 60, "NM:i:0", "AS:i:24", "cg:Z:12M", "cs:Z::12")
K13 = (SELF_QA +
       paf("qa", 12, 0, 12, "+", "t1", 200, 100, 114, 12, 14, 60, "NM:i:2", "AS:i:10", "cg:Z:4M2D8M", "cs:Z::4-tt:8") +
       paf("qa", 12, 9, 12, "+", "t2", 100, 50, 53, 3, 3, 60, "NM:i:0", "AS:i:6", "cg:Z:3M", "cs:Z::3") +
       paf("qa", 12, 0, 12, "-", "t3", 300, 200, 212, 11, 12, 60, "NM:i:1", "AS:i:20", "cg:Z:12M", "cs:Z::3*ct:8") +
       paf("qa", 12, 0, 12, "+", "t4", 400, 300, 313, 12, 13, 60, "NM:i:1", "AS:i:20", "cg:Z:8M1D4M", "cs:Z::8-g:4"))
K13_MSA = (">qa\nAACC--GGTT-AACC\n"
           ">t1:100-114+\nAACCttGGTT-AACC\n"
           ">t2:50-53+\n------------ACC\n"
           ">t3:200-212-\nAACC--GGTT-gACC\n"
           ">t4:300-313+\nAACC--GGTTgAACC\n")
K13_ERR = ("Skipping alignment of qry seq to itself.\n"
           ">MSA (5)\n" +
           " " * 14 + "v" * 15 + "\n"
           "         qa + AACC--GGTT-AACC\n"
           "t1:100-114+ + AACCttGGTT-AACC\n"
           "  t2:50-53+ + " + " " * 12 + "ACC\n"
           "t3:200-212- - AACC--GGTT-gACC\n"
           "t4:300-313+ + AACC--GGTTgAACC\n")
K11_ERR = (">MSA (4)\n" +
           " " * 14 + "v" * 16 + "\n"
           "         qa + AACC---GGTTAA-CC\n"
           "t3:100-114+ + AACCtt-GGTTAA-CC\n"
           "t4:100-114+ + AACCgggGGTT-A-CC\n"
           "t5:100-113+ + AACC---GGTTAAcCC\n")

# kat12_*: -v / -c with a self alignment of the query first
SELF_CDS = paf("cds", 30, 0, 30, "+", "cds", 30, 0, 30, 30, 30, 60, "NM:i:0", "AS:i:60", "cg:Z:30M", "cs:Z::30")
SKIP_MSG = "Skipping alignment of qry seq to itself.\n"
CLIP_PCT_ERR = "Error: invalid percent value (100) for -c option  (must be an integer between 1 and 99)!\n"


def line(s):
    return s.rstrip("\n")


CASES = {
    "kat1_forward": (FA1, K1, ["-r", "q.fa", "in.paf"], 0, K1_OUT, ""),
    "kat1_outfile": (FA1, K1, ["in.paf", "-r", "q.fa", "-o", "out.txt"], 0, "", ""),
    "kat2_reverse": (FA1, K2, ["-r", "q.fa", "in.paf"], 0, K2_OUT, ""),
    "kat3_status": (FA3, K3, ["-r", "q.fa", "in.paf"], 0, K3_OUT, K3_ERR),
    "kat4_fullgenome": (FA1, K1, ["-F", "-r", "q.fa", "in.paf"], 0, K4_OUT, ""),
    "kat7_near_start": (FA1, K7, ["-r", "q.fa", "in.paf"], 0, K7_OUT, ""),
    "kat8_tctx_walk": (FA1, K8, ["-r", "q.fa", "in.paf"], 0, K8_OUT, ""),
    "kat9_tctx_walk_reverse": (FA1, K9, ["-r", "q.fa", "in.paf"], 0, K9_OUT, ""),
    "kat10_general": (FA1, K10, ["-r", "q.fa", "in.paf"], 0, K10_OUT, ""),
    "kat6_msa_w": (FA6, K6, ["-o", "rep.txt", "-w", "msa.mfa", "-r", "q.fa", "in.paf"], 0, "", ""),
    "kat11_debug_msa": (FA6, K6, ["-D", "-o", "rep.txt", "-w", "msa.mfa", "-r", "q.fa", "in.paf"], 0, "", K11_ERR),
    "kat13_debug_msa_offsets": (FA6, K13, ["-o", "rep.txt", "-D", "-w", "msa.mfa", "-r", "q.fa", "in.paf"], 0, "",
                                K13_ERR),
    "kat14_debug_no_w": (FA3, K3, ["-D", "-r", "q.fa", "in.paf"], 0, K3_OUT, SKIP_MSG + K3_ERR),
    "kat12_verbose_c": (FA1, SELF_CDS + K1, ["-v", "-c", "5", "-r", "q.fa", "in.paf"], 0, K1_OUT,
                        "Max clipping set to 5 bases\n" + SKIP_MSG),
    "kat12_verbose_cpct": (FA1, SELF_CDS + K1, ["-v", "-c5%", "-r", "q.fa", "in.paf"], 0, K1_OUT,
                           "Percentual max clipping set to 5%\n" + SKIP_MSG),
    "kat12_quiet_unused_opts": (FA1, SELF_CDS + K1, ["-c", "7", "-s", "sum.txt", "-p", "x", "-m", "y", "-d", "z",
                                                     "-r", "q.fa", "in.paf"], 0, K1_OUT, ""),
    "err_clip_zero": (FA1, K1, ["-c", "0", "-r", "q.fa", "in.paf"], 1, "",
                      "Error: invalid -c <clipmax> (0) option provided (must be a positive integer)!\n"),
    "err_clip_pct": (FA1, K1, ["-v", "-c", "100%", "-r", "q.fa", "in.paf"], 1, "", CLIP_PCT_ERR),
    "kat5_noncoding": (FA1, K1, ["-N", "-r", "q.fa", "in.paf"], 0,
                       K4_OUT.replace(">cds:0-30--asm1", ">asm1"), ""),
    # pafreport.cpp:551-553 base check; records before the failing one are already reported
    "err_mismatch": (FA1, K1 + K1.replace("asm1", "asm9").replace("*ga", "*gc"), ["-r", "q.fa", "in.paf"], 1,
                     K1_OUT,
                     "Error: base mismatch C != qstr[4] (A) at line\n" +
                     line(K1.replace("asm1", "asm9").replace("*ga", "*gc")) + "\n"),
    # :620-622
    "err_spliced": (FA1, K1.replace(":4*ga:10-t:15", ":4~gt10ag:26"), ["-r", "q.fa", "in.paf"], 1, "",
                    "Error: spliced alignments not supported! at line:\n" +
                    line(K1.replace(":4*ga:10-t:15", ":4~gt10ag:26")) + "\n"),
    # :542 CS_ERROR (:474) with the cs position string
    "err_cs_parse": (FA1, K1.replace(":4*ga:10-t:15", ":4*ga:x10-t:15"), ["-r", "q.fa", "in.paf"], 1, "",
                     "Error parsing cs string from line: " + line(K1.replace(":4*ga:10-t:15", ":4*ga:x10-t:15")) +
                     " (cs position: x10-t:15)\n"),
    # :623-624
    "err_cs_op": (FA1, K1.replace(":4*ga:10-t:15", ":4*ga:10=t:15"), ["-r", "q.fa", "in.paf"], 1, "",
                  "Error: unhandled event at t:15 in cs, line:\n" +
                  line(K1.replace(":4*ga:10-t:15", ":4*ga:10=t:15")) + "\n"),
    # :715-716
    "err_tlen": (FA1, K1.replace("\t10\t41\t", "\t10\t42\t"), ["-r", "q.fa", "in.paf"], 1, "",
                 "Error: tseq alignment length mismatch (31 vs 32(42-10)) at line:" +
                 line(K1.replace("\t10\t41\t", "\t10\t42\t")) + "\n"),
    # :717-718 (cs/CIGAR consistent, PAF query span not)
    "err_qlen": (FA1, K1.replace("cds\t30\t0\t30", "cds\t30\t0\t29"), ["-r", "q.fa", "in.paf"], 1, "",
                 "Error: ref alignment length mismatch (30 vs 29-0) at line:" +
                 line(K1.replace("cds\t30\t0\t30", "cds\t30\t0\t29")) + "\n"),
    # :308-309
    "err_fields": (FA1, K1 + "cds\t30\t0\t30\t+\n", ["-r", "q.fa", "in.paf"], 1, K1_OUT,
                   "Error: invalid PAF fline (num. fields=5):\ncds\t30\t0\t30\t+\n"),
    # :356-358
    "err_rlen": (FA1, K1.replace("cds\t30\t", "cds\t31\t"), ["-r", "q.fa", "in.paf"], 1, "",
                 "Error: ref seq len in this PAF line (31) differs from loaded sequence length(30)!\n" +
                 line(K1.replace("cds\t30\t", "cds\t31\t")) + "\n"),
    # :347
    "err_noquery": (FA1, K1.replace("cds\t", "cdsX\t", 1), ["-r", "q.fa", "in.paf"], 1, "",
                    "Error: could not retrieve sequence for cdsX !\n"),
    # :711
    "err_cigar_op": (FA1, K1.replace("15M1D15M", "15M1Z15M"), ["-r", "q.fa", "in.paf"], 1, "",
                     "Error: unhandled cigar_op Z (len 1) in " + line(K1.replace("15M1D15M", "15M1Z15M")) + "\n"),
    # :521 with a NULL position string
    "err_nocigar": (FA1, K1.replace("cg:Z:15M1D15M", "xx:Z:15M1D15M"), ["-r", "q.fa", "in.paf"], 1, "",
                    "Error parsing cigar string from line: " + line(K1.replace("cg:Z:15M1D15M", "xx:Z:15M1D15M")) +
                    " (cigar position: (null))\n"),
    # :675-679 soft clip warning, then the report
    "warn_softclip": (FA1, K1.replace("cg:Z:15M1D15M", "cg:Z:2S13M3D15M"), ["-r", "q.fa", "in.paf"], 0,
                      K1_OUT, "Warning: soft clipping shouldn't be found in this application!\n" +
                      line(K1.replace("cg:Z:15M1D15M", "cg:Z:2S13M3D15M")) + "\n"),
    # CLI (:177-197, 251-252)
    "cli_no_r": (FA1, K1, ["in.paf"], 1, "", "Error: query FASTA file (-r) is required!\n"),
    "cli_G_F": (FA1, K1, ["-G", "-F", "-r", "q.fa", "in.paf"], 1, "", USAGE + " Error: cannot use both -G and -F!\n"),
    "cli_C_N": (FA1, K1, ["-C", "-N", "-r", "q.fa", "in.paf"], 1, "", USAGE + " Error: cannot use both -N and -C!\n"),
    "cli_bad_opt": (FA1, K1, ["-h", "-r", "q.fa", "in.paf"], 1, "", USAGE + "\nInvalid argument: -h\n"),
}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, (fa, pafs, args, rc, out, err) in CASES.items():
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "q.fa"), "w") as f:
            f.write(fa)
        with open(os.path.join(d, "in.paf"), "w") as f:
            f.write(pafs)
        spec = {"args": args, "rc": rc}
        if name == "kat1_outfile":
            spec["outfile"] = "out.txt"
            spec["outfile_expected"] = K1_OUT
        if name in ("kat6_msa_w", "kat11_debug_msa"):
            spec["outfile"] = "msa.mfa"
            spec["outfile_expected"] = K6_MSA
        if name == "kat13_debug_msa_offsets":
            spec["outfile"] = "msa.mfa"
            spec["outfile_expected"] = K13_MSA
        if name == "kat12_quiet_unused_opts":
            spec["absent"] = ["sum.txt", "x", "y", "z"]
        with open(os.path.join(d, "args.json"), "w") as f:
            json.dump(spec, f, indent=1)
        with open(os.path.join(d, "stdout"), "w") as f:
            f.write(out)
        with open(os.path.join(d, "stderr"), "w") as f:
            f.write(err)
    print(f"wrote {len(CASES)} cases to {OUT}")


if __name__ == "__main__":
    main()
