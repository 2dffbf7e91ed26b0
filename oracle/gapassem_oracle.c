/*
 * gapassem_oracle.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Plain-C restatement of the GapAssem column-consensus path of gpertea/pwasm:
 *   GSeqAlign(s1,s2)/addSeq          GapAssem.cpp:605-641, 694-716
 *   GSeqAlign::buildMSA              GapAssem.cpp:1088-1106
 *   GASeq::toMSA                     GapAssem.cpp:551-591
 *   GAlnColumn::addGap/addNuc        GapAssem.h:295-337
 *   GAlnColumn::bestChar + qsortnuc  GapAssem.cpp:1048-1069, 9-13
 *   GSeqAlign::refineMSA             GapAssem.cpp:1133-1183
 *   GSeqAlign::removeColumn          GapAssem.cpp:755-779
 *   GASeq::removeBase/removeClipGaps GapAssem.cpp:122-131, 522-549
 *   GSeqAlign::extendConsensus       GapAssem.cpp:1185-1198
 *   GASeq::refineClipping (X-drop)   GapAssem.cpp:182-349
 * It is literal (per-base scatter, qsort per column, O(rows*L) per removed column, the whole
 * gapped row rebuilt per refineClipping call), so only small layouts are practical.
 * Reads the reference makes outside its buffers (refineClipping's cons[cp] / gseq[sp] with an
 * index out of range — undefined there) read 0 here, and refineClipping with an empty consensus
 * (the reference dereferences its NULL consensus) changes nothing.
 *
 * PARITY STATUS: the reference cannot be built here (gclib absent); this restatement is
 * pinned by hand-derived known-answer layouts in tests/golden/ (parity otherwise unpinned).
 *
 *   GSeqAlign::writeACE / writeInfo  GapAssem.cpp:1200-1262, 1264-1367
 *   GSeqAlign::writeMSA (+finalize)  GapAssem.cpp:1039-1046, 1006-1012, 482-520, 89-101
 *   FastaSeq::write(f,NULL,NULL,s,60) gclib GFastaFile.h (absent here: its line layout — 60 per
 *                                    line, a newline after the last — is parity unpinned)
 * Usage: gapassem_oracle <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping]
 *                        [--ace F] [--info F] [--msa F]   (contig name "contig1")
 * Layout / result formats: tests/pwl_format.md.
 */
#include <ctype.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  char id[32];
  int offset, seqlen, clp5, clp3, numgaps;
  int revcompl;
  char* seq;
  short* ofs;
} row_t;

typedef struct {
  int cnt[6]; /* A C G T N - : GapAssem.h:263 order */
  int layers;
  int has_clip;
  char consensus;
} column_t;

static int g_remove_gaps = 0, g_refine_clip = 1;

/* GASeq::refineClipping (GapAssem.cpp:182-349), literal; clipL / clipR are the row's clp5 /
 * clp3 by orientation and are updated in place (also on the early "Warning" returns). */
static char at_c(const char* b, int n, int i) { return (i >= 0 && i < n) ? b[i] : 0; }
static void refine_clipping(row_t* s, const char* cons, int cons_len, int cpos, int skip_dels) {
  if (s->clp3 == 0 && s->clp5 == 0) return;
  if (cons_len == 0) return; /* no consensus: the reference reads through a NULL pointer (D11) */
  int* clipL = s->revcompl ? &s->clp3 : &s->clp5;
  int* clipR = s->revcompl ? &s->clp5 : &s->clp3;
  int seqlen = s->seqlen;
  int glen = seqlen + s->numgaps, allocsize = glen, gclipR = *clipR, gclipL = *clipL;
#define OFS(i) (((i) >= 0 && (i) < seqlen) ? s->ofs[(i)] : 0)
  if (skip_dels) {
    for (int i = 1; i <= *clipR; i++) {
      if (OFS(seqlen - i) < 0) allocsize++;
      else gclipR += OFS(seqlen - i);
    }
    for (int i = 0; i < *clipL; i++) {
      if (OFS(i) < 0) allocsize++;
      else gclipL += OFS(i);
    }
  } else {
    for (int i = 1; i <= *clipR; i++) gclipR += OFS(seqlen - i);
    for (int i = 0; i < *clipL; i++) gclipL += OFS(i);
  }
  int cap = allocsize > 0 ? allocsize : 0;
  int* gxpos = (int*)calloc((size_t)cap + 1, sizeof(int));
  char* gseq = (char*)calloc((size_t)cap + 1, 1);
  int gseqpos = 0;
  for (int i = 0; i < seqlen; i++) {
    if (s->ofs[i] < 0) {
      if (!skip_dels) continue;
      if (i >= *clipL && i < seqlen - *clipR) continue;
      glen++;
    }
    for (int j = 0; j < s->ofs[i]; j++) {
      if (gseqpos < cap) gseq[gseqpos] = '*';
      gseqpos++;
    }
    if (gseqpos < cap) {
      gseq[gseqpos] = s->seq[i];
      gxpos[gseqpos] = i;
    }
    gseqpos++;
  }
  if (glen != allocsize) {
    fprintf(stderr, "Length mismatch (allocsize %d vs. glen %d) while refineClipping for seq %s !\n", allocsize, glen,
            s->id);
    exit(1);
  }
#undef OFS
#define G(i) at_c(gseq, cap, (i))
#define C(i) at_c(cons, cons_len, (i))
  if (*clipR > 0) {
    int cp = cpos + glen - gclipR - 1, sp = glen - gclipR - 1;
    while (G(sp) != C(cp) || G(sp) == '*') {
      if (G(sp) != '*') (*clipR)++;
      sp--;
      cp--;
      if (sp < gclipL) {
        fprintf(stderr, "Warning: reached clipL trying to find an initial match on %s!\n", s->id);
        free(gseq);
        free(gxpos);
        return;
      }
    }
    int score = 1, maxscore = 1, startpos = sp, bestpos = sp;
    while (score > -16 && ++cp < cons_len && ++sp < glen) {
      if (G(sp) == C(cp)) {
        if (G(sp) != '*') {
          score += 1;
          if (score > maxscore) {
            bestpos = sp;
            maxscore = score;
          }
        }
      } else if (G(sp) != '*') {
        score += -3;
      }
    }
    if (bestpos > startpos) *clipR = seqlen - gxpos[bestpos] - 1;
  }
  if (*clipL > 0) {
    int cp = cpos + gclipL, sp = gclipL;
    while (G(sp) != C(cp) || G(sp) == '*') {
      if (G(sp) != '*') (*clipL)++;
      sp++;
      cp++;
      if (sp >= glen - gclipR) {
        fprintf(stderr, "Warning: reached clipR trying to find an initial match on %s!\n", s->id);
        free(gseq);
        free(gxpos);
        return;
      }
    }
    int score = 1, maxscore = 1, startpos = sp, bestpos = sp;
    while (score > -16 && --cp >= 0 && --sp >= 0) {
      if (G(sp) == C(cp)) {
        if (G(sp) != '*') {
          score += 1;
          if (score > maxscore) {
            bestpos = sp;
            maxscore = score;
          }
        }
      } else if (G(sp) != '*') {
        score += -3;
      }
    }
    if (bestpos < startpos) *clipL = gxpos[bestpos];
  }
#undef G
#undef C
  free(gseq);
  free(gxpos);
}

/* GASeq::removeClipGaps (GapAssem.cpp:522-549) */
static int remove_clip_gaps(row_t* s) {
  int clipL = s->revcompl ? s->clp3 : s->clp5;
  int clipR = s->revcompl ? s->clp5 : s->clp3;
  int dl = 0, dr = 0;
  for (int k = 0; k < s->seqlen; k++) {
    if (k <= clipL) {
      dl += s->ofs[k];
      s->ofs[k] = 0;
      continue;
    }
    if (k >= s->seqlen - clipR) {
      dr += s->ofs[k];
      s->ofs[k] = 0;
    }
  }
  s->offset += dl;
  s->numgaps -= (dl + dr);
  return dl + dr;
}

static void die(int code, const char* msg) {
  fputs(msg, stderr);
  exit(code);
}

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

/* GAlnColumn::addNuc (GapAssem.h:299-337) */
static void add_nuc(column_t* c, char b, int clipped) {
  if (clipped) {
    c->has_clip = 1;
    return;
  }
  switch (toupper((unsigned char)b)) {
    case 'A': c->cnt[0]++; break;
    case 'C': c->cnt[1]++; break;
    case 'G': c->cnt[2]++; break;
    case 'T': c->cnt[3]++; break;
    case '-':
    case '*': c->cnt[5]++; break;
    default: c->cnt[4]++;
  }
  c->layers++;
}

typedef struct {
  char c;
  int count;
} nuc_count;
static int qsortnuc(const void* p1, const void* p2) {
  const nuc_count* a = (const nuc_count*)p1;
  const nuc_count* b = (const nuc_count*)p2;
  return (a->count > b->count) ? -1 : ((a->count < b->count) ? 1 : 0);
}

/* GAlnColumn::bestChar (GapAssem.cpp:1048-1069); glibc qsort of 6 elements is stable */
static char best_char(column_t* c) {
  if (c->layers == 0) return 0;
  if (c->consensus) return c->consensus;
  nuc_count v[6] = {{'A', c->cnt[0]}, {'C', c->cnt[1]}, {'G', c->cnt[2]},
                    {'T', c->cnt[3]}, {'N', c->cnt[4]}, {'-', c->cnt[5]}};
  qsort(v, 6, sizeof(nuc_count), qsortnuc);
  int r = 0;
  char best = v[0].c;
  while ((best == '-' || best == 'N') && r + 1 < 6 && v[r].count == v[r + 1].count) {
    r++;
    best = v[r].c;
  }
  c->consensus = best;
  return best;
}

static const char* g_ace = NULL;
static const char* g_info = NULL;
static const char* g_msa = NULL;

static char comp_base(char c) { /* gclib ntComplement over the IUPAC pairs, identity otherwise */
  static const char* from = "AaCcTtGgUuMmRrWwSsYyKkVvHhDdBbNnXx-*";
  static const char* to = "TtGgAaCcAaKkYyWwSsRrMmBbDdHhVvNnXx-*";
  const char* p = strchr(from, c);
  return (c && p) ? to[p - from] : c;
}

/* GSeqAlign::writeACE (GapAssem.cpp:1200-1262); printGappedFasta :442-480 */
static void write_ace(FILE* f, const char* name, row_t* rows, uint32_t n, const char* cons, int cons_len,
                      int minoffset, int mincol) {
  int fwd = 0, rvs = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (rows[i].revcompl) rvs++;
    else fwd++;
  }
  fprintf(f, "CO %s %d %d 0 %c\n", name, cons_len, (int)n, rvs > fwd ? 'C' : 'U');
  for (int i = 0; i < cons_len; i++) { /* FastaSeq::write, 60 per line */
    if (i > 0 && i % 60 == 0) fputc('\n', f);
    fputc(cons[i], f);
  }
  fputc('\n', f);
  fprintf(f, "\nBQ \n\n");
  for (uint32_t i = 0; i < n; i++)
    fprintf(f, "AF %s %c %d\n", rows[i].id, rows[i].revcompl == 0 ? 'U' : 'C',
            (int)((unsigned)rows[i].offset - (unsigned)minoffset - (unsigned)mincol) + 1);
  fprintf(f, "\n");
  for (uint32_t i = 0; i < n; i++) {
    row_t* s = &rows[i];
    int gapped_len = s->seqlen + s->numgaps;
    fprintf(f, "RD %s %d 0 0\n", s->id, gapped_len);
    int printed = 0;
    for (int k = 0; k < s->seqlen; k++) {
      if (s->ofs[k] < 0) continue;
      for (int j = 0; j < s->ofs[k]; j++) {
        fputc('*', f);
        if (++printed == 60) {
          fputc('\n', f);
          printed = 0;
        }
      }
      fputc(s->seq[k], f);
      if (++printed == 60) {
        fputc('\n', f);
        printed = 0;
      }
    }
    if (printed < 60) fputc('\n', f);
    int clpl = s->revcompl == 0 ? s->clp5 : s->clp3, clpr = s->revcompl == 0 ? s->clp3 : s->clp5;
    int l = clpl, r = clpr;
    for (int j = 1; j <= r; j++) clpr += (s->seqlen - j >= 0) ? s->ofs[s->seqlen - j] : 0;
    for (int j = 0; j <= l; j++) clpl += (j < s->seqlen) ? s->ofs[j] : 0;
    int seql = clpl + 1, seqr = gapped_len - clpr;
    if (seqr < seql) {
      fprintf(stderr, "Bad trimming for %s of gapped len %d (%d, %d)\n", s->id, gapped_len, seql, seqr);
      seqr = seql + 1;
    }
    fprintf(f, "\nQA %d %d %d %d\nDS \n\n", seql, seqr, seql, seqr);
  }
}

/* GSeqAlign::writeInfo (GapAssem.cpp:1264-1367) */
static void write_info(FILE* f, const char* name, row_t* rows, uint32_t n, const char* cons, int cons_len,
                       int minoffset, int mincol) {
  fprintf(f, ">%s %d %s\n", name, (int)n, cons);
  for (uint32_t i = 0; i < n; i++) {
    row_t* s = &rows[i];
    char alndata[1 << 16];
    size_t an = 0;
    alndata[0] = 0;
    int gapped_len = s->seqlen + s->numgaps;
    int seqoffset = (int)((unsigned)s->offset - (unsigned)minoffset - (unsigned)mincol) + 1;
    int asml = seqoffset + 1, asmr = asml - 1;
    float pid = 0;
    int clpl = s->revcompl == 0 ? s->clp5 : s->clp3, clpr = s->revcompl == 0 ? s->clp3 : s->clp5;
    int aligned_len = 0, indel_ofs = 0;
    for (int j = s->clp5; j < s->seqlen - s->clp3; j++) {
      int indel = j >= 0 ? s->ofs[j] : 0;
      char indel_type = 0;
      asmr += indel + 1;
      if (indel < 0) {
        indel_type = 'd';
        indel = -indel;
      } else {
        if (indel > 0) indel_type = 'g';
        else indel_ofs++;
        char cc = (asmr - 1 >= 0 && asmr - 1 < cons_len) ? cons[asmr - 1] : 0;
        if (j >= 0 && toupper((unsigned char)s->seq[j]) == toupper((unsigned char)cc)) pid++;
        aligned_len++;
      }
      if (indel_type) {
        if (indel > 2) {
          if (an < sizeof alndata - 40) an += (size_t)snprintf(alndata + an, 40, "%d%c%d-", indel_ofs, indel_type, indel);
        } else {
          for (int q = 0; q < indel && an < sizeof alndata - 2; q++) alndata[an++] = indel_type;
          alndata[an] = 0;
        }
        indel_ofs = 0;
      }
    }
    pid = aligned_len ? (pid * 100.0f) / (float)aligned_len : -__builtin_nanf(""); /* x86 0/0: "-nan" */
    int seql = clpl + 1, seqr = s->seqlen - clpr;
    if (seqr < seql) {
      fprintf(stderr, "WARNING: Bad trimming for %s of gapped len %d (%d, %d)\n", s->id, gapped_len, seql, seqr);
      seqr = seql + 1;
    }
    if (s->revcompl) {
      int t = seqr;
      seqr = seql;
      seql = t;
    }
    fprintf(f, "%s %d %d %d %d %d %d %4.2f %s\n", s->id, s->seqlen, seqoffset, asml, asmr, seql, seqr, pid, alndata);
  }
}

/* GSeqAlign::writeMSA: finalize (prepSeq: reverse-complement revcompl rows) + printMFasta */
static void write_msa(FILE* f, row_t* rows, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    row_t* s = &rows[i];
    if (s->revcompl == 1) {
      for (int a = 0, b = s->seqlen - 1; a < b; a++, b--) {
        char t = s->seq[a];
        s->seq[a] = s->seq[b];
        s->seq[b] = t;
      }
      for (int k = 0; k < s->seqlen; k++) s->seq[k] = comp_base(s->seq[k]);
    }
    fprintf(f, ">%s\n", s->id);
    int printed = 0;
    for (int k = 0; k < s->offset; k++) {
      fputc('-', f);
      if (++printed == 60) {
        fputc('\n', f);
        printed = 0;
      }
    }
    for (int k = 0; k < s->seqlen; k++) {
      if (s->ofs[k] < 0) continue;
      for (int j = 0; j < s->ofs[k]; j++) {
        fputc('-', f);
        if (++printed == 60) {
          fputc('\n', f);
          printed = 0;
        }
      }
      fputc(s->seq[k], f);
      if (++printed == 60) {
        fputc('\n', f);
        printed = 0;
      }
    }
    if (printed < 60) fputc('\n', f);
  }
}

int main(int argc, char** argv) {
  if (argc < 3) die(2, "usage: gapassem_oracle <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping]\n");
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--remove-gaps")) g_remove_gaps = 1;
    else if (!strcmp(argv[i], "--no-refine-clipping")) g_refine_clip = 0;
    else if (!strcmp(argv[i], "--ace") && i + 1 < argc) g_ace = argv[++i];
    else if (!strcmp(argv[i], "--info") && i + 1 < argc) g_info = argv[++i];
    else if (!strcmp(argv[i], "--msa") && i + 1 < argc) g_msa = argv[++i];
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) die(2, "cannot open layout\n");
  char magic[4];
  uint32_t nrows;
  if (!rd(f, magic, 4) || memcmp(magic, "PWL1", 4) || !rd(f, &nrows, 4)) die(2, "bad layout header\n");
  row_t* rows = (row_t*)calloc(nrows ? nrows : 1, sizeof(row_t));
  for (uint32_t i = 0; i < nrows; i++) {
    int32_t h[5];
    if (!rd(f, h, sizeof h)) die(2, "bad row header\n");
    row_t* r = &rows[i];
    snprintf(r->id, sizeof r->id, "row%u", i);
    r->offset = h[0];
    r->seqlen = h[1];
    r->clp5 = h[2];
    r->clp3 = h[3];
    r->revcompl = h[4];
    r->seq = (char*)malloc((size_t)r->seqlen + 1);
    r->ofs = (short*)malloc(sizeof(short) * ((size_t)r->seqlen + 1));
    if (!rd(f, r->seq, (size_t)r->seqlen) || !rd(f, r->ofs, sizeof(short) * (size_t)r->seqlen))
      die(2, "truncated row\n");
    r->seq[r->seqlen] = 0;
    r->numgaps = 0;
    for (int k = 0; k < r->seqlen; k++) r->numgaps += r->ofs[k]; /* setGap bookkeeping */
  }
  fclose(f);
  if (nrows == 0) die(2, "empty layout\n");
  /* GSeqAlign(s1,s2) + addSeq: minoffset / length bookkeeping */
  int minoffset = INT_MAX, maxend = INT_MIN;
  for (uint32_t i = 0; i < nrows; i++) {
    if (rows[i].offset < minoffset) minoffset = rows[i].offset;
    int e = rows[i].offset + rows[i].seqlen + rows[i].numgaps; /* endOffset() */
    if (e > maxend) maxend = e;
  }
  int length = maxend - minoffset;
  if (length < 0) length = 0;
  /* buildMSA */
  column_t* cols = (column_t*)calloc((size_t)length + 1, sizeof(column_t));
  int mincol = INT_MAX, maxcol = 0;
  for (uint32_t i = 0; i < nrows; i++) {
    row_t* s = &rows[i];
    if (s->seqlen - s->clp3 - s->clp5 < 1)
      fprintf(stderr,
              "Warning: sequence %s (length %d) was trimmed too badly (%d,%d) -- should be removed from MSA w/ %s!\n",
              s->id, s->seqlen, s->clp5, s->clp3, rows[0].id);
    int clipL = s->revcompl ? s->clp3 : s->clp5;
    int clipR = s->revcompl ? s->clp5 : s->clp3;
    int rmin = INT_MAX, rmax = 0;
    int col = s->offset - minoffset;
    for (int k = 0; k < s->seqlen; k++) {
      int clipped = (k < clipL || k >= s->seqlen - clipR);
      if (!clipped && rmin == INT_MAX) rmin = col;
      for (int j = 0; j < s->ofs[k]; j++) {
        if (!clipped) {
          if (col < 0 || col >= length) {
            fprintf(stderr, "MSAColumns op[]: bad index %d (size=%d)\n", col, length);
            exit(1);
          }
          cols[col].cnt[5]++;
          cols[col].layers++;
        }
        col++;
      }
      if (col < 0 || col >= length) {
        fprintf(stderr, "MSAColumns op[]: bad index %d (size=%d)\n", col, length);
        exit(1);
      }
      add_nuc(&cols[col], s->seq[k], clipped);
      if (!clipped) rmax = col;
      col++;
    }
    if (rmin < mincol) mincol = rmin;
    if (rmax > maxcol) maxcol = rmax;
  }
  /* refineMSA */
  char* cons = (char*)malloc((size_t)length + 2);
  int cons_len = 0, cols_removed = 0;
  for (int c = mincol; c <= maxcol; c++) {
    char ch = best_char(&cols[c]);
    if (ch == 0) {
      fprintf(stderr, "WARNING: 0 coverage column %d (mincol=%d) found within alignment of %d seqs!\n", c, mincol,
              (int)nrows);
      for (uint32_t i = 0; i < nrows; i++) fprintf(stderr, "%s\n", rows[i].id);
      exit(5);
    }
    if (ch == '-' || ch == '*') {
      ch = '*';
      if (g_remove_gaps) { /* removeColumn(col - cols_removed) */
        int alpos = c - cols_removed + minoffset;
        for (uint32_t i = 0; i < nrows; i++) {
          row_t* s = &rows[i];
          int spos = 0, salpos = s->offset;
          if (salpos >= alpos) {
            s->offset--;
            continue;
          }
          while (spos < s->seqlen) {
            salpos += 1 + s->ofs[spos];
            if (salpos > alpos) break;
            spos++;
          }
          if (spos >= s->seqlen) continue;
          s->ofs[spos]--; /* removeBase */
          s->numgaps--;
        }
        length--;
        cols_removed++;
        continue;
      }
    }
    cons[cons_len++] = ch; /* extendConsensus */
  }
  cons[cons_len] = 0;
  /* refine clipping and remove gaps propagated in the clipping regions (GapAssem.cpp:1163-1181) */
  for (uint32_t i = 0; i < nrows; i++) {
    row_t* s = &rows[i];
    if (g_refine_clip) refine_clipping(s, cons, cons_len, s->offset - minoffset - mincol, 0);
    int grem = 0;
    if (g_remove_gaps) grem = remove_clip_gaps(s);
    if (grem != 0 && g_refine_clip) refine_clipping(s, cons, cons_len, s->offset - minoffset - mincol, 1);
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o) die(2, "cannot open output\n");
  int32_t h[6] = {length + cols_removed, minoffset, mincol == INT_MAX ? -1 : mincol, maxcol, cons_len, cols_removed};
  fwrite("PWC1", 1, 4, o);
  fwrite(h, sizeof h, 1, o);
  fwrite(cons, 1, (size_t)cons_len, o);
  for (int c = 0; c < length + cols_removed; c++) {
    int32_t v[6];
    for (int k = 0; k < 6; k++) v[k] = cols[c].cnt[k];
    fwrite(v, sizeof v, 1, o);
  }
  fwrite(&nrows, 4, 1, o);
  for (uint32_t i = 0; i < nrows; i++) {
    int32_t rh[4] = {rows[i].offset, rows[i].numgaps, rows[i].clp5, rows[i].clp3};
    fwrite(rh, sizeof rh, 1, o);
    fwrite(rows[i].ofs, sizeof(short), (size_t)rows[i].seqlen, o);
  }
  fclose(o);
  if (g_ace) {
    FILE* f2 = fopen(g_ace, "w");
    if (!f2) die(2, "cannot open ace output\n");
    write_ace(f2, "contig1", rows, nrows, cons, cons_len, minoffset, mincol);
    fclose(f2);
  }
  if (g_info) {
    FILE* f2 = fopen(g_info, "w");
    if (!f2) die(2, "cannot open info output\n");
    write_info(f2, "contig1", rows, nrows, cons, cons_len, minoffset, mincol);
    fclose(f2);
  }
  if (g_msa) {
    FILE* f2 = fopen(g_msa, "w");
    if (!f2) die(2, "cannot open msa output\n");
    write_msa(f2, rows, nrows);
    fclose(f2);
  }
  return 0;
}
