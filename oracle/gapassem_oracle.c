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
 * It is literal (per-base scatter, qsort per column, O(rows*L) per removed column),
 * so only small layouts are practical.  refineClipping (GapAssem.cpp:182-349) is not
 * restated: a layout with clipped rows must be run with refine-clipping disabled.
 *
 * PARITY STATUS: the reference cannot be built here (gclib absent); this restatement is
 * pinned by hand-derived known-answer layouts in tests/golden/ (parity otherwise unpinned).
 *
 * Usage: gapassem_oracle <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping]
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

int main(int argc, char** argv) {
  if (argc < 3) die(2, "usage: gapassem_oracle <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping]\n");
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--remove-gaps")) g_remove_gaps = 1;
    else if (!strcmp(argv[i], "--no-refine-clipping")) g_refine_clip = 0;
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
    if (g_refine_clip && (r->clp5 || r->clp3)) die(2, "refineClipping is not restated: use --no-refine-clipping\n");
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
  if (g_remove_gaps) /* removeClipGaps for every row (GapAssem.cpp:522-549) */
    for (uint32_t i = 0; i < nrows; i++) {
      row_t* s = &rows[i];
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
    int32_t rh[2] = {rows[i].offset, rows[i].numgaps};
    fwrite(rh, sizeof rh, 1, o);
    fwrite(rows[i].ofs, sizeof(short), (size_t)rows[i].seqlen, o);
  }
  fclose(o);
  return 0;
}
