/*
 * pafreport_oracle.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A single-threaded plain-C restatement of gpertea/pwasm `pafreport`
 * (/root/reference/pafreport.cpp) used as the parity checker for the HIP path and
 * as the `cpu_baseline` ("port") leg of bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may run it.
 *
 * PARITY STATUS: the reference itself cannot be built in this image (it needs gclib,
 * Makefile:3,61-62, which is absent; fetching it is a network operation).  This
 * restatement is pinned by hand-derived known-answer tests (tests/golden/kat_*),
 * each derived by reading the reference source line by line.  gclib semantics that
 * the reference relies on (GStr, parseInt, strsplit, GArgs, GLineReader, GFastaDb,
 * translateCodon, IUPAC complement) are restated from their documented behaviour;
 * where that behaviour is not observable here the result is "parity unpinned"
 * (see DESIGN.md §Oracle).  Inputs whose reference behaviour is undefined (reads past
 * the query buffer, zero-length indels, truncated cs ops, a missing cs tag) stop with
 * a documented error message; the product does the same.
 *
 * The algorithm is restated literally, including the reference's per-event copies of
 * the query suffix (pafreport.cpp:908) and the modseq copy (pafreport.cpp:802), so the
 * CPU timing reflects the reference's own cost model.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

/* ------------------------------------------------------------------ errors */
/* gclib GError: message to stderr, exit(1).  GMessage: message to stderr.
 * With --items <path> (test tooling for the multi-GPU shard merge) everything a
 * non-comment input line prints goes into one PWI1 item tagged with its 0-based line number. */
static FILE* g_errf;   /* stderr, or the current item's stderr buffer */
static FILE* g_items;  /* --items output */
static FILE* g_item_out;
static uint64_t g_item_line;
static char *g_ob, *g_eb;
static size_t g_on, g_en;

static void item_begin(uint64_t line) {
  g_item_line = line;
  g_item_out = open_memstream(&g_ob, &g_on);
  g_errf = open_memstream(&g_eb, &g_en);
}
static void item_end(int32_t status) {
  if (!g_items || !g_item_out) return;
  fclose(g_item_out);
  fclose(g_errf);
  uint32_t no = (uint32_t)g_on, ne = (uint32_t)g_en;
  if (no || ne || status >= 0) {
    fwrite(&g_item_line, 8, 1, g_items);
    fwrite(&status, 4, 1, g_items);
    fwrite(&no, 4, 1, g_items);
    fwrite(&ne, 4, 1, g_items);
    fwrite(g_ob, 1, no, g_items);
    fwrite(g_eb, 1, ne, g_items);
  }
  free(g_ob);
  free(g_eb);
  g_ob = g_eb = NULL;
  g_item_out = NULL;
  g_errf = stderr;
}
static void gerror(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(g_errf ? g_errf : stderr, fmt, ap);
  va_end(ap);
  if (g_items) {
    item_end(1);
    fclose(g_items);
    g_items = NULL;
  }
  exit(1);
}
static void gmessage(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(g_errf ? g_errf : stderr, fmt, ap);
  va_end(ap);
}

/* ------------------------------------------------------------------ strings */
typedef struct {
  char* s;
  int len;
  int cap;
} gstr;

static void gs_reserve(gstr* g, int need) {
  if (need + 1 <= g->cap) return;
  int nc = g->cap ? g->cap : 16;
  while (nc < need + 1) nc *= 2;
  g->s = (char*)realloc(g->s, (size_t)nc);
  if (!g->s) gerror("oracle: out of memory\n");
  g->cap = nc;
}
static void gs_init(gstr* g) {
  g->s = NULL;
  g->len = 0;
  g->cap = 0;
  gs_reserve(g, 8);
  g->s[0] = 0;
}
static void gs_free(gstr* g) {
  free(g->s);
  g->s = NULL;
  g->len = g->cap = 0;
}
static void gs_clear(gstr* g) {
  g->len = 0;
  g->s[0] = 0;
}
static void gs_appendn(gstr* g, const char* p, int n) {
  if (n <= 0) return;
  gs_reserve(g, g->len + n);
  memcpy(g->s + g->len, p, (size_t)n);
  g->len += n;
  g->s[g->len] = 0;
}
static void gs_appends(gstr* g, const char* p) { gs_appendn(g, p, (int)strlen(p)); }
static void gs_appendc(gstr* g, char c) {
  gs_reserve(g, g->len + 1);
  g->s[g->len++] = c;
  g->s[g->len] = 0;
}
static void gs_appendi(gstr* g, int v) { /* GStr::append(int) = "%d" */
  char b[24];
  snprintf(b, sizeof b, "%d", v);
  gs_appends(g, b);
}
static void gs_set(gstr* g, const char* p) {
  gs_clear(g);
  gs_appends(g, p);
}
static void gs_copy(gstr* dst, const gstr* src) {
  gs_clear(dst);
  gs_appendn(dst, src->s, src->len);
}
static void gs_upper(gstr* g) {
  for (int i = 0; i < g->len; i++) g->s[i] = (char)toupper((unsigned char)g->s[i]);
}
/* GStr::substr(idx,len): negative idx counts from the right; len<0 = to the end;
 * len is clipped to the end; an empty result for an out-of-range start. */
static void gs_substr(gstr* dst, const gstr* src, int idx, int len) {
  gs_clear(dst);
  if (idx < 0) idx += src->len;
  if (idx < 0) idx = 0;
  if (idx >= src->len) return;
  if (len < 0 || len > src->len - idx) len = src->len - idx;
  gs_appendn(dst, src->s + idx, len);
}
/* GStr::index(str): first occurrence or -1 */
static int gs_index(const gstr* g, const char* needle) {
  const char* p = strstr(g->s, needle);
  return p ? (int)(p - g->s) : -1;
}
static void gs_insert(gstr* g, const gstr* ins, int idx) {
  if (idx < 0) idx = 0;
  if (idx > g->len) idx = g->len;
  gs_reserve(g, g->len + ins->len);
  memmove(g->s + idx + ins->len, g->s + idx, (size_t)(g->len - idx + 1));
  memcpy(g->s + idx, ins->s, (size_t)ins->len);
  g->len += ins->len;
}
static void gs_cut(gstr* g, int idx, int len) {
  if (idx < 0 || idx >= g->len || len <= 0) return;
  if (len > g->len - idx) len = g->len - idx;
  memmove(g->s + idx, g->s + idx + len, (size_t)(g->len - idx - len + 1));
  g->len -= len;
}

/* ------------------------------------------------------------------ IUPAC complement
 * gclib gdna: IUPAC_DEFS / IUPAC_COMP map; identity for every other byte.
 * revCompl(GStr&) = tr(IUPAC_DEFS, IUPAC_COMP) + reverse (pafreport.cpp:469-472);
 * GASeq::reverseComplement = reverse + ntComplement (GapAssem.h:79-84). */
static const char IUPAC_DEFS[] = "AaCcTtGgUuMmRrWwSsYyKkVvHhDdBbNnXx-*";
static const char IUPAC_COMP[] = "TtGgAaCcAaKkYyWwSsRrMmBbDdHhVvNnXx-*";
static unsigned char g_comp[256];
static void comp_init(void) {
  for (int i = 0; i < 256; i++) g_comp[i] = (unsigned char)i;
  for (int i = 0; IUPAC_DEFS[i]; i++) g_comp[(unsigned char)IUPAC_DEFS[i]] = (unsigned char)IUPAC_COMP[i];
}
static void rev_compl(gstr* g) {
  for (int i = 0; i < g->len; i++) g->s[i] = (char)g_comp[(unsigned char)g->s[i]];
  for (int i = 0, j = g->len - 1; i < j; i++, j--) {
    char t = g->s[i];
    g->s[i] = g->s[j];
    g->s[j] = t;
  }
}

/* ------------------------------------------------------------------ translateCodon
 * gclib codons.cpp: NCBI table 1, stop = '.', unknown = 'X', input upper-cased.
 * Degenerate IUPAC codons translate to the amino acid shared by every expansion
 * (plus the Asx/Glx codes for RAY/SAR); for non-ACGT codons parity is UNPINNED. */
static const char* AA64 = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV.Y.YSSSS.CWCLFLF";
/* index = 16*b1 + 4*b2 + b3 with A=0 C=1 G=2 T=3 */
static int nt_mask(unsigned char c) {
  switch (c) {
    case 'A': return 1;
    case 'C': return 2;
    case 'G': return 4;
    case 'T': return 8;
    case 'R': return 1 | 4;
    case 'Y': return 2 | 8;
    case 'S': return 2 | 4;
    case 'W': return 1 | 8;
    case 'K': return 4 | 8;
    case 'M': return 1 | 2;
    case 'B': return 2 | 4 | 8;
    case 'D': return 1 | 4 | 8;
    case 'H': return 1 | 2 | 8;
    case 'V': return 1 | 2 | 4;
    case 'N': return 15;
    default: return 0;
  }
}
static char translate_codon(const char* p) {
  int m[3];
  for (int k = 0; k < 3; k++) {
    m[k] = nt_mask((unsigned char)toupper((unsigned char)p[k]));
    if (!m[k]) return 'X';
  }
  char aa = 0;
  for (int a = 0; a < 4; a++) {
    if (!(m[0] >> a & 1)) continue;
    for (int b = 0; b < 4; b++) {
      if (!(m[1] >> b & 1)) continue;
      for (int c = 0; c < 4; c++) {
        if (!(m[2] >> c & 1)) continue;
        char x = AA64[16 * a + 4 * b + c];
        if (aa == 0) aa = x;
        else if (aa != x) aa = '?';
      }
    }
  }
  if (aa != '?') return aa;
  /* ambiguity codes for Asx (AAY/GAY) and Glx (CAR/GAR) */
  int asx = (m[0] & ~5) == 0 && m[1] == 1 && (m[2] & ~10) == 0;
  int glx = (m[0] & ~6) == 0 && m[1] == 1 && (m[2] & ~5) == 0;
  if (asx && m[0] == 5) return 'B';
  if (glx && m[0] == 6) return 'Z';
  return 'X';
}
/* Codon at p, where bytes at or beyond `end` read as NUL (D6). */
static char translate_at(const char* base, int pos, int len) {
  char c[3];
  for (int k = 0; k < 3; k++) c[k] = (pos + k >= 0 && pos + k < len) ? base[pos + k] : 0;
  return translate_codon(c);
}

/* ------------------------------------------------------------------ gclib parseInt
 * skip blanks, optional sign, digits; false (p restored) when no digit follows. */
static int parse_int(char** pp, int* out) {
  char* p = *pp;
  while (*p == ' ' || *p == '\t') p++;
  char* start = p;
  if (*p == '-' || *p == '+') p++;
  char* dig = p;
  while (*p >= '0' && *p <= '9') p++;
  if (p == dig) return 0;
  *out = (int)strtol(start, NULL, 10);
  *pp = p;
  return 1;
}

/* ------------------------------------------------------------------ FASTA (GFastaDb) */
typedef struct {
  char* id;
  char* seq;
  int len;
} fa_rec;
typedef struct {
  fa_rec* r;
  int n, cap;
} fa_db;

static void fasta_load(fa_db* db, const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) gerror("Error: invalid FASTA file %s !\n", path);
  db->r = NULL;
  db->n = db->cap = 0;
  char* line = NULL;
  size_t lcap = 0;
  ssize_t ll;
  gstr cur;
  gs_init(&cur);
  int have = 0;
  while ((ll = getline(&line, &lcap, f)) >= 0) {
    while (ll > 0 && (line[ll - 1] == '\n' || line[ll - 1] == '\r')) line[--ll] = 0;
    if (line[0] == '>') {
      if (have) {
        db->r[db->n - 1].seq = strdup(cur.s);
        db->r[db->n - 1].len = cur.len;
      }
      if (db->n == db->cap) {
        db->cap = db->cap ? 2 * db->cap : 64;
        db->r = (fa_rec*)realloc(db->r, sizeof(fa_rec) * (size_t)db->cap);
      }
      char* p = line + 1;
      char* e = p;
      while (*e && !isspace((unsigned char)*e)) e++;
      db->r[db->n].id = strndup(p, (size_t)(e - p));
      db->r[db->n].seq = NULL;
      db->r[db->n].len = 0;
      db->n++;
      gs_clear(&cur);
      have = 1;
    } else if (have) {
      gs_appendn(&cur, line, (int)ll);
    }
  }
  if (have) {
    db->r[db->n - 1].seq = strdup(cur.s);
    db->r[db->n - 1].len = cur.len;
  }
  gs_free(&cur);
  free(line);
  fclose(f);
}
static fa_rec* fasta_fetch(fa_db* db, const char* id) {
  for (int i = 0; i < db->n; i++)
    if (strcmp(db->r[i].id, id) == 0) return &db->r[i];
  return NULL;
}

/* ------------------------------------------------------------------ q~t pair set */
typedef struct {
  char** k;
  int* v;
  size_t cap, n;
} strmap;
static uint64_t fnv(const char* s) {
  uint64_t h = 1469598103934665603ull;
  while (*s) h = (h ^ (unsigned char)*s++) * 1099511628211ull;
  return h;
}
static int* strmap_find(strmap* m, const char* key) {
  if (!m->cap) return NULL;
  size_t i = fnv(key) & (m->cap - 1);
  while (m->k[i]) {
    if (strcmp(m->k[i], key) == 0) return &m->v[i];
    i = (i + 1) & (m->cap - 1);
  }
  return NULL;
}
static void strmap_add(strmap* m, const char* key, int v) {
  if (2 * (m->n + 1) > m->cap) {
    size_t oc = m->cap;
    char** ok = m->k;
    int* ov = m->v;
    m->cap = oc ? 2 * oc : 1024;
    m->k = (char**)calloc(m->cap, sizeof(char*));
    m->v = (int*)calloc(m->cap, sizeof(int));
    m->n = 0;
    for (size_t i = 0; i < oc; i++)
      if (ok[i]) {
        size_t j = fnv(ok[i]) & (m->cap - 1);
        while (m->k[j]) j = (j + 1) & (m->cap - 1);
        m->k[j] = ok[i];
        m->v[j] = ov[i];
        m->n++;
      }
    free(ok);
    free(ov);
  }
  size_t i = fnv(key) & (m->cap - 1);
  while (m->k[i]) i = (i + 1) & (m->cap - 1);
  m->k[i] = strdup(key);
  m->v[i] = v;
  m->n++;
}

/* ------------------------------------------------------------------ PAF record */
typedef struct { /* AlnInfo, pafreport.cpp:54-88 */
  char reverse;
  const char* r_id;
  int r_len, r_alnstart, r_alnend;
  const char* t_id;
  int t_len, t_alnstart, t_alnend;
} aln_info;

typedef struct { /* TDiffInfo, pafreport.cpp:90-132 */
  char evt;
  int evtlen;
  gstr evtbases, evtsub;
  int rloc, tloc;
  gstr tctx;
} tdiff;

typedef struct {
  tdiff* d;
  int n, cap;
} tdiff_vec;

static tdiff* td_add(tdiff_vec* v) {
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 16;
    v->d = (tdiff*)realloc(v->d, sizeof(tdiff) * (size_t)v->cap);
  }
  tdiff* t = &v->d[v->n++];
  memset(t, 0, sizeof *t);
  gs_init(&t->evtbases);
  gs_init(&t->evtsub);
  gs_init(&t->tctx);
  return t;
}
static void td_free(tdiff_vec* v) {
  for (int i = 0; i < v->n; i++) {
    gs_free(&v->d[i].evtbases);
    gs_free(&v->d[i].evtsub);
    gs_free(&v->d[i].tctx);
  }
  free(v->d);
  v->d = NULL;
  v->n = v->cap = 0;
}

static const char* CIGAR_ERROR = "Error parsing cigar string from line: %s (cigar position: %s)\n";
static const char* CS_ERROR = "Error parsing cs string from line: %s (cs position: %s)\n";

/* ------------------------------------------------------------------ -w: GapAssem layout
 * Literal restatement of the progressive MSA construction pafreport -w performs
 * (pafreport.cpp:382-421, 447-450): GASeq::setGap/addGap (GapAssem.cpp:104-120),
 * GSeqAlign(s1,s2) (:605-641), addAlign (:645-690), addSeq (:694-716), injectGap (:720-753),
 * finalize/prepSeq (:1006-1012, 89-101) and writeMSA/printMFasta (:1039-1046, 482-520).
 * O(rows x L) per injected gap, exactly as the reference. */
typedef struct {
  int pos, len;
} gapdata; /* GapData, pafreport.cpp:48-52 */
typedef struct {
  gapdata* d;
  int n, cap;
} gapvec;
static void gv_add(gapvec* v, int pos, int len) {
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 16;
    v->d = (gapdata*)realloc(v->d, sizeof(gapdata) * (size_t)v->cap);
  }
  v->d[v->n].pos = pos;
  v->d[v->n].len = len;
  v->n++;
}

struct gsalign;
typedef struct {
  char* id;
  char* seq; /* NULL: not loaded (an instance of the query in one alignment) */
  int len;   /* loaded sequence length (0 when not loaded) */
  int seqlen;
  short* ofs;
  int numgaps, offset;
  char revcompl, prepped;
  struct gsalign* msa;
} gaseq;
typedef struct gsalign {
  gaseq** rows;
  int n, cap, length, minoffset;
} gsalign;

static gaseq* ga_new(const char* id, const char* seq, int slen, int offset) {
  gaseq* g = (gaseq*)calloc(1, sizeof(gaseq));
  g->id = strdup(id);
  if (seq) {
    g->seq = (char*)malloc((size_t)slen + 1);
    memcpy(g->seq, seq, (size_t)slen);
    g->seq[slen] = 0;
    g->len = slen;
  }
  g->seqlen = slen;
  g->ofs = (short*)calloc((size_t)(slen > 0 ? slen : 1), sizeof(short));
  g->offset = offset;
  return g;
}
static void ga_free(gaseq* g) {
  free(g->id);
  free(g->seq);
  free(g->ofs);
  free(g);
}
static void ga_setgap(gaseq* g, int pos, short gaplen) { /* GASeq::setGap :104-111 */
  if (pos < 0 || pos >= g->seqlen) gerror("Error: invalid gap position (%d) given for sequence %s\n", pos + 1, g->id);
  g->numgaps -= g->ofs[pos];
  g->ofs[pos] = gaplen;
  g->numgaps += gaplen;
}
static void ga_addgap(gaseq* g, int pos, short gapadd) { /* GASeq::addGap :114-120 */
  if (pos < 0 || pos >= g->seqlen) gerror("Error: invalid gap position (%d) given for sequence %s\n", pos + 1, g->id);
  g->numgaps += gapadd;
  g->ofs[pos] += gapadd;
}
static int ga_endoffset(const gaseq* g) { return g->offset + g->seqlen + g->numgaps; }
static void msa_add(gsalign* m, gaseq* s) {
  if (m->n == m->cap) {
    m->cap = m->cap ? 2 * m->cap : 8;
    m->rows = (gaseq**)realloc(m->rows, sizeof(gaseq*) * (size_t)m->cap);
  }
  m->rows[m->n++] = s;
}
static gsalign* msa_new2(gaseq* s1, gaseq* s2) { /* GSeqAlign(s1, s2) :605-641 */
  gsalign* m = (gsalign*)calloc(1, sizeof(gsalign));
  s1->msa = m;
  s2->msa = m;
  msa_add(m, s1);
  msa_add(m, s2);
  m->minoffset = s1->offset < s2->offset ? s1->offset : s2->offset;
  int e1 = ga_endoffset(s1), e2 = ga_endoffset(s2);
  m->length = (e1 > e2 ? e1 : e2) - m->minoffset;
  return m;
}
static void msa_inject_gap(gsalign* m, gaseq* seq, int pos, int xgap) { /* injectGap :720-753 */
  int alpos = seq->offset + pos;
  for (int i = 0; i <= pos; i++) alpos += seq->ofs[i];
  for (int i = 0; i < m->n; i++) {
    gaseq* s = m->rows[i];
    int spos = 0;
    if (s == seq) {
      spos = pos;
    } else {
      int salpos = s->offset;
      if (salpos >= alpos) {
        s->offset += xgap;
        continue;
      }
      while (spos < s->seqlen) {
        salpos += 1 + s->ofs[spos];
        if (salpos > alpos) break;
        spos++;
      }
      if (spos >= s->seqlen) continue;
    }
    ga_addgap(s, spos, (short)xgap);
  }
  m->length += xgap;
}
static void msa_add_seq(gsalign* m, gaseq* s, int soffs) { /* addSeq :694-716 (ng_ofs unused here) */
  s->offset = soffs;
  s->msa = m;
  msa_add(m, s);
  if (soffs < m->minoffset) {
    m->length += m->minoffset - soffs;
    m->minoffset = soffs;
  }
  if (ga_endoffset(s) - m->minoffset > m->length) m->length = ga_endoffset(s) - m->minoffset;
}
/* addAlign :645-690 (both instances of the query are forward here: no revComplement) */
static void msa_add_align(gsalign* m, gaseq* seq, gsalign* om, gaseq* oseq) {
  if (seq->seqlen != oseq->seqlen)
    gerror("GSeqAlign Error: invalid merge %s(len %d) vs %s(len %d)\n", seq->id, seq->seqlen, oseq->id, oseq->seqlen);
  for (int i = 0; i < seq->seqlen; i++) {
    int d = seq->ofs[i] - oseq->ofs[i];
    if (d > 0) msa_inject_gap(om, oseq, i, d);
    else if (d < 0) msa_inject_gap(m, seq, i, -d);
  }
  for (int i = 0; i < om->n; i++) {
    gaseq* s = om->rows[i];
    if (s == oseq) continue;
    msa_add_seq(m, s, seq->offset + s->offset - oseq->offset);
  }
  ga_free(oseq);
  free(om->rows);
  free(om);
}
/* finalize :1006-1012 -> prepSeq :89-101 (no deletions in pafreport: only the revcompl) */
static void msa_finalize(gsalign* m) {
  for (int i = 0; i < m->n; i++) {
    gaseq* s = m->rows[i];
    if (s->len == 0) gerror("Error: sequence for %s not loaded!\n", s->id);
    if (!s->prepped) {
      if (s->revcompl == 1) {
        gstr g;
        g.s = s->seq;
        g.len = s->len;
        rev_compl(&g);
      }
      s->prepped = 1;
    }
  }
}
/* GSeqAlign::print(f, 'v') :1013-1037 -> GASeq::printGappedSeq(f, minoffset) :412-440, the -D dump
 * of pafreport.cpp:443-446.  gclib's FastaSeq::getNameLen() is taken to be strlen(name) (gclib is
 * absent: an assumption).  Rows are never clipped in pafreport (clp5 = clp3 = 0), so
 * no base is lower-cased by the clip rule; tseq's own lower-case bases print as they are. */
static void msa_print(gsalign* m, FILE* f, char c) {
  msa_finalize(m);
  int max = 0;
  for (int i = 0; i < m->n; i++) {
    const int n = (int)strlen(m->rows[i]->id);
    if (n > max) max = n;
  }
  if (c != 0) {
    fprintf(f, "%*s %c ", max, " ", ' ');
    for (int k = 0; k < m->length; k++) fputc(c, f);
    fputc('\n', f);
  }
  for (int i = 0; i < m->n; i++) {
    gaseq* s = m->rows[i];
    fprintf(f, "%*s %c ", max, s->id, s->revcompl == 1 ? '-' : '+');
    if (s->len == 0 || s->len != s->seqlen)
      gerror("GASeq print Error: invalid sequence data '%s' (len=%d, seqlen=%d)\n", s->id, s->len, s->seqlen);
    for (int k = 0; k < s->offset - m->minoffset; k++) fputc(' ', f);
    for (int k = 0; k < s->seqlen; k++) {
      if (s->ofs[k] < 0) continue; /* deleted base */
      for (int j = 0; j < s->ofs[k]; j++) fputc('-', f);
      fputc(s->seq[k], f);
    }
    fputc('\n', f);
  }
}
/* writeMSA :1039-1046 -> finalize -> prepSeq (revcompl) -> printMFasta :482-520 */
static void msa_write(gsalign* m, FILE* f) {
  msa_finalize(m);
  for (int i = 0; i < m->n; i++) {
    gaseq* s = m->rows[i];
    const int llen = 60;
    fprintf(f, ">%s\n", s->id);
    int printed = 0;
    for (int k = 0; k < s->offset; k++) {
      fputc('-', f);
      if (++printed == llen) {
        fputc('\n', f);
        printed = 0;
      }
    }
    for (int k = 0; k < s->seqlen; k++) {
      if (s->ofs[k] < 0) continue;
      for (int j = 0; j < s->ofs[k]; j++) {
        fputc('-', f);
        if (++printed == llen) {
          fputc('\n', f);
          printed = 0;
        }
      }
      char c = s->seq[k];
      printed++;
      if (printed == llen) {
        fprintf(f, "%c\n", c);
        printed = 0;
      } else {
        fputc(c, f);
      }
    }
    if (printed < llen) fputc('\n', f);
  }
}

/* Decode: PAFAlignment::PAFAlignment, pafreport.cpp:477-719.
 * rs/rlen = the aligned-strand query (forward, or reverse complement for '-'). */
static void paf_decode(char** t, int tnum, const aln_info* al, const char* rs, int rlen, gstr* tseq,
                       const char* line, tdiff_vec* tdiffs, int* edist, int* alnscore, gapvec* rgaps, gapvec* tgaps) {
  int reverse = al->reverse;
  int offset = al->r_alnstart; /* :486-490 */
  if (reverse) offset = al->r_len - al->r_alnend;
  *edist = -1;
  *alnscore = 0;
  char* cigar = NULL;
  char* cs = NULL;
  int got = 0;
  for (int i = 12; i < tnum; ++i) { /* tag scan :495-520 */
    if (strncmp(t[i], "NM:i:", 5) == 0) {
      *edist = atoi(t[i] + 5);
      got |= 1;
      if (got == 15) break;
      continue;
    }
    if (strncmp(t[i], "AS:i:", 5) == 0) {
      *alnscore = atoi(t[i] + 5);
      got |= 2;
      if (got == 15) break;
      continue;
    }
    if (strncmp(t[i], "cg:Z:", 5) == 0) {
      free(cigar);
      cigar = strdup(t[i] + 5);
      got |= 4;
      if (got == 15) break;
      continue;
    }
    if (strncmp(t[i], "cs:Z:", 5) == 0) {
      free(cs);
      cs = strdup(t[i] + 5);
      got |= 8;
      if (got == 15) break;
      continue;
    }
  }
  if (cigar == NULL || cigar[0] == 0) gerror(CIGAR_ERROR, line, (const char*)0); /* :521 */
  if (cs == NULL) gerror("Error: cs tag missing at line:\n%s\n", line);         /* D4 */
  int qpos = 0, tpos = 0;
  int eff_t_len = al->t_alnend - al->t_alnstart;
  gs_clear(tseq);
  char* p = cs;
  while (*p != 0) { /* cs loop :536-626 */
    char op = *p;
    int cl = 0;
    p++;
    switch (op) {
      case ':': {
        if (!parse_int(&p, &cl)) gerror(CS_ERROR, line, p);
        if (cl < 0 || offset + qpos < 0 || offset + qpos + cl > rlen) /* D2 */
          gerror("Error: cs string extends beyond query sequence at line:\n%s\n", line);
        gs_appendn(tseq, rs + offset + qpos, cl);
        qpos += cl;
        tpos += cl;
        break;
      }
      case '*': {
        if (p[0] == 0 || p[1] == 0) gerror(CS_ERROR, line, p); /* D3 */
        char tch = (char)toupper((unsigned char)*p);
        ++p;
        char qch = (char)toupper((unsigned char)*p);
        ++p;
        int q_pos = offset + qpos;
        if (q_pos < 0 || q_pos > rlen) /* D2; rs[rlen] is the NUL terminator */
          gerror("Error: cs string extends beyond query sequence at line:\n%s\n", line);
        if (qch != rs[q_pos])
          gerror("Error: base mismatch %c != qstr[%d] (%c) at line\n%s\n", qch, q_pos, rs[q_pos], line);
        tdiff* last = tdiffs->n ? &tdiffs->d[tdiffs->n - 1] : NULL;
        if (last && last->evt == 'S' && last->rloc == q_pos - last->evtbases.len) { /* merge :556-560 */
          gs_appendc(&last->evtbases, (char)toupper((unsigned char)tch));
          gs_appendc(&last->evtsub, (char)toupper((unsigned char)qch));
        } else {
          tdiff* d = td_add(tdiffs);
          d->evt = 'S';
          d->evtlen = 1;
          d->rloc = q_pos;
          d->tloc = tpos;
          gs_appendc(&d->evtbases, (char)toupper((unsigned char)tch));
          gs_appendc(&d->evtsub, (char)toupper((unsigned char)qch));
        }
        gs_appendc(tseq, (char)tolower((unsigned char)tch));
        ++qpos;
        ++tpos;
        break;
      }
      case '-': { /* target-only bases => 'I' :579-601 */
        int s_pos = tpos;
        char tch;
        while (isalpha((unsigned char)(tch = (char)toupper((unsigned char)*p)))) {
          ++p;
          ++tpos;
          gs_appendc(tseq, (char)tolower((unsigned char)tch));
        }
        int e_len = tpos - s_pos;
        if (e_len == 0) gerror("Error: empty indel in cs string at line:\n%s\n", line); /* D1 */
        int q_pos = offset + qpos;
        tdiff* d = td_add(tdiffs);
        d->evt = 'I';
        d->evtlen = e_len;
        d->rloc = q_pos;
        d->tloc = s_pos;
        gs_appendn(&d->evtbases, tseq->s + tseq->len - e_len, e_len);
        if (reverse) {
          rev_compl(&d->evtbases);
          d->rloc = al->r_len - q_pos;
        }
        break;
      }
      case '+': { /* query-only bases => 'D' :602-619 */
        int s_pos = qpos;
        while (isalpha((unsigned char)toupper((unsigned char)*p))) {
          ++p;
          ++qpos;
        }
        int e_len = qpos - s_pos;
        if (e_len == 0) gerror("Error: empty indel in cs string at line:\n%s\n", line); /* D1 */
        int q_pos = s_pos + offset;
        if (q_pos < 0 || q_pos + e_len > rlen)
          gerror("Error: cs string extends beyond query sequence at line:\n%s\n", line); /* D2 */
        tdiff* d = td_add(tdiffs);
        d->evt = 'D';
        d->evtlen = e_len;
        d->rloc = q_pos;
        d->tloc = tpos;
        gs_appendn(&d->evtbases, rs + q_pos, e_len);
        if (reverse) {
          rev_compl(&d->evtbases);
          d->rloc = al->r_len - q_pos - e_len;
        }
        break;
      }
      case '~':
        gerror("Error: spliced alignments not supported! at line:\n%s\n", line);
        break;
      default:
        gerror("Error: unhandled event at %s in cs, line:\n%s\n", p, line);
    }
  }
  /* target context :628-643 */
  gstr tmp;
  gs_init(&tmp);
  for (int d = 0; d < tdiffs->n; d++) {
    tdiff* x = &tdiffs->d[d];
    int tc_start = x->tloc - 5; /* setTContext :120-128 */
    if (tc_start < 0) tc_start = 0;
    int evt_len = x->evtlen;
    if (x->evt == 'D') evt_len = 0;
    int tc_end = x->tloc + evt_len + 5;
    if (tc_end >= tseq->len) tc_end = tseq->len - 1;
    gs_substr(&tmp, tseq, tc_start, tc_end - tc_start);
    if (tc_end - tc_start == 0) gs_clear(&tmp);
    gs_copy(&x->tctx, &tmp);
    if (reverse) {
      rev_compl(&x->tctx);
      x->tloc = tseq->len - x->tloc;
      if (x->evt == 'S') {
        rev_compl(&x->evtbases);
        rev_compl(&x->evtsub);
        x->rloc = al->r_len - x->rloc - x->evtbases.len;
      }
    }
  }
  gs_free(&tmp);
  if (reverse) { /* tdiffs.Reverse() :643 */
    for (int i = 0, j = tdiffs->n - 1; i < j; i++, j--) {
      tdiff s = tdiffs->d[i];
      tdiffs->d[i] = tdiffs->d[j];
      tdiffs->d[j] = s;
    }
  }
  /* CIGAR :645-718 (gap lists rgaps / tgaps are only consumed by -w) */
  rgaps->n = tgaps->n = 0;
  p = cigar;
  qpos = 0;
  tpos = 0;
  while (*p != '\0') {
    int cl = 0;
    if (!parse_int(&p, &cl)) gerror(CIGAR_ERROR, line, p);
    char cop = *p;
    if (cop == '\0') gerror(CIGAR_ERROR, line, p);
    switch (cop) {
      case 'X':
      case 'M':
      case '=':
        tpos += cl;
        qpos += cl;
        break;
      case 'P':
      case 'H':
        break;
      case 'S':
        qpos += cl;
        gmessage("Warning: soft clipping shouldn't be found in this application!\n%s\n", line);
        break;
      case 'I': /* gap in the target :685-691 */
        gv_add(tgaps, reverse ? eff_t_len - tpos : tpos, cl);
        qpos += cl;
        break;
      case 'D': /* gap in the query :692-700 */
      case 'N': /* :701-711 */
        gv_add(rgaps, reverse ? al->r_len - (offset + qpos) : offset + qpos, cl);
        tpos += cl;
        break;
      default:
        gerror("Error: unhandled cigar_op %c (len %d) in %s\n", cop, cl, line);
    }
    ++p;
  }
  if (eff_t_len != tpos || tseq->len != tpos)
    gerror("Error: tseq alignment length mismatch (%d vs %d(%d-%d)) at line:%s\n", tpos, eff_t_len,
           al->t_alnend, al->t_alnstart, line);
  if (al->r_alnend - al->r_alnstart != qpos)
    gerror("Error: ref alignment length mismatch (%d vs %d-%d) at line:%s\n", qpos, al->r_alnend,
           al->r_alnstart, line);
  free(cigar);
  free(cs);
}

/* ------------------------------------------------------------------ classify */
static const char* const METMOT[] = {"CCTGG", "CCAGG", "GATC", "GTAC", NULL}; /* :41 */

/* getRefContext, pafreport.cpp:721-733 */
static int get_ref_context(const char* ref, int L, int rloc, gstr* rctx) {
  int ctxstart = rloc - 4;
  int evtloc = 4;
  if (ctxstart < 0) {
    evtloc += ctxstart;
    ctxstart = 0;
  } else if (ctxstart + 8 >= L) {
    evtloc += L - ctxstart - 9;
    ctxstart = L - 9;
  }
  if (ctxstart < 0 || ctxstart + 9 > L) gerror("Error: query sequence too short for a 9-nt context\n"); /* D5 */
  gs_appendn(rctx, ref + ctxstart, 9);
  gs_upper(rctx);
  return evtloc;
}

/* hpolyCheck, pafreport.cpp:735-748 */
static int hpoly_check(const tdiff* d, const gstr* rctx, int rctxloc) {
  if (d->evtbases.len > 1) {
    char c = d->evtbases.s[0];
    for (int i = 1; i < d->evtbases.len; i++)
      if (c != d->evtbases.s[i]) return 0;
  }
  char ch = d->evtbases.s[0];
  char seed[5] = {ch, ch, ch, ch, 0};
  int l = gs_index(rctx, seed);
  return (l >= 0 && l <= rctxloc && l + 4 >= rctxloc);
}

/* mmotifCheck, pafreport.cpp:751-763 */
static int mmotif_check(gstr* stat, const gstr* rctx) {
  for (int m = 0; METMOT[m]; ++m) {
    if (gs_index(rctx, METMOT[m]) >= 0) {
      gs_set(stat, "motif ");
      gs_appends(stat, METMOT[m]);
      return m + 1;
    }
  }
  return 0;
}

/* predictImpact, pafreport.cpp:801-883 (literal: copies modseq from the suffix) */
static void predict_impact(gstr* txt, const tdiff* di, const gstr* r_trseq, int r_offset) {
  gstr modseq;
  gs_init(&modseq);
  gs_copy(&modseq, r_trseq);
  if (di->evt == 'S') {
    int aaofs = -1;
    int* aamods = (int*)malloc(sizeof(int) * (size_t)(di->evtbases.len + 1));
    int naa = 0;
    for (int i = 0; i < di->evtbases.len; ++i) {
      int idx = di->rloc - r_offset + i;
      if (idx < 0 || idx >= modseq.len) gerror("GStr: index out of range\n");
      if (toupper((unsigned char)modseq.s[idx]) != toupper((unsigned char)di->evtsub.s[i]))
        gerror("Error: modseq[%d] not matching di.evtsub[%d] !\n", idx, i);
      modseq.s[idx] = di->evtbases.s[i];
      int ao = idx / 3;
      if (ao != aaofs) {
        aaofs = ao;
        aamods[naa++] = ao;
      }
    }
    int cdiff = 0;
    for (int i = 0; i < naa; ++i) {
      char aa = translate_at(r_trseq->s, aamods[i] * 3, r_trseq->len);
      char maa = translate_at(modseq.s, aamods[i] * 3, modseq.len);
      if (aa != maa) {
        if (cdiff) gs_appends(txt, ", ");
        gs_appends(txt, "AA");
        int aapos = aamods[i] + di->rloc / 3;
        gs_appendi(txt, aapos);
        gs_appendc(txt, '|');
        gs_appendc(txt, aa);
        gs_appendc(txt, ':');
        gs_appendc(txt, maa);
        ++cdiff;
        if (maa == '.') {
          gs_appends(txt, "|premature stop at AA");
          gs_appendi(txt, aapos);
        }
      }
    }
    if (txt->len == 0) gs_appends(txt, "synonymous");
    free(aamods);
    gs_free(&modseq);
    return;
  }
  if (di->evt == 'I') gs_insert(&modseq, &di->evtbases, di->rloc - r_offset);
  else if (di->evt == 'D') gs_cut(&modseq, di->rloc - r_offset, di->evtlen);
  else gerror("Error: unrecognized editing event (%c)!\n", di->evt);
  int aamodc = 0;
  gstr aa4, maa4;
  gs_init(&aa4);
  gs_init(&maa4);
  for (int i = 0; i + 2 < modseq.len; i += 3) {
    char aamod = translate_codon(modseq.s + i);
    if (aamod == '.') {
      gs_appends(txt, "premature stop at AA");
      gs_appendi(txt, 1 + (i + r_offset) / 3);
      break;
    }
    if (i > 0 && aamodc < 4) {
      ++aamodc;
      if (i + 2 < r_trseq->len) gs_appendc(&aa4, translate_codon(r_trseq->s + i));
      gs_appendc(&maa4, aamod);
    }
  }
  if (txt->len == 0 && aa4.len > 0 && maa4.len > 0) {
    gs_appends(txt, "frame shift ");
    gs_appendn(txt, aa4.s, aa4.len);
    gs_appendc(txt, '+');
    gs_appendc(txt, ':');
    gs_appendn(txt, maa4.s, maa4.len);
    gs_appendc(txt, '+');
  }
  gs_free(&aa4);
  gs_free(&maa4);
  gs_free(&modseq);
}

static int g_skip_codan = 0;
static int g_elide_dead = 0; /* --elide-dead (parity tooling) */

/* printDiffInfo, pafreport.cpp:885-955; ref = forward upper-case query */
static void print_diff_info(FILE* f, const char* rlabel, const char* tlabel, const aln_info* al, int alnscore,
                            int edist, tdiff_vec* tdiffs, const char* ref, int L) {
  double cov = ((al->r_alnend - al->r_alnstart) * 100.00) / al->r_len;
  if (rlabel[0] == 0)
    fprintf(f, ">%s coverage:%.2f score=%d edit_distance=%d\n", tlabel, cov, alnscore, edist);
  else
    fprintf(f, ">%s--%s coverage:%.2f score=%d edit_distance=%d\n", rlabel, tlabel, cov, alnscore, edist);
  gstr status, rctx, r_trseq, impact, tcontext, evtbases, evtsub;
  gs_init(&status);
  gs_init(&rctx);
  gs_init(&r_trseq);
  gs_init(&impact);
  gs_init(&tcontext);
  gs_init(&evtbases);
  gs_init(&evtsub);
  for (int i = 0; i < tdiffs->n; ++i) {
    tdiff* di = &tdiffs->d[i];
    gs_upper(&di->evtbases);
    int aapos = di->rloc / 3;
    char aa = translate_at(ref, 3 * aapos, L);
    ++aapos;
    gs_clear(&status);
    gs_clear(&rctx);
    int rctxloc = get_ref_context(ref, L, di->rloc, &rctx);
    if (hpoly_check(di, &rctx, rctxloc)) gs_set(&status, "homopolymer");
    int r_trloc = 3 * (aapos - 2);
    if (r_trloc < 0) r_trloc = 0;
    /* GStr r_trseq(ref + r_trloc, evtlen): the 2nd argument is a capacity, so the
       whole suffix is copied (pafreport.cpp:908) */
    gs_clear(&r_trseq);
    /* (--elide-dead, parity tooling: with the codon pass skipped the copy is never read, so a
       parity run may skip it; the CPU baseline keeps the reference's literal cost) */
    if (r_trloc < L && !(g_skip_codan && g_elide_dead)) gs_appendn(&r_trseq, ref + r_trloc, L - r_trloc);
    if (status.len == 0) mmotif_check(&status, &rctx);
    gs_clear(&impact);
    if (!g_skip_codan) predict_impact(&impact, di, &r_trseq, r_trloc);
    if (status.len == 0) gs_set(&status, "[unknown]");
    gs_copy(&tcontext, &di->tctx);
    const int MAX_EVLEN = 12;
    if (tcontext.len > 10 + MAX_EVLEN) {
      int dlen = tcontext.len - 10;
      gs_clear(&tcontext);
      gs_appendn(&tcontext, di->tctx.s, 5);
      gs_appendc(&tcontext, '[');
      gs_appendi(&tcontext, dlen);
      gs_appendc(&tcontext, ']');
      gs_appendn(&tcontext, di->tctx.s + di->tctx.len - 5, 5);
    }
    gs_copy(&evtbases, &di->evtbases);
    if (evtbases.len > MAX_EVLEN) {
      int dlen = evtbases.len;
      gs_set(&evtbases, "[");
      gs_appendi(&evtbases, dlen);
      gs_appendc(&evtbases, ']');
    }
    gs_copy(&evtsub, &di->evtsub);
    if (evtsub.len > MAX_EVLEN) {
      int dlen = evtsub.len;
      gs_set(&evtsub, "[");
      gs_appendi(&evtsub, dlen);
      gs_appendc(&evtsub, ']');
    }
    if (di->evt == 'S')
      fprintf(f, "%c\t%d\t%d(%c)\t%s:%s\t%d\t%s\t%s\t%s\t%s\n", di->evt, di->rloc + 1, aapos, aa, evtsub.s,
              evtbases.s, di->tloc + 1, tcontext.s, rctx.s, status.s, impact.s);
    else if (di->evt == 'I')
      fprintf(f, "%c\t%d\t%d(%c)\t:%s\t%d\t%s\t%s\t%s\t%s\n", di->evt, di->rloc + 1, aapos, aa, evtbases.s,
              di->tloc + 1, tcontext.s, rctx.s, status.s, impact.s);
    else
      fprintf(f, "%c\t%d\t%d(%c)\t%s:\t%d\t%s\t%s\t%s\t%s\n", di->evt, di->rloc + 1, aapos, aa, evtbases.s,
              di->tloc + 1, tcontext.s, rctx.s, status.s, impact.s);
  }
  gs_free(&status);
  gs_free(&rctx);
  gs_free(&r_trseq);
  gs_free(&impact);
  gs_free(&tcontext);
  gs_free(&evtbases);
  gs_free(&evtsub);
}

/* ------------------------------------------------------------------ CLI (GArgs) */
#define USAGE                                                             \
  "Usage:\n\
 pafreport <paf_with_cg_cs> -r <refseq.fa> [-s <summary.txt>]\n\
    [-o <diff_report.dfa>][-w <outfile.mfa>] [-G|-F|-C|-N]\n\
    \n\
   <paf_with_cg_cs> is the input PAF file with high quality query sequence(s)\n\
      aligned to many target sequences using minimap2 --cs\n\
   -r provide the fasta file with query sequence(s) (required)\n\
   -o write difference data for each alignment into <diff_report.dfa>\n\
   -s write event summary counts into <summary.txt>\n\
   -w write MSA as multifasta into <outfile.mfa>\n\
   -G gene CDS analysis mode (default for query<100K; assumes -C)\n\
   -F full genome alignment mode (default for query>100Kb; assumes -N)\n\
   -C perform codon impact analysis\n\
   -N skip codon impact analysis\n"

typedef struct {
  const char* val[128];
  int set[128];
  const char* nonopt[64];
  int n_nonopt;
  int err;
} gargs;

/* GArgs(argc, argv, "DGFCNvd:p:r:o:m:w:c:s:"): single-letter switches (groupable),
 * value options as "-ovalue" or "-o value"; returns index of the first invalid arg. */
static void gargs_parse(gargs* a, int argc, char** argv, const char* fmt) {
  memset(a, 0, sizeof *a);
  for (int i = 1; i < argc; i++) {
    char* p = argv[i];
    if (p[0] == '-' && p[1] != 0) {
      for (int k = 1; p[k]; k++) {
        unsigned char c = (unsigned char)p[k];
        const char* f = (c < 128 && c != ':') ? strchr(fmt, c) : NULL;
        if (!f) {
          a->err = i;
          return;
        }
        if (f[1] == ':') {
          if (p[k + 1]) a->val[c] = p + k + 1;
          else if (i + 1 < argc) a->val[c] = argv[++i];
          else {
            a->err = i;
            return;
          }
          a->set[c] = 1;
          break;
        }
        a->set[c] = 1;
        a->val[c] = "";
      }
    } else if (a->n_nonopt < 64) {
      a->nonopt[a->n_nonopt++] = p;
    }
  }
}

/* strsplit(line, t, '\t'): in-place tab split */
static int strsplit_tab(char* s, char*** fields, int* cap) {
  int n = 0;
  int after = 1;
  for (int i = 0; s[i]; i++) {
    if (after) {
      if (n == *cap) {
        *cap = *cap ? 2 * *cap : 32;
        *fields = (char**)realloc(*fields, sizeof(char*) * (size_t)*cap);
      }
      (*fields)[n++] = s + i;
    }
    after = 0;
    if (s[i] == '\t') {
      s[i] = 0;
      after = 1;
    }
  }
  return n;
}

/* GLineReader::getLine: \n, \r or \r\n terminate a line; returns NULL at EOF */
static char* get_line(FILE* f, gstr* buf) {
  gs_clear(buf);
  int c;
  while ((c = getc(f)) != EOF) {
    if (c == '\n' || c == '\r') {
      if (c == '\r') {
        int d = getc(f);
        if (d != '\n' && d != EOF) ungetc(d, f);
      }
      return buf->s;
    }
    gs_appendc(buf, (char)c);
  }
  if (buf->len == 0) return NULL;
  return buf->s;
}

int main(int argc, char* argv[]) {
  comp_init();
  g_errf = stderr;
  const char* items_path = NULL;
  long long range_a = 0, range_b = -1;
  /* test tooling, not pafreport options (they precede the pafreport arguments):
   *   --items PATH    line-tagged item stream (PWI1) instead of the report
   *   --range A:B     only the PAF lines that start in bytes [A, B) (chunked parity runs)
   *   --elide-dead    skip the query-suffix copy that nothing reads when the codon pass is off */
  for (;;) {
    if (argc > 2 && strcmp(argv[1], "--items") == 0) {
      items_path = argv[2];
    } else if (argc > 2 && strcmp(argv[1], "--range") == 0) {
      if (sscanf(argv[2], "%lld:%lld", &range_a, &range_b) != 2 || range_a < 0 || range_b < range_a)
        gerror("--range A:B\n");
    } else if (argc > 1 && strcmp(argv[1], "--elide-dead") == 0) {
      g_elide_dead = 1;
      argv[1] = argv[0];
      argc -= 1;
      argv += 1;
      continue;
    } else {
      break;
    }
    argv[2] = argv[0];
    argc -= 2;
    argv += 2;
  }
  gargs args;
  gargs_parse(&args, argc, argv, "DGFCNvd:p:r:o:m:w:c:s:");
  if (args.err > 0) {
    gmessage("%s\nInvalid argument: %s\n", USAGE, argv[args.err]);
    exit(1);
  }
  int debug_mode = args.set['D'];
  int fullgenome = args.set['F'];
  int gene_cds = args.set['G'];
  if (fullgenome && gene_cds) {
    gmessage("%s Error: cannot use both -G and -F!\n", USAGE);
    exit(1);
  }
  int force_coding = args.set['C'];
  int force_noncoding = args.set['N'];
  if (force_coding && force_noncoding) {
    gmessage("%s Error: cannot use both -N and -C!\n", USAGE);
    exit(1);
  }
  int verbose = args.set['v'] || debug_mode;
  FILE* inf = stdin;
  if (args.n_nonopt > 0 && args.nonopt[0][0]) {
    inf = fopen(args.nonopt[0], "r");
    if (!inf) gerror("Cannot open input file %s!\n", args.nonopt[0]);
  }
  if (range_b >= 0 && range_a > 0) { /* start after the line break before byte A */
    if (fseeko(inf, (off_t)(range_a - 1), SEEK_SET) != 0) gerror("--range: cannot seek\n");
    int c;
    while ((c = getc(inf)) != EOF && c != '\n') {
    }
  }
  if (args.set['c'] && args.val['c'][0]) { /* -c clipmax: parsed, never consumed (:217-240) */
    char cbuf[64];
    snprintf(cbuf, sizeof cbuf, "%s", args.val['c']);
    size_t cl = strlen(cbuf);
    int ispercent = cl > 0 && cbuf[cl - 1] == '%';
    if (ispercent)
      while (cl > 0 && cbuf[cl - 1] == '%') cbuf[--cl] = 0;
    int c = atoi(cbuf);
    if (c <= 0) gerror("Error: invalid -c <clipmax> (%d) option provided (must be a positive integer)!\n", c);
    if (ispercent && c > 99)
      gerror("Error: invalid percent value (%d) for -c option  (must be an integer between 1 and 99)!\n", c);
    if (ispercent) {
      float clipmax = (float)c / 100;
      int maxp = (int)(100 * clipmax + 0.5f);
      if (verbose) fprintf(stderr, "Percentual max clipping set to %d%%\n", maxp);
    } else if (verbose)
      fprintf(stderr, "Max clipping set to %d bases\n", c);
  }
  FILE* freport = stdout;
  if (args.set['o'] && args.val['o'][0]) {
    freport = fopen(args.val['o'], "w");
    if (!freport) gerror("Cannot open file %s for writing!\n", args.val['o']);
  }
  const char* fa = args.set['r'] ? args.val['r'] : "";
  if (!fa[0]) gerror("Error: query FASTA file (-r) is required!\n");
  struct stat st;
  long long fsize = (stat(fa, &st) == 0) ? (long long)st.st_size : -1;
  if (fsize <= 0) gerror("Error: invalid FASTA file %s !\n", fa);
  fa_db qfasta;
  fasta_load(&qfasta, fa);
  if (!fullgenome && !gene_cds && fsize > 120000) fullgenome = 1;
  g_skip_codan = (fullgenome || force_noncoding);
  if (!g_skip_codan && !force_coding && fsize > 120000) g_skip_codan = 1;
  FILE* fmsa = NULL;
  if (args.set['w'] && args.val['w'][0]) { /* :263-273 */
    if (fullgenome) {
      gmessage("%s Error: can only generate MSA for -G mode!\n", USAGE);
      exit(1);
    }
    fmsa = fopen(args.val['w'], "w");
    if (!fmsa) gerror("Cannot open file %s for writing!\n", args.val['w']);
  }
  gapvec rgaps = {0}, tgaps = {0};
  gaseq* ga_ref = NULL; /* GASeq of the current query (:341-351); NULL until it is first used */
  gsalign* ref_msa = NULL; /* refMSA */
  strmap alnpairs = {0};
  gstr lbuf, lstr, tseq, qtpair, tlabel, rlabel;
  gs_init(&lbuf);
  gs_init(&lstr);
  gs_init(&tseq);
  gs_init(&qtpair);
  gs_init(&tlabel);
  gs_init(&rlabel);
  char** t = NULL;
  int tcap = 0;
  fa_rec* refseq = NULL;
  char* refseq_rc = NULL; /* reverse complement of the current query */
  char* line;
  if (items_path) {
    g_items = fopen(items_path, "wb");
    if (!g_items) gerror("Cannot open file %s for writing!\n", items_path);
    fwrite("PWI1", 1, 4, g_items);
  }
  uint64_t line_no = 0;
  for (; (range_b < 0 || ftello(inf) < (off_t)range_b) && (line = get_line(inf, &lbuf)) != NULL;
       line_no++, item_end(-1)) { /* :303-436 */
    if (g_items) {
      item_begin(line_no);
      freport = g_item_out;
    }
    if (line[0] == '#') continue;
    gs_set(&lstr, line);
    int numt = strsplit_tab(line, &t, &tcap);
    if (numt < 15) gerror("Error: invalid PAF fline (num. fields=%d):\n%s\n", numt, lstr.s);
    aln_info al;
    al.reverse = (t[4][0] == '-') ? 1 : 0;
    al.r_id = t[0];
    al.r_len = atoi(t[1]);
    al.r_alnstart = atoi(t[2]);
    al.r_alnend = atoi(t[3]);
    al.t_id = t[5];
    al.t_len = atoi(t[6]);
    al.t_alnstart = atoi(t[7]);
    al.t_alnend = atoi(t[8]);
    if (strcmp(al.r_id, al.t_id) == 0) {
      if (verbose) gmessage("Skipping alignment of qry seq to itself.\n");
      continue;
    }
    if (!fullgenome) { /* gene-mode q~t dedupe :319-334 */
      gs_set(&qtpair, al.r_id);
      gs_appendc(&qtpair, '~');
      gs_appends(&qtpair, al.t_id);
      int* vc = strmap_find(&alnpairs, qtpair.s);
      if (!vc) strmap_add(&alnpairs, qtpair.s, 0);
      else {
        ++(*vc);
        if (*vc == 1) gmessage("Warning: alignment %s to %s already seen, ignoring \n", al.r_id, al.t_id);
        continue;
      }
    }
    if (refseq == NULL || strcmp(refseq->id, al.r_id) != 0) { /* :338-354 */
      ga_ref = NULL; /* a new GASeq for the query: its msa starts empty (rseqs is never filled) */
      fa_rec* r = fasta_fetch(&qfasta, al.r_id);
      if (!r) gerror("Error: could not retrieve sequence for %s !\n", al.r_id);
      refseq = r;
      for (int i = 0; i < r->len; i++) r->seq[i] = (char)toupper((unsigned char)r->seq[i]);
      free(refseq_rc);
      refseq_rc = (char*)malloc((size_t)r->len + 1);
      for (int i = 0; i < r->len; i++) refseq_rc[i] = (char)g_comp[(unsigned char)r->seq[r->len - 1 - i]];
      refseq_rc[r->len] = 0;
    }
    if (al.r_len != refseq->len)
      gerror("Error: ref seq len in this PAF line (%d) differs from loaded sequence length(%d)!\n%s\n", al.r_len,
             refseq->len, lstr.s);
    const char* r_seq = al.reverse ? refseq_rc : refseq->seq;
    tdiff_vec tdiffs = {0};
    int edist, alnscore;
    paf_decode(t, numt, &al, r_seq, refseq->len, &tseq, lstr.s, &tdiffs, &edist, &alnscore, &rgaps, &tgaps);
    gs_set(&tlabel, al.t_id);
    gs_set(&rlabel, al.r_id);
    if (fullgenome) {
      gs_appendc(&rlabel, ':');
      gs_appendi(&rlabel, al.r_alnstart);
      gs_appendc(&rlabel, '-');
      gs_appendi(&rlabel, al.r_alnend);
    }
    gs_appends(&tlabel, ":");
    gs_appendi(&tlabel, al.t_alnstart);
    gs_appendc(&tlabel, '-');
    gs_appendi(&tlabel, al.t_alnend);
    gs_appendc(&tlabel, al.reverse ? '-' : '+');
    if (qfasta.n == 1 && !fullgenome) gs_clear(&rlabel);
    print_diff_info(freport, rlabel.s, tlabel.s, &al, alnscore, edist, &tdiffs, refseq->seq, refseq->len);
    td_free(&tdiffs);
    if (fmsa) { /* :382-421 */
      gaseq* taseq = ga_new(tlabel.s, tseq.s, tseq.len, al.r_alnstart);
      taseq->revcompl = (char)al.reverse;
      if (ga_ref == NULL) ga_ref = ga_new(refseq->id, refseq->seq, refseq->len, 0);
      gaseq* rseq = ga_ref;
      const int first = ga_ref->msa == NULL;
      if (!first) rseq = ga_new(refseq->id, NULL, al.r_len, 0);
      for (int g = 0; g < rgaps.n; g++) ga_setgap(rseq, rgaps.d[g].pos, (short)rgaps.d[g].len);
      for (int g = 0; g < tgaps.n; g++) ga_setgap(taseq, tgaps.d[g].pos, (short)tgaps.d[g].len);
      gsalign* newmsa = msa_new2(rseq, taseq);
      if (first) ref_msa = newmsa;
      else {
        msa_add_align(ga_ref->msa, ga_ref, newmsa, rseq);
        ref_msa = ga_ref->msa;
      }
    }
  }
  /* :443-446 -D: the MSA dump on stderr before it is written (without -w, or with no alignment,
   * refMSA is NULL and the reference dereferences it: nothing is printed here, D7 / D10) */
  if (debug_mode && ref_msa) {
    fprintf(g_errf, ">MSA (%d)\n", ref_msa->n);
    msa_print(ref_msa, g_errf, 'v');
  }
  if (fmsa) { /* :447-450 (no alignment at all: the reference dereferences NULL; here: empty file, D10) */
    if (ref_msa) msa_write(ref_msa, fmsa);
    fclose(fmsa);
  }
  if (g_items) {
    fclose(g_items);
  } else if (freport != stdout) {
    fclose(freport);
  }
  if (inf != stdin) fclose(inf);
  return 0;
}
