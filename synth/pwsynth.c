/*
 * pwsynth.c — deterministic synthetic inputs for tests and bench.py (tooling, not product).
 *
 *   pwsynth paf    --config K [--scale F] [--seed S] --fa out.fa --paf out.paf [knobs]
 *                  (cfg3 / cfg4: [--threads T] — per-record random streams, so a multi-threaded
 *                  run writes the same bytes; cfg3 also [--shard r/N]: a shard writes exactly
 *                  the lines of the full file it owns)
 *   pwsynth layout --config 5 [--scale F] [--seed S] --out layout.pwl [knobs]
 *
 * PAF records are minimap2-style (`-c --cs`): 12 columns + NM/ms/AS/nn/tp/cm/s1/s2/de/rl/cg/cs
 * tags, short-form cs (":n", "*tq", "+query-only", "-target-only", lower-case bases), a CIGAR
 * whose M/I/D runs match the cs ops.  The query (CDS, PAF column 1) is the sequence pafreport
 * analyses; for '-' records the cs walks the reverse complement of the query, as minimap2 does
 * and as pafreport.cpp:486-490,536-626 expects.
 *
 * Error model: per aligned query base an event with probability `err`;
 * 45% 1+bp query-only (cs '+', pafreport 'D'), 35% target-only (cs '-', pafreport 'I'), 20%
 * substitution; indels 4x likelier inside homopolymers >= 3; indel length geometric(p=0.7)
 * capped at 20.  The first/last `margin` aligned bases are kept as matches (minimap2 never
 * opens or closes an alignment with an indel).  Knobs add the edge cases the tests need.
 */
#include <math.h>
#include <pthread.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread uint64_t g_rng; /* per thread: cfg3 records are generated in parallel */
static uint64_t rnd64(void) { /* splitmix64 */
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double rndu(void) { return (double)(rnd64() >> 11) * (1.0 / 9007199254740992.0); }
static int rndi(int lo, int hi) { return lo + (int)(rnd64() % (uint64_t)(hi - lo + 1)); } /* inclusive */

static const char NT[4] = {'A', 'C', 'G', 'T'};
static char comp(char c) {
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    case 'a': return 't';
    case 'c': return 'g';
    case 'g': return 'c';
    case 't': return 'a';
    default: return c;
  }
}
static int is_stop(const char* c) {
  return (c[0] == 'T' && c[1] == 'A' && (c[2] == 'A' || c[2] == 'G')) || (c[0] == 'T' && c[1] == 'G' && c[2] == 'A');
}

typedef struct {
  char* buf;
  size_t len, cap;
} sbuf;
static void sb_res(sbuf* b, size_t n) {
  if (b->len + n + 1 > b->cap) {
    size_t c = b->cap ? b->cap : 4096;
    while (c < b->len + n + 1) c *= 2;
    b->buf = (char*)realloc(b->buf, c);
    b->cap = c;
  }
}
static void sb_putn(sbuf* b, const char* p, size_t n) {
  sb_res(b, n);
  memcpy(b->buf + b->len, p, n);
  b->len += n;
  b->buf[b->len] = 0;
}
static void sb_putc(sbuf* b, char c) { sb_putn(b, &c, 1); }
static void sb_printf(sbuf* b, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void sb_printf(sbuf* b, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  char tmp[512];
  int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  sb_putn(b, tmp, (size_t)n);
}

typedef struct {
  int config;
  double scale;
  uint64_t seed;
  int ncds, len_min, len_max, recs_per_cds, contig_min, contig_max;
  double err, rev, partial, p_sub, p_del, p_ins, hp_boost, p_subrun, p_longindel, p_inframe;
  int margin, motif_plant, long_mode;
  int threads, shard, nshards; /* cfg3: worker threads; --shard r/N keeps the target-genome shard r */
  double p_dup, p_self, p_comment, p_softclip;
  const char* fa;
  const char* paf;
  const char* out;
  /* layout knobs */
  int rows, ref_len, row_min, row_max;
  double ref_gap, row_gap, n_frac;
  double clip_frac, del_frac; /* layout: rows with clipped ends; deleted bases (ofs -1) */
} opts_t;

static void set_config(opts_t* o) {
  o->err = 0.01;
  o->rev = 0.5;
  o->partial = 0.1;
  o->p_del = 0.45;
  o->p_ins = 0.35;
  o->p_sub = 0.20;
  o->hp_boost = 4.0;
  o->p_subrun = 0.1;
  o->p_longindel = 0.0;
  o->p_inframe = 0.0;
  o->margin = 6;
  o->motif_plant = 0;
  o->long_mode = 0;
  o->contig_min = 50000;
  o->contig_max = 200000;
  switch (o->config) {
    case 1: /* 1 x ~1.5 kb CDS vs ~20 assemblies */
      o->ncds = 1;
      o->len_min = o->len_max = 1503;
      o->recs_per_cds = 20;
      break;
    case 2: /* 100k records over 1,000 CDS of 1-5 kb (=0 mod 3), 100 targets each */
      o->ncds = 1000;
      o->len_min = 1000;
      o->len_max = 5000;
      o->recs_per_cds = 100;
      break;
    case 3: /* 200-gene panel (300-3000 nt) x 50,000 assemblies */
      o->ncds = 200;
      o->len_min = 300;
      o->len_max = 3000;
      o->recs_per_cds = 50000;
      break;
    case 4: /* 100 contigs of 1-5 Mb x 100 targets, dense cs, auto -F */
      o->ncds = 100;
      o->len_min = 1000000;
      o->len_max = 5000000;
      o->recs_per_cds = 100;
      o->contig_min = 6000000;
      o->contig_max = 8000000;
      o->long_mode = 1;
      o->partial = 0.0;
      break;
    case 5:
      o->rows = 200;
      o->ref_len = 1000000;
      o->row_min = 500000;
      o->row_max = 1000000;
      o->ref_gap = 0.005;
      o->row_gap = 0.005;
      o->n_frac = 0.001;
      break;
    default: /* 0 = edge-case mix for tests */
      o->ncds = 6;
      o->len_min = 300;
      o->len_max = 900;
      o->recs_per_cds = 12;
      o->err = 0.03;
      o->p_subrun = 0.35;
      o->p_longindel = 0.15;
      o->p_inframe = 0.25;
      o->margin = 1;
      o->motif_plant = 1;
      o->partial = 0.4;
      o->p_dup = 0.05;
      o->p_self = 0.03;
      o->p_comment = 0.03;
      o->p_softclip = 0.0;
      o->contig_min = 2000;
      o->contig_max = 5000;
      break;
  }
}

/* random CDS: ATG + sense codons + stop; length = 0 mod 3 */
static void make_cds(char* s, int L, int plant) {
  memcpy(s, "ATG", 3);
  for (int i = 3; i < L - 3; i += 3) {
    do {
      for (int k = 0; k < 3; k++) s[i + k] = NT[rnd64() & 3];
    } while (is_stop(s + i));
  }
  const char* stops[3] = {"TAA", "TAG", "TGA"};
  memcpy(s + L - 3, stops[rnd64() % 3], 3);
  if (plant) { /* plant motifs and homopolymers so the classifier sees every status */
    static const char* mot[] = {"CCTGG", "CCAGG", "GATC", "GTAC", "AAAAA", "CCCCC", "GGGGG", "TTTTT"};
    for (int n = 0; n < L / 60; n++) {
      const char* m = mot[rnd64() % 8];
      int ml = (int)strlen(m);
      int p = rndi(3, L - 4 - ml);
      memcpy(s + p, m, (size_t)ml);
    }
    for (int i = 3; i < L - 3; i += 3) /* planting may create stops: repair in frame 0 */
      if (is_stop(s + i)) s[i] = 'C';
  }
  s[L] = 0;
}

static int geom_len(void) {
  int k = 1;
  while (k < 20 && rndu() < 0.3) k++;
  return k;
}

/* One alignment: query segment Q'[qs, qe) (aligned strand) -> cs/cigar/target bases. */
typedef struct {
  sbuf cs, cg;
  int tlen_aln, nm, nmatch, alnlen;
} aln_out;

static void cig_push(sbuf* cg, char* last, int* run, char op, int n) {
  if (*last == op) {
    *run += n;
    return;
  }
  if (*last) sb_printf(cg, "%d%c", *run, *last);
  *last = op;
  *run = n;
}

static void simulate(const opts_t* o, const char* Q, int qs, int qe, aln_out* a) {
  a->cs.len = 0;
  a->cg.len = 0;
  if (a->cs.buf) a->cs.buf[0] = 0;
  if (a->cg.buf) a->cg.buf[0] = 0;
  a->tlen_aln = a->nm = a->nmatch = a->alnlen = 0;
  char clast = 0;
  int crun = 0;
  int mrun = 0; /* pending ':' run */
  int q = qs;
  char tmp[64];
  while (q < qe) {
    int inner = (q - qs >= o->margin) && (qe - q > o->margin);
    double rate = o->err;
    int hp = 1;
    while (q + hp < qe && Q[q + hp] == Q[q]) hp++;
    int in_hp = (hp >= 3) || (q > qs && Q[q - 1] == Q[q] && q > qs + 1 && Q[q - 2] == Q[q]);
    double u = rndu();
    double pind = o->p_del + o->p_ins;
    double boost = in_hp ? o->hp_boost : 1.0;
    double tot = o->p_sub + pind * boost;
    if (!inner || u >= rate * tot / (o->p_sub + pind)) { /* match */
      mrun++;
      q++;
      a->tlen_aln++;
      a->nmatch++;
      a->alnlen++;
      cig_push(&a->cg, &clast, &crun, 'M', 1);
      continue;
    }
    double v = rndu() * tot;
    if (mrun) {
      sb_printf(&a->cs, ":%d", mrun);
      mrun = 0;
    }
    if (v < o->p_sub) { /* substitution run */
      int n = 1;
      while (rndu() < o->p_subrun && q + n < qe - o->margin) n++;
      for (int k = 0; k < n; k++) {
        char qc = Q[q + k];
        char tc;
        do tc = NT[rnd64() & 3];
        while (tc == qc);
        tmp[0] = '*';
        tmp[1] = (char)(tc | 0x20);
        tmp[2] = (char)(qc | 0x20);
        sb_putn(&a->cs, tmp, 3);
      }
      q += n;
      a->tlen_aln += n;
      a->nm += n;
      a->alnlen += n;
      cig_push(&a->cg, &clast, &crun, 'M', n);
    } else {
      int len = geom_len();
      if (rndu() < o->p_longindel) len = rndi(13, 60);
      if (rndu() < o->p_inframe) len = 3 * rndi(1, 4);
      int is_del = (v - o->p_sub) < o->p_del * boost;
      if (is_del) { /* query-only bases: cs '+' */
        if (q + len > qe - o->margin) len = qe - o->margin - q;
        if (len < 1) {
          mrun++;
          q++;
          a->tlen_aln++;
          a->nmatch++;
          a->alnlen++;
          cig_push(&a->cg, &clast, &crun, 'M', 1);
          continue;
        }
        sb_putc(&a->cs, '+');
        for (int k = 0; k < len; k++) sb_putc(&a->cs, (char)(Q[q + k] | 0x20));
        q += len;
        a->nm += len;
        a->alnlen += len;
        cig_push(&a->cg, &clast, &crun, 'I', len);
      } else { /* target-only bases: cs '-' */
        sb_putc(&a->cs, '-');
        for (int k = 0; k < len; k++) {
          char b = in_hp ? Q[q] : NT[rnd64() & 3];
          sb_putc(&a->cs, (char)(b | 0x20));
        }
        a->tlen_aln += len;
        a->nm += len;
        a->alnlen += len;
        cig_push(&a->cg, &clast, &crun, 'D', len);
        /* the base at q is still to be aligned */
      }
    }
  }
  if (mrun) sb_printf(&a->cs, ":%d", mrun);
  if (clast) sb_printf(&a->cg, "%d%c", crun, clast);
}

/* CRC-32 (IEEE, = zlib.crc32): a record's shard is crc32(target name) % N, the rule of
 * pwasm_amd/shard.py and pw_batch_from_files_shard. */
static uint32_t crc32_ieee(const char* p, size_t n) {
  static uint32_t tab[256];
  static int init = 0;
  if (!init) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    init = 1;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = tab[(c ^ (uint8_t)p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

typedef struct {
  const opts_t* o;
  char** cds;
  char** rcs;
  const int* clen;
  int recs;
} paf_ctx;

/* One PAF record (query i, target r) appended to `out`. */
static void gen_record(const paf_ctx* c, int i, int r, aln_out* a, sbuf* line, sbuf* out) {
  const opts_t* o = c->o;
  int L = c->clen[i];
  int rev = rndu() < o->rev;
  int qs = 0, qe = L;
  if (rndu() < o->partial && L > 120) {
    qs = rndi(0, L / 4);
    qe = L - rndi(0, L / 4);
    if (qe - qs < 60) {
      qs = 0;
      qe = L;
    }
  }
  /* aligned strand coordinates: cs walks rc from offset = L - qend */
  const char* Q = rev ? c->rcs[i] : c->cds[i];
  int as = rev ? L - qe : qs, ae = rev ? L - qs : qe;
  simulate(o, Q, as, ae, a);
  int tlen = rndi(o->contig_min, o->contig_max);
  if (tlen < a->tlen_aln + 10) tlen = a->tlen_aln + 10;
  int ts = rndi(0, tlen - a->tlen_aln);
  int te = ts + a->tlen_aln;
  char tname[64];
  if (o->config == 0 && rndu() < o->p_self) snprintf(tname, sizeof tname, "cds%d", i);
  else snprintf(tname, sizeof tname, "asm%d_ctg%d", r, i % 7);
  line->len = 0;
  if (o->config == 0 && rndu() < o->p_comment) sb_printf(line, "# comment line %d\n", r);
  int as_score = 2 * a->nmatch - 4 * a->nm;
  sb_printf(line, "cds%d\t%d\t%d\t%d\t%c\t%s\t%d\t%d\t%d\t%d\t%d\t60\t", i, L, qs, qe, rev ? '-' : '+', tname,
            tlen, ts, te, a->nmatch, a->alnlen);
  sb_printf(line, "NM:i:%d\tms:i:%d\tAS:i:%d\tnn:i:0\ttp:A:P\tcm:i:%d\ts1:i:%d\ts2:i:0\tde:f:%.4f\trl:i:0\tcg:Z:",
            a->nm, as_score, as_score, a->nmatch / 10, a->nmatch, (double)a->nm / (a->alnlen ? a->alnlen : 1));
  sb_putn(line, a->cg.buf, a->cg.len);
  sb_putn(line, "\tcs:Z:", 6);
  sb_putn(line, a->cs.buf, a->cs.len);
  sb_putc(line, '\n');
  sb_putn(out, line->buf, line->len);
  if (o->config == 0 && rndu() < o->p_dup) sb_putn(out, line->buf, line->len); /* duplicate q~t pair */
}

/* cfg3 / cfg4: record k = i * recs + r draws from its own stream (seed, k), so any subset of the
 * records (a shard) or any split over threads generates the same bytes. */
typedef struct {
  const paf_ctx* c;
  long long k0, k1;
  sbuf out;
  long long n;
} blk_job;

static void* gen_block(void* arg) {
  blk_job* j = (blk_job*)arg;
  const paf_ctx* c = j->c;
  const opts_t* o = c->o;
  aln_out a;
  memset(&a, 0, sizeof a);
  sbuf line = {0};
  j->out.len = 0;
  j->n = 0;
  for (long long k = j->k0; k < j->k1; k++) {
    const int i = (int)(k / c->recs), r = (int)(k % c->recs);
    if (o->nshards > 1) {
      char tname[64];
      int tn = snprintf(tname, sizeof tname, "asm%d_ctg%d", r, i % 7);
      if (crc32_ieee(tname, (size_t)tn) % (uint32_t)o->nshards != (uint32_t)o->shard) continue;
    }
    g_rng = (o->seed * 0x2545F4914F6CDD1Dull + 12345) ^ ((uint64_t)k * 0xD1B54A32D192ED03ull);
    rnd64();
    gen_record(c, i, r, &a, &line, &j->out);
    j->n++;
  }
  free(line.buf);
  free(a.cs.buf);
  free(a.cg.buf);
  return NULL;
}

static int cmd_paf(opts_t* o) {
  int ncds = o->ncds;
  int recs = (int)llround(o->recs_per_cds * o->scale);
  if (recs < 1) recs = 1;
  if (o->config == 4 || o->config == 3) {
    /* scale the number of queries first for the heavy configs */
    ncds = (int)llround(o->ncds * (o->scale < 1 ? sqrt(o->scale) : 1.0));
    if (ncds < 1) ncds = 1;
    recs = (int)llround((double)o->recs_per_cds * o->ncds * o->scale / ncds);
    if (recs < 1) recs = 1;
  }
  FILE* ff = fopen(o->fa, "wb");
  FILE* fp = fopen(o->paf, "wb");
  if (!ff || !fp) {
    fprintf(stderr, "pwsynth: cannot open outputs\n");
    return 2;
  }
  char** cds = (char**)calloc((size_t)ncds, sizeof(char*));
  char** rcs = (char**)calloc((size_t)ncds, sizeof(char*));
  int* clen = (int*)calloc((size_t)ncds, sizeof(int));
  for (int i = 0; i < ncds; i++) {
    int L = rndi(o->len_min / 3, o->len_max / 3) * 3;
    if (L < 30) L = 30;
    clen[i] = L;
    cds[i] = (char*)malloc((size_t)L + 1);
    make_cds(cds[i], L, o->motif_plant);
    fprintf(ff, ">cds%d gene %d\n", i, i);
    for (int k = 0; k < L; k += 70) fprintf(ff, "%.*s\n", (L - k) < 70 ? (L - k) : 70, cds[i] + k);
  }
  fclose(ff);
  paf_ctx c = {o, cds, rcs, clen, recs};
  long long nrec = 0;
  if (o->config == 3 || o->config == 4) { /* per-record streams over worker threads */
    for (int i = 0; i < ncds; i++) {
      rcs[i] = (char*)malloc((size_t)clen[i] + 1);
      for (int k = 0; k < clen[i]; k++) rcs[i][k] = comp(cds[i][clen[i] - 1 - k]);
      rcs[i][clen[i]] = 0;
    }
    const long long total = (long long)ncds * recs;
    int T = o->threads > 0 ? o->threads : 16;
    const long long B = o->config == 4 ? 2 : 4096; /* records per job (cfg4 records are Mb each) */
    blk_job* jobs = (blk_job*)calloc((size_t)T, sizeof(blk_job));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    for (long long k0 = 0; k0 < total; k0 += B * T) {
      int nj = 0;
      for (int t = 0; t < T && k0 + B * t < total; t++, nj++) {
        jobs[t].c = &c;
        jobs[t].k0 = k0 + B * t;
        jobs[t].k1 = jobs[t].k0 + B < total ? jobs[t].k0 + B : total;
        pthread_create(&th[t], NULL, gen_block, &jobs[t]);
      }
      for (int t = 0; t < nj; t++) {
        pthread_join(th[t], NULL);
        fwrite(jobs[t].out.buf, 1, jobs[t].out.len, fp);
        nrec += jobs[t].n;
      }
    }
    for (int t = 0; t < T; t++) free(jobs[t].out.buf);
    free(jobs);
    free(th);
  } else {
    aln_out a;
    memset(&a, 0, sizeof a);
    sbuf line = {0}, out = {0};
    for (int i = 0; i < ncds; i++) {
      int L = clen[i];
      rcs[i] = (char*)malloc((size_t)L + 1);
      for (int k = 0; k < L; k++) rcs[i][k] = comp(cds[i][L - 1 - k]);
      rcs[i][L] = 0;
      for (int r = 0; r < recs; r++) {
        out.len = 0;
        gen_record(&c, i, r, &a, &line, &out);
        fwrite(out.buf, 1, out.len, fp);
        nrec++;
      }
      free(rcs[i]);
      rcs[i] = NULL;
    }
  }
  fclose(fp);
  fprintf(stderr, "pwsynth: %lld records, %d queries\n", nrec, ncds);
  return 0;
}

/* ---- GapAssem layout (PWL1, tests/pwl_format.md): row 0 = the reference with insertion
 * blocks (ref_gap per position, 1-5 columns); rows 1.. cover U[row_min,row_max] reference
 * positions, fill part of some insertion blocks with their own bases, delete ~row_gap of their
 * reference bases (a gap column in that row) and carry ~n_frac N bases + 1% mismatches.
 * --clip P: a row gets clp5 / clp3 in [0, len/8] with probability P; --dels P: a base gets
 * ofs -1 (deleted) with probability P. */
static int cmd_layout(opts_t* o) {
  int rows = o->rows;
  int L = (int)llround(o->ref_len * o->scale);
  if (L < 50) L = 50;
  int rmin = (int)llround(o->row_min * o->scale), rmax = (int)llround(o->row_max * o->scale);
  if (rmin < 10) rmin = 10;
  if (rmax < rmin) rmax = rmin;
  if (rmax > L) rmax = L;
  if (rmin > rmax) rmin = rmax;
  FILE* f = fopen(o->out, "wb");
  if (!f) return 2;
  uint32_t nr = (uint32_t)rows;
  fwrite("PWL1", 1, 4, f);
  fwrite(&nr, 4, 1, f);
  size_t cap = (size_t)L * 6 + 16;
  char* seq = (char*)malloc(cap);
  short* ofs = (short*)malloc(sizeof(short) * cap);
  short* refgap = (short*)calloc((size_t)L, sizeof(short));
  char* ref = (char*)malloc((size_t)L);
  for (int i = 0; i < L; i++) ref[i] = NT[rnd64() & 3];
  for (int i = 1; i < L; i++)
    if (rndu() < o->ref_gap) refgap[i] = (short)rndi(1, 5);
  long long* colof = (long long*)malloc(sizeof(long long) * (size_t)L); /* column of ref base i */
  long long c = 0;
  for (int i = 0; i < L; i++) {
    c += refgap[i];
    colof[i] = c;
    c++;
  }
  for (int r = 0; r < rows; r++) {
    int start = 0, len = L;
    if (r > 0) {
      len = rndi(rmin, rmax);
      start = rndi(0, L - len);
    }
    int n = 0, pending = 0;
    for (int p = start; p < start + len; p++) {
      if (p > start) {
        int g = refgap[p];
        if (r > 0 && g > 0 && rndu() < 0.5) {
          int own = rndi(1, g);
          pending += g - own;
          for (int k = 0; k < own; k++) {
            seq[n] = NT[rnd64() & 3];
            ofs[n++] = (short)pending;
            pending = 0;
          }
        } else pending += g;
        if (r > 0 && p < start + len - 1 && rndu() < o->row_gap) { /* row lacks this base */
          pending += 1;
          continue;
        }
      }
      char b = ref[p];
      if (r > 0) {
        double u = rndu();
        if (u < o->n_frac) b = 'N';
        else if (u < o->n_frac + 0.01) b = NT[rnd64() & 3];
      }
      seq[n] = b;
      ofs[n++] = (short)pending;
      pending = 0;
    }
    int32_t c5 = 0, c3 = 0;
    if (r > 0 && o->clip_frac > 0 && rndu() < o->clip_frac) { /* (no draws when the option is off) */
      c5 = rndi(0, n / 8);
      c3 = rndi(0, n / 8);
    }
    if (r > 0 && o->del_frac > 0)
      for (int i = 1; i + 1 < n; i++)
        if (ofs[i] == 0 && rndu() < o->del_frac) ofs[i] = -1;
    int32_t h[5] = {(int32_t)colof[start], n, c5, c3, (r % 3 == 1) ? 1 : 0};
    fwrite(h, sizeof h, 1, f);
    fwrite(seq, 1, (size_t)n, f);
    fwrite(ofs, sizeof(short), (size_t)n, f);
  }
  fclose(f);
  free(seq);
  free(ofs);
  free(refgap);
  free(ref);
  free(colof);
  fprintf(stderr, "pwsynth: layout %d rows, ref %d\n", rows, L);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: pwsynth paf|layout --config K [...]\n");
    return 2;
  }
  opts_t o;
  memset(&o, 0, sizeof o);
  o.scale = 1.0;
  o.config = -1;
  o.seed = 1;
  for (int i = 2; i < argc; i++)
    if (!strcmp(argv[i], "--config") && i + 1 < argc) o.config = atoi(argv[i + 1]);
  if (o.config < 0) o.config = 0;
  set_config(&o);
  int seed_set = 0;
  for (int i = 2; i + 1 < argc; i += 2) {
    const char* k = argv[i];
    const char* v = argv[i + 1];
    if (!strcmp(k, "--config")) continue;
    else if (!strcmp(k, "--scale")) o.scale = atof(v);
    else if (!strcmp(k, "--seed")) {
      o.seed = strtoull(v, NULL, 10);
      seed_set = 1;
    } else if (!strcmp(k, "--fa")) o.fa = v;
    else if (!strcmp(k, "--paf")) o.paf = v;
    else if (!strcmp(k, "--out")) o.out = v;
    else if (!strcmp(k, "--ncds")) o.ncds = atoi(v);
    else if (!strcmp(k, "--len-min")) o.len_min = atoi(v);
    else if (!strcmp(k, "--len-max")) o.len_max = atoi(v);
    else if (!strcmp(k, "--recs")) o.recs_per_cds = atoi(v);
    else if (!strcmp(k, "--err")) o.err = atof(v);
    else if (!strcmp(k, "--rev")) o.rev = atof(v);
    else if (!strcmp(k, "--partial")) o.partial = atof(v);
    else if (!strcmp(k, "--subrun")) o.p_subrun = atof(v);
    else if (!strcmp(k, "--psub")) o.p_sub = atof(v);
    else if (!strcmp(k, "--pdel")) o.p_del = atof(v);
    else if (!strcmp(k, "--pins")) o.p_ins = atof(v);
    else if (!strcmp(k, "--longindel")) o.p_longindel = atof(v);
    else if (!strcmp(k, "--inframe")) o.p_inframe = atof(v);
    else if (!strcmp(k, "--margin")) o.margin = atoi(v);
    else if (!strcmp(k, "--plant")) o.motif_plant = atoi(v);
    else if (!strcmp(k, "--contig-min")) o.contig_min = atoi(v);
    else if (!strcmp(k, "--contig-max")) o.contig_max = atoi(v);
    else if (!strcmp(k, "--rows")) o.rows = atoi(v);
    else if (!strcmp(k, "--ref-len")) o.ref_len = atoi(v);
    else if (!strcmp(k, "--row-min")) o.row_min = atoi(v);
    else if (!strcmp(k, "--row-max")) o.row_max = atoi(v);
    else if (!strcmp(k, "--clip")) o.clip_frac = atof(v);
    else if (!strcmp(k, "--dels")) o.del_frac = atof(v);
    else if (!strcmp(k, "--threads")) o.threads = atoi(v);
    else if (!strcmp(k, "--shard")) {
      if (sscanf(v, "%d/%d", &o.shard, &o.nshards) != 2 || o.nshards < 1 || o.shard < 0 || o.shard >= o.nshards) {
        fprintf(stderr, "pwsynth: --shard r/N\n");
        return 2;
      }
    }
    else {
      fprintf(stderr, "pwsynth: unknown option %s\n", k);
      return 2;
    }
  }
  if (!seed_set) o.seed = (uint64_t)(o.config > 0 ? o.config : 7);
  if (o.nshards > 1 && o.config != 3) {
    fprintf(stderr, "pwsynth: --shard is for --config 3 (per-record streams)\n");
    return 2;
  }
  g_rng = o.seed * 0x2545F4914F6CDD1Dull + 12345;
  if (!strcmp(argv[1], "paf")) {
    if (!o.fa || !o.paf) {
      fprintf(stderr, "pwsynth paf: --fa and --paf required\n");
      return 2;
    }
    return cmd_paf(&o);
  }
  if (!strcmp(argv[1], "layout")) {
    if (!o.out) {
      fprintf(stderr, "pwsynth layout: --out required\n");
      return 2;
    }
    if (o.rows == 0) {
      o.rows = 200;
      o.ref_len = o.ref_len ? o.ref_len : 1000000;
      o.row_min = o.row_min ? o.row_min : 500000;
      o.row_max = o.row_max ? o.row_max : 1000000;
      o.ref_gap = 0.005;
      o.row_gap = 0.005;
      o.n_frac = 0.001;
    }
    if (o.ref_gap == 0) {
      o.ref_gap = 0.005;
      o.row_gap = 0.005;
      o.n_frac = 0.001;
    }
    return cmd_layout(&o);
  }
  fprintf(stderr, "pwsynth: unknown command %s\n", argv[1]);
  return 2;
}
