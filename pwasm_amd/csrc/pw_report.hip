// pw_report.hip — the MI355X hot path of pafreport: cs decode -> event classifier -> codon
// consequence -> report-line rendering, fused into one kernel (gfx950, wave64).
//
// Reference behaviour restated here (gpertea/pwasm, /root/reference):
//   decode            PAFAlignment::PAFAlignment           pafreport.cpp:526-643
//   target context    TDiffInfo::setTContext + '-' fixups  pafreport.cpp:120-128, 628-643
//   ref context       getRefContext                        pafreport.cpp:721-733
//   homopolymer/motif hpolyCheck / mmotifCheck             pafreport.cpp:735-763
//   codon consequence predictImpact                        pafreport.cpp:801-883
//   event line        printDiffInfo (event loop)           pafreport.cpp:893-954
//
// Layout: one 64-lane wavefront (= one 64-thread workgroup) owns one PAF record at a time and
// walks its packed op stream in SEGMENTS of up to 128 ops (2 per lane):
//   1. coalesced load of the segment's op words; wave prefix-scan of (query, target, literal)
//      advances -> every op's start coordinates;
//   2. the segment is cut where its query span or literal span would overflow the LDS windows,
//      then staged in LDS with 16-byte loads: op words (+16-op halo each side), per-op starts,
//      the literal bytes and the forward-query window its events can touch (span + 64 bytes
//      each side).  Byte accesses hit LDS; one outside a window (long indels at a segment edge)
//      falls back to the global copy, so windows change speed, never results;
//   3. ballot of SUB ops -> S-run heads (pafreport merges directly consecutive '*' ops,
//      pafreport.cpp:556-560; `:0` ops are dropped by the pre-pass so "consecutive" is exact);
//      heads are compacted into an event list, one event per lane;
//   4. each lane computes its event and writes the report line, field by field as the values
//      become known, into its own 112-byte LDS line buffer (stores are unconditional: a
//      masked-off character goes to the lane's junk byte, so there is no per-character branch);
//   5. a wave prefix-scan of line lengths places the lines in the record's text slot (events of
//      '-' records back-to-front = the reference's tdiffs.Reverse(), pafreport.cpp:643) and the
//      lines are gathered 16 bytes per lane into full-width global stores.
// Rare, divergent work is not done in the wave (where one lane taking a slow path stalls all 64):
// a target context that needs an op walk, and a line longer than its buffer (an S run with many
// changed codons), get their bytes reserved and are queued for fixup_kernel, launched behind.
// Workgroups are persistent (grid-stride over records): the 4.6 KB of byte tables are staged
// into LDS once per workgroup.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "pw_tables.h"
#include "pwasm_amd.h"

namespace pw {

// LDS pointers carry their address space explicitly: a generic pointer here makes hipcc merge
// "LDS hit ? lds[o] : global[i]" into one flat load (global latency + vmcnt waits).
#define LDS __attribute__((address_space(3)))
typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // 16-byte copies

__constant__ Tables c_tables = build_tables();

constexpr int kWave = 64;
constexpr int kSegOps = 128;    // ops per segment (2 per lane)
constexpr int kOpHalo = 16;     // op words staged before / after a segment
constexpr int kQW = 4096;       // forward-query window per wave (bytes)
constexpr int kQPad = 64;       // context reach beyond a segment's query span
constexpr int kLW = 1024;       // literal window per wave (bytes)
constexpr int kLPad = 64;
constexpr int kLine = 112;      // per-lane report-line buffer (bytes)
constexpr int kMap = kWave * kLine / 16 + 2;  // chunk-map entries (rounds without long lines)
constexpr int kMaxEv = 12;      // MAX_EVLEN, pafreport.cpp:919
constexpr int32_t kNoStop = INT32_MAX;
// Timing-only ablations for experiment builds (tools/exp_build.sh); 0 in the product build.
#ifndef PW_ABL
#define PW_ABL 0
#endif

struct WaveLds {
  uint8_t line[kWave * kLine];  // per-lane line buffers
  uint8_t qw[kQW];
  uint8_t lw[kLW];
  uint32_t opw[kSegOps + 2 * kOpHalo];
  int32_t qs[kSegOps];
  int32_t ts[kSegOps];
  uint32_t ls[kSegOps];
  uint32_t ostart[kWave + 1];   // line starts in output order
  uint8_t junk[kWave];
  uint8_t olane[kWave];         // lane of the k-th line in output order
  uint8_t cmap[kMap];           // 16-byte output chunk -> output index of its first line
  uint16_t evl[kSegOps];
};

struct Lds {
  Tables tab;
  WaveLds w;
};

// ------------------------------------------------------------------ wave primitives
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}
__device__ __forceinline__ uint32_t bcast(uint32_t v, int src) { return __shfl(v, src, kWave); }
// LDS written by some lanes and read by others of the same (single-wave) workgroup
__device__ __forceinline__ void wave_sync() { __syncthreads(); }

// ------------------------------------------------------------------ record context
struct Rec {
  const uint32_t* ops;      // this record's ops (global)
  const uint8_t* lits;      // global literal array
  const uint8_t* R;         // forward query (global)
  const int32_t* NS;        // next-stop table of this query (or null)
  const LDS Tables* tab;    // LDS tables
  const LDS uint8_t* qw;    // LDS forward-query window
  const LDS uint8_t* lw;    // LDS literal window
  const LDS uint32_t* opw;  // LDS op words
  int L;                    // query length
  int offset;               // start on the aligned strand
  int T;                    // tseq length
  uint32_t n_ops;
  int qlo;                  // forward position of qw[0]
  uint32_t l_lo, l_n;       // literal window [l_lo, l_lo + l_n)
  int op_lo;                // record op index of opw[0]
  uint32_t op_n;
  bool rev;
};

__device__ __forceinline__ uint8_t Rc(const Rec& r, int x) {
  if ((unsigned)x >= (unsigned)r.L) return 0;
  const unsigned o = (unsigned)(x - r.qlo);
  return o < (unsigned)kQW ? r.qw[o] : r.R[x];
}
__device__ __forceinline__ uint8_t litb(const Rec& r, uint32_t i) {
  const uint32_t o = i - r.l_lo;
  return o < r.l_n ? r.lw[o] : r.lits[i];
}
__device__ __forceinline__ uint32_t opword(const Rec& r, uint32_t j) {
  const unsigned o = (unsigned)((int)j - r.op_lo);
  return o < r.op_n ? r.opw[o] : r.ops[j];
}

// aligned-strand query char at p (refseq_rc for '-' records, pafreport.cpp:352-362); p == L
// reads the NUL terminator as the reference does.
__device__ __forceinline__ uint8_t aligned_char(const Rec& r, int p) {
  if ((unsigned)p >= (unsigned)r.L) return 0;
  return r.rev ? r.tab->comp[Rc(r, r.L - 1 - p)] : Rc(r, p);
}

// translateCodon: three bases of {A,C,G,T} in either case take one lookup in codon64 (no
// dependent table reads); anything else goes through the IUPAC mask tables.
__device__ __forceinline__ bool is_acgt(uint32_t c) {
  // letters 0x40-0x7F whose low 5 bits are 1 (A), 3 (C), 7 (G) or 20 (T)
  return (c & 0xC0u) == 0x40u && ((0x0010008Au >> (c & 0x1Fu)) & 1u);
}
__device__ __forceinline__ uint8_t translate(const LDS Tables* t, uint8_t a, uint8_t b, uint8_t c) {
  if (is_acgt(a) && is_acgt(b) && is_acgt(c))
    return t->codon64[((a >> 1) & 3u) << 4 | ((b >> 1) & 3u) << 2 | ((c >> 1) & 3u)];
  return t->codon[(t->nt[a] << 8) | (t->nt[b] << 4) | t->nt[c]];
}

__device__ __forceinline__ uint32_t op_tadv(uint32_t w) {
  uint32_t t = w >> 30, n = w & 0x3FFFFFFFu;
  return (t == PW_OP_MATCH || t == PW_OP_INS) ? n : (t == PW_OP_SUB ? 1u : 0u);
}
__device__ __forceinline__ uint32_t op_qadv(uint32_t w) {
  uint32_t t = w >> 30, n = w & 0x3FFFFFFFu;
  return (t == PW_OP_MATCH || t == PW_OP_DEL) ? n : (t == PW_OP_SUB ? 1u : 0u);
}
__device__ __forceinline__ uint32_t op_ladv(uint32_t w) {
  uint32_t t = w >> 30, n = w & 0x3FFFFFFFu;
  return t == PW_OP_SUB ? 2u : (t == PW_OP_INS ? n : 0u);
}
__device__ __forceinline__ uint8_t to_upper(uint8_t c) { return (c >= 'a' && c <= 'z') ? c - 32 : c; }
__device__ __forceinline__ uint8_t to_lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
// comp[comp[c]] without the tables: the IUPAC complement is an involution except U/u -> A/a -> T/t
__device__ __forceinline__ uint8_t comp2(uint8_t c) { return (c | 0x20) == 'u' ? (uint8_t)(c - 1) : c; }

// ------------------------------------------------------------------ event
struct Event {
  uint32_t type;  // PW_OP_SUB / INS / DEL
  int n;          // evtbases length (S-run length, I/D length)
  int q_pos;      // offset + qpos at creation (aligned strand)
  uint32_t ls;    // literal start of the head op
  int rloc;       // final (printed - 1)
  int r_trloc;
};

// evtbases[i] in final orientation, upper case (pafreport.cpp:563,594-596,612-614,637,895)
__device__ __forceinline__ uint8_t ev_base(const Rec& r, const Event& e, int i) {
  if (e.type == PW_OP_SUB) return r.rev ? r.tab->comp[litb(r, e.ls + 2 * (e.n - 1 - i))] : litb(r, e.ls + 2 * i);
  if (e.type == PW_OP_INS) return r.rev ? r.tab->comp[litb(r, e.ls + (e.n - 1 - i))] : litb(r, e.ls + i);
  return r.rev ? comp2(Rc(r, e.rloc + i)) : Rc(r, e.q_pos + i);
}
// evtsub[i] (S only)
__device__ __forceinline__ uint8_t ev_sub(const Rec& r, const Event& e, int i) {
  return r.rev ? r.tab->comp[litb(r, e.ls + 2 * (e.n - 1 - i) + 1)] : litb(r, e.ls + 2 * i + 1);
}

// ------------------------------------------------------------------ line sinks
// LineSink writes into the lane's LDS line buffer; a store past the buffer or a masked-off
// character goes to the lane's junk byte (no branch).  GlobalSink (fixup_kernel) writes
// the line straight to its place in the text slot.
struct LineSink {
  LDS uint8_t* buf;
  LDS uint8_t* junk;
  int pos;
  __device__ __forceinline__ void put(uint8_t c) {
    *(pos < kLine ? buf + pos : junk) = c;
    pos++;
  }
  __device__ __forceinline__ void put_if(bool pred, uint8_t c) {
    *((pred && pos < kLine) ? buf + pos : junk) = c;
    pos += pred ? 1 : 0;
  }
  __device__ __forceinline__ void put_at(int i, uint8_t c) { *(i < kLine ? buf + i : junk) = c; }
};
struct GlobalSink {
  uint8_t* p;
  int pos;
  __device__ __forceinline__ void put(uint8_t c) { p[pos++] = c; }
  __device__ __forceinline__ void put_if(bool pred, uint8_t c) {
    if (pred) p[pos++] = c;
  }
  __device__ __forceinline__ void put_at(int i, uint8_t c) { p[i] = c; }
};

// Write tseq[p0, p1) (the target segment, pafreport.cpp:543,575,588 — never materialised) to
// line positions base.. : in order for '+' records, reverse-complemented for '-' records
// (revCompl of tctx, pafreport.cpp:631).  Walks the op stream run by run from the cursor.
struct Cursor {
  uint32_t j;
  int ts, qs;
  uint32_t ls, w;
};
template <class S>
__device__ __forceinline__ void emit_tseq(S& k, const Rec& r, Cursor c, int p0, int p1, int base) {
  while (c.ts > p0 && c.j > 0) {  // step back to the op holding p0
    c.j--;
    c.w = opword(r, c.j);
    c.ts -= (int)op_tadv(c.w);
    c.qs -= (int)op_qadv(c.w);
    c.ls -= op_ladv(c.w);
  }
  int p = p0;
  while (p < p1) {
    const int tl = (int)op_tadv(c.w);
    if (p >= c.ts + tl && c.j + 1 < r.n_ops) {
      c.ts += tl;
      c.qs += (int)op_qadv(c.w);
      c.ls += op_ladv(c.w);
      c.j++;
      c.w = opword(r, c.j);
      continue;
    }
    int pe = c.ts + tl;
    if (pe > p1 || pe <= p) pe = p1;  // (pe <= p: past the last op; cannot happen on valid input)
    const uint32_t t = c.w >> 30;
    for (; p < pe; p++) {
      const int off = p - c.ts;
      uint8_t ch;
      if (t == PW_OP_MATCH) {
        const int x = r.offset + c.qs + off;  // aligned-strand query position
        ch = r.rev ? comp2(Rc(r, r.L - 1 - x)) : Rc(r, x);
        if (x >= r.L) ch = 0;
      } else {
        ch = to_lower(litb(r, t == PW_OP_SUB ? c.ls : c.ls + off));
        if (r.rev) ch = r.tab->comp[ch];
      }
      k.put_at(r.rev ? base + (p1 - 1 - p) : base + (p - p0), ch);
    }
  }
}

// "%d" of a non-negative int
template <class S>
__device__ __forceinline__ void wr_dig(S& k, uint32_t v) {
#if PW_ABL & 8
  k.put('1'); k.put('2'); k.put('3'); k.put((uint8_t)('0' + (v & 7)));
  return;
#endif
  if (v >= 100000u) {
    for (uint32_t P = 1000000000u; P >= 100000u; P /= 10u) k.put_if(v >= P, (uint8_t)('0' + (v / P) % 10u));
  }
#pragma unroll
  for (uint32_t P = 10000u; P >= 10u; P /= 10u) k.put_if(v >= P, (uint8_t)('0' + (v / P) % 10u));
  k.put((uint8_t)('0' + v % 10u));
}
template <class S, int N>
__device__ __forceinline__ void wr_lit(S& k, const char (&s)[N]) {
#pragma unroll
  for (int i = 0; i < N - 1; i++) k.put((uint8_t)s[i]);
}

// evtbases length of the event headed by op j: the run of directly consecutive '*' ops
// (pafreport.cpp:556-560) or the indel length
__device__ __forceinline__ int event_len(const Rec& r, uint32_t j, uint32_t wd) {
  if ((wd >> 30) != PW_OP_SUB) return (int)(wd & 0x3FFFFFFFu);
  int n = 1;
  uint32_t kk = j + 1;
  while (kk < r.n_ops && (opword(r, kk) >> 30) == PW_OP_SUB) {
    n++;
    kk++;
  }
  return n;
}

// Length of the tctx field for a context of cl target bases (abbreviated past 10+MAX_EVLEN).
__device__ __forceinline__ int tctx_field_len(int cl) {
  if (cl <= 10 + kMaxEv) return cl;
  const uint32_t v = (uint32_t)(cl - 10);
  return 12 + 1 + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) + (v >= 1000000u) +
         (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}

// The tctx field (setTContext, pafreport.cpp:120-128; revCompl :631; abbreviation :918-927).
// Fast path — match runs of >= 5 on both sides (the common case): query bytes, the event's own
// target bases, query bytes, no op walk.  Otherwise the context is gathered by walking the op
// stream; with `defer` that walk is not done here: the field's bytes are skipped (its length is
// known) and the return value is its position in the line, for fixup_kernel to fill.
template <class S>
__device__ __forceinline__ int emit_tctx(S& k, const Rec& r, uint32_t typ, int n, uint32_t j, uint32_t wd, int qs,
                                         int ts, uint32_t ls, bool defer) {
  const int qp = r.offset + qs;
  const int evtlen = typ == PW_OP_SUB ? 1 : n;  // merged S keeps evtlen 1 (pafreport.cpp:562)
  int tcs = ts - 5;
  if (tcs < 0) tcs = 0;
  int tce = ts + (typ == PW_OP_DEL ? 0 : evtlen) + 5;
  if (tce >= r.T) tce = r.T - 1;
  int cl = tce - tcs;
  if (cl < 0) cl = 0;
  const int ll = ts - tcs;                                          // target bases before
  const int nm = typ == PW_OP_DEL ? 0 : (typ == PW_OP_SUB ? 1 : n);  // the event's own
  const int rl = tce - (ts + nm);                                   // bases after
  const uint32_t pw = (ll > 0 && j > 0) ? opword(r, j - 1) : 0u;
  const uint32_t aw = (rl > 0 && j + 1 < r.n_ops) ? opword(r, j + 1) : 0u;
  const bool fast = cl <= 10 + kMaxEv && (typ != PW_OP_SUB || n == 1) && rl >= 0 &&
                    (ll == 0 || (j > 0 && (pw >> 30) == PW_OP_MATCH && (int)(pw & 0x3FFFFFFFu) >= ll)) &&
                    (rl == 0 || (j + 1 < r.n_ops && (aw >> 30) == PW_OP_MATCH && (int)(aw & 0x3FFFFFFFu) >= rl));
  if (fast) {
    // aligned query start after the event; '-' records read the forward query in the other
    // order (revCompl of tctx: comp(comp(x)) = x up to U)
    const int qpa = qp + (typ == PW_OP_SUB ? 1 : (typ == PW_OP_DEL ? n : 0));
    const int f1 = r.rev ? r.L - qpa - rl : qp - ll, n1 = r.rev ? rl : ll;
    const int f2 = r.rev ? r.L - qp : qpa, n2 = r.rev ? ll : rl;
    uint8_t c1[5], c2[5];
#pragma unroll
    for (int q = 0; q < 5; q++) {
      c1[q] = Rc(r, f1 + q);
      c2[q] = Rc(r, f2 + q);
    }
#pragma unroll
    for (int q = 0; q < 5; q++) k.put_if(q < n1, r.rev ? comp2(c1[q]) : c1[q]);
    for (int q = 0; q < nm; q++) {
      uint8_t ch = to_lower(litb(r, ls + (typ == PW_OP_SUB ? 0u : (uint32_t)(r.rev ? nm - 1 - q : q))));
      k.put(r.rev ? r.tab->comp[ch] : ch);
    }
#pragma unroll
    for (int q = 0; q < 5; q++) k.put_if(q < n2, r.rev ? comp2(c2[q]) : c2[q]);
    return -1;
  }
  if (defer) {
    const int at = k.pos;
    k.pos += tctx_field_len(cl);
    return at;
  }
  Cursor cur;
  cur.j = j;
  cur.ts = ts;
  cur.qs = qs;
  cur.ls = ls;
  cur.w = wd;
  if (cl <= 10 + kMaxEv) {
    emit_tseq(k, r, cur, tcs, tce, k.pos);
    k.pos += cl;
  } else {  // first5[len-10]last5 of the (oriented) context
    emit_tseq(k, r, cur, r.rev ? tce - 5 : tcs, r.rev ? tce : tcs + 5, k.pos);
    k.pos += 5;
    k.put('[');
    wr_dig(k, (uint32_t)(cl - 10));
    k.put(']');
    emit_tseq(k, r, cur, r.rev ? tcs : tce - 5, r.rev ? tcs + 5 : tce, k.pos);
    k.pos += 5;
  }
  return -1;
}

// S consequence, one codon of modseq (predictImpact, pafreport.cpp:811-826)
__device__ __forceinline__ void sub_codon(const Rec& r, const Event& e, int ao, uint8_t& aa, uint8_t& maa) {
  const int p0 = e.rloc - e.r_trloc;
  uint8_t m[3], o[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int pos = 3 * ao + j;
    o[j] = Rc(r, e.r_trloc + pos);
    m[j] = (pos >= p0 && pos < p0 + e.n) ? ev_base(r, e, pos - p0) : o[j];
  }
  aa = translate(r.tab, o[0], o[1], o[2]);
  maa = translate(r.tab, m[0], m[1], m[2]);
}

// Indel consequence: predictImpact insert/cut + stop scan (pafreport.cpp:843-882), written to
// the sink.  modseq = Q[r_trloc, rloc) + X + Q[s, L) with X the inserted bases (I) or nothing
// (D; s = rloc + len).  Codons touching the prefix / X / the first five codons are translated
// explicitly; past that, modseq codons are query codons and the first stop is one lookup in the
// next-stop table.
template <class S>
__device__ __forceinline__ void indel_impact(S& k, const Rec& r, const Event& e) {
  const int a = e.rloc - e.r_trloc;
  const int x = (e.type == PW_OP_INS) ? e.n : 0;
  const int dl = (e.type == PW_OP_DEL) ? e.n : 0;
  const int sfx = e.rloc + dl;
  const int M = (r.L - e.r_trloc) + x - dl;
  const int trlen = r.L - e.r_trloc;
  int stop_i = -1;
  uint32_t aa4 = 0, maa4 = 0;
  int aa4n = 0, maa4n = 0;
  if (a + x <= 15) {
    // the reference scans codons i = 0,3,..,12 (while i+2 < M), stopping at the first stop;
    // here all five codons and the four reference codons are read and translated at once
    // (independent reads, no loop-carried latency) and the scan is replayed on the results
    uint8_t m[15];
#pragma unroll
    for (int p = 0; p < 15; p++) {
      const uint8_t q = Rc(r, p < a ? e.r_trloc + p : sfx + p - a - x);
      const int ii = p - a;
      const uint32_t li = e.ls + (uint32_t)(r.rev ? x - 1 - ii : ii);
      const uint8_t ib = (ii >= 0 && ii < x) ? litb(r, li) : (uint8_t)0;
      m[p] = (ii >= 0 && ii < x) ? (r.rev ? r.tab->comp[ib] : ib) : q;
    }
    uint8_t mm[5], rr[5];
#pragma unroll
    for (int c = 0; c < 5; c++) {
      mm[c] = translate(r.tab, m[3 * c], m[3 * c + 1], m[3 * c + 2]);
      rr[c] = c == 0 ? 0 : translate(r.tab, Rc(r, e.r_trloc + 3 * c), Rc(r, e.r_trloc + 3 * c + 1),
                                     Rc(r, e.r_trloc + 3 * c + 2));
    }
    int stopc = 5, nvalid = 0;
#pragma unroll
    for (int c = 4; c >= 0; c--) {
      const bool valid = 3 * c + 2 < M;
      if (valid && mm[c] == '.') stopc = c;
      nvalid += valid ? 1 : 0;
    }
    const int last = stopc < nvalid ? stopc : nvalid;  // codons scanned without a stop: [0, last)
#pragma unroll
    for (int c = 1; c < 5; c++) {
      if (c < last) {
        if (3 * c + 2 < trlen) {
          aa4 |= (uint32_t)rr[c] << (8 * aa4n);
          aa4n++;
        }
        maa4 |= (uint32_t)mm[c] << (8 * maa4n);
        maa4n++;
      }
    }
    if (stopc < nvalid) {
      stop_i = 3 * stopc;
    } else if (nvalid == 5 && 15 + 2 < M && r.NS) {
      const int k0 = sfx + (15 - a - x);
      if (k0 >= 0 && k0 < r.L) {
        const int st = r.NS[k0];
        if (st != kNoStop) stop_i = st - sfx + a + x;
      }
    }
  } else {  // long insertion: the reference loop as is
    const int E = a + x;
    int i = 0;
    for (; i + 2 < M && i < E; i += 3) {
      uint8_t m[3];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const int p = i + j;
        m[j] = (p < a) ? Rc(r, e.r_trloc + p) : (p < a + x ? ev_base(r, e, p - a) : Rc(r, sfx + p - a - x));
      }
      const uint8_t mm = translate(r.tab, m[0], m[1], m[2]);
      if (mm == '.') {
        stop_i = i;
        break;
      }
      if (i > 0 && maa4n < 4) {
        if (i + 2 < trlen) {
          aa4 |= (uint32_t)translate(r.tab, Rc(r, e.r_trloc + i), Rc(r, e.r_trloc + i + 1),
                                     Rc(r, e.r_trloc + i + 2))
                 << (8 * aa4n);
          aa4n++;
        }
        maa4 |= (uint32_t)mm << (8 * maa4n);
        maa4n++;
      }
    }
    if (stop_i < 0 && i + 2 < M && r.NS) {
      const int k0 = sfx + (i - a - x);
      if (k0 >= 0 && k0 < r.L) {
        const int st = r.NS[k0];
        if (st != kNoStop) stop_i = st - sfx + a + x;
      }
    }
  }
  if (stop_i >= 0) {
    wr_lit(k, "premature stop at AA");
    wr_dig(k, (uint32_t)(1 + (stop_i + e.r_trloc) / 3));
  } else if (aa4n > 0 && maa4n > 0) {
    wr_lit(k, "frame shift ");
#pragma unroll
    for (int q = 0; q < 4; q++) k.put_if(q < aa4n, (uint8_t)(aa4 >> (8 * q)));
    k.put('+');
    k.put(':');
#pragma unroll
    for (int q = 0; q < 4; q++) k.put_if(q < maa4n, (uint8_t)(maa4 >> (8 * q)));
    k.put('+');
  }
}

// Compute the event whose head op is `j` (record op index), segment slot `idx`, and write its
// report line (printDiffInfo, pafreport.cpp:886-953) to the sink as the fields become known.
// Returns the evtsub index failing the modseq check (pafreport.cpp:811-814), or -1; `rel`
// receives rloc - r_trloc for the error message.
template <class S>
__device__ __forceinline__ int emit_event(S& k, const Rec& r, uint32_t j, uint32_t wd, int qs, int ts, uint32_t ls,
                                          bool skip, bool defer, int& rel, int& tpos) {
  Event e;
  const uint32_t typ = wd >> 30;
  const int qp = r.offset + qs;
  e.type = typ;
  e.q_pos = qp;
  e.ls = ls;
  e.n = event_len(r, j, wd);
  int tloc;
  if (!r.rev) {
    e.rloc = qp;
    tloc = ts;
  } else {  // pafreport.cpp:597, 615, 633, 639
    e.rloc = (typ == PW_OP_INS) ? r.L - qp : r.L - qp - e.n;
    tloc = r.T - ts;
  }
  // amino acid at the event (pafreport.cpp:897-899)
  const int aap0 = e.rloc / 3;
  const uint8_t aa = translate(r.tab, Rc(r, 3 * aap0), Rc(r, 3 * aap0 + 1), Rc(r, 3 * aap0 + 2));
  e.r_trloc = aap0 > 0 ? 3 * (aap0 - 1) : 0;  // 3*(aapos-2), clipped at 0
  rel = e.rloc - e.r_trloc;

  // ---- "E\trloc\taapos(aa)\t"
  k.put(typ == PW_OP_SUB ? 'S' : (typ == PW_OP_INS ? 'I' : 'D'));
  k.put('\t');
  wr_dig(k, (uint32_t)(e.rloc + 1));
  k.put('\t');
  wr_dig(k, (uint32_t)(aap0 + 1));
  k.put('(');
  k.put(aa);
  k.put(')');
  k.put('\t');
  // ---- bases field ("[n]" past MAX_EVLEN, pafreport.cpp:928-941); homopolymer uniformity
  const bool big = e.n > kMaxEv;
#if PW_ABL & 32
  const uint8_t b0 = 'A';
  const bool same = e.n == 1;
  k.put('A'); k.put(':'); k.put('C');
#else
  if (typ == PW_OP_SUB) {
    if (big) {
      k.put('[');
      wr_dig(k, (uint32_t)e.n);
      k.put(']');
    } else {
      for (int i = 0; i < e.n; i++) k.put(ev_sub(r, e, i));
    }
  }
  if (typ != PW_OP_DEL) k.put(':');
  const uint8_t b0 = ev_base(r, e, 0);
  bool same = true;
  if (big) {
    k.put('[');
    wr_dig(k, (uint32_t)e.n);
    k.put(']');
    for (int i = 1; i < e.n; i++) same = same && ev_base(r, e, i) == b0;
  } else {
    for (int i = 0; i < e.n; i++) {
      const uint8_t b = ev_base(r, e, i);
      same = same && b == b0;
      k.put(b);
    }
  }
  if (typ == PW_OP_DEL) k.put(':');
#endif
  k.put('\t');
  wr_dig(k, (uint32_t)(tloc + 1));
  k.put('\t');
  // ---- target context (setTContext :120-128, revCompl :631, abbreviation :918-927)
  tpos = emit_tctx(k, r, typ, e.n, j, wd, qs, ts, ls, defer);
  k.put('\t');
  // ---- query context (getRefContext, pafreport.cpp:721-733) + status
#if PW_ABL & 4
  wr_lit(k, "ACGTACGTA\t[unknown]");
  (void)same;
  (void)b0;
#else
  int c0 = e.rloc - 4, eloc = 4;
  if (c0 < 0) {
    eloc += c0;
    c0 = 0;
  } else if (c0 + 8 >= r.L) {
    eloc += r.L - c0 - 9;
    c0 = r.L - 9;
  }
  if (c0 < 0) c0 = 0;  // L < 9 is reported by the host
  uint32_t rw0 = 0, rw1 = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint8_t c = Rc(r, c0 + q);
    k.put(c);
    rw0 |= (uint32_t)c << (8 * q);
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint8_t c = Rc(r, c0 + 4 + q);
    k.put(c);
    rw1 |= (uint32_t)c << (8 * q);
  }
  const uint32_t rw2 = Rc(r, c0 + 8);
  k.put((uint8_t)rw2);
  k.put('\t');
  {
    // homopolymer seed "cccc": first occurrence in the context (hpolyCheck, :742-746); motifs:
    // first in list order anywhere in it (mmotifCheck, :751-763)
    const uint64_t lo = (uint64_t)rw0 | ((uint64_t)rw1 << 32);
    int l = -1;
    bool m0 = false, m1 = false, m2 = false, m3 = false;
#pragma unroll
    for (int p = 5; p >= 0; p--) {
      const uint32_t v4 = p <= 4 ? (uint32_t)(lo >> (8 * p)) : ((rw1 >> 8) | (rw2 << 24));
      const uint32_t c4 = p < 4 ? (uint32_t)(lo >> (8 * (p + 4))) & 0xFFu : (p == 4 ? rw2 : 0u);
      if (v4 == 0x01010101u * b0) l = p;
      m0 = m0 || (v4 == 0x47544343u && c4 == 'G');  // "CCTGG"
      m1 = m1 || (v4 == 0x47414343u && c4 == 'G');  // "CCAGG"
      m2 = m2 || v4 == 0x43544147u;                 // "GATC"
      m3 = m3 || v4 == 0x43415447u;                 // "GTAC"
    }
    const int st = (same && l >= 0 && l <= eloc && l + 4 >= eloc) ? 1 : (m0 ? 2 : (m1 ? 3 : (m2 ? 4 : (m3 ? 5 : 0))));
    const LDS uint8_t* sw = r.tab->status[st];  // one table row, no divergent literal writes
    const int sl = sw[11];
#pragma unroll
    for (int q = 0; q < 11; q++) k.put_if(q < sl, sw[q]);
  }
#endif
  k.put('\t');
  // ---- codon consequence (predictImpact, pafreport.cpp:801-883)
  int modseq_err = -1;
#if PW_ABL & 2
  if (!skip) wr_lit(k, "synonymous");
  if (false) {
#else
  if (!skip) {
#endif
#if PW_ABL & 128
    if (typ == PW_OP_SUB) {
      wr_lit(k, "synonymous");
    } else
#endif
#if PW_ABL & 256
    if (typ != PW_OP_SUB) {
      wr_lit(k, "premature stop at AA1");
    } else
#endif
    if (typ == PW_OP_SUB) {
      for (int i = 0; i < e.n; i++)
        if (modseq_err < 0 && to_upper(Rc(r, e.rloc + i)) != to_upper(ev_sub(r, e, i))) modseq_err = i;
      const int p0 = e.rloc - e.r_trloc;
      bool any = false;
      for (int ao = p0 / 3; ao <= (p0 + e.n - 1) / 3; ao++) {
        uint8_t caa, cmaa;
        sub_codon(r, e, ao, caa, cmaa);
        if (caa != cmaa) {
          if (any) wr_lit(k, ", ");
          wr_lit(k, "AA");
          const uint32_t ap = (uint32_t)(ao + e.rloc / 3);
          wr_dig(k, ap);
          k.put('|');
          k.put(caa);
          k.put(':');
          k.put(cmaa);
          if (cmaa == '.') {
            wr_lit(k, "|premature stop at AA");
            wr_dig(k, ap);
          }
          any = true;
        }
      }
      if (!any) wr_lit(k, "synonymous");
    } else {
      indel_impact(k, r, e);
    }
  }
  k.put('\n');
  return modseq_err;
}

// ------------------------------------------------------------------ per-record driver
// Work left for fixup_kernel: a target context that needs the op walk (pos = its position in
// the line) or a whole line longer than the LDS line buffer (pos = kFixLine).
struct Fixup {
  uint32_t ai, j;
  int32_t qs, ts;
  uint32_t ls, pos;
  uint64_t dst;  // text offset of the line
};
constexpr uint32_t kFixLine = 0x80000000u;
struct FixList {
  Fixup* list;
  uint32_t* count;
  uint32_t cap;
};

__device__ __forceinline__ void process_record(const pw_report_args& A, const FixList& F, LDS Lds* S, uint32_t ai,
                                               int lane) {
  LDS WaveLds* w = &S->w;
  const pw_aln_desc d = A.desc[ai];
  const uint32_t qi = d.ref & 0x7FFFFFFFu;
  Rec r;
  r.ops = A.ops + d.op_begin;
  r.lits = A.lits;
  r.R = A.qseq + A.qoff[qi];
  r.L = A.qlen[qi];
  r.NS = A.next_stop ? A.next_stop + A.qoff[qi] : nullptr;
  r.tab = &S->tab;
  r.qw = w->qw;
  r.lw = w->lw;
  r.opw = w->opw;
  r.offset = d.offset;
  r.T = d.t_len;
  r.n_ops = d.n_ops;
  r.rev = (d.ref & PW_REF_REVERSE) != 0;
  const bool skip = A.skip_codan != 0;
  const uint64_t slot_lo = d.text_begin;
  const uint64_t slot_hi = (ai + 1 < A.n_alns) ? A.desc[ai + 1].text_begin : A.text_total;
  uint64_t out_lo = slot_lo, out_hi = slot_hi;

  int qc = 0, tc = 0;
  uint32_t lc = d.lit_begin;
  bool prev_sub = false, fix_overflow = false;
  uint32_t ev_idx = 0;
  int me_first = INT_MAX, me_last = -1, me_fa = 0, me_fb = 0, me_la = 0, me_lb = 0;  // modseq errors
  LDS uint8_t* my_line = w->line + lane * kLine;

  for (uint32_t sb = 0; sb < r.n_ops;) {
    // ---- 1. op words + scan (2 ops per lane, op sb + 64k + lane)
    uint32_t wd[2], qa[2], ta[2], la[2];
    int qs[2], ts[2];
    uint32_t ls[2];
    uint32_t qtot = 0, ttot = 0, ltot = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t j = sb + 64 * k + lane;
      wd[k] = j < r.n_ops ? r.ops[j] : 0u;
      qa[k] = op_qadv(wd[k]);
      ta[k] = op_tadv(wd[k]);
      la[k] = op_ladv(wd[k]);
      const uint32_t qi_ = wave_incl_scan(qa[k], lane), ti_ = wave_incl_scan(ta[k], lane),
                     li_ = wave_incl_scan(la[k], lane);
      qs[k] = qc + (int)(qtot + qi_ - qa[k]);
      ts[k] = tc + (int)(ttot + ti_ - ta[k]);
      ls[k] = lc + ltot + li_ - la[k];
      qtot += bcast(qi_, 63);
      ttot += bcast(ti_, 63);
      ltot += bcast(li_, 63);
    }
    // ---- 2. segment length: query / literal spans must fit the windows
    uint32_t nseg = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t j = sb + 64 * k + lane;
      const bool fits = j < r.n_ops && (uint32_t)(qs[k] + (int)qa[k] - qc) <= (uint32_t)(kQW - 2 * kQPad - 16) &&
                        (ls[k] + la[k] - lc) <= (uint32_t)(kLW - 2 * kLPad - 16);
      nseg += (uint32_t)__popcll(__ballot(fits));
    }
    if (nseg == 0) nseg = 1;
    // ---- 3. stage op words (+halo), starts
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t idx = 64 * k + lane;
      if (idx < nseg) {
        w->opw[kOpHalo + idx] = wd[k];
        w->qs[idx] = qs[k];
        w->ts[idx] = ts[k];
        w->ls[idx] = ls[k];
      }
    }
    if (lane < 2 * kOpHalo) {
      const int j = lane < kOpHalo ? (int)sb - kOpHalo + lane : (int)(sb + nseg) + (lane - kOpHalo);
      const uint32_t v = (j >= 0 && (uint32_t)j < r.n_ops) ? r.ops[j] : 0u;
      w->opw[lane < kOpHalo ? lane : kOpHalo + nseg + (lane - kOpHalo)] = v;
    }
    r.op_lo = (int)sb - kOpHalo;
    r.op_n = nseg + 2 * kOpHalo;
    uint32_t sq = 0, st = 0, sl = 0;  // segment totals
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const bool in = (uint32_t)(64 * k + lane) < nseg;
      sq += in ? qa[k] : 0u;
      st += in ? ta[k] : 0u;
      sl += in ? la[k] : 0u;
    }
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
      sq += __shfl_xor(sq, dd, kWave);
      st += __shfl_xor(st, dd, kWave);
      sl += __shfl_xor(sl, dd, kWave);
    }
    // ---- 4. forward-query window: aligned span [offset+qc-pad, offset+qc+sq+pad)
    {
      const int a0q = r.offset + qc - kQPad, a1q = r.offset + qc + (int)sq + kQPad;
      int f0 = r.rev ? r.L - a1q : a0q;
      if (f0 < 0) f0 = 0;
      if (f0 > r.L) f0 = r.L;
      const uintptr_t abs0 = (uintptr_t)(r.R + f0) & ~(uintptr_t)15;
      r.qlo = (int)((intptr_t)abs0 - (intptr_t)r.R);
      const intptr_t avail = (intptr_t)(r.R + r.L) - (intptr_t)abs0;  // bytes up to the query end
      int nbytes = (int)((avail + 15) & ~(intptr_t)15);
      if (nbytes > kQW) nbytes = kQW;
      for (int o = lane * 16; o < nbytes; o += kWave * 16)
        *reinterpret_cast<LDS v4u*>(w->qw + o) = *reinterpret_cast<const v4u*>(abs0 + o);
    }
    // ---- 5. literal window [lc - pad, lc + sl + pad)
    {
      const uint32_t l0 = lc > (uint32_t)kLPad ? lc - kLPad : 0u;
      const uintptr_t abs0 = (uintptr_t)(r.lits + l0) & ~(uintptr_t)15;
      r.l_lo = (uint32_t)((const uint8_t*)abs0 - r.lits);
      uint32_t nbytes = (lc + sl + kLPad - r.l_lo + 15) & ~15u;
      if (nbytes > (uint32_t)kLW) nbytes = kLW;
      r.l_n = nbytes;
      for (uint32_t o = lane * 16; o < nbytes; o += kWave * 16)
        *reinterpret_cast<LDS v4u*>(w->lw + o) = *reinterpret_cast<const v4u*>(abs0 + o);
    }
    wave_sync();

    // ---- 6. base check of every '*' op (pafreport.cpp:550-554) and S-run heads
    uint64_t hm[2];
    uint32_t sm_prev = prev_sub ? 1u : 0u;
    int bad_idx = INT_MAX;
    int bad_qp = 0, bad_q = 0, bad_r = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t idx = 64 * k + lane;
      const bool in = idx < nseg;
      const uint32_t typ = wd[k] >> 30;
      const bool is_sub = in && typ == PW_OP_SUB;
      const uint64_t subm = __ballot(is_sub);
      const bool prevsub = lane == 0 ? sm_prev != 0 : ((subm >> (lane - 1)) & 1ull) != 0;
      sm_prev = (uint32_t)((subm >> 63) & 1ull);
      hm[k] = __ballot(in && (typ == PW_OP_INS || typ == PW_OP_DEL || (is_sub && !prevsub)));
      bool bad = false;
      uint8_t qch = 0, rch = 0;
      const int qp = r.offset + qs[k];
      if (is_sub) {
        qch = litb(r, ls[k] + 1);
        rch = aligned_char(r, qp);
        bad = qch != rch;
      }
      const uint64_t bm = __ballot(bad);
      if (bm && bad_idx == INT_MAX) {
        const int fl = __builtin_ctzll(bm);
        bad_idx = 64 * k + fl;
        bad_qp = __shfl(qp, fl, kWave);
        bad_q = __shfl((int)qch, fl, kWave);
        bad_r = __shfl((int)rch, fl, kWave);
      }
    }
    if (bad_idx != INT_MAX) {
      if (lane == 0) {
        pw_aln_result res;
        res.text_off = slot_lo;
        res.text_len = 0;
        res.n_events = 0;
        res.err = PW_REC_MISMATCH;
        res.err_a = bad_qp;
        res.err_b = bad_q;
        res.err_c = bad_r;
        A.results[ai] = res;
      }
      return;
    }
    // compact the heads into the event list
    const uint32_t n0 = (uint32_t)__popcll(hm[0]);
    const uint32_t nev = n0 + (uint32_t)__popcll(hm[1]);
    {
      const uint64_t lt = (1ull << lane) - 1ull;
      if ((hm[0] >> lane) & 1ull) w->evl[__popcll(hm[0] & lt)] = (uint16_t)lane;
      if ((hm[1] >> lane) & 1ull) w->evl[n0 + __popcll(hm[1] & lt)] = (uint16_t)(64 + lane);
    }
    wave_sync();
    prev_sub = (w->opw[kOpHalo + nseg - 1] >> 30) == PW_OP_SUB;  // carry into the next segment

    // ---- 7. events, 64 per round: each lane writes its line into its LDS line buffer
    for (uint32_t e0 = 0; e0 < nev; e0 += kWave) {
      const uint32_t ei = e0 + lane;
      const bool act = ei < nev;
      const uint32_t idx = act ? w->evl[ei] : 0u;
      int linelen = 0, merr = -1, rel = 0, tpos = -1;
      if (act) {
        LineSink k;
        k.buf = my_line;
        k.junk = w->junk + lane;
        k.pos = 0;
        merr = emit_event(k, r, sb + idx, w->opw[kOpHalo + idx], w->qs[idx], w->ts[idx], w->ls[idx], skip, true,
                          rel, tpos);
        linelen = k.pos;
      }
      // modseq errors: first / last failing event of the record (in creation order)
      {
        const uint64_t fm = __ballot(merr >= 0);
        if (fm) {
          const int lo = __builtin_ctzll(fm), hi = 63 - __builtin_clzll(fm);
          const int fi_lo = __shfl(merr, lo, kWave), fi_hi = __shfl(merr, hi, kWave);
          const int rl_lo = __shfl(rel, lo, kWave), rl_hi = __shfl(rel, hi, kWave);
          const int gi_lo = (int)(ev_idx + e0) + lo, gi_hi = (int)(ev_idx + e0) + hi;
          if (gi_lo < me_first) {
            me_first = gi_lo;
            me_fa = rl_lo + fi_lo;
            me_fb = fi_lo;
          }
          if (gi_hi > me_last) {
            me_last = gi_hi;
            me_la = rl_hi + fi_hi;
            me_lb = fi_hi;
          }
        }
      }
      const uint32_t incl = wave_incl_scan((uint32_t)linelen, lane);
      const uint32_t B = bcast(incl, kWave - 1);
      const uint32_t my_off = r.rev ? (B - incl) : (incl - (uint32_t)linelen);
      if (B == 0) continue;
      if (out_hi - out_lo < B) {  // host slot bound violated: report, never write outside the slot
        if (lane == 0) {
          pw_aln_result res = {};
          res.text_off = slot_lo;
          res.err = 3;
          A.results[ai] = res;
        }
        return;
      }
      uint64_t g0;
      if (!r.rev) {
        g0 = out_lo;
        out_lo += B;
      } else {
        out_hi -= B;
        g0 = out_hi;
      }
      // deferred work -> fixup list (one wave-aggregated atomic)
      {
        const bool need = act && (linelen > kLine || tpos >= 0);
        const uint64_t nm = __ballot(need);
        if (nm) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(F.count, (uint32_t)__popcll(nm));
          base = bcast(base, 0);
          const uint32_t slot = base + (uint32_t)__popcll(nm & ((1ull << lane) - 1ull));
          if (need && slot < F.cap) {
            Fixup f;
            f.ai = ai;
            f.j = sb + idx;
            f.qs = w->qs[idx];
            f.ts = w->ts[idx];
            f.ls = w->ls[idx];
            f.pos = linelen > kLine ? kFixLine : (uint32_t)tpos;
            f.dst = g0 + my_off;
            F.list[slot] = f;
          }
          fix_overflow = fix_overflow || (__ballot(need && slot >= F.cap) != 0ull);
        }
      }
      // line starts in output order (k-th line = lane k, or lane 63-k for '-' records) and the
      // chunk map: 16-byte chunk ci of the aligned destination -> line holding its first byte
      uint8_t* const dst = A.text + g0;
      const uint32_t shift = (uint32_t)((uintptr_t)dst & 15);
      uint8_t* const gb = dst - shift;  // 16-byte aligned
      const uint32_t end = shift + B;
      {
        const int oi = r.rev ? kWave - 1 - lane : lane;
        w->ostart[oi] = my_off;
        w->olane[oi] = (uint8_t)lane;
        if (lane == 0) w->ostart[kWave] = B;
        if (linelen > 0) {
          const uint32_t c1 = (my_off + (uint32_t)linelen + shift + 15) >> 4;
          if (my_off == 0) w->cmap[0] = (uint8_t)oi;
          for (uint32_t ci = (my_off + shift + 15) >> 4; ci < c1 && ci < (uint32_t)kMap; ci++) w->cmap[ci] = (uint8_t)oi;
        }
      }
      wave_sync();
#if PW_ABL & 16
      if (true) {
        wave_sync();
        continue;
      }
#endif
      // gather: each lane assembles 16 output bytes from (at most a few) line buffers with
      // aligned dword reads + byte-align shifts, then one 16-byte store
      for (uint32_t c = (uint32_t)lane * 16; c < end; c += kWave * 16) {
        const int cb = (int)c - (int)shift;  // output byte at chunk position 0 (< 0 in chunk 0)
        uint32_t b = cb < 0 ? 0u : (uint32_t)cb;
        const uint32_t be = (c + 16 - shift < B) ? c + 16 - shift : B;
        int oi;
        if ((c >> 4) < (uint32_t)kMap) {
          oi = w->cmap[c >> 4];
        } else {  // past the map (rounds with long lines): last line starting at or before b
          oi = 0;
#pragma unroll
          for (int step = 32; step >= 1; step >>= 1)
            if (oi + step <= kWave - 1 && w->ostart[oi + step] <= b) oi += step;
        }
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        while (b < be) {
          const uint32_t s0 = w->ostart[oi], s1 = w->ostart[oi + 1];
          const uint32_t pe = s1 < be ? s1 : be;
          if (pe > b) {
            int x = cb - (int)s0;          // line offset at chunk position 0, >= -15
            if (x > kLine) x = kLine;      // long line: garbage here, fixup_kernel rewrites it
            const int a = (int)w->olane[oi] * kLine + x;
            const LDS uint32_t* src = reinterpret_cast<const LDS uint32_t*>(w->line + (a & ~3));
            const uint32_t sh = (uint32_t)a & 3u;
            uint32_t d[5];
#pragma unroll
            for (int i = 0; i < 5; i++) d[i] = src[i];
            const uint32_t qlo = (uint32_t)((int)b - cb), qhi = (uint32_t)((int)pe - cb);
            const uint32_t m16 = ((1u << qhi) - 1u) & ~((1u << qlo) - 1u);
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const uint32_t nib = (m16 >> (4 * i)) & 15u;
              const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;
              v[i] |= __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & bm;
            }
          }
          b = pe > b ? pe : b;
          oi++;
        }
        if (c >= shift && c + 16 <= end) {
          v4u vv;
          vv.x = v[0];
          vv.y = v[1];
          vv.z = v[2];
          vv.w = v[3];
          *reinterpret_cast<v4u*>(gb + c) = vv;
        } else {
          const uint32_t lo = c < shift ? shift : c, hi = (c + 16 < end) ? c + 16 : end;
          for (uint32_t bb = lo; bb < hi; bb++) gb[bb] = (uint8_t)(v[(bb - c) >> 2] >> (8 * ((bb - c) & 3)));
        }
      }
      wave_sync();
    }

    // ---- 8. carries
    qc += (int)sq;
    tc += (int)st;
    lc += sl;
    ev_idx += nev;
    sb += nseg;
  }

  if (lane == 0) {
    pw_aln_result res;
    res.text_off = r.rev ? out_hi : slot_lo;
    res.text_len = (uint32_t)(r.rev ? (slot_hi - out_hi) : (out_lo - slot_lo));
    res.n_events = ev_idx;
    res.err = fix_overflow ? 3 : PW_REC_OK;
    res.err_a = res.err_b = res.err_c = 0;
    if (me_last >= 0) {  // first failing event in OUTPUT order
      res.err |= PW_REC_MODSEQ;
      if (!r.rev) {
        res.err_a = me_fa;
        res.err_b = me_fb;
        res.err_c = me_first;
      } else {
        res.err_a = me_la;
        res.err_b = me_lb;
        res.err_c = (int)ev_idx - 1 - me_last;
      }
    }
    A.results[ai] = res;
  }
}

__device__ __forceinline__ void stage_tables(LDS Lds* sp, int lane) {
  const v4u* src = reinterpret_cast<const v4u*>(&c_tables);
  LDS v4u* dst = reinterpret_cast<LDS v4u*>(&sp->tab);
  for (int i = lane; i < (int)(sizeof(Tables) / 16); i += kWave) dst[i] = src[i];
}

__global__ __launch_bounds__(kWave) void report_kernel(pw_report_args A, FixList F) {
  __shared__ __attribute__((aligned(16))) Lds s;
  LDS Lds* sp = (LDS Lds*)&s;
  const int lane = threadIdx.x;
  stage_tables(sp, lane);
  __syncthreads();
  for (uint32_t ai = blockIdx.x; ai < A.n_alns; ai += gridDim.x) {
    process_record(A, F, sp, ai, lane);
    __syncthreads();
  }
}

// Deferred work of report_kernel, one entry per thread: the op-walk target contexts and the
// lines longer than the LDS line buffer, written in place (their bytes were reserved).  The
// record is read straight from global memory (empty LDS windows).
__global__ __launch_bounds__(256) void fixup_kernel(pw_report_args A, FixList F) {
  __shared__ __attribute__((aligned(16))) Tables tab;
  {
    const v4u* src = reinterpret_cast<const v4u*>(&c_tables);
    LDS v4u* dst = reinterpret_cast<LDS v4u*>((LDS Tables*)&tab);
    for (int i = threadIdx.x; i < (int)(sizeof(Tables) / 16); i += 256) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t n = min(*F.count, F.cap);
  const bool skip = A.skip_codan != 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const Fixup f = F.list[i];
    const pw_aln_desc d = A.desc[f.ai];
    const uint32_t qi = d.ref & 0x7FFFFFFFu;
    Rec r;
    r.ops = A.ops + d.op_begin;
    r.lits = A.lits;
    r.R = A.qseq + A.qoff[qi];
    r.L = A.qlen[qi];
    r.NS = A.next_stop ? A.next_stop + A.qoff[qi] : nullptr;
    r.tab = (const LDS Tables*)&tab;
    r.qw = r.lw = (const LDS uint8_t*)&tab;  // windows empty: every read goes to global memory
    r.opw = (const LDS uint32_t*)&tab;
    r.qlo = -(1 << 30);
    r.l_lo = 0;
    r.l_n = 0;
    r.op_lo = 0;
    r.op_n = 0;
    r.offset = d.offset;
    r.T = d.t_len;
    r.n_ops = d.n_ops;
    r.rev = (d.ref & PW_REF_REVERSE) != 0;
    const uint32_t wd = r.ops[f.j];
    GlobalSink g;
    g.pos = 0;
    if (f.pos == kFixLine) {
      g.p = A.text + f.dst;
      int rel, tpos;
      emit_event(g, r, f.j, wd, f.qs, f.ts, f.ls, skip, false, rel, tpos);
    } else {
      g.p = A.text + f.dst + f.pos;
      emit_tctx(g, r, wd >> 30, event_len(r, f.j, wd), f.j, wd, f.qs, f.ts, f.ls, false);
    }
  }
}

// ------------------------------------------------------------------ next-stop table
// One 256-thread workgroup per query; tiles of 768 positions from the end, each thread owns
// three consecutive positions (one per frame); per frame a suffix-min scan over the tile.
__global__ __launch_bounds__(256) void stop_table_kernel(const uint8_t* qseq, const uint64_t* qoff,
                                                         const int32_t* qlen, uint32_t nq, int32_t* ns) {
  __shared__ Tables tab;
  __shared__ int32_t sm[3][256];
  __shared__ int32_t carry[3];
  const int t = threadIdx.x;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&c_tables);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&tab);
    for (int i = t; i < (int)(sizeof(Tables) / 4); i += 256) dst[i] = src[i];
  }
  for (uint32_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
    const uint8_t* R = qseq + qoff[qi];
    int32_t* out = ns + qoff[qi];
    const int L = qlen[qi];
    if (t < 3) carry[t] = kNoStop;
    __syncthreads();
    const int ntile = (L + 767) / 768;
    for (int tile = ntile - 1; tile >= 0; tile--) {
      const int base = tile * 768;
#pragma unroll
      for (int f = 0; f < 3; f++) {
        const int p = base + 3 * t + f;
        int32_t v = kNoStop;
        if (p + 2 < L) {
          uint8_t c = tab.codon[(tab.nt[R[p]] << 8) | (tab.nt[R[p + 1]] << 4) | tab.nt[R[p + 2]]];
          if (c == '.') v = p;
        }
        sm[f][t] = v;
      }
      __syncthreads();
      for (int dd = 1; dd < 256; dd <<= 1) {  // suffix min over t
        int32_t v[3];
#pragma unroll
        for (int f = 0; f < 3; f++) v[f] = (t + dd < 256) ? sm[f][t + dd] : kNoStop;
        __syncthreads();
#pragma unroll
        for (int f = 0; f < 3; f++) sm[f][t] = min(sm[f][t], v[f]);
        __syncthreads();
      }
#pragma unroll
      for (int f = 0; f < 3; f++) {
        const int p = base + 3 * t + f;
        const int32_t v = min(sm[f][t], carry[f]);
        if (p < L) out[p] = v;
      }
      __syncthreads();
      if (t < 3) carry[t] = min(carry[t], sm[t][0]);
      __syncthreads();
    }
  }
}

}  // namespace pw

extern "C" uint64_t pw_report_workspace_bytes(uint64_t n_events_max) {
  return 64u + sizeof(pw::Fixup) * (n_events_max ? n_events_max : 1u);
}

extern "C" int pw_report_events(const pw_report_args* args, void* stream) {
  if (!args || !args->desc || !args->ops || !args->qseq || !args->qoff || !args->qlen || !args->results ||
      (!args->text && args->text_total))
    return PW_E_ARG;
  if (!args->skip_codan && !args->next_stop) return PW_E_ARG;
  if (!args->workspace || args->workspace_bytes < pw_report_workspace_bytes(1) ||
      ((uintptr_t)args->workspace & 15))
    return PW_E_ARG;
  if (args->n_alns == 0) return PW_OK;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  pw::FixList F;
  F.count = static_cast<uint32_t*>(args->workspace);
  F.list = reinterpret_cast<pw::Fixup*>(static_cast<uint8_t*>(args->workspace) + 64);
  const uint64_t cap = (args->workspace_bytes - 64) / sizeof(pw::Fixup);
  F.cap = cap > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cap;
  if (hipMemsetAsync(F.count, 0, sizeof(uint32_t), (hipStream_t)stream) != hipSuccess) return PW_E_HIP;
  const uint32_t max_blocks = (uint32_t)ncu * 16u;
  const uint32_t grid = args->n_alns < max_blocks ? args->n_alns : max_blocks;
  hipLaunchKernelGGL(pw::report_kernel, dim3(grid), dim3(pw::kWave), 0, (hipStream_t)stream, *args, F);
  hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu * 2u), dim3(256), 0, (hipStream_t)stream, *args, F);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

extern "C" int pw_stop_table_build(const uint8_t* qseq, const uint64_t* qoff, const int32_t* qlen, uint32_t nq,
                                   int32_t* next_stop, void* stream) {
  if (!qseq || !qoff || !qlen || !next_stop) return PW_E_ARG;
  if (nq == 0) return PW_OK;
  const uint32_t grid = nq < 4096u ? nq : 4096u;
  hipLaunchKernelGGL(pw::stop_table_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, qseq, qoff, qlen, nq,
                     next_stop);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}
