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
// walks its packed op stream in chunks of 64 ops, one op per lane:
//   1. wave prefix-scan of (q, t, literal) advances -> each op's query/target/literal start;
//   2. ballot of SUB ops -> S-run heads (pafreport merges directly consecutive '*' ops,
//      pafreport.cpp:556-560; `:0` ops are dropped by the pre-pass so "consecutive" is exact);
//   3. each head lane owns one event: final coordinates, target context (gathered from the
//      op stream + query, never materialising tseq), 9-nt query context, status, amino acid,
//      codon consequence (O(1) per indel via the next-stop table), and renders its report line
//      twice (count, then write) into a per-wave LDS staging window;
//   4. the wave copies the window to the record's text slot (events of '-' records are written
//      back-to-front, which is the reference's tdiffs.Reverse(), pafreport.cpp:643).
// Workgroups are persistent (grid-stride over records) so the 4.6 KB of byte tables are
// staged into LDS once per workgroup.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "pw_tables.h"
#include "pwasm_amd.h"

namespace pw {

__constant__ Tables c_tables = build_tables();

constexpr int kWave = 64;
constexpr int kStage = 4096;  // LDS staging window per wave (bytes)
constexpr int kCtx = 24;      // per-lane target-context scratch (bytes)
constexpr int kMaxEv = 12;    // MAX_EVLEN, pafreport.cpp:919
constexpr int32_t kNoStop = INT32_MAX;

struct Lds {
  Tables tab;                        // 4608 B
  uint8_t stage[kStage];             // 4096 B
  uint8_t ctx[kWave * kCtx];         // 1536 B
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

// ------------------------------------------------------------------ record context
struct Rec {
  const uint32_t* ops;   // this record's ops
  const uint8_t* lits;   // global literal array
  const uint8_t* R;      // forward query
  const int32_t* NS;     // next-stop table of this query (or null)
  int L;                 // query length
  int offset;            // start on the aligned strand
  int T;                 // tseq length
  uint32_t n_ops;
  bool rev;
};

__device__ __forceinline__ uint8_t Rc(const Rec& r, int x) { return (x >= 0 && x < r.L) ? r.R[x] : 0; }

// aligned-strand query char at p (refseq_rc for '-' records, pafreport.cpp:352-362); p == L
// reads the NUL terminator as the reference does.
__device__ __forceinline__ uint8_t aligned_char(const Rec& r, const Lds& s, int p) {
  if (p < 0 || p >= r.L) return 0;
  return r.rev ? s.tab.comp[r.R[r.L - 1 - p]] : r.R[p];
}

__device__ __forceinline__ uint8_t translate(const Lds& s, uint8_t a, uint8_t b, uint8_t c) {
  return s.tab.codon[(s.tab.nt[a] << 8) | (s.tab.nt[b] << 4) | s.tab.nt[c]];
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

// ------------------------------------------------------------------ one event (head lane)
struct Event {
  uint32_t type;   // PW_OP_SUB / INS / DEL
  int n;           // evtbases length (S-run length, I/D length)
  int q_pos;       // offset + qpos at creation (aligned strand)
  uint32_t ls;     // literal start of the head op
  int rloc, tloc;  // final (printed - 1)
  int ctx_len;     // tctx length before abbreviation
  int rctx0, rctx_loc;
  int status;      // 0 unknown, 1 homopolymer, 2..5 motif
  uint8_t aa;
  int aapos;       // printed aapos (rloc/3 + 1)
  int r_trloc;
  // I/D impact (computed once)
  int imp_kind;    // 0 none, 1 stop, 2 frame shift, 3 empty
  int imp_val;
  uint32_t aa4, maa4;
  int aa4n, maa4n;
};

// evtbases[i] in final orientation, upper case (pafreport.cpp:563,594-596,612-614,637,895)
__device__ __forceinline__ uint8_t ev_base(const Rec& r, const Lds& s, const Event& e, int i) {
  if (e.type == PW_OP_SUB) {
    return r.rev ? s.tab.comp[r.lits[e.ls + 2 * (e.n - 1 - i)]] : r.lits[e.ls + 2 * i];
  } else if (e.type == PW_OP_INS) {
    return r.rev ? s.tab.comp[r.lits[e.ls + (e.n - 1 - i)]] : r.lits[e.ls + i];
  }
  return r.rev ? s.tab.comp[s.tab.comp[Rc(r, e.rloc + i)]] : Rc(r, e.q_pos + i);
}
// evtsub[i] (S only)
__device__ __forceinline__ uint8_t ev_sub(const Rec& r, const Lds& s, const Event& e, int i) {
  return r.rev ? s.tab.comp[r.lits[e.ls + 2 * (e.n - 1 - i) + 1]] : r.lits[e.ls + 2 * i + 1];
}
__device__ __forceinline__ uint8_t to_upper(uint8_t c) { return (c >= 'a' && c <= 'z') ? c - 32 : c; }
__device__ __forceinline__ uint8_t to_lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Gather tseq[p0, p1) (tseq = the target segment, pafreport.cpp:543,575,588) by walking the op
// stream from the event's head op; writes into dst[0..).
struct Cursor {
  uint32_t j;
  int ts, qs;
  uint32_t ls, w;
};
__device__ void gather_tseq(const Rec& r, const Lds& s, Cursor c, int p0, int p1, uint8_t* dst) {
  while (c.ts > p0 && c.j > 0) {  // step back to the op holding p0
    c.j--;
    c.w = r.ops[c.j];
    c.ts -= (int)op_tadv(c.w);
    c.qs -= (int)op_qadv(c.w);
    c.ls -= op_ladv(c.w);
  }
  int k = 0;
  for (int p = p0; p < p1; p++) {
    while (p >= c.ts + (int)op_tadv(c.w) && c.j + 1 < r.n_ops) {
      c.ts += (int)op_tadv(c.w);
      c.qs += (int)op_qadv(c.w);
      c.ls += op_ladv(c.w);
      c.j++;
      c.w = r.ops[c.j];
    }
    uint32_t t = c.w >> 30;
    int off = p - c.ts;
    uint8_t ch;
    if (t == PW_OP_MATCH) ch = aligned_char(r, s, r.offset + c.qs + off);
    else if (t == PW_OP_SUB) ch = to_lower(r.lits[c.ls]);
    else ch = to_lower(r.lits[c.ls + off]);
    dst[k++] = ch;
  }
}

// ------------------------------------------------------------------ rendering sinks
struct CountSink {
  int n = 0;
  __device__ __forceinline__ void put(uint8_t) { n++; }
};
struct WriteSink {
  uint8_t* buf;
  int pos, lo, hi;
  __device__ __forceinline__ void put(uint8_t c) {
    if (pos >= lo && pos < hi) buf[pos - lo] = c;
    pos++;
  }
};
template <class S>
__device__ __forceinline__ void put_str(S& k, const char* p) {
  while (*p) k.put((uint8_t)*p++);
}
template <class S>
__device__ __forceinline__ void put_int(S& k, int v) {
  if (v < 0) {
    k.put('-');
    v = -v;  // values here are > INT_MIN
  }
  char b[11];
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) k.put((uint8_t)b[--n]);
}

__constant__ char kMotif[4][6] = {"CCTGG", "CCAGG", "GATC", "GTAC"};  // pafreport.cpp:41

template <class S>
__device__ void put_bases(S& k, const Rec& r, const Lds& s, const Event& e, bool sub) {
  if (e.n > kMaxEv) {
    k.put('[');
    put_int(k, e.n);
    k.put(']');
    return;
  }
  for (int i = 0; i < e.n; i++) k.put(sub ? ev_sub(r, s, e, i) : ev_base(r, s, e, i));
}

// S consequence: predictImpact substitution branch (pafreport.cpp:804-841)
template <class S>
__device__ void put_sub_impact(S& k, const Rec& r, const Lds& s, const Event& e) {
  int p0 = e.rloc - e.r_trloc;
  int first = p0 / 3, last = (p0 + e.n - 1) / 3;
  bool any = false;
  for (int ao = first; ao <= last; ao++) {
    uint8_t m[3], o[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      int pos = 3 * ao + j;
      o[j] = Rc(r, e.r_trloc + pos);
      m[j] = (pos >= p0 && pos < p0 + e.n) ? ev_base(r, s, e, pos - p0) : o[j];
    }
    uint8_t aa = translate(s, o[0], o[1], o[2]);
    uint8_t maa = translate(s, m[0], m[1], m[2]);
    if (aa != maa) {
      if (any) put_str(k, ", ");
      put_str(k, "AA");
      int aapos = ao + e.rloc / 3;
      put_int(k, aapos);
      k.put('|');
      k.put(aa);
      k.put(':');
      k.put(maa);
      any = true;
      if (maa == '.') {
        put_str(k, "|premature stop at AA");
        put_int(k, aapos);
      }
    }
  }
  if (!any) put_str(k, "synonymous");
}

template <class S>
__device__ void render(S& k, const Rec& r, const Lds& s, const Event& e, const uint8_t* ctx, bool skip_codan) {
  k.put(e.type == PW_OP_SUB ? 'S' : (e.type == PW_OP_INS ? 'I' : 'D'));
  k.put('\t');
  put_int(k, e.rloc + 1);
  k.put('\t');
  put_int(k, e.aapos);
  k.put('(');
  k.put(e.aa);
  k.put(')');
  k.put('\t');
  if (e.type == PW_OP_SUB) {
    put_bases(k, r, s, e, true);
    k.put(':');
    put_bases(k, r, s, e, false);
  } else if (e.type == PW_OP_INS) {
    k.put(':');
    put_bases(k, r, s, e, false);
  } else {
    put_bases(k, r, s, e, false);
    k.put(':');
  }
  k.put('\t');
  put_int(k, e.tloc + 1);
  k.put('\t');
  const int l = e.ctx_len;  // tctx, abbreviated past 22 (pafreport.cpp:918-927)
  if (l <= 10 + kMaxEv) {
    for (int j = 0; j < l; j++) k.put(r.rev ? s.tab.comp[ctx[l - 1 - j]] : ctx[j]);
  } else {
    for (int j = 0; j < 5; j++) k.put(r.rev ? s.tab.comp[ctx[9 - j]] : ctx[j]);
    k.put('[');
    put_int(k, l - 10);
    k.put(']');
    for (int j = 0; j < 5; j++) k.put(r.rev ? s.tab.comp[ctx[4 - j]] : ctx[5 + j]);
  }
  k.put('\t');
  for (int j = 0; j < 9; j++) k.put(r.R[e.rctx0 + j]);
  k.put('\t');
  if (e.status == 0) put_str(k, "[unknown]");
  else if (e.status == 1) put_str(k, "homopolymer");
  else {
    put_str(k, "motif ");
    put_str(k, kMotif[e.status - 2]);
  }
  k.put('\t');
  if (!skip_codan) {
    if (e.type == PW_OP_SUB) put_sub_impact(k, r, s, e);
    else if (e.imp_kind == 1) {
      put_str(k, "premature stop at AA");
      put_int(k, e.imp_val);
    } else if (e.imp_kind == 2) {
      put_str(k, "frame shift ");
      for (int j = 0; j < e.aa4n; j++) k.put((uint8_t)(e.aa4 >> (8 * j)));
      k.put('+');
      k.put(':');
      for (int j = 0; j < e.maa4n; j++) k.put((uint8_t)(e.maa4 >> (8 * j)));
      k.put('+');
    }
  }
  k.put('\n');
}

// Indel consequence: predictImpact insert/cut + stop scan (pafreport.cpp:843-882).  The
// modified sequence is modseq = Q[r_trloc, rloc) + X + Q[s, L) with X the inserted bases
// (I) or nothing (D; s = rloc + len).  Codons touching the prefix / X / the first five codons
// are translated explicitly; past that, modseq codons are query codons and the first stop is
// one lookup in the next-stop table.
__device__ void indel_impact(const Rec& r, const Lds& s, Event& e) {
  const int a = e.rloc - e.r_trloc;
  const int x = (e.type == PW_OP_INS) ? e.n : 0;
  const int dl = (e.type == PW_OP_DEL) ? e.n : 0;
  const int sfx = e.rloc + dl;
  const int M = (r.L - e.r_trloc) + x - dl;
  const int trlen = r.L - e.r_trloc;
  int E = a + x;
  if (E < 15) E = 15;
  int stop_i = -1;
  e.aa4 = e.maa4 = 0;
  e.aa4n = e.maa4n = 0;
  int i = 0;
  for (; i + 2 < M && i < E; i += 3) {
    uint8_t m[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      int p = i + j;
      m[j] = (p < a) ? Rc(r, e.r_trloc + p) : (p < a + x ? ev_base(r, s, e, p - a) : Rc(r, sfx + p - a - x));
    }
    uint8_t mm = translate(s, m[0], m[1], m[2]);
    if (mm == '.') {
      stop_i = i;
      break;
    }
    if (i > 0 && e.maa4n < 4) {
      if (i + 2 < trlen) {
        e.aa4 |= (uint32_t)translate(s, Rc(r, e.r_trloc + i), Rc(r, e.r_trloc + i + 1), Rc(r, e.r_trloc + i + 2))
                 << (8 * e.aa4n);
        e.aa4n++;
      }
      e.maa4 |= (uint32_t)mm << (8 * e.maa4n);
      e.maa4n++;
    }
  }
  if (stop_i < 0 && i + 2 < M && r.NS) {
    int k0 = sfx + (i - a - x);
    if (k0 >= 0 && k0 < r.L) {
      int st = r.NS[k0];
      if (st != kNoStop) stop_i = st - sfx + a + x;
    }
  }
  if (stop_i >= 0) {
    e.imp_kind = 1;
    e.imp_val = 1 + (stop_i + e.r_trloc) / 3;
  } else if (e.aa4n > 0 && e.maa4n > 0) {
    e.imp_kind = 2;
  } else {
    e.imp_kind = 3;
  }
}

// ------------------------------------------------------------------ per-record driver
__device__ void process_record(const pw_report_args& A, Lds& s, uint32_t ai, int lane) {
  const pw_aln_desc d = A.desc[ai];
  const uint32_t qi = d.ref & 0x7FFFFFFFu;
  Rec r;
  r.ops = A.ops + d.op_begin;
  r.lits = A.lits;
  r.R = A.qseq + A.qoff[qi];
  r.L = A.qlen[qi];
  r.NS = A.next_stop ? A.next_stop + A.qoff[qi] : nullptr;
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
  bool prev_sub = false;
  uint32_t ev_base_idx = 0;
  int me_first = INT_MAX, me_last = -1, me_fa = 0, me_fb = 0, me_la = 0, me_lb = 0;  // modseq errors
  uint8_t* ctx = s.ctx + lane * kCtx;

  for (uint32_t base = 0; base < r.n_ops; base += kWave) {
    const uint32_t k = base + lane;
    const bool valid = k < r.n_ops;
    const uint32_t w = valid ? r.ops[k] : 0u;
    const uint32_t typ = w >> 30, len = w & 0x3FFFFFFFu;
    const uint32_t qadv = op_qadv(w), tadv = op_tadv(w), ladv = op_ladv(w);
    const uint32_t qi_ = wave_incl_scan(qadv, lane);
    const uint32_t ti_ = wave_incl_scan(tadv, lane);
    const uint32_t li_ = wave_incl_scan(ladv, lane);
    const int qs = qc + (int)(qi_ - qadv);
    const int ts = tc + (int)(ti_ - tadv);
    const uint32_t ls = lc + (li_ - ladv);
    const bool is_sub = valid && typ == PW_OP_SUB;
    const uint64_t submask = __ballot(is_sub);
    const bool prevsub = lane == 0 ? prev_sub : ((submask >> (lane - 1)) & 1ull) != 0;
    const bool head = valid && (typ == PW_OP_INS || typ == PW_OP_DEL || (is_sub && !prevsub));

    // base check of every '*' op (pafreport.cpp:550-554)
    bool bad = false;
    uint8_t qch = 0, rch = 0;
    const int qp = r.offset + qs;
    if (is_sub) {
      qch = r.lits[ls + 1];
      rch = aligned_char(r, s, qp);
      bad = qch != rch;
    }
    const uint64_t badmask = __ballot(bad);
    if (badmask) {
      const int fl = __builtin_ctzll(badmask);
      if (lane == fl) {
        pw_aln_result res;
        res.text_off = slot_lo;
        res.text_len = 0;
        res.n_events = 0;
        res.err = PW_REC_MISMATCH;
        res.err_a = qp;
        res.err_b = qch;
        res.err_c = rch;
        A.results[ai] = res;
      }
      return;
    }

    // ---- event fields (head lanes)
    Event e;
    int linelen = 0;
    if (head) {
      e.type = typ;
      e.q_pos = qp;
      e.ls = ls;
      if (is_sub) {
        int n = 1;
        const uint64_t after = (lane == 63) ? 0ull : (submask >> (lane + 1));
        const int avail = 63 - lane;
        const int ones = (int)__builtin_ctzll(~after);  // consecutive SUB lanes after this one
        n += ones < avail ? ones : avail;
        if (lane + n == kWave) {  // run reaches the chunk end: continue in the op stream
          uint32_t j = base + kWave;
          while (j < r.n_ops && (r.ops[j] >> 30) == PW_OP_SUB) {
            n++;
            j++;
          }
        }
        e.n = n;
      } else {
        e.n = (int)len;
      }
      // final coordinates (pafreport.cpp:562,593-598,611-616,630-640)
      const int evtlen = is_sub ? 1 : e.n;
      if (!r.rev) {
        e.rloc = qp;
        e.tloc = ts;
      } else {
        e.rloc = (typ == PW_OP_INS) ? r.L - qp : r.L - qp - e.n;
        e.tloc = r.T - ts;
      }
      // target context (setTContext, pafreport.cpp:120-128)
      int tcs = ts - 5;
      if (tcs < 0) tcs = 0;
      int tce = ts + (typ == PW_OP_DEL ? 0 : evtlen) + 5;
      if (tce >= r.T) tce = r.T - 1;
      int cl = tce - tcs;
      if (cl < 0) cl = 0;
      e.ctx_len = cl;
      Cursor cur;
      cur.j = k;
      cur.ts = ts;
      cur.qs = qs;
      cur.ls = ls;
      cur.w = w;
      if (cl <= 10 + kMaxEv) {
        gather_tseq(r, s, cur, tcs, tce, ctx);
      } else {
        gather_tseq(r, s, cur, tcs, tcs + 5, ctx);
        gather_tseq(r, s, cur, tce - 5, tce, ctx + 5);
      }
      // query context (getRefContext, pafreport.cpp:721-733)
      int c0 = e.rloc - 4, eloc = 4;
      if (c0 < 0) {
        eloc += c0;
        c0 = 0;
      } else if (c0 + 8 >= r.L) {
        eloc += r.L - c0 - 9;
        c0 = r.L - 9;
      }
      if (c0 < 0) c0 = 0;  // L < 9 is rejected on the host
      e.rctx0 = c0;
      e.rctx_loc = eloc;
      uint8_t rc9[9];
#pragma unroll
      for (int j = 0; j < 9; j++) rc9[j] = Rc(r, c0 + j);
      // homopolymer (hpolyCheck, pafreport.cpp:735-748)
      const uint8_t b0 = ev_base(r, s, e, 0);
      bool same = true;
      for (int i = 1; i < e.n && same; i++) same = ev_base(r, s, e, i) == b0;
      e.status = 0;
      if (same) {
        int l = -1;
        for (int p = 0; p + 4 <= 9 && l < 0; p++)
          if (rc9[p] == b0 && rc9[p + 1] == b0 && rc9[p + 2] == b0 && rc9[p + 3] == b0) l = p;
        if (l >= 0 && l <= eloc && l + 4 >= eloc) e.status = 1;
      }
      if (e.status == 0) {  // mmotifCheck: first motif in list order found anywhere
        for (int m = 0; m < 4 && e.status == 0; m++) {
          const char* mo = kMotif[m];
          const int ml = (m < 2) ? 5 : 4;
          for (int p = 0; p + ml <= 9; p++) {
            bool hit = true;
            for (int q = 0; q < ml; q++) hit = hit && rc9[p + q] == (uint8_t)mo[q];
            if (hit) {
              e.status = 2 + m;
              break;
            }
          }
        }
      }
      // amino acid at the event (pafreport.cpp:897-899)
      const int aap0 = e.rloc / 3;
      e.aa = translate(s, Rc(r, 3 * aap0), Rc(r, 3 * aap0 + 1), Rc(r, 3 * aap0 + 2));
      e.aapos = aap0 + 1;
      e.r_trloc = 3 * (e.aapos - 2);
      if (e.r_trloc < 0) e.r_trloc = 0;
      e.imp_kind = 0;
      if (!skip) {
        if (is_sub) {  // modseq check (pafreport.cpp:811-814)
          for (int i = 0; i < e.n; i++) {
            if (to_upper(Rc(r, e.rloc + i)) != to_upper(ev_sub(r, s, e, i))) {
              e.imp_kind = -1 - i;  // failing evtsub index, resolved after the chunk scan
              break;
            }
          }
        } else {
          indel_impact(r, s, e);
        }
      }
      CountSink cnt;
      render(cnt, r, s, e, ctx, skip);
      linelen = cnt.n;
    }

    // ---- chunk block placement
    const uint64_t headmask = __ballot(head);
    const uint32_t nh = (uint32_t)__popcll(headmask);
    const uint32_t incl = wave_incl_scan((uint32_t)linelen, lane);
    const uint32_t B = bcast(incl, kWave - 1);
    const int my_off = r.rev ? (int)(B - incl) : (int)(incl - (uint32_t)linelen);
    // modseq errors: keep the first / last failing event index
    {
      int fail_i = (head && e.type == PW_OP_SUB && e.imp_kind < 0) ? (-1 - e.imp_kind) : -1;
      const uint64_t fm = __ballot(fail_i >= 0);
      if (fm) {
        const int lo = __builtin_ctzll(fm), hi = 63 - __builtin_clzll(fm);
        const int gi_lo = (int)ev_base_idx + (int)__popcll(headmask & ((1ull << lo) - 1ull));
        const int gi_hi = (int)ev_base_idx + (int)__popcll(headmask & ((1ull << hi) - 1ull));
        const int fi_lo = __shfl(fail_i, lo, kWave), fi_hi = __shfl(fail_i, hi, kWave);
        const int rl_lo = __shfl(head ? e.rloc : 0, lo, kWave), rl_hi = __shfl(head ? e.rloc : 0, hi, kWave);
        const int tr_lo = __shfl(head ? e.r_trloc : 0, lo, kWave), tr_hi = __shfl(head ? e.r_trloc : 0, hi, kWave);
        if (gi_lo < me_first) {
          me_first = gi_lo;
          me_fa = rl_lo - tr_lo + fi_lo;
          me_fb = fi_lo;
        }
        if (gi_hi > me_last) {
          me_last = gi_hi;
          me_la = rl_hi - tr_hi + fi_hi;
          me_lb = fi_hi;
        }
      }
      if (head && e.type == PW_OP_SUB && e.imp_kind < 0) e.imp_kind = 0;
    }

    if (B > 0) {
      uint64_t g0;
      if (!r.rev) {
        g0 = out_lo;
        out_lo += B;
      } else {
        out_hi -= B;
        g0 = out_hi;
      }
      for (uint32_t w0 = 0; w0 < B; w0 += kStage) {
        const uint32_t wn = (B - w0) < (uint32_t)kStage ? (B - w0) : (uint32_t)kStage;
        if (head && (uint32_t)(my_off + linelen) > w0 && (uint32_t)my_off < w0 + wn) {
          WriteSink ws;
          ws.buf = s.stage;
          ws.pos = my_off;
          ws.lo = (int)w0;
          ws.hi = (int)(w0 + wn);
          render(ws, r, s, e, ctx, skip);
        }
        __syncthreads();
        uint8_t* dst = A.text + g0 + w0;
        for (uint32_t i = lane; i < wn; i += kWave) dst[i] = s.stage[i];
        __syncthreads();
      }
    }

    // ---- carries
    qc += (int)bcast(qi_, kWave - 1);
    tc += (int)bcast(ti_, kWave - 1);
    lc += bcast(li_, kWave - 1);
    prev_sub = ((submask >> 63) & 1ull) != 0;
    ev_base_idx += nh;
  }

  if (lane == 0) {
    pw_aln_result res;
    res.text_off = r.rev ? out_hi : slot_lo;
    res.text_len = (uint32_t)(r.rev ? (slot_hi - out_hi) : (out_lo - slot_lo));
    res.n_events = ev_base_idx;
    res.err = PW_REC_OK;
    res.err_a = res.err_b = res.err_c = 0;
    if (me_last >= 0) {  // first failing event in OUTPUT order
      res.err = PW_REC_MODSEQ;
      if (!r.rev) {
        res.err_a = me_fa;
        res.err_b = me_fb;
        res.err_c = me_first;
      } else {
        res.err_a = me_la;
        res.err_b = me_lb;
        res.err_c = (int)ev_base_idx - 1 - me_last;
      }
    }
    A.results[ai] = res;
  }
}

__global__ __launch_bounds__(kWave) void report_kernel(pw_report_args A) {
  __shared__ __attribute__((aligned(16))) Lds s;
  const int lane = threadIdx.x;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&c_tables);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&s.tab);
    for (int i = lane; i < (int)(sizeof(Tables) / 4); i += kWave) dst[i] = src[i];
  }
  __syncthreads();
  for (uint32_t ai = blockIdx.x; ai < A.n_alns; ai += gridDim.x) {
    process_record(A, s, ai, lane);
    __syncthreads();
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

extern "C" int pw_report_events(const pw_report_args* args, void* stream) {
  if (!args || !args->desc || !args->ops || !args->qseq || !args->qoff || !args->qlen || !args->results ||
      (!args->text && args->text_total))
    return PW_E_ARG;
  if (!args->skip_codan && !args->next_stop) return PW_E_ARG;
  if (args->n_alns == 0) return PW_OK;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  const uint32_t max_blocks = (uint32_t)ncu * 16u;
  const uint32_t grid = args->n_alns < max_blocks ? args->n_alns : max_blocks;
  hipLaunchKernelGGL(pw::report_kernel, dim3(grid), dim3(pw::kWave), 0, (hipStream_t)stream, *args);
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
