// pw_report.hip — the MI355X hot path of pafreport: cs decode -> event classifier -> codon
// consequence -> report-line rendering (gfx950, wave64).
//
// Reference behaviour restated here (gpertea/pwasm, /root/reference):
//   decode            PAFAlignment::PAFAlignment           pafreport.cpp:526-643
//   target context    TDiffInfo::setTContext + '-' fixups  pafreport.cpp:120-128, 628-643
//   ref context       getRefContext                        pafreport.cpp:721-733
//   homopolymer/motif hpolyCheck / mmotifCheck             pafreport.cpp:735-763
//   codon consequence predictImpact                        pafreport.cpp:801-883
//   event line        printDiffInfo (event loop)           pafreport.cpp:893-954
//
// One pass (pw_report_events) is these launches on one stream (pw_stop_table_build, the
// per-query next-stop table, may run on a side stream: pw_report_events_after):
//
//  plan_kernel,     only when a record has more than PW_BLOCK_OPS (2048) ops: such records are cut
//  carry_kernel     into blocks of 2048 ops; one wavefront per block sums its query / target /
//                   literal advance and event heads, so blocks can be decoded independently.
//  index_kernel     one wavefront per PAF record (per block of a long record): DPP wave prefix
//                   scans over the packed op stream give every op its query / target / literal
//                   coordinates (the sequential walk of pafreport.cpp:536-626), '*' ops are
//                   base-checked by ballot, directly consecutive '*' ops merged into one S event
//                   (:556-560), and every event is written as a 32-byte Hot record (+ a 16-byte
//                   Cold record for a record's first / last line) into its record's event slots,
//                   already in OUTPUT order ('-' records fill their slots back to front =
//                   tdiffs.Reverse(), :643).  Events whose target context needs an op walk are
//                   flagged for tctx_kernel.
//  tctx_kernel      a wavefront scans the flag bytes of its 256-slot groups (one group ahead),
//                   queues the flagged slots in an LDS list that carries across groups, and takes
//                   them 64 at a time, one event per lane: the lane walks its op stream through
//                   LDS windows (setTContext, :120-128) and writes a 32-byte pre-rendered
//                   target-context record.
//  render_kernel    lane-dense: wavefront g takes chunks g, g + NW, ... of 64 consecutive event
//                   slots (static stride, no work queue); each lane renders its event's report
//                   line into an LDS line buffer from its Hot record and a 48-byte forward-query
//                   window staged per lane (loaded one chunk ahead); a wave whose lanes all
//                   qualify renders through the RecFast instantiation (every read in registers
//                   or the window, no fallbacks).  A DPP scan of the line lengths places the
//                   lines in the chunk's page and the wave writes them with 16-byte stores.
//  fixup_kernel     lines longer than the line buffer (~0.06 %), rendered again straight to
//                   their reserved place in the page.
//  finalize_kernel  per-record results (text length across pages, event count, errors).
//
// The text is one contiguous stream of event lines in record order; record headers are
// formatted by the host (the only floating-point value, coverage:%.2f).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <limits.h>
#include <stdint.h>

#include "pw_tables.h"
#include "pwasm_amd.h"
#include "pw_wave.h"

namespace pw {

// LDS pointers carry their address space explicitly: a generic pointer here makes hipcc merge
// "LDS hit ? lds[o] : global[i]" into one flat load (global latency + vmcnt waits).
#define LDS __attribute__((address_space(3)))
typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // 16-byte copies
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v4a4 __attribute__((ext_vector_type(4), aligned(4)));  // 16 bytes at a dword address

__constant__ Tables c_tables = build_tables();

constexpr int kWave = 64;
constexpr int kWaves = 4;       // wavefronts per workgroup (independent; they share the tables)
constexpr int kSegOps = 128;    // index_kernel: ops per segment (2 per lane)
constexpr int kOpHalo = 16;     // index_kernel: op words staged before / after a segment
constexpr int kQWin = 48;       // render_kernel: forward-query window per lane (bytes)
constexpr int kQStride = 56;    // ... its LDS stride (14 dwords: same-offset dword reads at most 2-way)
constexpr int kLine = 108;      // render_kernel: report lines up to this long are built in LDS (all but ~1 in 10^4 at cfg2)
constexpr int kLSlack = 40;     // ... + slack: a field block writes at most 35 bytes past its start (the
                                // bases + tloc block of a 12-base S run), so none needs a bounds check
static_assert(kLine + kLSlack <= 148, "line buffer stride");
// Lines longer than kLine: a fast wave's line grows past its line buffer into its own query-window
// column (up to kAppMax bytes, below) and render stores the wave's first such line itself; the
// wave's other long lines of up to kLong bytes (kLongCap per wave) are emitted again after the
// wave's last chunk (render's epilogue), the rest by fixup_kernel
constexpr int kLong = 252;
constexpr int kLongCap = 4;
constexpr uint32_t kDropOff = 0xFFFFFF00u;  // a buffer-store offset past any range: the store is dropped
// the report text is written non-temporal (cache policy nt): no kernel reads it again, and left to
// the default policy its 303 MB per cfg2 pass linger dirty in the caches the next kernels (and the
// next pass's index / tctx) read through — round 5, same call: render 213 -> 197 us, index 126 ->
// 117, tctx 75 -> 71, pass 0.439 -> 0.408 ms (sc1, write-through that drops the line: no change)
constexpr int kTextPolicy = 2;
constexpr int kLStride = 148;  // line buffer stride (37 dwords, odd: lanes at the same line position hit 32 banks)
// (render's copy-out builds an in-place page, <= PW_PAGE_BYTES, over the wave's line buffers)
static_assert(kWave * kLStride >= PW_PAGE_BYTES, "the LDS page image must fit the wave's line buffers");
constexpr int kMaxEv = 12;      // MAX_EVLEN, pafreport.cpp:919
constexpr int32_t kNoStop = INT32_MAX;
constexpr uint32_t kNoEv = 0xFFFFFFFFu;  // empty event slot (merged '*' runs, failed records)
constexpr uint32_t kNBig = (1u << 19) - 1;  // evtbases length field saturates here
constexpr uint32_t kFnAcgt = 1u << 19;      // query + record literals all A/C/G/T (PW_REF_ACGT)
constexpr int kTx = 32;         // pre-rendered target-context record (length byte + field)
constexpr int kIndexOcc = 5;    // index_kernel: waves per SIMD the register budget is sized for
constexpr int kPairOcc = 4;     // index_pair_kernel: (two records per wave hold more live state: 128 VGPRs)
constexpr int kRenderOcc = 3;   // render_kernel: workgroups per CU (LDS-limited)

// Render record of one event (index_kernel -> render_kernel, tctx_kernel, fixup_kernel), decoded.
//   fn: type (31-30) | reverse (29) | fast tctx (28) | first line of its record (27) |
//       last line (26) | ll (25-23) | rl (22-20) | A/C/G/T only (19) | evtbases length (18-0,
//       saturated)
//   l0, l1: the event's first 8 literal bytes (SUB: target,query pairs; INS: inserted bases)
// In memory it is 32 bytes {fn, qp, tloc, ls | qb, L, l0, l1}, or — when the batch's query
// positions and indices fit (pw_report_args.hot_pbits = P != 0) — 16 bytes {fn, qi << P | qp, tloc,
// ls}: the query's start and length then come from qoff / qlen, the literal bytes from lits (loads
// the readers issue a stage before they need them).  fn is word 0 of either.
struct Hot {
  uint32_t qb;    // forward query start in qseq, in 16-byte units (qoff is 16-byte aligned)
  int32_t L;      // query length
  int32_t qp;     // offset + qpos at the event (aligned strand)
  int32_t tloc;   // printed tloc - 1 (pafreport.cpp:639)
  uint32_t ls;    // literal start
  uint32_t fn;
  uint32_t l0, l1;
};
// Cold record, 16 bytes: written only for a record's first / last line and saturated lengths.
struct Cold {
  uint32_t ai, j;  // record, head op
  int32_t qs, ts;  // query / target position at the head op
};
__device__ __forceinline__ uint32_t hot_fn(uint32_t typ, bool rev, bool fast, bool first, bool last, int ll, int rl,
                                           bool acgt, uint32_t n) {
  return typ << 30 | (rev ? 1u << 29 : 0u) | (fast ? 1u << 28 : 0u) | (first ? 1u << 27 : 0u) |
         (last ? 1u << 26 : 0u) | (uint32_t)(ll & 7) << 23 | (uint32_t)(rl & 7) << 20 | (acgt ? kFnAcgt : 0u) |
         (n < kNBig ? n : kNBig);
}

// Byte tables read per event (LDS copy per workgroup).  The IUPAC code / 4096-entry codon
// tables are only needed off {A,C,G,T} and are read from c_tables.
struct SmallTables {
  uint8_t comp[256];
  uint8_t codon64[64];
  uint8_t status[8][12];
  uint8_t dig2[200];  // "00" .. "99"
};

// ------------------------------------------------------------------ wave primitives
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int) { return wave_scan_incl(v); }
__device__ __forceinline__ uint32_t bcast(uint32_t v, int src) { return __shfl(v, src, kWave); }
// LDS written by some lanes of a wavefront and read by others of the SAME wavefront (the
// waves of a workgroup are independent): LDS operations of one wave execute in order, so only
// the compiler has to be kept from moving memory operations across this point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Global-address-space views (loads through them are global_load, not flat: a flat load also
// counts on lgkmcnt, so the next LDS wait would wait for it too)
#define PW_GLOBAL __attribute__((address_space(1)))
typedef const PW_GLOBAL uint8_t* GU8;
typedef PW_GLOBAL const v4u GV4;

// Prefetched registers are first touched where they are consumed, one or two chunks later: an
// empty asm that "rewrites" them there keeps the compiler from folding any use into the block
// that issued the load.  Every prefetch load is unconditional (a clamped or dummy address when
// the value is not needed): a load inside a branch costs an s_waitcnt vmcnt(0) at the join,
// since the count of loads issued after it differs between the paths.
__device__ __forceinline__ void pin(v4u& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }

// ------------------------------------------------------------------ record context
struct Rec {
  const uint32_t* ops;      // this record's ops (global)
  const uint8_t* lits;      // global literal array
  const uint8_t* R;         // forward query (global)
  const int32_t* NS;        // next-stop table of this query (or null)
  const LDS SmallTables* tab;
  const LDS uint8_t* qw;    // LDS forward-query window
  int qlo;                  // forward position of qw[0]
  int qn;                   // window bytes (0 = no window)
  const LDS uint32_t* opw;  // LDS op-word window (index_kernel)
  int op_lo;                // record op index of opw[0]
  uint32_t op_n;            // window ops (0 = none)
  uint32_t lit0, lit1;      // literal bytes [ls0, ls0 + ln) in registers (render_kernel)
  uint32_t ls0, ln;
  const LDS uint8_t* lw;    // LDS literal window [l_lo, l_lo + l_n) (index_kernel)
  uint32_t l_lo, l_n;
  int L;                    // query length
  int offset;               // start on the aligned strand
  int T;                    // tseq length
  uint32_t n_ops;
  bool rev;
  bool acgt;                // query and the record's literals are all A/C/G/T (register fast paths)
  static constexpr bool kFast = false;
};
// A render lane whose every read is known to hit its registers or its LDS query window (the
// render_kernel predicate fast_lane()): query bytes straight from the window, literal bytes from
// the Hot record's 8, codons from the A/C/G/T table, and every byte-wise fallback compiled out.
// A wavefront takes this instantiation of emit_event when all its lanes qualify.
struct RecFast : Rec {
  static constexpr bool kFast = true;
};

// Query byte x of the forward query, 0 outside [0, L) (the NUL / missing bytes).  The LDS
// window holds zeros where it extends past the query, so a window hit needs no bounds check.
// (outside the window: rare, kept out of line so the hot paths stay small)
__device__ __noinline__ uint8_t rc_global(const uint8_t* R, int L, int x) {
  return (unsigned)x < (unsigned)L ? R[x] : (uint8_t)0;
}
__device__ __forceinline__ uint8_t Rc(const Rec& r, int x) {
  const unsigned o = (unsigned)(x - r.qlo);
  if (o < (unsigned)r.qn) return r.qw[o];
  return rc_global(r.R, r.L, x);
}
__device__ __forceinline__ uint8_t Rc(const RecFast& r, int x) { return r.qw[x - r.qlo]; }
__device__ __noinline__ uint8_t lit_global(const uint8_t* lits, uint32_t i) { return lits[i]; }
__device__ __forceinline__ uint8_t litb(const Rec& r, uint32_t i) {
  const uint32_t o = i - r.ls0;
  if (o < r.ln) return (uint8_t)((o < 4 ? r.lit0 : r.lit1) >> (8 * (o & 3)));
  const uint32_t ow = i - r.l_lo;
  if (ow < r.l_n) return r.lw[ow];
  return lit_global(r.lits, i);
}
__device__ __forceinline__ uint8_t litb(const RecFast& r, uint32_t i) {
  const uint32_t o = i - r.ls0;
  return (uint8_t)((o < 4 ? r.lit0 : r.lit1) >> (8 * (o & 3)));
}
__device__ __forceinline__ uint32_t opword(const Rec& r, uint32_t j) {
  const unsigned o = (unsigned)((int)j - r.op_lo);
  return o < r.op_n ? r.opw[o] : r.ops[j];
}

// aligned-strand query char at p (refseq_rc for '-' records, pafreport.cpp:352-362); p == L
// reads the NUL terminator as the reference does.
__device__ __forceinline__ uint8_t aligned_char_g(const uint8_t* R, int L, bool rev, const LDS SmallTables* t, int p) {
  if ((unsigned)p >= (unsigned)L) return 0;
  return rev ? t->comp[R[L - 1 - p]] : R[p];
}

// translateCodon: three bases of {A,C,G,T} in either case take one lookup in codon64 (no
// dependent table reads); anything else goes through the IUPAC mask tables.
__device__ __forceinline__ bool is_acgt(uint32_t c) {
  // letters 0x40-0x7F whose low 5 bits are 1 (A), 3 (C), 7 (G) or 20 (T)
  return (c & 0xC0u) == 0x40u && ((0x0010008Au >> (c & 0x1Fu)) & 1u);
}
// (off {A,C,G,T}: rare, kept out of line so its table reads do not hold registers in the callers)
__device__ __noinline__ uint8_t translate_iupac(uint32_t a, uint32_t b, uint32_t c) {
  return c_tables.codon[(c_tables.nt[a] << 8) | (c_tables.nt[b] << 4) | c_tables.nt[c]];
}
__device__ __forceinline__ uint8_t translate(const LDS SmallTables* t, uint8_t a, uint8_t b, uint8_t c) {
  if (is_acgt(a) && is_acgt(b) && is_acgt(c))
    return t->codon64[((a >> 1) & 3u) << 4 | ((b >> 1) & 3u) << 2 | ((c >> 1) & 3u)];
  return translate_iupac(a, b, c);
}
// translateCodon as the record's lane needs it (a fast lane's bytes are all A/C/G/T)
template <class R>
__device__ __forceinline__ uint8_t tr(const R& r, uint8_t a, uint8_t b, uint8_t c) {
  if constexpr (R::kFast) return r.tab->codon64[((a >> 1) & 3u) << 4 | ((b >> 1) & 3u) << 2 | ((c >> 1) & 3u)];
  else return translate(r.tab, a, b, c);
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

// What a line needs besides the record: the event's coordinates and how to produce its tctx.
struct EvIn {
  uint32_t typ;
  int n, qp, tloc;
  uint32_t ls;
  int tmode;          // 0 fast (ll / rl), 1 pre-rendered by tctx_kernel (tx)
  int ll, rl;
  uint32_t tx[6];     // length byte + field (tmode 1): the tx record's first 24 bytes
  int ns_pre;         // next_stop entry the indel scan needs, loaded ahead (kNsNone: not loaded)
};
constexpr int kNsNone = INT_MIN;

// evtbases[i] in final orientation, upper case (pafreport.cpp:563,594-596,612-614,637,895)
template <class R>
__device__ __forceinline__ uint8_t ev_base(const R& r, const Event& e, int i) {
  if (e.type == PW_OP_SUB) return r.rev ? r.tab->comp[litb(r, e.ls + 2 * (e.n - 1 - i))] : litb(r, e.ls + 2 * i);
  if (e.type == PW_OP_INS) return r.rev ? r.tab->comp[litb(r, e.ls + (e.n - 1 - i))] : litb(r, e.ls + i);
  return r.rev ? comp2(Rc(r, e.rloc + i)) : Rc(r, e.q_pos + i);
}
// evtsub[i] (S only)
template <class R>
__device__ __forceinline__ uint8_t ev_sub(const R& r, const Event& e, int i) {
  return r.rev ? r.tab->comp[litb(r, e.ls + 2 * (e.n - 1 - i) + 1)] : litb(r, e.ls + 2 * i + 1);
}

// ---- 16-byte register images of query / modified-sequence bytes (indel fast path)
typedef unsigned __int128 u128;
// bytes qw[off, off + 16) of an LDS window (off >= 0; up to 4 bytes past off + 16 are read)
__device__ __forceinline__ u128 lds16(const LDS uint8_t* qw, int off) {
  const LDS uint32_t* p = reinterpret_cast<const LDS uint32_t*>(qw + (off & ~3));
  const uint32_t sh = (uint32_t)off & 3u;
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 5; i++) d[i] = p[i];
  u128 v = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) v |= (u128)__builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) << (32 * i);
  return v;
}
__device__ __forceinline__ u128 low_bytes(int n) {  // bytes [0, n) set, 0 <= n <= 15
  return n <= 0 ? (u128)0 : (((u128)1 << (8 * n)) - 1);
}
__device__ __forceinline__ uint32_t byte_at(u128 v, int p) { return (uint32_t)(v >> (8 * p)) & 0xFFu; }
// every byte of v in [0, 15) is one of A, C, G, T (upper case: query and literals are)
__device__ __forceinline__ bool acgt15(u128 v) {
  bool ok = true;
#pragma unroll
  for (int p = 0; p < 15; p++) ok = ok && is_acgt(byte_at(v, p));
  return ok;
}
// translateCodon of the codon at byte p of v (all ACGT): 2-bit codes, one codon64 lookup
__device__ __forceinline__ uint8_t codon_at(const LDS SmallTables* t, u128 v, int p) {
  const uint32_t c0 = (byte_at(v, p) >> 1) & 3u, c1 = (byte_at(v, p + 1) >> 1) & 3u, c2 = (byte_at(v, p + 2) >> 1) & 3u;
  return t->codon64[c0 << 4 | c1 << 2 | c2];
}
// complement of A/C/G/T bytes (A<->T: ^0x15, C<->G: ^0x04; bit 1 tells them apart).  Maps no
// other byte onto A/C/G/T, so a validity check after it still rejects non-ACGT input.
__device__ __forceinline__ uint32_t comp_acgt4(uint32_t v) {
  const uint32_t t = (v >> 1) & 0x01010101u, u = t ^ 0x01010101u;  // (0 / 1 per byte: shifts, no carries)
  return v ^ (t << 2 | u | u << 2 | u << 4);
}
__device__ __forceinline__ uint64_t comp_acgt8(uint64_t v) {
  return (uint64_t)comp_acgt4((uint32_t)v) | (uint64_t)comp_acgt4((uint32_t)(v >> 32)) << 32;
}

// bytes qw[off, off + 8) of an LDS window (off >= 0)
__device__ __forceinline__ uint64_t lds8(const LDS uint8_t* qw, int off) {
  const LDS uint32_t* p = reinterpret_cast<const LDS uint32_t*>(qw + (off & ~3));
  const uint32_t sh = (uint32_t)off & 3u;
  const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
  return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32;
}

// ------------------------------------------------------------------ line sinks
// LineSink writes into the lane's LDS line buffer; a store past the buffer or a masked-off
// character goes to the lane's junk byte (no branch).  A field is written through block(room,
// f): when `room` bytes are left it gets a RawSink — no per-character bounds check, a masked
// character is stored anyway and then overwritten, and runs of characters fold into the
// immediate offsets of the byte stores.  GlobalSink writes straight to global memory
// (fixup_kernel lines).
// Line bytes are stored one ds_write_b8 each through a volatile pointer: left alone, the compiler
// merges runs of byte stores at fixed offsets into ds_write_b64/b96/b128 at byte-aligned
// addresses, which the LDS replays at 64 cycles per wave-instruction (SQ_LDS_UNALIGNED_STALL).
__device__ __forceinline__ void st8(LDS uint8_t* p, uint8_t c) { *(volatile LDS uint8_t*)p = c; }
struct RawSink {
  LDS uint8_t* buf;
  int pos;
  __device__ __forceinline__ void put(uint8_t c) {
    st8(buf + pos, c);
    pos++;
  }
  __device__ __forceinline__ void put_if(bool pred, uint8_t c) {
    st8(buf + pos, c);
    pos += pred ? 1 : 0;
  }
  __device__ __forceinline__ void put_at(int i, uint8_t c) { st8(buf + i, c); }
  // bytes 1.. of w, n of them (n <= 4 * N - 1): all stored at fixed offsets, then pos += n
  template <int N>
  __device__ __forceinline__ void put_span(const uint32_t (&w)[N], int n) {
#pragma unroll
    for (int q = 0; q < 4 * N - 1; q++) st8(buf + pos + q, (uint8_t)(w[(q + 1) >> 2] >> (8 * ((q + 1) & 3))));
    pos += n;
  }
  // the first n bytes of w (all 4N stored at fixed offsets; the block reserved them)
  template <int N>
  __device__ __forceinline__ void put_bytes(const uint32_t (&w)[N], int n) {
#pragma unroll
    for (int q = 0; q < 4 * N; q++) st8(buf + pos + q, (uint8_t)(w[q >> 2] >> (8 * (q & 3))));
    pos += n;
  }
  template <class F>
  __device__ __forceinline__ void block(int, F&& f) {
    f(*this);
  }
};
template <class S, int N>
__device__ __forceinline__ void put_span_checked(S& k, const uint32_t (&w)[N], int n) {
#pragma unroll
  for (int q = 0; q < 4 * N - 1; q++) k.put_if(q < n, (uint8_t)(w[(q + 1) >> 2] >> (8 * ((q + 1) & 3))));
}
template <class S, int N>
__device__ __forceinline__ void put_bytes_checked(S& k, const uint32_t (&w)[N], int n) {
#pragma unroll
  for (int q = 0; q < 4 * N; q++) k.put_if(q < n, (uint8_t)(w[q >> 2] >> (8 * (q & 3))));
}
template <int CAP>
struct LdsSink {
  LDS uint8_t* buf;
  LDS uint8_t* junk;
  int pos;
  __device__ __forceinline__ void put(uint8_t c) {
    *(pos < CAP ? buf + pos : junk) = c;
    pos++;
  }
  __device__ __forceinline__ void put_if(bool pred, uint8_t c) {
    *((pred && pos < CAP) ? buf + pos : junk) = c;
    pos += pred ? 1 : 0;
  }
  __device__ __forceinline__ void put_at(int i, uint8_t c) { *(i < CAP ? buf + i : junk) = c; }
  template <int N>
  __device__ __forceinline__ void put_span(const uint32_t (&w)[N], int n) {
    put_span_checked(*this, w, n);
  }
  template <int N>
  __device__ __forceinline__ void put_bytes(const uint32_t (&w)[N], int n) {
    put_bytes_checked(*this, w, n);
  }
  template <class F>
  __device__ __forceinline__ void block(int room, F&& f) {
    if (pos + room <= CAP) {
      RawSink u{buf, pos};
      f(u);
      pos = u.pos;
    } else {
      f(*this);
    }
  }
};
// ClampSink: render_kernel's line buffer (kLine bytes + kLSlack).  Every field goes through a
// block of at most 35 bytes written with a RawSink (no per-character checks): a block starting
// at pos <= kLine ends inside the slack; once pos passes kLine the line is long (fixup_kernel
// rewrites it) and the block is folded back onto the slack.
struct ClampSink {
  LDS uint8_t* line;
  int pos;
  int lim;  // kLine (the lane's line buffer) or kLong - kLSlack (render's epilogue)
  template <class F>
  __device__ __forceinline__ void block(int, F&& f) {
    const int p0 = pos < lim ? pos : lim;
    RawSink u{line + (p0 - pos), pos};
    f(u);
    pos = u.pos;
  }
  __device__ __forceinline__ void put(uint8_t c) {
    st8(line + (pos < lim ? pos : lim), c);
    pos++;
  }
};
typedef ClampSink LineSink;
struct GlobalSink {
  PW_GLOBAL uint8_t* p;
  int pos;
  __device__ __forceinline__ void put(uint8_t c) { p[pos++] = c; }
  __device__ __forceinline__ void put_if(bool pred, uint8_t c) {
    if (pred) p[pos++] = c;
  }
  __device__ __forceinline__ void put_at(int i, uint8_t c) { p[i] = c; }
  template <int N>
  __device__ __forceinline__ void put_span(const uint32_t (&w)[N], int n) {
    put_span_checked(*this, w, n);
  }
  template <int N>
  __device__ __forceinline__ void put_bytes(const uint32_t (&w)[N], int n) {
    put_bytes_checked(*this, w, n);
  }
  template <class F>
  __device__ __forceinline__ void block(int, F&& f) {
    f(*this);
  }
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
    if (t == PW_OP_MATCH) {
      // a match run inside the query and the window: its query bytes as 8-byte images (one LDS
      // round trip per 8 bytes instead of one per byte: a byte read could not pass the previous
      // byte's store to the sink, which may alias it)
      const int xa = r.offset + c.qs + (p - c.ts), cnt = pe - p;
      const int fs = r.rev ? r.L - xa - cnt : xa;  // first forward position of the run's bytes
      const int o = fs - r.qlo;
      if (xa >= 0 && xa + cnt <= r.L && o >= 0 && o + cnt <= r.qn) {
        for (int q = 0; q < cnt; q += 8) {
          const uint64_t v = lds8(r.qw, o + q);
#pragma unroll
          for (int b = 0; b < 8; b++) {
            if (q + b >= cnt) break;
            const uint8_t f = (uint8_t)(v >> (8 * b));
            // forward byte fs + q + b: aligned position xa + q + b ('+'), or L - 1 - (fs + q + b)
            // = xa + cnt - 1 - (q + b) ('-', complemented)
            const int pp = r.rev ? p + cnt - 1 - (q + b) : p + q + b;
            k.put_at(r.rev ? base + (p1 - 1 - pp) : base + (pp - p0), r.rev ? comp2(f) : f);
          }
        }
        p = pe;
        continue;
      }
    }
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

// "%d" of a non-negative int, digit by digit (numbers >= 10^8, abbreviation lengths: rare).  Inline:
// an out-of-line call taking the sink by reference put the sink in a scratch segment (no report
// kernel has one now)
template <class S>
__device__ __forceinline__ void wr_dig(S& k, uint32_t v) {
  for (uint32_t P = 1000000000u; P >= 10u; P /= 10u) k.put_if(v >= P, (uint8_t)('0' + (v / P) % 10u));
  k.put((uint8_t)('0' + v % 10u));
}
// "%d" through the digit-pair table for v < 10^8 (up to four LDS reads, the digits stored at
// fixed offsets; needs 8 bytes of room)
template <class S>
__device__ __forceinline__ void wr_num(S& k, const LDS SmallTables* t, uint32_t v) {
  const LDS uint16_t* d2 = reinterpret_cast<const LDS uint16_t*>(t->dig2);
  if (v < 10000u) {
    const uint32_t hi = v / 100u, lo = v - 100u * hi;
    const uint32_t p = (uint32_t)d2[hi] | (uint32_t)d2[lo] << 16;
    const int nd = 1 + (v >= 10u) + (v >= 100u) + (v >= 1000u);
    const uint32_t w[1] = {p >> (8 * (4 - nd))};
    k.put_bytes(w, nd);
  } else if (v < 100000000u) {
    const uint32_t h = v / 10000u, l = v - 10000u * h;
    const uint32_t hh = h / 100u, hl = h - 100u * hh, lh = l / 100u, ll = l - 100u * lh;
    const uint64_t p = (uint64_t)d2[hh] | (uint64_t)d2[hl] << 16 | (uint64_t)d2[lh] << 32 | (uint64_t)d2[ll] << 48;
    const int nd = 5 + (h >= 10u) + (h >= 100u) + (h >= 1000u);
    const uint64_t q = p >> (8 * (8 - nd));
    const uint32_t w[2] = {(uint32_t)q, (uint32_t)(q >> 32)};
    k.put_bytes(w, nd);
  } else {
    wr_dig(k, v);
  }
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

// Target-context geometry of an event (setTContext, pafreport.cpp:120-128): context [tcs, tce)
// of cl bases, ll target bases before the event, nm of its own, rl after.
struct TGeom {
  int tcs, tce, cl, ll, nm, rl;
};
__device__ __forceinline__ TGeom tgeom(int T, uint32_t typ, int n, int ts) {
  TGeom g;
  const int evtlen = typ == PW_OP_SUB ? 1 : n;  // merged S keeps evtlen 1 (pafreport.cpp:562)
  g.tcs = ts - 5;
  if (g.tcs < 0) g.tcs = 0;
  g.tce = ts + (typ == PW_OP_DEL ? 0 : evtlen) + 5;
  if (g.tce >= T) g.tce = T - 1;
  g.cl = g.tce - g.tcs;
  if (g.cl < 0) g.cl = 0;
  g.ll = ts - g.tcs;
  g.nm = typ == PW_OP_DEL ? 0 : (typ == PW_OP_SUB ? 1 : n);
  g.rl = g.tce - (ts + g.nm);
  return g;
}
// Fast target context: match runs on both sides cover it (the common case), so it is query
// bytes, the event's own target bases, query bytes — no op walk.  pw / aw: the op words before
// the event and after its head op.
__device__ __forceinline__ bool tctx_fast(const TGeom& g, uint32_t typ, int n, uint32_t pw, bool has_pw, uint32_t aw,
                                          bool has_aw) {
  return g.cl <= 10 + kMaxEv && (typ != PW_OP_SUB || n == 1) && g.rl >= 0 &&
         (g.ll == 0 || (has_pw && (pw >> 30) == PW_OP_MATCH && (int)(pw & 0x3FFFFFFFu) >= g.ll)) &&
         (g.rl == 0 || (has_aw && (aw >> 30) == PW_OP_MATCH && (int)(aw & 0x3FFFFFFFu) >= g.rl));
}

// The tctx field, fast form: ll query bytes, the event's own target bases, rl query bytes.
template <class S, class R>
__device__ __forceinline__ void emit_tctx_fast(S& k, const R& r, uint32_t typ, int n, int qp, uint32_t ls, int ll,
                                               int rl) {
  const int nm = typ == PW_OP_DEL ? 0 : (typ == PW_OP_SUB ? 1 : n);
  // aligned query start after the event; '-' records read the forward query in the other
  // order (revCompl of tctx: comp(comp(x)) = x up to U)
  const int qpa = qp + (typ == PW_OP_SUB ? 1 : (typ == PW_OP_DEL ? n : 0));
  const int f1 = r.rev ? r.L - qpa - rl : qp - ll, n1 = r.rev ? rl : ll;
  const int f2 = r.rev ? r.L - qp : qpa, n2 = r.rev ? ll : rl;
  const int o1 = f1 - r.qlo, o2 = f2 - r.qlo;
  if (R::kFast || (r.acgt && r.qn == kQWin && o1 >= 0 && o2 >= 0 && o1 + 8 <= kQWin && o2 + 8 <= kQWin && r.ln == 8 &&
                    ls == r.ls0 && nm <= 8)) {
    // register images (comp2 is the identity on A/C/G/T): 8 query bytes each side, the event's
    // target bases from the literal registers, lower case
    const uint64_t a = lds8(r.qw, o1), b = lds8(r.qw, o2);
    const uint64_t l64 = (uint64_t)r.lit1 << 32 | r.lit0;
    uint64_t m = typ == PW_OP_SUB ? (l64 & 0xFFull) : l64;
    if (r.rev) m = nm > 0 ? comp_acgt8(__builtin_bswap64(m) >> (8 * (8 - nm))) : 0ull;
    m |= 0x2020202020202020ull;
    const uint32_t wa[2] = {(uint32_t)a, (uint32_t)(a >> 32)}, wm[2] = {(uint32_t)m, (uint32_t)(m >> 32)},
                   wb[2] = {(uint32_t)b, (uint32_t)(b >> 32)};
    k.put_bytes(wa, n1);
    k.put_bytes(wm, nm);
    k.put_bytes(wb, n2);
    return;
  }
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
}

// The tctx field by walking the op stream (setTContext, pafreport.cpp:120-128; revCompl :631;
// abbreviation first5[len-10]last5, :918-927).
template <class S>
__device__ __forceinline__ void emit_tctx_walk(S& k, const Rec& r, uint32_t typ, int n, uint32_t j, uint32_t wd,
                                               int qs, int ts, uint32_t ls) {
  const TGeom g = tgeom(r.T, typ, n, ts);
  Cursor cur;
  cur.j = j;
  cur.ts = ts;
  cur.qs = qs;
  cur.ls = ls;
  cur.w = wd;
  if (g.cl <= 10 + kMaxEv) {
    emit_tseq(k, r, cur, g.tcs, g.tce, k.pos);
    k.pos += g.cl;
  } else {
    emit_tseq(k, r, cur, r.rev ? g.tce - 5 : g.tcs, r.rev ? g.tce : g.tcs + 5, k.pos);
    k.pos += 5;
    k.put('[');
    wr_dig(k, (uint32_t)(g.cl - 10));
    k.put(']');
    emit_tseq(k, r, cur, r.rev ? g.tcs : g.tce - 5, r.rev ? g.tcs + 5 : g.tce, k.pos);
    k.pos += 5;
  }
}

// S consequence, one codon of modseq (predictImpact, pafreport.cpp:811-826)
template <class R>
__device__ __forceinline__ void sub_codon(const R& r, const Event& e, int ao, uint8_t& aa, uint8_t& maa) {
  const int p0 = e.rloc - e.r_trloc;
  uint8_t m[3], o[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const int pos = 3 * ao + j;
    o[j] = Rc(r, e.r_trloc + pos);
    m[j] = (pos >= p0 && pos < p0 + e.n) ? ev_base(r, e, pos - p0) : o[j];
  }
  aa = tr(r, o[0], o[1], o[2]);
  maa = tr(r, m[0], m[1], m[2]);
}

// The five codons of modseq and the four reference codons after the first (predictImpact's
// scan, pafreport.cpp:854-870) from register images when the event's neighbourhood is in the
// LDS window, inside the query and all A/C/G/T (the common case; anything else -> false and
// the byte-wise path).  m(p) = Q[r_trloc + p] (p < a), X[p - a] (a <= p < a + x),
// Q[r_trloc + p + dl - x] (after the event).
template <class R>
__device__ __forceinline__ bool indel_codons_fast(const R& r, const Event& e, int a, int x, int dl, uint8_t (&mm)[5],
                                                  uint8_t (&rr)[5]) {
  if constexpr (!R::kFast) {
    if (!r.acgt || r.qn != kQWin || x > 8 || a + x > 15) return false;
    if (x > 0 && (r.ln != 8 || e.ls != r.ls0)) return false;  // inserted bases not in registers
  }
  const int o0 = e.r_trloc - r.qlo, o1 = o0 + dl - x;
  if (!R::kFast && (o0 < 0 || o1 < 0 || o0 + 16 > kQWin || o1 + 16 > kQWin)) return false;
  const u128 q0 = lds16(r.qw, o0), q1 = lds16(r.qw, o1);
  u128 xs = 0;
  if (x > 0) {
    const uint64_t l64 = (uint64_t)r.lit1 << 32 | r.lit0;
    uint64_t xv = r.rev ? comp_acgt8(__builtin_bswap64(l64) >> (8 * (8 - x))) : l64;
    if (x < 8) xv &= (1ull << (8 * x)) - 1ull;
    xs = (u128)xv << (8 * a);
  }
  const u128 ma = low_bytes(a), mx = low_bytes(a + x) & ~ma;
  const u128 m = (q0 & ma) | (xs & mx) | (q1 & ~(ma | mx));
  // (bytes past the query end are the zero padding: they only reach codons the scan does not
  // use, 3c + 2 >= |modseq| or >= |r_trseq|)
#pragma unroll
  for (int c = 0; c < 5; c++) {
    mm[c] = codon_at(r.tab, m, 3 * c);
    rr[c] = c == 0 ? 0 : codon_at(r.tab, q0, 3 * c);
  }
  return true;
}

// S run of n <= 4 (predictImpact's substitution branch, pafreport.cpp:806-838) from register
// images: q0 = Q[r_trloc, +16), m = q0 with evtbases at [p0, p0 + n); the modseq check
// (:811-814) compares q0 with evtsub.  false -> the byte-wise path.
__device__ __forceinline__ uint32_t pack_even4(uint64_t v) {  // bytes 0, 2, 4, 6 of v
  return (uint32_t)(v & 0xFFu) | (uint32_t)((v >> 8) & 0xFF00u) | (uint32_t)((v >> 16) & 0xFF0000u) |
         (uint32_t)((v >> 24) & 0xFF000000u);
}
template <class R>
__device__ __forceinline__ bool sub_image(const R& r, const Event& e, int p0, u128& q0, u128& m, int& modseq_err) {
  // (codons up to byte 8 of q0 are read: all inside the query, none reaches the NUL)
  if (!R::kFast && (!r.acgt || r.qn != kQWin || e.n > 4 || r.ln != 8 || e.ls != r.ls0 || e.r_trloc + 9 > r.L))
    return false;
  const int o0 = e.r_trloc - r.qlo;
  if (!R::kFast && (o0 < 0 || o0 + 16 > kQWin)) return false;
  q0 = lds16(r.qw, o0);
  const uint64_t l64 = (uint64_t)r.lit1 << 32 | r.lit0;  // (target, query) pairs
  uint32_t alt = pack_even4(l64), sub = pack_even4(l64 >> 8);
  const int n = e.n;
  if (r.rev) {  // evtbases / evtsub reversed and complemented (pafreport.cpp:636-637)
    alt = comp_acgt4(__builtin_bswap32(alt) >> (8 * (4 - n)));
    sub = comp_acgt4(__builtin_bswap32(sub) >> (8 * (4 - n)));
  }
  const uint32_t nm = n == 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
  const u128 place = (u128)nm << (8 * p0);
  m = (q0 & ~place) | ((u128)(alt & nm) << (8 * p0));
  const uint32_t diff = ((uint32_t)(q0 >> (8 * p0)) ^ sub) & nm;
  modseq_err = diff ? (int)(__builtin_ctz(diff) >> 3) : -1;
  return true;
}

// Indel consequence: predictImpact insert/cut + stop scan (pafreport.cpp:843-882), written to
// the sink.  modseq = Q[r_trloc, rloc) + X + Q[s, L) with X the inserted bases (I) or nothing
// (D; s = rloc + len).  Codons touching the prefix / X / the first five codons are translated
// explicitly; past that, modseq codons are query codons and the first stop is one lookup in the
// next-stop table.
template <class S, class R>
__device__ __forceinline__ void indel_impact(S& k, const R& r, const Event& e, int ns_pre) {
  const int a = e.rloc - e.r_trloc;
  const int x = (e.type == PW_OP_INS) ? e.n : 0;
  const int dl = (e.type == PW_OP_DEL) ? e.n : 0;
  const int sfx = e.rloc + dl;
  const int M = (r.L - e.r_trloc) + x - dl;
  const int trlen = r.L - e.r_trloc;
  int stop_i = -1;
  uint32_t aa4 = 0, maa4 = 0;
  int aa4n = 0, maa4n = 0;
  if (R::kFast || a + x <= 15) {  // (a fast lane's insertion is at most 8 bases)
    // the reference scans codons i = 0,3,..,12 (while i+2 < M), stopping at the first stop;
    // here all five codons and the four reference codons are read and translated at once
    // (independent reads, no loop-carried latency) and the scan is replayed on the results
    uint8_t mm[5], rr[5];
    if (!indel_codons_fast(r, e, a, x, dl, mm, rr)) {
      uint8_t m[15];
#pragma unroll
      for (int p = 0; p < 15; p++) {
        const uint8_t q = Rc(r, p < a ? e.r_trloc + p : sfx + p - a - x);
        const int ii = p - a;
        const uint32_t li = e.ls + (uint32_t)(r.rev ? x - 1 - ii : ii);
        const uint8_t ib = (ii >= 0 && ii < x) ? litb(r, li) : (uint8_t)0;
        m[p] = (ii >= 0 && ii < x) ? (r.rev ? r.tab->comp[ib] : ib) : q;
      }
#pragma unroll
      for (int c = 0; c < 5; c++) {
        mm[c] = tr(r, m[3 * c], m[3 * c + 1], m[3 * c + 2]);
        rr[c] = c == 0 ? 0 : tr(r, Rc(r, e.r_trloc + 3 * c), Rc(r, e.r_trloc + 3 * c + 1),
                                       Rc(r, e.r_trloc + 3 * c + 2));
      }
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
        const int st = ns_pre != kNsNone ? ns_pre : r.NS[k0];
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
      const uint8_t mm = tr(r, m[0], m[1], m[2]);
      if (mm == '.') {
        stop_i = i;
        break;
      }
      if (i > 0 && maa4n < 4) {
        if (i + 2 < trlen) {
          aa4 |= (uint32_t)tr(r, Rc(r, e.r_trloc + i), Rc(r, e.r_trloc + i + 1),
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
    k.block(30, [&](auto& o) {
      wr_lit(o, "premature stop at AA");
      wr_num(o, r.tab, (uint32_t)(1 + (stop_i + e.r_trloc) / 3));
    });
  } else if (aa4n > 0 && maa4n > 0) {
    k.block(23, [&](auto& o) {
      wr_lit(o, "frame shift ");
#pragma unroll
      for (int q = 0; q < 4; q++) o.put_if(q < aa4n, (uint8_t)(aa4 >> (8 * q)));
      o.put('+');
      o.put(':');
#pragma unroll
      for (int q = 0; q < 4; q++) o.put_if(q < maa4n, (uint8_t)(maa4 >> (8 * q)));
      o.put('+');
    });
  }
}

// forward-query position the event's reads centre on (its final rloc, pafreport.cpp:597,615,633)
__device__ __forceinline__ int event_rloc(int L, bool rev, uint32_t typ, int qp, int n) {
  if (!rev) return qp;
  return (typ == PW_OP_INS) ? L - qp : L - qp - n;
}

// Write one event's report line (printDiffInfo, pafreport.cpp:886-953) to the sink as the
// fields become known.  Returns the evtsub index failing the modseq check
// (pafreport.cpp:811-814), or -1; `rel` receives rloc - r_trloc for the error message.
template <class S, class R>
__device__ __forceinline__ int emit_event(S& k, const R& r, const EvIn& in, bool skip, int& rel) {
  Event e;
  const uint32_t typ = in.typ;
  e.type = typ;
  e.q_pos = in.qp;
  e.ls = in.ls;
  e.n = in.n;
  e.rloc = event_rloc(r.L, r.rev, typ, in.qp, in.n);
  // amino acid at the event (pafreport.cpp:897-899)
  const int aap0 = e.rloc / 3;
  const uint8_t aa = tr(r, Rc(r, 3 * aap0), Rc(r, 3 * aap0 + 1), Rc(r, 3 * aap0 + 2));
  e.r_trloc = aap0 > 0 ? 3 * (aap0 - 1) : 0;  // 3*(aapos-2), clipped at 0
  rel = e.rloc - e.r_trloc;

  // ---- "E\trloc\taapos(aa)\t"
  k.block(27, [&](auto& o) {
      o.put(typ == PW_OP_SUB ? 'S' : (typ == PW_OP_INS ? 'I' : 'D'));
      o.put('\t');
      wr_num(o, r.tab, (uint32_t)(e.rloc + 1));
      o.put('\t');
      wr_num(o, r.tab, (uint32_t)(aap0 + 1));
      o.put('(');
      o.put(aa);
      o.put(')');
      o.put('\t');
    });
  // ---- bases field ("[n]" past MAX_EVLEN, pafreport.cpp:928-941); homopolymer uniformity; tloc
  const bool big = !R::kFast && e.n > kMaxEv;
  const uint8_t b0 = ev_base(r, e, 0);
  bool same = true;
  if (big)
    for (int i = 1; i < e.n; i++) same = same && ev_base(r, e, i) == b0;
  k.block((big ? 27 : 2 * e.n + 1) + 12, [&](auto& o) {
    if (typ == PW_OP_SUB) {
      if (big) {
        o.put('[');
        wr_dig(o, (uint32_t)e.n);
        o.put(']');
      } else {
        for (int i = 0; i < e.n; i++) o.put(ev_sub(r, e, i));
      }
    }
    if (typ != PW_OP_DEL) o.put(':');
    if (big) {
      o.put('[');
      wr_dig(o, (uint32_t)e.n);
      o.put(']');
    } else {
      for (int i = 0; i < e.n; i++) {
        const uint8_t b = ev_base(r, e, i);
        same = same && b == b0;
        o.put(b);
      }
    }
    if (typ == PW_OP_DEL) o.put(':');
    o.put('\t');
    wr_num(o, r.tab, (uint32_t)(in.tloc + 1));
    o.put('\t');
  });
  // ---- target context (setTContext :120-128, revCompl :631, abbreviation :918-927)
  {
    k.block(10 + kMaxEv + 4, [&](auto& o) {
      if (in.tmode == 0) {
        emit_tctx_fast(o, r, typ, e.n, in.qp, in.ls, in.ll, in.rl);
      } else {
        o.put_span(in.tx, (int)(in.tx[0] & 0xFFu));
      }
    });
  }
  k.put('\t');
  // ---- query context (getRefContext, pafreport.cpp:721-733) + status
  int c0 = e.rloc - 4, eloc = 4;
  if (c0 < 0) {
    eloc += c0;
    c0 = 0;
  } else if (c0 + 8 >= r.L) {
    eloc += r.L - c0 - 9;
    c0 = r.L - 9;
  }
  if (c0 < 0) c0 = 0;  // L < 9 is reported by the host
  {
    uint32_t rw0 = 0, rw1 = 0, rw2 = 0;
    const int oc = c0 - r.qlo;
    if (R::kFast || (r.qn == kQWin && oc >= 0 && oc + 16 <= kQWin)) {  // one image from the window
      const u128 im = lds16(r.qw, oc);
      rw0 = (uint32_t)im;
      rw1 = (uint32_t)(im >> 32);
      rw2 = (uint32_t)(im >> 64) & 0xFFu;
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        rw0 |= (uint32_t)Rc(r, c0 + q) << (8 * q);
        rw1 |= (uint32_t)Rc(r, c0 + 4 + q) << (8 * q);
      }
      rw2 = Rc(r, c0 + 8);
    }
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
    const LDS uint32_t* sw = reinterpret_cast<const LDS uint32_t*>(r.tab->status[st]);  // one table row
    const uint32_t sv[3] = {sw[0], sw[1], sw[2]};
    const int sl = (int)(sv[2] >> 24);
    const uint32_t rv[3] = {rw0, rw1, rw2 | (uint32_t)'\t' << 8};
    k.block(23, [&](auto& o) {
      o.put_bytes(rv, 10);
      o.put_bytes(sv, sl);
      o.put('\t');
    });
  }
  // ---- codon consequence (predictImpact, pafreport.cpp:801-883)
  int modseq_err = -1;
  if (!skip) {
    if (typ == PW_OP_SUB) {
      const int p0 = e.rloc - e.r_trloc;
      u128 q0 = 0, mi = 0;
      const bool fs = sub_image(r, e, p0, q0, mi, modseq_err);
      if (!fs)
        for (int i = 0; i < e.n; i++)
          if (modseq_err < 0 && to_upper(Rc(r, e.rloc + i)) != to_upper(ev_sub(r, e, i))) modseq_err = i;
      bool any = false;
      for (int ao = p0 / 3; ao <= (p0 + e.n - 1) / 3; ao++) {
        uint8_t caa, cmaa;
        if (fs) {
          caa = codon_at(r.tab, q0, 3 * ao);
          cmaa = codon_at(r.tab, mi, 3 * ao);
        } else {
          sub_codon(r, e, ao, caa, cmaa);
        }
        if (caa != cmaa) {
          const uint32_t ap = (uint32_t)(ao + e.rloc / 3);
          k.block(18, [&](auto& o) {
            if (any) wr_lit(o, ", ");
            wr_lit(o, "AA");
            wr_num(o, r.tab, ap);
            o.put('|');
            o.put(caa);
            o.put(':');
            o.put(cmaa);
          });
          if (cmaa == '.')
            k.block(31, [&](auto& o) {
              wr_lit(o, "|premature stop at AA");
              wr_num(o, r.tab, ap);
            });
          any = true;
        }
      }
      if (!any) k.block(10, [&](auto& o) { wr_lit(o, "synonymous"); });
    } else {
      indel_impact(k, r, e, in.ns_pre);
    }
  }
  k.put('\n');
  return modseq_err;
}

// ------------------------------------------------------------------ render fast path: dword lines
// The RecFast case of emit_event (every read in registers or the lane's query window, A/C/G/T,
// numbers below 10^8) restated with register images: each field is composed in VGPRs (numbers by
// SWAR decimal conversion, bases from the literal registers or the window, codons by one multiply
// per codon index) and appended to the lane's line buffer as whole dwords — the partial dword at
// the line end is read back and merged with v_perm, so a 16-byte field costs one read, five perms
// and three stores instead of sixteen byte stores.  Same bytes as emit_event (pafreport.cpp:886-953).
// The fast path's line buffers and query windows are lane-interleaved: dword k of a lane's buffer
// is at k * kTS dwords + lane (kTS = 64: a wave's buffers as rows of 256 bytes).  Every lane's
// dword access then hits bank lane mod 32 whatever its line position or window offset — with
// per-lane contiguous buffers those positions are data-dependent and a wave's dword accesses met
// 2-4-way bank conflicts (render: 37 % of its LDS cycles).
constexpr int kTS = kWave;
struct DLine {
  LDS uint8_t* buf;  // the lane's dword column of the wave's interleaved line buffers (kLine + kLSlack bytes)
  int pos;
};
// The wave's interleaved buffers and windows are kIlvRows rows, the query windows last: a line
// grows past its buffer into its own window column, which emit_fast has read for the last time by
// then (a line reaches ~101 bytes at most before the codon consequence, whose window reads come
// first).  Past kAppMax an append is folded back (that line goes elsewhere): every append writes
// at most 7 dwords.
constexpr int kIlvRows = (kLStride + kQStride) / 4;
constexpr int kAppMax = (kIlvRows - 7) * 4;
// append bytes [0, n) of f (4D bytes; bytes past n may be anything) at the line end
template <int D>
__device__ __forceinline__ void app(DLine& L, const uint32_t (&f)[D], int n) {
  const int p = L.pos;
  const int a = min(p & ~3, kAppMax);
  const uint32_t sh = (uint32_t)p & 3u;
  LDS uint32_t* d = reinterpret_cast<LDS uint32_t*>(L.buf) + (a >> 2) * kTS;
  const uint32_t cur = d[0];  // bytes [a, p) of the line
  // result byte j of dword i = stream byte 4i + j - sh: selector 4 - sh + j over {f[i], f[i - 1]};
  // dword 0 keeps its first sh bytes from cur
  const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, sh, 0u);  // (byte 0 of sh in every byte)
  const uint32_t m = (uint32_t)((1ull << (8 * sh)) - 1ull);
  const uint32_t sel0 = (sel & ~m) | (0x03020100u & m);
  uint32_t g[D + 1];
  g[0] = __builtin_amdgcn_perm(f[0], cur, sel0);
#pragma unroll
  for (int i = 1; i < D; i++) g[i] = __builtin_amdgcn_perm(f[i], f[i - 1], sel);
  g[D] = __builtin_amdgcn_perm(0u, f[D - 1], sel);
#pragma unroll
  for (int i = 0; i <= D; i++) d[i * kTS] = g[i];
  L.pos = p + n;
}
// OR the bytes of w into img at byte offset k (k + the bytes w uses <= 4N)
template <int N>
__device__ __forceinline__ void or_at(uint32_t (&img)[N], uint32_t w, int k) {
  const uint64_t v = (uint64_t)w << (8 * (k & 3));
  const int q = k >> 2;
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
  for (int i = 0; i < N; i++) img[i] |= (q == i ? lo : 0u) | (q == i - 1 ? hi : 0u);
}
__device__ __forceinline__ uint32_t keep32(uint32_t v, int n) {  // bytes [0, n) of v (n clamped to [0, 4])
  return n >= 4 ? v : (n <= 0 ? 0u : (v & ((1u << (8 * n)) - 1u)));
}
__device__ __forceinline__ uint64_t keep64(uint64_t v, int n) {  // bytes [0, n) of v (n clamped to [0, 8])
  return n >= 8 ? v : (n <= 0 ? 0ull : (v & ((1ull << (8 * n)) - 1ull)));
}
// N dwords of a lane-interleaved LDS window (qw: the lane's column) from byte offset off (off >=
// -8; reads one dword past them)
template <int N>
__device__ __forceinline__ void lds_img(const LDS uint8_t* qw, int off, uint32_t (&o)[N]) {
  const LDS uint32_t* p = reinterpret_cast<const LDS uint32_t*>(qw) + (off >> 2) * kTS;
  const uint32_t sh = (uint32_t)off & 3u;
  uint32_t d[N + 1];
#pragma unroll
  for (int i = 0; i <= N; i++) d[i] = p[i * kTS];
#pragma unroll
  for (int i = 0; i < N; i++) o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}
// "%u" of v < 10^8 by SWAR: two 4-digit halves, each split into 2-digit pairs (x / 100 =
// x * 5243 >> 19) and tens (y * 103 >> 10) — the digits in memory order in lo | hi << 32, nd of them
struct Num {
  uint32_t lo, hi;
  int nd;
};
// (24-bit multiplies: every operand here is below 2^24, and v_mul_u32_u24 is full rate)
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return __umul24(a, b); }
__device__ __forceinline__ uint32_t dig4(uint32_t x) {  // x < 10^4 -> 4 digit values, first in byte 0
  const uint32_t q = mul24(x, 5243u) >> 19;
  const uint32_t p = q | (x - mul24(100u, q)) << 16;
  const uint32_t t = (mul24(p, 103u) >> 10) & 0x000F000Fu;
  return t | (p - mul24(10u, t)) << 8;
}
__device__ __forceinline__ Num fmt8(uint32_t v) {
  const uint32_t h = __umulhi(v, 3518437209u) >> 13;  // v / 10^4 (exact for v < 10^8)
  const uint64_t raw = (uint64_t)dig4(h) | (uint64_t)dig4(v - mul24(10000u, h)) << 32;
  const uint32_t lo = (uint32_t)raw, hi = (uint32_t)(raw >> 32);
  // leading zero digits = trailing zero bytes of raw (at least one digit stays)
  int z = (lo ? __builtin_ctz(lo) : 32 + (hi ? __builtin_ctz(hi) : 32)) >> 3;
  z = z > 7 ? 7 : z;
  const uint64_t s = (raw + 0x3030303030303030ull) >> (8 * z);
  Num r;
  r.lo = (uint32_t)s;
  r.hi = (uint32_t)(s >> 32);
  r.nd = 8 - z;
  return r;
}
// codon64 index of the three bases in bytes 0-2 of w (A/C/G/T: code (c >> 1) & 3)
__device__ __forceinline__ uint32_t cidx(uint32_t w) {
  const uint32_t c = (w >> 1) & 0x00030303u;
  return (mul24(c, 0x00100401u) >> 16) & 63u;  // (low 32 bits of the product: bits 16-21 are exact)
}
// constant text as dwords
template <int N>
struct Txt {
  uint32_t w[(N + 2) / 4];
};
template <int N>
__host__ __device__ constexpr Txt<N> txt(const char (&s)[N]) {
  Txt<N> t{};
  for (int i = 0; i < N - 1; i++) t.w[i >> 2] |= (uint32_t)(uint8_t)s[i] << (8 * (i & 3));
  return t;
}

// One event's line (the fast case); returns the modseq error index (S) or -1, rel as emit_event.
__device__ __forceinline__ int emit_fast(DLine& L, const LDS uint8_t* qw, int qlo, const LDS SmallTables* tab,
                                         const EvIn& in, bool rev, int Lq, uint32_t l0, uint32_t l1,
                                         const int32_t* NS, bool skip, int& rel) {
  const uint32_t typ = in.typ;
  const int n = in.n;
  const bool isS = typ == PW_OP_SUB, isI = typ == PW_OP_INS, isD = typ == PW_OP_DEL;
  const int rloc = event_rloc(Lq, rev, typ, in.qp, n);
  const int aap0 = rloc / 3;
  const int rt = 3 * (aap0 - 1);  // r_trloc (rloc >= 4 here)
  rel = rloc - rt;
  const uint64_t l64 = (uint64_t)l1 << 32 | l0;
  const LDS uint8_t* c64 = tab->codon64;

  // ---- "E\trloc\taapos(aa)\t" (pafreport.cpp:897-899, 918)
  {
    uint32_t aw[1];
    lds_img(qw, 3 * aap0 - qlo, aw);
    const uint32_t aa = c64[cidx(aw[0])];
    const Num a1 = fmt8((uint32_t)rloc + 1u);
    const uint32_t tc = isS ? 'S' : (isI ? 'I' : 'D');
    uint32_t f1[3] = {tc | (uint32_t)'\t' << 8 | a1.lo << 16, a1.lo >> 16 | a1.hi << 16, a1.hi >> 16};
    or_at(f1, '\t', 2 + a1.nd);
    app(L, f1, 3 + a1.nd);
    const Num a2 = fmt8((uint32_t)aap0 + 1u);
    uint32_t f2[3] = {a2.lo, a2.hi, 0u};
    or_at(f2, (uint32_t)'(' | aa << 8 | (uint32_t)')' << 16 | (uint32_t)'\t' << 24, a2.nd);
    app(L, f2, a2.nd + 4);
  }
  // ---- bases ("SUB:BASES", ":INS", "DEL:"), evtbases in final orientation (:563, 594-596,
  // 612-614, 637, 928-941); b0 / same for hpolyCheck
  uint32_t alt = 0, sub = 0;
  uint32_t b0;
  bool same;
  if (isS) {  // (target, query) literal pairs
    alt = pack_even4(l64);
    sub = pack_even4(l64 >> 8);
    if (rev) {
      alt = comp_acgt4(__builtin_bswap32(alt) >> (8 * (4 - n)));
      sub = comp_acgt4(__builtin_bswap32(sub) >> (8 * (4 - n)));
    }
    alt = keep32(alt, n);
    sub = keep32(sub, n);
    b0 = alt & 0xFFu;
    same = keep32(alt ^ (b0 * 0x01010101u), n) == 0u;
    const uint64_t s1 = (uint64_t)sub | (uint64_t)':' << (8 * n), s2 = (uint64_t)alt | (uint64_t)'\t' << (8 * n);
    const uint32_t g1[2] = {(uint32_t)s1, (uint32_t)(s1 >> 32)}, g2[2] = {(uint32_t)s2, (uint32_t)(s2 >> 32)};
    app(L, g1, n + 1);
    app(L, g2, n + 1);
  } else if (isI) {  // inserted target bases
    const uint64_t b = keep64(rev ? comp_acgt8(__builtin_bswap64(l64) >> (8 * (8 - n))) : l64, n);
    b0 = (uint32_t)b & 0xFFu;
    same = keep64(b ^ (b0 * 0x0101010101010101ull), n) == 0ull;
    const uint32_t blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    uint32_t g[3] = {(uint32_t)':' | blo << 8, blo >> 24 | bhi << 8, bhi >> 24};
    or_at(g, '\t', n + 1);
    app(L, g, n + 2);
  } else {  // deleted query bases, Q[rloc, rloc + n) on either strand (comp2 is the identity on A/C/G/T)
    uint32_t w[3];
    lds_img(qw, rloc - qlo, w);
    uint32_t g[4] = {w[0], w[1], w[2], 0u};
    b0 = g[0] & 0xFFu;
    const uint32_t bb = b0 * 0x01010101u;
    same = keep32(g[0] ^ bb, n) == 0u && keep32(g[1] ^ bb, n - 4) == 0u && keep32(g[2] ^ bb, n - 8) == 0u;
    g[0] = keep32(g[0], n);
    g[1] = n > 4 ? keep32(g[1], n - 4) : 0u;
    g[2] = n > 8 ? keep32(g[2], n - 8) : 0u;
    or_at(g, (uint32_t)':' | (uint32_t)'\t' << 8, n);
    app(L, g, n + 2);
  }
  {  // ---- tloc + 1
    const Num a4 = fmt8((uint32_t)in.tloc + 1u);
    uint32_t f4[3] = {a4.lo, a4.hi, 0u};
    or_at(f4, '\t', a4.nd);
    app(L, f4, a4.nd + 1);
  }
  // ---- target context (setTContext :120-128, revCompl :631): fast form or the tx record
  if (in.tmode == 0) {
    const int nm = isD ? 0 : (isS ? 1 : n);
    const int qpa = in.qp + (isS ? 1 : (isD ? n : 0));
    const int f1 = rev ? Lq - qpa - in.rl : in.qp - in.ll, n1 = rev ? in.rl : in.ll;
    const int f2 = rev ? Lq - in.qp : qpa, n2 = rev ? in.ll : in.rl;
    uint32_t a[2], b[2];
    lds_img(qw, f1 - qlo, a);
    lds_img(qw, f2 - qlo, b);
    uint64_t mv = isS ? (l64 & 0xFFull) : l64;
    if (rev) mv = nm > 0 ? comp_acgt8(__builtin_bswap64(mv) >> (8 * (8 - nm))) : 0ull;
    mv |= 0x2020202020202020ull;
    const uint32_t g[2] = {(uint32_t)mv, (uint32_t)(mv >> 32)};
    app(L, a, n1);
    app(L, g, nm);
    app(L, b, n2);
  } else {  // length byte + field
    const uint32_t t[7] = {in.tx[0], in.tx[1], in.tx[2], in.tx[3], in.tx[4], in.tx[5], 0u};
    uint32_t g[6];
#pragma unroll
    for (int i = 0; i < 6; i++) g[i] = __builtin_amdgcn_alignbyte(t[i + 1], t[i], 1u);
    app(L, g, (int)(in.tx[0] & 0xFFu));
  }
  // ---- "\tRCTX\tstatus" (getRefContext :721-733, hpolyCheck :735-748, mmotifCheck :751-763)
  {
    int c0 = rloc - 4, eloc = 4;
    if (c0 + 8 >= Lq) {
      eloc += Lq - c0 - 9;
      c0 = Lq - 9;
    }
    uint32_t rw[3];
    lds_img(qw, c0 - qlo, rw);
    const uint32_t rw2 = rw[2] & 0xFFu;
    const uint64_t lo = (uint64_t)rw[0] | ((uint64_t)rw[1] << 32);
    int l = -1;
    bool m0 = false, m1 = false, m2 = false, m3 = false;
#pragma unroll
    for (int p = 5; p >= 0; p--) {
      const uint32_t v4 = p <= 4 ? (uint32_t)(lo >> (8 * p)) : ((rw[1] >> 8) | (rw2 << 24));
      const uint32_t c4 = p < 4 ? (uint32_t)(lo >> (8 * (p + 4))) & 0xFFu : (p == 4 ? rw2 : 0u);
      if (v4 == 0x01010101u * b0) l = p;
      m0 = m0 || (v4 == 0x47544343u && c4 == 'G');  // "CCTGG"
      m1 = m1 || (v4 == 0x47414343u && c4 == 'G');  // "CCAGG"
      m2 = m2 || v4 == 0x43544147u;                 // "GATC"
      m3 = m3 || v4 == 0x43415447u;                 // "GTAC"
    }
    const int st = (same && l >= 0 && l <= eloc && l + 4 >= eloc) ? 1 : (m0 ? 2 : (m1 ? 3 : (m2 ? 4 : (m3 ? 5 : 0))));
    const uint32_t f6[3] = {(uint32_t)'\t' | rw[0] << 8, rw[0] >> 24 | rw[1] << 8,
                            rw[1] >> 24 | rw2 << 8 | (uint32_t)'\t' << 16};
    app(L, f6, 11);
    const LDS uint32_t* sw = reinterpret_cast<const LDS uint32_t*>(tab->status[st]);
    const uint32_t sv[3] = {sw[0], sw[1], sw[2]};
    app(L, sv, (int)(sv[2] >> 24));
  }
  // ---- codon consequence (predictImpact, pafreport.cpp:801-883)
  int merr = -1;
  if (skip) {
    const uint32_t e[1] = {(uint32_t)'\t' | (uint32_t)'\n' << 8};
    app(L, e, 2);
    return -1;
  }
  if (isS) {  // codons ao = 1, 2 of modseq (r_trloc + 3 .. + 8): bytes 3-10 of Q[r_trloc ..] in t
    uint32_t q[3];
    lds_img(qw, rt - qlo, q);
    const uint64_t t = (uint64_t)(q[0] >> 24) | (uint64_t)q[1] << 8 | (uint64_t)q[2] << 40;
    const int sh = 8 * (rel - 3);  // evtbases at modseq byte rel (3..5)
    const uint32_t nmask = keep32(0xFFFFFFFFu, n);
    const uint32_t diff = ((uint32_t)(t >> sh) ^ sub) & nmask;  // modseq check (:811-814)
    merr = diff ? (int)(__builtin_ctz(diff) >> 3) : -1;
    const uint64_t mt = (t & ~((uint64_t)nmask << sh)) | ((uint64_t)alt << sh);
    const uint32_t caa1 = c64[cidx((uint32_t)t)], cmaa1 = c64[cidx((uint32_t)mt)];
    const uint32_t caa2 = c64[cidx((uint32_t)(t >> 24))], cmaa2 = c64[cidx((uint32_t)(mt >> 24))];
    const bool ch1 = caa1 != cmaa1, ch2 = rel + n - 1 >= 6 && caa2 != cmaa2;
    if (!ch1 && !ch2) {
      constexpr Txt<13> syn = txt("\tsynonymous\n");
      app(L, syn.w, 12);
      return merr;
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const bool ch = k == 0 ? ch1 : ch2;
      if (!ch) continue;
      const uint32_t caa = k == 0 ? caa1 : caa2, cmaa = k == 0 ? cmaa1 : cmaa2;
      const bool first = k == 0 || !ch1;
      const uint32_t pf[1] = {first ? 0x0041'4109u : 0x4141'202Cu};  // "\tAA" / ", AA"
      app(L, pf, first ? 3 : 4);
      const Num an = fmt8((uint32_t)(aap0 + 1 + k));  // ap = ao + rloc / 3
      uint32_t g[3] = {an.lo, an.hi, 0u};
      or_at(g, (uint32_t)'|' | caa << 8 | (uint32_t)':' << 16 | cmaa << 24, an.nd);
      app(L, g, an.nd + 4);
      if (cmaa == '.') {
        constexpr Txt<22> ps = txt("|premature stop at AA");
        app(L, ps.w, 21);
        const uint32_t d[2] = {an.lo, an.hi};
        app(L, d, an.nd);
      }
    }
    const uint32_t e[1] = {'\n'};
    app(L, e, 1);
    return merr;
  }
  // indel: modseq = Q[r_trloc, rloc) + X + Q[rloc + dl, ..), codons 0-4 and reference codons 1-4
  const int a = rel;
  const int x = isI ? n : 0, dl = isD ? n : 0;
  const int sfx = rloc + dl;
  const int M = (Lq - rt) + x - dl;
  const int trlen = Lq - rt;
  uint32_t q0[4], q1[4];
  lds_img(qw, rt - qlo, q0);
  lds_img(qw, rt - qlo + dl - x, q1);
  const uint64_t X = isI ? keep64(rev ? comp_acgt8(__builtin_bswap64(l64) >> (8 * (8 - x))) : l64, x) : 0ull;
  // X << 8a over four dwords (a = 3..5)
  const uint32_t xs[4] = {(uint32_t)(X << (8 * a)), (uint32_t)((X << (8 * a)) >> 32), (uint32_t)(X >> (64 - 8 * a)),
                          a == 5 ? (uint32_t)(X >> 56) : 0u};
  uint32_t mw[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int ca = min(max(a - 4 * i, 0), 4), cx = min(max(a + x - 4 * i, 0), 4);
    const uint32_t ma = (uint32_t)((1ull << (8 * ca)) - 1ull), mx = (uint32_t)((1ull << (8 * cx)) - 1ull) & ~ma;
    mw[i] = (q0[i] & ma) | (xs[i] & mx) | (q1[i] & ~(ma | mx));
  }
  uint32_t mm[5], rr[5];
  {
    const uint32_t mc[5] = {mw[0], __builtin_amdgcn_alignbyte(mw[1], mw[0], 3u),
                            __builtin_amdgcn_alignbyte(mw[2], mw[1], 2u), mw[2] >> 8, mw[3]};
    const uint32_t rc[5] = {0u, __builtin_amdgcn_alignbyte(q0[1], q0[0], 3u),
                            __builtin_amdgcn_alignbyte(q0[2], q0[1], 2u), q0[2] >> 8, q0[3]};
#pragma unroll
    for (int c = 0; c < 5; c++) {
      mm[c] = c64[cidx(mc[c])];
      rr[c] = c == 0 ? 0u : (uint32_t)c64[cidx(rc[c])];
    }
  }
  // (bytes past the query end are the zero padding: they only reach codons the scan does not use)
  int stopc = 5, nvalid = 0;
#pragma unroll
  for (int c = 4; c >= 0; c--) {
    const bool valid = 3 * c + 2 < M;
    if (valid && mm[c] == '.') stopc = c;
    nvalid += valid ? 1 : 0;
  }
  const int last = stopc < nvalid ? stopc : nvalid;
  uint32_t aa4 = 0, maa4 = 0;
  int aa4n = 0, maa4n = 0;
#pragma unroll
  for (int c = 1; c < 5; c++) {
    if (c < last) {
      if (3 * c + 2 < trlen) {
        aa4 |= rr[c] << (8 * aa4n);
        aa4n++;
      }
      maa4 |= mm[c] << (8 * maa4n);
      maa4n++;
    }
  }
  int stop_i = -1;
  if (stopc < nvalid) {
    stop_i = 3 * stopc;
  } else if (nvalid == 5 && 15 + 2 < M && NS) {
    const int k0 = sfx + (15 - a - x);
    if (k0 >= 0 && k0 < Lq) {
      const int st = in.ns_pre != kNsNone ? in.ns_pre : NS[k0];
      if (st != kNoStop) stop_i = st - sfx + a + x;
    }
  }
  if (stop_i >= 0) {
    constexpr Txt<22> ps = txt("\tpremature stop at AA");
    app(L, ps.w, 21);
    const Num an = fmt8((uint32_t)(1 + (stop_i + rt) / 3));
    uint32_t g[3] = {an.lo, an.hi, 0u};
    or_at(g, '\n', an.nd);
    app(L, g, an.nd + 1);
  } else if (aa4n > 0 && maa4n > 0) {
    constexpr Txt<14> fs = txt("\tframe shift ");
    app(L, fs.w, 13);
    const uint64_t u = (uint64_t)aa4 | (uint64_t)('+' | ':' << 8) << (8 * aa4n);
    const uint64_t v = (uint64_t)maa4 | (uint64_t)('+' | '\n' << 8) << (8 * maa4n);
    const uint32_t gu[2] = {(uint32_t)u, (uint32_t)(u >> 32)}, gv[2] = {(uint32_t)v, (uint32_t)(v >> 32)};
    app(L, gu, aa4n + 2);
    app(L, gv, maa4n + 2);
  } else {
    const uint32_t e[1] = {(uint32_t)'\t' | (uint32_t)'\n' << 8};
    app(L, e, 2);
  }
  return merr;
}

// ------------------------------------------------------------------ workspace
// Device scratch of one pass (pw_report_workspace_bytes):
//   ctr      u32 [1] long-line count, [2] overflow flags; u64 at byte 16: arena bytes used
//   rec_mod  per record: modseq error key (first failing line in output order)
//   hot/cold per event slot (Hot, Cold); tx: pre-rendered target contexts
//   sflag    per slot: 1 = tctx_kernel renders its target context (index_kernel writes every slot's)
//   fix      long-line list
struct Fixup {
  uint32_t s, pad;
  uint64_t dst;  // text offset of the line
};

// render_kernel: the bytes a page keeps free after its text (a line's last 16-byte store may reach
// 12 bytes past its end)
constexpr uint32_t kPageSlack = 16;
struct Work {
  uint32_t* ctr;
  unsigned long long* arena_used;
  uint64_t* rec_mod;
  uint32_t* hotw;     // event records: slot s at word s << hot_sh (fn = that word)
  uint32_t hot_sh;    // 3 (32-byte records) or 2 (16-byte records: hot_pbits != 0)
  uint32_t hot_pbits;
  Cold* cold;
  uint8_t* tx;
  uint8_t* sflag;
  Fixup* fix;         // per slot: the destination of a long line (written only for long lines)
  uint64_t* lmask;    // per chunk: lanes whose line is longer than the LDS line buffer
  // records of more than kBlkOps ops, decoded block by block (plan_kernel / carry_kernel):
  uint32_t* rec_blk;  // per record: its first entry in blist, or kNoBlk
  uint32_t* rec_bad;  // per record: the first block (>= 1) with a base mismatch (atomicMin), or kNoBlk
  uint64_t* blist;    // entries record << 32 | block, a record's blocks consecutive
  v4u* bcarry;        // per entry: query / target / literal advance and event heads of the block
  v4u* berr;          // per entry (blocks >= 1): mismatch details {err, q_pos, query char, aligned char}
  uint32_t blk_cap;
  uint32_t ns_grid;   // index's first workgroups that build next_stop (PW_REPORT_BUILD_NEXT_STOP), 0 = none
  uint32_t clear_ctr; // index clears the counters (no memset launch: a batch without long records)
  uint64_t n_slots, n_chunks;
  uint64_t arena0;  // first arena byte in text (= n_chunks * PW_PAGE_BYTES)
};
constexpr int kBlkOps = PW_BLOCK_OPS;   // ops per block of a long record (16 segments)
constexpr uint32_t kNoBlk = 0xFFFFFFFFu;

__host__ __device__ inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// layout of the workspace; returns its size (base may be null to only size it)
__host__ __device__ inline uint64_t work_layout(uint8_t* base, uint64_t n_slots, uint64_t n_alns, Work* w) {
  const uint64_t n_chunks = (n_slots + kWave - 1) / kWave;
  const uint64_t ns = n_chunks * kWave;  // slot arrays padded to whole chunks
  uint64_t o = 256;
  const uint64_t o_rm = o;
  o = align_up(o + 8 * n_alns, 256);
  const uint64_t o_hot = o;
  o = align_up(o + sizeof(Hot) * ns, 256);
  const uint64_t o_cold = o;
  o = align_up(o + sizeof(Cold) * ns, 256);
  const uint64_t o_tx = o;
  o = align_up(o + (uint64_t)kTx * ns, 256);
  const uint64_t o_sflag = o;
  o = align_up(o + ns, 256);
  const uint64_t o_fix = o;
  o = align_up(o + sizeof(Fixup) * ns, 256);
  const uint64_t o_lmask = o;
  o = align_up(o + 8 * (n_chunks ? n_chunks : 1), 256);
  // block list capacity: a record of n > kBlkOps ops has ceil(n / kBlkOps) < 2n / kBlkOps blocks,
  // and a well-formed record has n <= 2 * (its event slots) + 1 ops; a record that does not get
  // room is decoded by one wavefront
  const uint64_t bcap = 4 * (n_slots + n_alns) / kBlkOps + 64;
  const uint64_t o_rblk = o;
  o = align_up(o + 8 * n_alns, 256);
  const uint64_t o_blist = o;
  o = align_up(o + 8 * bcap, 256);
  const uint64_t o_bcarry = o;
  o = align_up(o + 16 * bcap, 256);
  const uint64_t o_berr = o;
  o = align_up(o + 16 * bcap, 256);
  if (w && base) {
    w->ctr = reinterpret_cast<uint32_t*>(base);
    w->arena_used = reinterpret_cast<unsigned long long*>(base + 16);
    w->rec_mod = reinterpret_cast<uint64_t*>(base + o_rm);
    w->hotw = reinterpret_cast<uint32_t*>(base + o_hot);
    w->hot_sh = 3;
    w->hot_pbits = 0;
    w->cold = reinterpret_cast<Cold*>(base + o_cold);
    w->tx = base + o_tx;
    w->sflag = base + o_sflag;
    w->fix = reinterpret_cast<Fixup*>(base + o_fix);
    w->lmask = reinterpret_cast<uint64_t*>(base + o_lmask);
    w->rec_blk = reinterpret_cast<uint32_t*>(base + o_rblk);
    w->rec_bad = w->rec_blk + n_alns;
    w->blist = reinterpret_cast<uint64_t*>(base + o_blist);
    w->bcarry = reinterpret_cast<v4u*>(base + o_bcarry);
    w->berr = reinterpret_cast<v4u*>(base + o_berr);
    w->blk_cap = (uint32_t)(bcap < 0xFFFFFFF0ull ? bcap : 0xFFFFFFF0ull);
    w->ns_grid = 0;
    w->clear_ctr = 0;
    w->n_slots = n_slots;
    w->n_chunks = n_chunks;
    w->arena0 = n_chunks * (uint64_t)PW_PAGE_BYTES;
  }
  return o;
}

// the fn word of slot s (empty slots, last-line flags)
__device__ __forceinline__ uint32_t& hot_fn(const Work& W, uint64_t s) { return W.hotw[s << W.hot_sh]; }
// index_kernel's store of an event's record (qi: its query index)
__device__ __forceinline__ void store_hot(const Work& W, uint64_t s, const Hot& h, uint32_t qi) {
  v4u* p = reinterpret_cast<v4u*>(W.hotw + (s << W.hot_sh));
  if (W.hot_pbits) {
    p[0] = (v4u){h.fn, qi << W.hot_pbits | (uint32_t)h.qp, (uint32_t)h.tloc, h.ls};
  } else {
    p[0] = (v4u){h.fn, (uint32_t)h.qp, (uint32_t)h.tloc, h.ls};
    p[1] = (v4u){h.qb, (uint32_t)h.L, h.l0, h.l1};
  }
}
// a 16-byte record's query index / query position (0 for empty slots, whose other words are stale)
__device__ __forceinline__ uint32_t hot16_qi(const Work& W, uint32_t fn, uint32_t w1) {
  return fn == kNoEv ? 0u : w1 >> W.hot_pbits;
}
__device__ __forceinline__ uint32_t hot16_qp(const Work& W, uint32_t w1) { return w1 & ((1u << W.hot_pbits) - 1u); }
// the first 8 literal bytes from ls, given the three dwords from ls & ~3
__device__ __forceinline__ void lit8(uint32_t ls, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t& l0, uint32_t& l1) {
  l0 = __builtin_amdgcn_alignbyte(d1, d0, ls & 3u);
  l1 = __builtin_amdgcn_alignbyte(d2, d1, ls & 3u);
}
// the whole record of slot s with its dependent loads (tctx_kernel, fixup_kernel)
__device__ __forceinline__ Hot load_hot_full(const pw_report_args& A, const Work& W, uint64_t s) {
  const v4u a = reinterpret_cast<const v4u*>(W.hotw + (s << W.hot_sh))[0];
  Hot h;
  h.fn = a.x;
  h.tloc = (int32_t)a.z;
  h.ls = a.x == kNoEv ? 0u : a.w;
  if (W.hot_pbits) {
    const uint32_t qi = hot16_qi(W, a.x, a.y);
    h.qp = (int32_t)hot16_qp(W, a.y);
    h.qb = (uint32_t)(A.qoff[qi] >> 4);
    h.L = A.qlen[qi];
    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(A.lits) + (h.ls >> 2);
    lit8(h.ls, l32[0], l32[1], l32[2], h.l0, h.l1);
  } else {
    const v4u b = reinterpret_cast<const v4u*>(W.hotw + (s << W.hot_sh))[1];
    h.qp = (int32_t)a.y;
    h.qb = b.x;
    h.L = (int32_t)b.y;
    h.l0 = b.z;
    h.l1 = b.w;
  }
  return h;
}

// (every caller runs 256 threads: each thread issues its three loads before any store, so the
// staging costs one memory round trip, not three)
__device__ __forceinline__ void stage_small_tables(LDS SmallTables* dst, int tid, int nthreads) {
  const uint8_t* s = reinterpret_cast<const uint8_t*>(&c_tables);
  LDS uint8_t* d = reinterpret_cast<LDS uint8_t*>(dst);
  for (int i0 = 0; i0 < 256; i0 += nthreads) {
    const int i = i0 + tid;
    const uint8_t b0 = s[offsetof(Tables, comp) + (i < 256 ? i : 255)];
    const uint8_t b1 = s[offsetof(Tables, codon64) + (i < 64 ? i : 63)];
    const uint8_t b2 = s[offsetof(Tables, status) + (i < 96 ? i : 95)];
    if (i < 256) d[offsetof(SmallTables, comp) + i] = b0;
    if (i < 64) d[offsetof(SmallTables, codon64) + i] = b1;
    if (i < 96) d[offsetof(SmallTables, status) + i] = b2;
    if (i < 100) {
      d[offsetof(SmallTables, dig2) + 2 * i] = (uint8_t)('0' + i / 10);
      d[offsetof(SmallTables, dig2) + 2 * i + 1] = (uint8_t)('0' + i % 10);
    }
  }
}

// ------------------------------------------------------------------ next-stop table
// ns[p] = the first q >= p with q = p (mod 3) where codon Q[q, q+3) is a stop (kNoStop if none).
// One 256-thread workgroup per query; tiles of 768 positions from the end.  Thread t owns the
// three positions base + 3 * (255 - t) + f, so lanes in increasing order walk the tile
// backwards: a DPP prefix-minimum over the lanes is the suffix minimum over positions, per frame
// (positions 3j + f of a thread share the frame f + base mod 3); the four waves combine through
// LDS, the tiles through a carry.  Workgroup b of nb takes queries b, b + nb, ... (its own launch,
// pw_stop_table_build, or the first workgroups of index_kernel with PW_REPORT_BUILD_NEXT_STOP).
__device__ __forceinline__ void stop_table_wg(const uint8_t* qseq, const uint64_t* qoff, const int32_t* qlen, uint32_t nq,
                                              int32_t* ns, const LDS SmallTables* tp, uint32_t b, uint32_t nb) {
  __shared__ int32_t wm[kWaves][3];
  const int t = threadIdx.x, wv = t / kWave;
  for (uint32_t qi = b; qi < nq; qi += nb) {
    const uint8_t* R = qseq + qoff[qi];
    int32_t* out = ns + qoff[qi];
    const int L = qlen[qi];
    int carry[3] = {kNoStop, kNoStop, kNoStop};
    const int ntile = (L + 767) / 768;
    for (int tile = ntile - 1; tile >= 0; tile--) {
      const int pb = tile * 768 + 3 * (255 - t);
      // five bytes from pb (indices clamped to L: the query is followed by zero bytes)
      uint8_t bq[5];
#pragma unroll
      for (int q = 0; q < 5; q++) bq[q] = R[pb + q < L ? pb + q : L];
      int sm[3];
#pragma unroll
      for (int f = 0; f < 3; f++) {
        const int p = pb + f;
        const int v = (p + 2 < L && translate(tp, bq[f], bq[f + 1], bq[f + 2]) == '.') ? p : kNoStop;
        sm[f] = wave_min_incl(v);
      }
      if ((t & (kWave - 1)) == kWave - 1) {
#pragma unroll
        for (int f = 0; f < 3; f++) wm[wv][f] = sm[f];
      }
      __syncthreads();
      // positions above this wave's: the waves before it in this tile, then the tiles above
#pragma unroll
      for (int f = 0; f < 3; f++) {
        int above = carry[f];
        for (int w2 = 0; w2 < wv; w2++) above = min(above, wm[w2][f]);
        const int p = pb + f;
        if (p < L) out[p] = min(sm[f], above);
      }
#pragma unroll
      for (int f = 0; f < 3; f++)
        for (int w2 = 0; w2 < kWaves; w2++) carry[f] = min(carry[f], wm[w2][f]);
      __syncthreads();
    }
  }
}
__global__ __launch_bounds__(256) void stop_table_kernel(const uint8_t* qseq, const uint64_t* qoff,
                                                         const int32_t* qlen, uint32_t nq, int32_t* ns) {
  __shared__ SmallTables tab;
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, 256);
  __syncthreads();
  stop_table_wg(qseq, qoff, qlen, nq, ns, tp, blockIdx.x, gridDim.x);
}

// index_kernel / index_pair_kernel's start: next_stop workgroups, the counters.  Returns the
// workgroup's index among the decode workgroups (-1: it built next_stop and is done).
__device__ __forceinline__ int index_prologue(const pw_report_args& A, const Work& W, const LDS SmallTables* tp) {
  if (blockIdx.x < W.ns_grid) {
    stop_table_wg(A.qseq, A.qoff, A.qlen, A.n_queries, const_cast<int32_t*>(A.next_stop), tp, blockIdx.x, W.ns_grid);
    return -1;
  }
  // (render is the first kernel that uses ctr[0..2] and the arena counter: a memset launch less)
  if (W.clear_ctr && blockIdx.x == W.ns_grid && threadIdx.x < 8) W.ctr[threadIdx.x] = 0u;
  return (int)(blockIdx.x - W.ns_grid);
}

// ------------------------------------------------------------------ index_kernel
constexpr int kOpWin = kSegOps + 2 * kOpHalo;
struct IndexWave {
  uint32_t opw[kOpWin + 8];        // op words of the segment + halo (index_pair_kernel: two records' ops)
};

__device__ __forceinline__ int ndigits(uint32_t v) {
  return 1 + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) + (v >= 1000000u) +
         (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}

// A record's head, loaded one record ahead (index_kernel's loop): descriptor, query location,
// next record's first event slot and the first 128 op words (2 per lane).
struct RecPre {
  pw_aln_desc d;
  uint64_t qb, ev_next;
  int L;
  uint32_t w0, w1;
  bool last;  // ai is the batch's last record (ev_next = n_ev_slots)
};
// All loads unconditional (clamped / dummy addresses; see pin()): the values are selected when
// the record is processed, one record later.
__device__ __forceinline__ void rec_pre(const pw_report_args& A, uint32_t ai, const pw_aln_desc& d, int lane,
                                        RecPre& p) {
  p.d = d;
  const uint32_t qi = d.ref & PW_REF_QMASK;
  p.qb = A.qoff[qi];
  p.L = A.qlen[qi];
  p.last = ai + 1 >= A.n_alns;
  p.ev_next = A.desc[p.last ? ai : ai + 1].ev_begin;
  const uint32_t* ops = A.ops + d.op_begin;
  const uint32_t* dummy = reinterpret_cast<const uint32_t*>(A.desc);
  p.w0 = *((uint32_t)lane < d.n_ops ? ops + lane : dummy);
  p.w1 = *((uint32_t)(lane + 64) < d.n_ops ? ops + lane + 64 : dummy);
}
__device__ __forceinline__ void rec_pre_ready(const pw_report_args& A, RecPre& p, int lane) {
  asm volatile("" : "+v"(p.qb), "+v"(p.ev_next), "+v"(p.L), "+v"(p.w0), "+v"(p.w1));
  if (p.last) p.ev_next = A.n_ev_slots;
  if ((uint32_t)lane >= p.d.n_ops) p.w0 = 0u;
  if ((uint32_t)(lane + 64) >= p.d.n_ops) p.w1 = 0u;
}

// A descriptor loaded two records ahead stays in VGPRs (a uniform load is otherwise moved to
// SGPRs at once, which waits for it — and, vmcnt being in order, for every store before it)
struct DescRaw {
  v4u a, b;
};
__device__ __forceinline__ DescRaw load_desc(const pw_report_args& A, uint32_t i) {
  const v4u* p = reinterpret_cast<const v4u*>(A.desc + i);
  DescRaw r;
  r.a = p[0];
  r.b = p[1];
  return r;
}
__device__ __forceinline__ pw_aln_desc unpack_desc(const DescRaw& r) {
  pw_aln_desc d;
  d.op_begin = __builtin_amdgcn_readfirstlane(r.a.x);
  d.n_ops = __builtin_amdgcn_readfirstlane(r.a.y);
  d.lit_begin = __builtin_amdgcn_readfirstlane(r.a.z);
  d.ref = __builtin_amdgcn_readfirstlane(r.a.w);
  d.offset = (int32_t)__builtin_amdgcn_readfirstlane(r.b.x);
  d.t_len = (int32_t)__builtin_amdgcn_readfirstlane(r.b.y);
  d.ev_begin = (uint64_t)__builtin_amdgcn_readfirstlane(r.b.z) | (uint64_t)__builtin_amdgcn_readfirstlane(r.b.w) << 32;
  return d;
}

// The op range a wavefront decodes: a whole record, or one block of a record of more than
// kBlkOps ops (its coordinates and event count at the block start from carry_kernel's totals of
// the blocks before it; the record's event count is then known up front, so its last line is
// flagged when written).
struct IdxBlk {
  uint32_t sb0, sb1;   // ops [sb0, sb1) of the record
  int qc, tc;          // query / target position at sb0
  uint32_t lc;         // literal index at sb0
  uint32_t ev0;        // events created before sb0
  uint32_t ev1;        // ... before sb1 (blocked)
  uint32_t tot;        // events of the record (blocked)
  uint32_t k, bidx;    // block index in the record, its blist entry
  bool prev_sub;       // the op before sb0 is a '*'
  bool blocked;
};
__device__ __forceinline__ IdxBlk whole_record(const pw_aln_desc& d) {
  IdxBlk B;
  B.sb0 = 0;
  B.sb1 = d.n_ops;
  B.qc = B.tc = 0;
  B.lc = d.lit_begin;
  B.ev0 = B.ev1 = B.tot = 0;
  B.k = B.bidx = 0;
  B.prev_sub = false;
  B.blocked = false;
  return B;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return wave_last(wave_scan_incl(v)); }
// block k of a record whose blocks are blist entries [base, base + nb): prefix of the carries
__device__ __forceinline__ IdxBlk block_of(const Work& W, const pw_aln_desc& d, uint32_t base, uint32_t nb, uint32_t k,
                                          int lane) {
  IdxBlk B;
  uint32_t q = 0, t = 0, l = 0, e = 0, tot = 0, ek = 0;
  for (uint32_t j0 = 0; j0 < nb; j0 += kWave) {
    const uint32_t j = j0 + (uint32_t)lane;
    v4u c = W.bcarry[base + (j < nb ? j : 0u)];
    if (j >= nb) c = (v4u){0u, 0u, 0u, 0u};
    const bool b = j < k;
    q += wave_sum(b ? c.x : 0u);
    t += wave_sum(b ? c.y : 0u);
    l += wave_sum(b ? c.z : 0u);
    e += wave_sum(b ? c.w : 0u);
    ek += wave_sum(j == k ? c.w : 0u);
    tot += wave_sum(c.w);
  }
  B.sb0 = k * (uint32_t)kBlkOps;
  B.sb1 = d.n_ops - B.sb0 < (uint32_t)kBlkOps ? d.n_ops : B.sb0 + (uint32_t)kBlkOps;
  B.qc = (int)q;
  B.tc = (int)t;
  B.lc = d.lit_begin + l;
  B.ev0 = e;
  B.ev1 = e + ek;
  B.tot = tot;
  B.k = k;
  B.bidx = base + k;
  B.prev_sub = false;  // (set by the caller from the op before sb0)
  B.blocked = true;
  return B;
}

__device__ __forceinline__ void index_record(const pw_report_args& A, const Work& W, const LDS SmallTables* tab,
                                             LDS IndexWave* w, uint32_t ai, int lane, const RecPre& pre,
                                             const IdxBlk& B) {
  const pw_aln_desc d = pre.d;
  const uint32_t* ops = A.ops + d.op_begin;
  const uint64_t qb = pre.qb;
  const uint8_t* R = A.qseq + qb;
  // the render record keeps qb / 16 in 32 bits and the event slots [ev_begin, next ev_begin)
  // must be a non-empty-or-empty range inside the batch (pwasm_amd.h, pw_report_args)
  const bool layout_ok = (qb & 15u) == 0 && (qb >> 36) == 0 && pre.ev_next >= d.ev_begin && pre.ev_next <= A.n_ev_slots;
  const int L = pre.L;
  const bool rev = (d.ref & PW_REF_REVERSE) != 0;
  const int T = d.t_len;
  const uint32_t n_ops = d.n_ops;
  const uint64_t evb = d.ev_begin;
  const uint64_t ev_next = pre.ev_next;
  const uint32_t nmax = layout_ok ? (uint32_t)(ev_next - evb) : 0u;
  const uint32_t* lits32 = reinterpret_cast<const uint32_t*>(A.lits);

  int qc = B.qc, tc = B.tc;
  uint32_t lc = B.lc;
  bool prev_sub = B.prev_sub;
  uint32_t ev = B.ev0, ev_last_seg = 0;  // events created; by the last segment processed
  int err = layout_ok ? PW_REC_OK : PW_REC_LAYOUT, err_a = 0, err_b = 0, err_c = 0;
  const uint32_t qi = d.ref & PW_REF_QMASK;
  bool bad_hot = false;

  for (uint32_t sb = B.sb0; layout_ok && sb < B.sb1; sb += kSegOps) {
    const uint32_t nseg = (B.sb1 - sb) < (uint32_t)kSegOps ? (B.sb1 - sb) : (uint32_t)kSegOps;
    const bool two = nseg > (uint32_t)kWave;  // (uniform) a segment of <= 64 ops skips its empty second half
    // ---- op words (2 per lane) + wave scans of the query / target / literal advances
    uint32_t wd[2];
    int qs[2], ts[2];
    uint32_t ls[2];
    uint32_t qtot = 0, ttot = 0, ltot = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t idx = 64 * k + lane;
      if (k == 1 && !two) {
        wd[1] = 0u;
        qs[1] = qc + (int)qtot;
        ts[1] = tc + (int)ttot;
        ls[1] = lc + ltot;
        continue;
      }
      if (sb == 0) {
        wd[k] = k == 0 ? pre.w0 : pre.w1;
      } else {  // (clamped index: an unconditional load, waited for inside this branch: a wait at
                // the join would also hold the first segment for the next record's prefetch)
        uint32_t w = ops[idx < nseg ? sb + idx : sb];
        asm volatile("" : "+v"(w));
        wd[k] = idx < nseg ? w : 0u;
      }
      const uint32_t qa = idx < nseg ? op_qadv(wd[k]) : 0u, ta = idx < nseg ? op_tadv(wd[k]) : 0u,
                     la = idx < nseg ? op_ladv(wd[k]) : 0u;
      const uint32_t qi_ = wave_incl_scan(qa, lane), ti_ = wave_incl_scan(ta, lane), li_ = wave_incl_scan(la, lane);
      qs[k] = qc + (int)(qtot + qi_ - qa);
      ts[k] = tc + (int)(ttot + ti_ - ta);
      ls[k] = lc + ltot + li_ - la;
      qtot += wave_last(qi_);
      ttot += wave_last(ti_);
      ltot += wave_last(li_);
      w->opw[kOpHalo + idx] = wd[k];
    }
    // halo: the op words just before / after the segment (tctx_fast's neighbours; lanes 0 and 1),
    // loaded with the segment's other reads below and stored once they are in
    const int hj = lane == 0 ? (int)sb - 1 : (int)(sb + nseg);
    const bool hok = lane < 2 && hj >= 0 && (uint32_t)hj < n_ops;
    uint32_t halo = ops[hok ? (uint32_t)hj : sb];
    // ---- the segment's global reads, issued together before any is used (clamped indices, so
    // no load sits in a branch): per op the query base and the cs query base of a '*' op, and the
    // first 8 literal bytes of an event head (lits and qseq are readable PW_DEV_PAD bytes past
    // their ends, and every query is followed by zero padding)
    uint8_t qlit[2], qref[2];
    uint32_t lw[2][3];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !two) {
        qref[1] = qlit[1] = 0;
        lw[1][0] = lw[1][1] = lw[1][2] = 0u;
        continue;
      }
      const int qp = d.offset + qs[k];
      const int qc = qp < 0 ? 0 : (qp >= L ? (L > 0 ? L - 1 : 0) : qp);
      qref[k] = R[rev ? (L > 0 ? L - 1 - qc : 0) : qc];
      qlit[k] = A.lits[ls[k] + 1];
      const uint32_t la = ls[k] >> 2;
#pragma unroll
      for (int q = 0; q < 3; q++) lw[k][q] = lits32[la + q];
    }
    // ---- base check of every '*' op (pafreport.cpp:550-554) and event heads
    uint64_t subm[2], hm[2];
    int bad_idx = INT_MAX;
    uint32_t sm_prev = prev_sub ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !two) {
        subm[1] = hm[1] = 0ull;
        continue;
      }
      const uint32_t idx = 64 * k + lane;
      const bool in = idx < nseg;
      const uint32_t typ = wd[k] >> 30;
      const bool is_sub = in && typ == PW_OP_SUB;
      subm[k] = __ballot(is_sub);
      const bool prevsub = lane == 0 ? sm_prev != 0 : ((subm[k] >> (lane - 1)) & 1ull) != 0;
      sm_prev = (uint32_t)((subm[k] >> 63) & 1ull);
      hm[k] = __ballot(in && (typ == PW_OP_INS || typ == PW_OP_DEL || (is_sub && !prevsub)));
      const int qp = d.offset + qs[k];
      // aligned-strand query char at qp (refseq_rc for '-' records; 0 past the end)
      const uint8_t rch = (unsigned)qp >= (unsigned)L ? (uint8_t)0 : (rev ? tab->comp[qref[k]] : qref[k]);
      const uint8_t qch = qlit[k];
      const bool bad = is_sub && qch != rch;
      const uint64_t bm = __ballot(bad);
      if (bm && bad_idx == INT_MAX) {
        const int fl = __builtin_ctzll(bm);
        bad_idx = 64 * k + fl;
        err_a = __shfl(qp, fl, kWave);
        err_b = __shfl((int)qch, fl, kWave);
        err_c = __shfl((int)rch, fl, kWave);
      }
    }
    if (lane < 2) w->opw[lane == 0 ? kOpHalo - 1 : kOpHalo + (int)nseg] = hok ? halo : 0u;
    wave_sync();
    if (bad_idx != INT_MAX) {
      err = PW_REC_MISMATCH;
      break;
    }
    // every event head's first 8 literal bytes, for both halves now: a load first consumed after
    // the first half's Hot stores would make the compiler wait for those stores too (vmcnt(0))
    uint32_t hl0[2], hl1[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t sh = ls[k] & 3u;
      hl0[k] = __builtin_amdgcn_alignbyte(lw[k][1], lw[k][0], sh);
      hl1[k] = __builtin_amdgcn_alignbyte(lw[k][2], lw[k][1], sh);
      asm volatile("" : "+v"(hl0[k]), "+v"(hl1[k]));  // (kept here, not sunk into the store branch)
    }
    // ---- events of this segment: creation index, S-run length, target context
    const uint32_t n0 = (uint32_t)__popcll(hm[0]);
    const uint32_t nev = n0 + (uint32_t)__popcll(hm[1]);
    const bool fin = sb + (uint32_t)kSegOps >= n_ops;  // the record's last segment
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (k == 1 && !two) continue;
      const uint32_t idx = 64 * k + lane;
      const uint32_t typ = wd[k] >> 30;
      uint64_t s = 0;
      TGeom g;
      uint32_t n = 0;
      if ((hm[k] >> lane) & 1ull) {
        if (typ != PW_OP_SUB) {
          n = wd[k] & 0x3FFFFFFFu;
        } else {  // run of '*' ops from idx: first non-'*' op at or after it
          const uint64_t ns0 = ~subm[0], ns1 = ~subm[1];
          uint32_t end;
          const uint64_t r0 = k == 0 ? (ns0 >> lane) : 0ull;
          if (k == 0 && r0) end = (uint32_t)lane + (uint32_t)__builtin_ctzll(r0);
          else {
            const uint64_t r1 = k == 0 ? ns1 : (ns1 >> lane);
            end = r1 ? (k == 0 ? 64u + (uint32_t)__builtin_ctzll(r1)
                               : 64u + (uint32_t)lane + (uint32_t)__builtin_ctzll(r1))
                     : 128u;
          }
          n = end - idx;
          if (end >= 128u) {  // the run continues past the segment
            uint32_t jj = sb + 128u;
            while (jj < n_ops && (ops[jj] >> 30) == PW_OP_SUB) {
              n++;
              jj++;
            }
          }
        }
        const uint32_t j = sb + idx;
        g = tgeom(T, typ, (int)n, ts[k]);
        const uint32_t pw = w->opw[kOpHalo + idx - 1], aw = w->opw[kOpHalo + idx + 1];
        const bool fast = tctx_fast(g, typ, (int)n, pw, j > 0, aw, j + 1 < n_ops);
        const uint32_t kidx = ev + (k == 0 ? (uint32_t)__popcll(hm[0] & lt) : n0 + (uint32_t)__popcll(hm[1] & lt));
        if (kidx < nmax) {
          s = rev ? evb + nmax - 1 - kidx : evb + kidx;
          // first / last line of the record in output order: the first created event, and the
          // last created one when this is the record's last segment (else flagged once the
          // record is done, below)
          const bool lastc = B.blocked ? kidx + 1 == B.tot : (fin && kidx + 1 == ev + nev);
          const bool first = rev ? lastc : kidx == 0, last = rev ? kidx == 0 : lastc;
          Hot hh;
          hh.qb = (uint32_t)(qb >> 4);
          hh.L = L;
          hh.qp = d.offset + qs[k];
          hh.tloc = rev ? T - ts[k] : ts[k];
          hh.ls = ls[k];
          hh.fn = hot_fn(typ, rev, fast, first, last, fast ? g.ll : 0, fast ? g.rl : 0, (d.ref & PW_REF_ACGT) != 0, n);
          hh.l0 = hl0[k];
          hh.l1 = hl1[k];
          if (W.hot_pbits && (((uint32_t)hh.qp >> W.hot_pbits) | (qi >> (32 - W.hot_pbits)))) {  // (hot_pbits contract)
            hh.fn = kNoEv;
            bad_hot = true;
          }
          store_hot(W, s, hh, qi);
          W.sflag[s] = fast ? (uint8_t)0 : (uint8_t)1;  // (every slot's flag is written: no memset)
          // the Cold record: read for the first / last line, saturated lengths and — the walk's
          // start (record, head op, its query / target position) — by tctx_kernel for target
          // contexts that are not a plain query copy (another event within 5 bases, an S run, a
          // long insertion; flagged above); one 16-byte store shared by all of them
          if (kidx == 0 || lastc || n >= kNBig || !fast) {
            Cold cd;
            cd.ai = ai;
            cd.j = j;
            cd.qs = qs[k];
            cd.ts = ts[k];
            W.cold[s] = cd;
          }
        }
      }
    }
    ev += nev;
    ev_last_seg = nev;
    prev_sub = (w->opw[kOpHalo + nseg - 1] >> 30) == PW_OP_SUB;
    qc += (int)qtot;
    tc += (int)ttot;
    lc += ltot;
    wave_sync();
  }
  if (__ballot(bad_hot) != 0 && err == PW_REC_OK) err = PW_REC_LAYOUT;
  if (B.blocked) {
    // slots nobody writes: this block's after a mismatch, and (last block) those past the
    // record's last event; creation index e sits in slot evb + e ('+') or evb + nmax - 1 - e ('-')
    const uint32_t f0 = ev < nmax ? ev : nmax, f1 = B.ev1 < nmax ? B.ev1 : nmax;
    if (f1 > f0) {
      const uint64_t a0 = rev ? evb + nmax - f1 : evb + f0, a1 = rev ? evb + nmax - f0 : evb + f1;
      for (uint64_t s = a0 + lane; s < a1; s += kWave) {
        hot_fn(W, s) = kNoEv;
        W.sflag[s] = 0;
      }
    }
    if (B.sb1 == n_ops && B.tot < nmax) {
      const uint64_t a0 = rev ? evb : evb + B.tot, a1 = rev ? evb + nmax - B.tot : evb + nmax;
      for (uint64_t s = a0 + lane; s < a1; s += kWave) {
        hot_fn(W, s) = kNoEv;
        W.sflag[s] = 0;
      }
    }
    if (lane == 0) {
      if (B.k == 0) {
        pw_aln_result res;
        res.text_off = res.text_end = 0;
        res.page_first = res.page_last = 0;
        res.text_len = 0;
        res.n_events = B.tot < nmax ? B.tot : nmax;
        res.err = err == PW_REC_OK && B.tot > nmax ? PW_REC_OVERFLOW : err;
        res.err_a = err_a;
        res.err_b = err_b;
        res.err_c = err_c;
        A.results[ai] = res;
        W.rec_mod[ai] = ~0ull;
      } else if (err != PW_REC_OK) {  // (finalize_kernel takes the first failing block)
        W.berr[B.bidx] = (v4u){(uint32_t)err, (uint32_t)err_a, (uint32_t)err_b, (uint32_t)err_c};
        atomicMin(&W.rec_bad[ai], B.k);
      }
    }
    return;
  }
  if (!layout_ok && pre.ev_next >= evb && pre.ev_next <= A.n_ev_slots)  // (contract violation: no events)
    for (uint64_t s = evb + lane; s < pre.ev_next; s += kWave) {
      hot_fn(W, s) = kNoEv;
      W.sflag[s] = 0;
    }
  const bool ev_over = ev > nmax;
  if (ev_over) {  // host event bound violated (cannot happen: every head is a counted op)
    err = PW_REC_OVERFLOW;
    ev = nmax;
  }
  // empty slots: merged '*' runs, or everything after a failure
  const uint64_t h0 = rev ? evb : evb + ev, h1 = rev ? evb + nmax - ev : evb + nmax;  // (none if !layout_ok)
  for (uint64_t s = h0 + lane; s < h1; s += kWave) {
    hot_fn(W, s) = kNoEv;
    W.sflag[s] = 0;
  }
  // the last created event was flagged when written unless the last segment had no event head
  // (or the event bound was violated): then flag it now, after this wave's store of its record
  if (lane == 0 && ev > 0 && err == PW_REC_OK && (ev_last_seg == 0 || ev_over)) {
    const uint64_t s_last = rev ? evb + nmax - ev : evb + ev - 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's store of that record first
    atomicOr(&hot_fn(W, s_last), rev ? 1u << 27 : 1u << 26);
    W.cold[s_last].ai = ai;
  }
  if (lane == 0) {
    pw_aln_result res;
    res.text_off = res.text_end = 0;
    res.page_first = res.page_last = 0;
    res.text_len = 0;
    res.n_events = ev;
    res.err = err;
    res.err_a = err_a;
    res.err_b = err_b;
    res.err_c = err_c;
    A.results[ai] = res;
    W.rec_mod[ai] = ~0ull;
  }
}

// index_kernel's (and index_pair_kernel's) end: blocks 1.. of the long records, spread over all
// wavefronts (a record of 1-5 Mb walked by one wave would be the whole kernel's critical path), and
// the padding slots of the last chunk (empty)
__device__ __forceinline__ void index_long_blocks(const pw_report_args& A, const Work& W, const LDS SmallTables* tp,
                                                  LDS IndexWave* w, int lane, int wv, uint32_t stride, bool planned,
                                                  uint32_t bid) {
  if (planned) {
    const uint32_t nbl = W.ctr[3] < W.blk_cap ? W.ctr[3] : W.blk_cap;
    for (uint32_t i = bid * kWaves + wv; i < nbl; i += stride) {
      const uint64_t e = W.blist[i];
      const uint32_t bai = (uint32_t)(e >> 32), k = (uint32_t)e;
      if (k == 0) continue;
      RecPre p;
      rec_pre(A, bai, A.desc[bai], lane, p);
      rec_pre_ready(A, p, lane);
      IdxBlk B = block_of(W, p.d, i - k, (p.d.n_ops + kBlkOps - 1) / kBlkOps, k, lane);
      B.prev_sub = (A.ops[p.d.op_begin + B.sb0 - 1] >> 30) == PW_OP_SUB;
      index_record(A, W, tp, w, bai, lane, p, B);
    }
  }
  const uint64_t pad0 = A.n_ev_slots, pad1 = W.n_chunks * kWave;
  if (bid == 0)
    for (uint64_t s = pad0 + threadIdx.x; s < pad1; s += kWave * kWaves) {
      hot_fn(W, s) = kNoEv;
      W.sflag[s] = 0;
    }
}

__global__ __launch_bounds__(kWave* kWaves, kIndexOcc) void index_kernel(pw_report_args A, Work W) {
  __shared__ SmallTables tab;
  __shared__ IndexWave iw[kWaves];
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, kWave * kWaves);
  __syncthreads();
  const int bid_ = index_prologue(A, W, tp);
  if (bid_ < 0) return;
  const uint32_t bid = (uint32_t)bid_;
  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  LDS IndexWave* w = (LDS IndexWave*)&iw[wv];
  // records ai, ai + stride, ...: the next record's head loads are issued before this record is
  // processed (its descriptor two records ahead), so their latency overlaps the work
  const uint32_t stride = (gridDim.x - W.ns_grid) * kWaves;
  const bool planned = A.max_rec_ops == 0 || A.max_rec_ops > (uint32_t)kBlkOps;  // plan_kernel ran
  uint32_t ai = bid * kWaves + wv;
  if (ai < A.n_alns) {
    // (indices past the batch are clamped to its last record: the loads stay unconditional)
    const uint32_t nm1 = A.n_alns - 1;
    RecPre cur;
    rec_pre(A, ai, A.desc[ai], lane, cur);
    DescRaw dn = load_desc(A, ai + stride < A.n_alns ? ai + stride : nm1);
    rec_pre_ready(A, cur, lane);
    pin(dn.a);
    pin(dn.b);
    for (; ai < A.n_alns; ai += stride) {
      const uint32_t an = ai + stride;
      RecPre nxt;
      rec_pre(A, an < A.n_alns ? an : nm1, unpack_desc(dn), lane, nxt);
      DescRaw dnn = load_desc(A, an + stride < A.n_alns ? an + stride : nm1);
      IdxBlk B = whole_record(cur.d);
      if (planned && cur.d.n_ops > (uint32_t)kBlkOps) {  // a long record: this wave decodes its block 0
        const uint32_t base = W.rec_blk[ai];
        if (base != kNoBlk)
          B = block_of(W, cur.d, base, (cur.d.n_ops + kBlkOps - 1) / kBlkOps, 0u, lane);
      }
      index_record(A, W, tp, w, ai, lane, cur, B);
      // (first consumed here, where the record's segment loads have already waited for them:
      // consumed at the top of the next iteration, the wait would also cover this record's stores)
      rec_pre_ready(A, nxt, lane);
      pin(dnn.a);
      pin(dnn.b);
      cur = nxt;
      dn = dnn;
    }
  }
  index_long_blocks(A, W, tp, w, lane, wv, stride, planned, bid);
}

// ------------------------------------------------------------------ index_kernel, two short records per wave
// Records of at most kPairOps ops (most of a gene panel's — cfg3 averages ~40 — where one record
// per wavefront left the wave's fixed per-record work, not the ops, as index_kernel's cost) go two
// to a wavefront, one per 32-lane half, every op at once (2 per lane).  The per-op work is
// index_record's for a record that fits one segment; the scans stop at the half (no row_bcast:31
// step), the ballots are read per half and the record fields are per lane.
constexpr uint32_t kPairOps = 64;
__device__ __forceinline__ uint32_t half_scan_incl(uint32_t v) {
  v += dpp_or_zero<0x111>(v);       // row_shr:1
  v += dpp_or_zero<0x112>(v);       // row_shr:2
  v += dpp_or_zero<0x114>(v);       // row_shr:4
  v += dpp_or_zero<0x118>(v);       // row_shr:8
  v += dpp_or_zero<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3: each half's second row
  return v;
}
__device__ __forceinline__ uint32_t half_last(uint32_t v, int lane) {  // lane 31's / lane 63's value
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 31), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  return lane < 32 ? a : b;
}
__device__ __forceinline__ uint32_t half_bits(uint64_t m, int lane) { return (uint32_t)(m >> (lane & 32)); }

// the head of a pair unit's record ri (valid: ri < n_alns), every value per lane
struct PairHead {
  pw_aln_desc d;
  uint64_t qb, ev_next;
  int L;
  uint32_t w0, w1;
};
__device__ __forceinline__ void pair_head(const pw_report_args& A, uint32_t ri, int hl, PairHead& p) {
  const uint32_t r = ri < A.n_alns ? ri : A.n_alns - 1;
  p.d = A.desc[r];
  const uint32_t qi = p.d.ref & PW_REF_QMASK;
  p.qb = A.qoff[qi];
  p.L = A.qlen[qi];
  p.ev_next = r + 1 < A.n_alns ? A.desc[r + 1].ev_begin : A.n_ev_slots;
  const uint32_t* ops = A.ops + p.d.op_begin;
  const uint32_t n = p.d.n_ops;
  const uint32_t* dummy = reinterpret_cast<const uint32_t*>(A.desc);  // (a readable word for lanes past the ops)
  p.w0 = *((uint32_t)hl < n ? ops + hl : dummy);
  p.w1 = *((uint32_t)(hl + 32) < n ? ops + hl + 32 : dummy);
  if ((uint32_t)hl >= n) p.w0 = 0u;
  if ((uint32_t)(hl + 32) >= n) p.w1 = 0u;
}

// the two records of a pair unit (record ri of this lane's half; valid = it exists)
__device__ __forceinline__ void index_pair(const pw_report_args& A, const Work& W, const LDS SmallTables* tab,
                                           LDS IndexWave* w, uint32_t ai, bool valid, int lane, const PairHead& P) {
  const int hl = lane & 31, half = lane >> 5;
  const pw_aln_desc& d = P.d;
  const uint64_t qb = P.qb;
  const uint8_t* R = A.qseq + qb;
  const bool layout_ok = (qb & 15u) == 0 && (qb >> 36) == 0 && P.ev_next >= d.ev_begin && P.ev_next <= A.n_ev_slots;
  const int L = P.L;
  const bool rev = (d.ref & PW_REF_REVERSE) != 0;
  const int T = d.t_len;
  const uint32_t n_ops = valid && layout_ok ? d.n_ops : 0u;
  const uint64_t evb = d.ev_begin;
  const uint32_t nmax = layout_ok ? (uint32_t)(P.ev_next - evb) : 0u;
  const uint32_t* lits32 = reinterpret_cast<const uint32_t*>(A.lits);
  LDS uint32_t* opw = w->opw + kOpHalo + 80 * half;  // this half's op words (opw[-1] and opw[64]: 0)
  // ---- op words + half scans of the query / target / literal advances
  uint32_t wd[2];
  int qs[2], ts[2];
  uint32_t ls[2];
  uint32_t qtot = 0, ttot = 0, ltot = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t idx = 32 * k + hl;
    wd[k] = idx < n_ops ? (k == 0 ? P.w0 : P.w1) : 0u;
    const uint32_t qa = op_qadv(wd[k]), ta = op_tadv(wd[k]), la = op_ladv(wd[k]);  // (0 for a 0 word... see below)
    const uint32_t qa_ = idx < n_ops ? qa : 0u, ta_ = idx < n_ops ? ta : 0u, la_ = idx < n_ops ? la : 0u;
    const uint32_t qi_ = half_scan_incl(qa_), ti_ = half_scan_incl(ta_), li_ = half_scan_incl(la_);
    qs[k] = (int)(qtot + qi_ - qa_);
    ts[k] = (int)(ttot + ti_ - ta_);
    ls[k] = d.lit_begin + ltot + li_ - la_;
    qtot += half_last(qi_, lane);
    ttot += half_last(ti_, lane);
    ltot += half_last(li_, lane);
    opw[idx] = wd[k];
  }
  if (hl == 0) {
    opw[-1] = 0u;
    opw[64] = 0u;
  }
  // ---- per op: query base, cs query base of a '*' op, the first 8 literal bytes of an event head
  uint8_t qlit[2], qref[2];
  uint32_t lw[2][3];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int qp = d.offset + qs[k];
    const int qc = qp < 0 ? 0 : (qp >= L ? (L > 0 ? L - 1 : 0) : qp);
    qref[k] = R[rev ? (L > 0 ? L - 1 - qc : 0) : qc];
    qlit[k] = A.lits[ls[k] + 1];
    const uint32_t la = ls[k] >> 2;
#pragma unroll
    for (int q = 0; q < 3; q++) lw[k][q] = lits32[la + q];
  }
  // ---- base check of every '*' op (pafreport.cpp:550-554) and event heads, per half
  uint32_t subm[2], hm[2];
  int bad_idx = INT_MAX;
  int err_a = 0, err_b = 0, err_c = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t idx = 32 * k + hl;
    const bool in = idx < n_ops;
    const uint32_t typ = wd[k] >> 30;
    const bool is_sub = in && typ == PW_OP_SUB;
    subm[k] = half_bits(__ballot(is_sub), lane);
    const bool prevsub = hl == 0 ? (k == 1 && ((subm[0] >> 31) & 1u) != 0) : ((subm[k] >> (hl - 1)) & 1u) != 0;
    hm[k] = half_bits(__ballot(in && (typ == PW_OP_INS || typ == PW_OP_DEL || (is_sub && !prevsub))), lane);
    const int qp = d.offset + qs[k];
    const uint8_t rch = (unsigned)qp >= (unsigned)L ? (uint8_t)0 : (rev ? tab->comp[qref[k]] : qref[k]);
    const uint8_t qch = qlit[k];
    const bool bad = is_sub && qch != rch;
    const uint32_t bm = half_bits(__ballot(bad), lane);
    const int fl = __builtin_ctz(bm | 0x80000000u);  // (31 when none: a lane in range)
    const int src = (lane & 32) + fl;
    const int ea = __shfl(qp, src, kWave), eb = __shfl((int)qch, src, kWave), ec = __shfl((int)rch, src, kWave);
    if (bm && bad_idx == INT_MAX) {
      bad_idx = 32 * k + fl;
      err_a = ea;
      err_b = eb;
      err_c = ec;
    }
  }
  wave_sync();
  uint32_t hl0[2], hl1[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t sh = ls[k] & 3u;
    hl0[k] = __builtin_amdgcn_alignbyte(lw[k][1], lw[k][0], sh);
    hl1[k] = __builtin_amdgcn_alignbyte(lw[k][2], lw[k][1], sh);
  }
  // ---- events (none after a mismatch: the record ends at its first one)
  const bool ok = bad_idx == INT_MAX;
  bool bad_hot = false;
  const uint32_t n0 = (uint32_t)__popc(hm[0]);
  const uint32_t nev = ok ? n0 + (uint32_t)__popc(hm[1]) : 0u;
  const uint32_t lt = (1u << hl) - 1u;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const uint32_t idx = 32 * k + hl;
    const uint32_t typ = wd[k] >> 30;
    if (ok && ((hm[k] >> hl) & 1u)) {
      uint32_t n;
      if (typ != PW_OP_SUB) {
        n = wd[k] & 0x3FFFFFFFu;
      } else {  // run of '*' ops from idx: first non-'*' op at or after it (ops past the record are not '*')
        const uint32_t ns0 = ~subm[0], ns1 = ~subm[1];
        uint32_t end;
        const uint32_t r0 = k == 0 ? (ns0 >> hl) : 0u;
        if (k == 0 && r0) end = (uint32_t)hl + (uint32_t)__builtin_ctz(r0);
        else {
          const uint32_t r1 = k == 0 ? ns1 : (ns1 >> hl);
          end = r1 ? (k == 0 ? 32u + (uint32_t)__builtin_ctz(r1) : 32u + (uint32_t)hl + (uint32_t)__builtin_ctz(r1)) : 64u;
        }
        n = end - idx;
      }
      const TGeom g = tgeom(T, typ, (int)n, ts[k]);
      const uint32_t pw = opw[(int)idx - 1], aw = opw[idx + 1];
      const bool fast = tctx_fast(g, typ, (int)n, pw, idx > 0, aw, idx + 1 < n_ops);
      const uint32_t kidx = k == 0 ? (uint32_t)__popc(hm[0] & lt) : n0 + (uint32_t)__popc(hm[1] & lt);
      if (kidx < nmax) {
        const uint64_t s = rev ? evb + nmax - 1 - kidx : evb + kidx;
        const bool lastc = kidx + 1 == nev;
        const bool first = rev ? lastc : kidx == 0, last = rev ? kidx == 0 : lastc;
        Hot hh;
        hh.qb = (uint32_t)(qb >> 4);
        hh.L = L;
        hh.qp = d.offset + qs[k];
        hh.tloc = rev ? T - ts[k] : ts[k];
        hh.ls = ls[k];
        hh.fn = hot_fn(typ, rev, fast, first, last, fast ? g.ll : 0, fast ? g.rl : 0, (d.ref & PW_REF_ACGT) != 0, n);
        hh.l0 = hl0[k];
        hh.l1 = hl1[k];
        const uint32_t qi = d.ref & PW_REF_QMASK;
        if (W.hot_pbits && (((uint32_t)hh.qp >> W.hot_pbits) | (qi >> (32 - W.hot_pbits)))) {  // (hot_pbits contract)
          hh.fn = kNoEv;
          bad_hot = true;
        }
        store_hot(W, s, hh, qi);
        W.sflag[s] = fast ? (uint8_t)0 : (uint8_t)1;
        if (kidx == 0 || lastc || n >= kNBig || !fast) {  // (and tctx_kernel's walk start)
          Cold cd;
          cd.ai = ai;
          cd.j = idx;
          cd.qs = qs[k];
          cd.ts = ts[k];
          W.cold[s] = cd;
        }
      }
    }
  }
  // ---- empty slots, results
  int err = !layout_ok ? PW_REC_LAYOUT : (ok ? PW_REC_OK : PW_REC_MISMATCH);
  if (half_bits(__ballot(bad_hot), lane) != 0u && err == PW_REC_OK) err = PW_REC_LAYOUT;
  uint32_t ev = nev;
  if (ev > nmax) {  // host event bound violated (cannot happen: every head is a counted op)
    err = PW_REC_OVERFLOW;
    ev = nmax;
  }
  if (valid) {
    if (!layout_ok) {
      if (P.ev_next >= evb && P.ev_next <= A.n_ev_slots)
        for (uint64_t s = evb + (uint64_t)hl; s < P.ev_next; s += 32) {
          hot_fn(W, s) = kNoEv;
          W.sflag[s] = 0;
        }
    } else {
      const uint64_t h0 = rev ? evb : evb + ev, h1 = rev ? evb + nmax - ev : evb + nmax;
      for (uint64_t s = h0 + (uint64_t)hl; s < h1; s += 32) {
        hot_fn(W, s) = kNoEv;
        W.sflag[s] = 0;
      }
    }
    if (hl == 0) {
      pw_aln_result res;
      res.text_off = res.text_end = 0;
      res.page_first = res.page_last = 0;
      res.text_len = 0;
      res.n_events = ev;
      res.err = err;
      res.err_a = err_a;
      res.err_b = err_b;
      res.err_c = err_c;
      A.results[ai] = res;
      W.rec_mod[ai] = ~0ull;
    }
  }
  wave_sync();
}

// one record of a unit that is not a pair (index_kernel's per-record step, without its prefetch)
__device__ __forceinline__ void index_one(const pw_report_args& A, const Work& W, const LDS SmallTables* tab,
                                          LDS IndexWave* w, uint32_t ai, int lane, bool planned) {
  RecPre p;
  rec_pre(A, ai, A.desc[ai], lane, p);
  rec_pre_ready(A, p, lane);
  IdxBlk B = whole_record(p.d);
  if (planned && p.d.n_ops > (uint32_t)kBlkOps) {
    const uint32_t base = W.rec_blk[ai];
    if (base != kNoBlk) B = block_of(W, p.d, base, (p.d.n_ops + kBlkOps - 1) / kBlkOps, 0u, lane);
  }
  index_record(A, W, tab, w, ai, lane, p, B);
}

__global__ __launch_bounds__(kWave* kWaves, kPairOcc) void index_pair_kernel(pw_report_args A, Work W) {
  __shared__ SmallTables tab;
  __shared__ IndexWave iw[kWaves];
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, kWave * kWaves);
  __syncthreads();
  const int bid_ = index_prologue(A, W, tp);
  if (bid_ < 0) return;
  const uint32_t bid = (uint32_t)bid_;
  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int hl = lane & 31;
  LDS IndexWave* w = (LDS IndexWave*)&iw[wv];
  const uint32_t stride = (gridDim.x - W.ns_grid) * kWaves;
  const bool planned = A.max_rec_ops == 0 || A.max_rec_ops > (uint32_t)kBlkOps;
  const uint32_t nu = (A.n_alns + 1) / 2;  // units of two records
  uint32_t u = bid * kWaves + wv;
  if (u < nu) {
    // the next unit's heads are loaded while this one is processed
    PairHead cur;
    pair_head(A, 2 * u + (uint32_t)(lane >> 5), hl, cur);
    for (; u < nu; u += stride) {
      const uint32_t un = u + stride;
      const uint32_t nx = 2 * (un < nu ? un : u) + (uint32_t)(lane >> 5);
      const uint32_t ai = 2 * u + (uint32_t)(lane >> 5);
      const bool valid = ai < A.n_alns;
      const uint32_t n_a = (uint32_t)__builtin_amdgcn_readlane((int)cur.d.n_ops, 0);
      const uint32_t n_b = (uint32_t)__builtin_amdgcn_readlane((int)cur.d.n_ops, 32);
      const bool b_ok = 2 * u + 1 < A.n_alns;
      if (n_a <= kPairOps && (!b_ok || n_b <= kPairOps)) {
        PairHead nxt;  // (the next unit's heads in flight while this pair is decoded)
        pair_head(A, nx, hl, nxt);
        index_pair(A, W, tp, w, ai, valid, lane, cur);
        cur = nxt;
      } else {  // (no head prefetch across the single-record path: it holds index_record's registers)
#pragma unroll 1
        for (uint32_t x = 2 * u; x < 2 * u + (b_ok ? 2u : 1u); x++) index_one(A, W, tp, w, x, lane, planned);
        pair_head(A, nx, hl, cur);
      }
    }
  }
  index_long_blocks(A, W, tp, w, lane, wv, stride, planned, bid);
}

// ------------------------------------------------------------------ long records: plan + carries
// plan_kernel: a thread per record; a record of more than kBlkOps ops reserves ceil(n / kBlkOps)
// consecutive blist entries (no room: it is decoded by one wavefront, and the entries it did get
// are marked block 0, which nobody decodes twice).
__global__ __launch_bounds__(256) void plan_kernel(pw_report_args A, Work W) {
  const uint32_t ai = blockIdx.x * 256 + threadIdx.x;
  if (ai >= A.n_alns) return;
  W.rec_bad[ai] = kNoBlk;
  const uint32_t n = A.desc[ai].n_ops;
  uint32_t base = kNoBlk;
  if (n > (uint32_t)kBlkOps) {
    const uint32_t nb = (n + kBlkOps - 1) / kBlkOps;
    const uint32_t b = atomicAdd(&W.ctr[3], nb);
    const bool fits = (uint64_t)b + nb <= W.blk_cap;
    for (uint32_t k = 0; k < nb && (uint64_t)b + k < W.blk_cap; k++)
      W.blist[b + k] = (uint64_t)ai << 32 | (fits ? k : 0u);
    if (fits) base = b;
  }
  W.rec_blk[ai] = base;
}

// carry_kernel: a wavefront per blist entry — the block's query / target / literal advance and
// its event heads (an indel op, or a '*' op not directly after another, pafreport.cpp:556-560),
// the quantities index_kernel's scans accumulate.
__global__ __launch_bounds__(kWave* kWaves) void carry_kernel(pw_report_args A, Work W) {
  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t nbl = W.ctr[3] < W.blk_cap ? W.ctr[3] : W.blk_cap;
  for (uint32_t i = blockIdx.x * kWaves + wv; i < nbl; i += gridDim.x * kWaves) {
    const uint64_t e = W.blist[i];
    const uint32_t ai = (uint32_t)(e >> 32), k = (uint32_t)e;
    const pw_aln_desc d = A.desc[ai];
    const uint32_t* ops = A.ops + d.op_begin;
    const uint32_t j0 = k * (uint32_t)kBlkOps;
    const uint32_t j1 = d.n_ops - j0 < (uint32_t)kBlkOps ? d.n_ops : j0 + (uint32_t)kBlkOps;
    uint32_t prev = j0 > 0 && (ops[j0 - 1] >> 30) == PW_OP_SUB ? 1u : 0u;
    uint32_t q = 0, t = 0, l = 0, h = 0;
    for (uint32_t jb = j0; jb < j1; jb += 4 * kWave) {
      uint32_t wd[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t j = jb + 64 * u + (uint32_t)lane;
        wd[u] = ops[j < j1 ? j : j0];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint32_t j = jb + 64 * u + (uint32_t)lane;
        const bool in = j < j1;
        const uint32_t w = in ? wd[u] : 0u, typ = w >> 30;
        const bool is_sub = in && typ == PW_OP_SUB;
        const uint64_t m = __ballot(is_sub);
        const bool prevsub = lane == 0 ? prev != 0 : ((m >> (lane - 1)) & 1ull) != 0;
        prev = (uint32_t)((m >> 63) & 1ull);
        q += in ? op_qadv(w) : 0u;
        t += in ? op_tadv(w) : 0u;
        l += in ? op_ladv(w) : 0u;
        h += (in && (typ == PW_OP_INS || typ == PW_OP_DEL || (is_sub && !prevsub))) ? 1u : 0u;
      }
    }
    q = wave_sum(q);
    t = wave_sum(t);
    l = wave_sum(l);
    h = wave_sum(h);
    if (lane == 0) W.bcarry[i] = (v4u){q, t, l, h};
  }
}

// ------------------------------------------------------------------ render_kernel
struct RenderWave {
  uint8_t line[kWave * kLStride];   // per-lane line buffers
  uint8_t qw[kWave * kQStride];     // per-lane forward-query windows
  Fixup lst[kLongCap];              // long lines for the epilogue
};
// kRenderOcc = 3 workgroups per CU: LDS is allocated in blocks larger than 1 KB (measured: a
// 53,864-byte workgroup ran render at 2 per CU, +50 % time; 53,096 at 3), so the bound is kept at
// 26 blocks of 2 KB
static_assert(sizeof(SmallTables) + kWaves * sizeof(RenderWave) <= 26 * 2048, "render LDS: 3 workgroups per CU");

// the record owning event slot s: the last one whose first slot is <= s (error path only)
// (arguments by value: a reference to the kernel arguments would put a copy of them in scratch)
__device__ __noinline__ uint32_t rec_of_slot(const pw_aln_desc* desc, uint32_t n_alns, uint64_t s) {
  uint32_t lo = 0, hi = n_alns - 1;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo + 1) / 2;
    if (desc[mid].ev_begin <= s) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}


// the raw record of chunk c's lane (the second half only for 32-byte records)
template <bool kH16>
struct HotRaw {
  v4u a, b;
};
template <>
struct HotRaw<true> {
  v4u a;
};
template <bool kH16>
__device__ __forceinline__ HotRaw<kH16> load_hot(const Work& W, uint64_t c, int lane) {
  const uint64_t cc = c < W.n_chunks ? c : W.n_chunks - 1;  // (W.n_chunks >= 1 when render runs)
  const v4u* p = reinterpret_cast<const v4u*>(W.hotw) + ((cc * kWave + (uint64_t)lane) << (kH16 ? 0 : 1));
  HotRaw<kH16> r;
  r.a = p[0];
  if constexpr (!kH16) r.b = p[1];
  return r;
}
// a 16-byte record's query: start (16-byte units) and length, loaded a stage ahead of its use
struct QInfo {
  uint32_t qb;
  int32_t L;
};
__device__ __forceinline__ QInfo load_qinfo(const pw_report_args& A, const Work& W, const HotRaw<true>& r) {
  const uint32_t qi = hot16_qi(W, r.a.x, r.a.y);
  QInfo q;
  q.qb = (uint32_t)(A.qoff[qi] >> 4);
  q.L = A.qlen[qi];
  return q;
}
__device__ __forceinline__ void pin(QInfo& q) { asm volatile("" : "+v"(q.qb), "+v"(q.L)); }
// The record is copied out of the load's registers here, before the next prefetch is issued (an
// explicit move into other registers, ordered as memory): left to hipcc, the copy sinks to the
// loop latch, after the next load, whose result then needs other registers and a move of its own
// at the latch — which waits for that load and exposes the prefetch's whole latency.  (16-byte
// records: l0 / l1 are filled from the literal words render_pre loads, once they are in.)
template <bool kH16>
__device__ __forceinline__ Hot decode_hot(const Work& W, const HotRaw<kH16>& r, const QInfo& q, bool valid) {
  Hot h;
  uint32_t fn, qp, tl, w3;
  asm volatile("v_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\tv_mov_b32 %2, %6\n\tv_mov_b32 %3, %7"
               : "=&v"(fn), "=&v"(qp), "=&v"(tl), "=&v"(w3)
               : "v"(r.a.x), "v"(r.a.y), "v"(r.a.z), "v"(r.a.w)
               : "memory");
  h.tloc = (int32_t)tl;
  h.ls = fn == kNoEv ? 0u : w3;
  if constexpr (kH16) {
    h.qp = (int32_t)hot16_qp(W, qp);
    h.qb = q.qb;
    h.L = q.L;
    h.l0 = h.l1 = 0u;
  } else {
    uint32_t qb, L, l0, l1;
    asm volatile("v_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\tv_mov_b32 %2, %6\n\tv_mov_b32 %3, %7"
                 : "=&v"(qb), "=&v"(L), "=&v"(l0), "=&v"(l1)
                 : "v"(r.b.x), "v"(r.b.y), "v"(r.b.z), "v"(r.b.w)
                 : "memory");
    h.qp = (int32_t)qp;
    h.qb = qb;
    h.L = (int32_t)L;
    h.l0 = l0;
    h.l1 = l1;
  }
  h.fn = valid ? fn : kNoEv;
  return h;
}

// What a lane needs from global memory before its line can be rendered besides the Hot record:
// the forward-query window, the tx record, the next-stop entry and, for a record's first / last
// line, the record index.  Issued for chunk c + NW while chunk c writes its page (the Hot record
// of c + NW was loaded one chunk earlier), so the latency hides behind a whole output phase.
struct RenderPre {
  v4u q[kQWin / 16];  // 48 forward-query bytes from the 16-byte aligned qlo
  v4u t0, t1;         // tx record (pre-rendered target context; garbage unless the slot has one)
  uint32_t ai;        // record of a first / last line (garbage otherwise)
  uint32_t ns_raw;    // next-stop entry (used when ns_ok)
  int qlo;            // forward position of q[0]
  int n;              // evtbases length (resolved when the Hot field saturates)
  bool ns_ok;
  uint32_t lw[3];     // 16-byte records: the literal words from ls & ~3 (the event's first 8 literal bytes)
};
template <bool kH16>
__device__ __forceinline__ void render_pre(const pw_report_args& A, const Work& W, const Hot& h, uint64_t s, bool skip,
                                           RenderPre& p) {
  if constexpr (kH16) {
    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(A.lits) + (h.ls >> 2);
#pragma unroll
    for (int q = 0; q < 3; q++) p.lw[q] = l32[q];
  }
  const bool ev = h.fn != kNoEv;
  const uint32_t typ = h.fn >> 30;
  const bool rev = (h.fn >> 29) & 1u;
  int n = (int)(h.fn & kNBig);
  // the tx record only for a pre-rendered target context, the Cold record only for a record's first
  // / last line: other lanes read slot 0's (valid memory, an L2 hit, unused) — an unconditional
  // load either way, without the HBM traffic of records nobody uses
  const uint64_t se_tx = (ev && !((h.fn >> 28) & 1u)) ? s : 0;
  const uint64_t se_cold = (ev && (h.fn & (3u << 26))) ? s : 0;
  {
    const v4u* tp4 = reinterpret_cast<const v4u*>(W.tx + (uint64_t)kTx * se_tx);
    p.t0 = tp4[0];
    p.t1 = tp4[1];
  }
  p.ai = W.cold[se_cold].ai;
  if (ev && (uint32_t)n == kNBig) {  // saturated length: from the op stream (rare; dependent loads)
    const Cold cd = W.cold[s];
    const pw_aln_desc d = A.desc[cd.ai];
    Rec r;
    r.ops = A.ops + d.op_begin;
    r.n_ops = d.n_ops;
    r.op_n = 0;
    r.op_lo = 0;
    r.opw = nullptr;
    n = event_len(r, cd.j, r.ops[cd.j]);
  }
  p.n = n;
  // 48 forward-query bytes from 8 before the event (16-byte aligned; covers [rloc - 8, rloc + 25],
  // the reads of all but long deletions)
  const uint8_t* R = ev ? A.qseq + ((uint64_t)h.qb << 4) : A.qseq;
  const int rl = ev ? event_rloc(h.L, rev, typ, h.qp, n) : 0;
  int x0 = rl - 8;
  if (x0 < 0) x0 = 0;
  // (R is 16-byte aligned: qseq is, and queries start at 16-byte multiples.  Pointer arithmetic,
  // not an integer round trip, keeps the loads global_load: flat loads would also count on
  // lgkmcnt and make every LDS wait of the output phase wait for them.)
  const int x0a = x0 & ~15;
  const v4u* a0 = reinterpret_cast<const v4u*>(R + x0a);
#pragma unroll
  for (int q = 0; q < kQWin / 16; q++) p.q[q] = a0[q];
  p.qlo = x0a;
  const int aap0 = rl / 3, rt = aap0 > 0 ? 3 * (aap0 - 1) : 0, a = rl - rt;
  const int x = typ == PW_OP_INS ? n : 0, dl = typ == PW_OP_DEL ? n : 0;
  const int k0 = rl + dl + (15 - a - x);
  p.ns_ok = ev && typ != PW_OP_SUB && A.next_stop && !skip && a + x <= 15 && (h.L - rt) + x - dl > 17 && k0 >= 0 &&
            k0 < h.L;
  const int32_t* nsp = p.ns_ok ? A.next_stop + ((uint64_t)h.qb << 4) + (uint64_t)k0 : (const int32_t*)A.qseq;
  p.ns_raw = (uint32_t)*nsp;
}
// the prefetched registers, first touched here
template <bool kH16>
__device__ __forceinline__ void render_pre_ready(RenderPre& p) {
#pragma unroll
  for (int q = 0; q < kQWin / 16; q++) pin(p.q[q]);
  pin(p.t0);
  pin(p.t1);
  pin(p.ai);
  pin(p.ns_raw);
  if constexpr (kH16) {
#pragma unroll
    for (int q = 0; q < 3; q++) pin(p.lw[q]);
  }
}

// One line, whole, from its slot's records (a long line: fixup_kernel, render's epilogue): the
// windows render stages (query bytes around the event, the tx record) plus kFxLit literal bytes go
// to the LDS buffers qwb (kQWin bytes) and lwb (kFxLit), the line to the sink
constexpr int kFxLit = 32;
template <class S>
__device__ __forceinline__ void long_line(const pw_report_args& A, const Work& W, const LDS SmallTables* tp, uint64_t s,
                                          LDS uint8_t* qwb, LDS uint8_t* lwb, S& g, bool skip) {
  const Hot h = load_hot_full(A, W, s);
  const uint32_t typ = h.fn >> 30;
  const bool rev = (h.fn >> 29) & 1u;
  const bool use_tx = !((h.fn >> 28) & 1u);
  int ne = (int)(h.fn & kNBig);
  Rec r;
  r.lits = A.lits;
  r.R = A.qseq + ((uint64_t)h.qb << 4);
  r.L = h.L;
  r.NS = A.next_stop ? A.next_stop + ((uint64_t)h.qb << 4) : nullptr;
  r.tab = tp;
  r.opw = nullptr;
  r.op_lo = 0;
  r.op_n = 0;
  r.lit0 = h.l0;
  r.lit1 = h.l1;
  r.ls0 = h.ls;
  r.ln = 8;
  r.rev = rev;
  r.acgt = (h.fn & kFnAcgt) != 0;
  r.offset = 0;
  r.T = 0;
  r.ops = nullptr;
  r.n_ops = 0;
  if ((uint32_t)ne == kNBig) {  // saturated length: from the op stream
    const Cold cd = W.cold[s];
    const pw_aln_desc d = A.desc[cd.ai];
    r.ops = A.ops + d.op_begin;
    r.n_ops = d.n_ops;
    ne = event_len(r, cd.j, r.ops[cd.j]);
  }
  // windows: tx record, 48 query bytes from 8 before the event, 32 literal bytes from ls
  v4u t0 = {0u, 0u, 0u, 0u}, t1 = t0;
  if (use_tx) {
    const v4u* tp4 = reinterpret_cast<const v4u*>(W.tx + (uint64_t)kTx * s);
    t0 = tp4[0];
    t1 = tp4[1];
  }
  const int rl = event_rloc(r.L, rev, typ, h.qp, ne);
  int x0 = rl - 8;
  if (x0 < 0) x0 = 0;
  const int x0a = x0 & ~15;  // (r.R is 16-byte aligned)
  const GV4* a0 = reinterpret_cast<const GV4*>((GU8)(r.R) + x0a);
#pragma unroll
  for (int q = 0; q < kQWin / 16; q++) *reinterpret_cast<LDS v4u*>(qwb + 16 * q) = a0[q];
  r.qw = qwb;
  r.qlo = x0a;
  r.qn = kQWin;
  const uint32_t l0 = h.ls & ~3u;
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(A.lits) + l0 / 4;
#pragma unroll
  for (int q = 0; q < kFxLit / 4; q++) reinterpret_cast<LDS uint32_t*>(lwb)[q] = l32[q];
  r.lw = lwb;
  r.l_lo = l0;
  r.l_n = kFxLit;
  EvIn in;
  in.typ = typ;
  in.n = ne;
  in.qp = h.qp;
  in.tloc = h.tloc;
  in.ls = h.ls;
  in.tmode = use_tx ? 1 : 0;
  in.ll = (int)((h.fn >> 23) & 7u);
  in.rl = (int)((h.fn >> 20) & 7u);
  in.tx[0] = t0.x, in.tx[1] = t0.y, in.tx[2] = t0.z, in.tx[3] = t0.w, in.tx[4] = t1.x, in.tx[5] = t1.y;
  in.ns_pre = kNsNone;
  int rel;
  emit_event(g, r, in, skip, rel);
}

// render's epilogue: the wave's listed long lines, one per lane (buffers over the wave's line /
// window area: the line at 256 lane, its literal window at 1024 + 32 lane, its query window at
// qwb), then stored byte by byte over the wave once the wave's page stores have completed
__device__ __forceinline__ void render_long_lines(const pw_report_args& A, const Work& W, const LDS SmallTables* tp,
                                               LDS RenderWave* w, LDS uint8_t* my_qw, int n_long, int lane, bool skip) {
  int len = 0;
  if (lane < n_long) {
    const uint32_t ls = w->lst[lane].s;
    LineSink ks;
    ks.line = w->line + 256 * lane;
    ks.pos = 0;
    ks.lim = kLong - kLSlack;
    long_line(A, W, tp, ls, my_qw, w->line + 1024 + kFxLit * lane, ks, skip);
    len = ks.pos;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int j = 0; j < n_long; j++) {
    const uint64_t dst = w->lst[j].dst;
    const int n = __builtin_amdgcn_readlane(len, j);
    const uint32_t v = reinterpret_cast<const LDS uint32_t*>(w->line + 256 * j)[lane];
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * lane + i < n) __builtin_nontemporal_store((uint8_t)(v >> (8 * i)), A.text + dst + 4 * lane + i);
  }
}

// Chunks are assigned statically (wave g takes chunks g, g + NW, ...): no work queue, no
// inter-wave communication.  Each chunk's lines form one text page (PW_PAGE_BYTES at
// chunk * PW_PAGE_BYTES, or an arena allocation when they do not fit).  Hot records are loaded
// two chunks ahead, the rest of a lane's inputs one chunk ahead (render_pre).
template <bool kH16>
__global__ __launch_bounds__(kWave* kWaves, kRenderOcc) void render_kernel(pw_report_args A, Work W) {
  __shared__ SmallTables tab;
  __shared__ __attribute__((aligned(16))) RenderWave rw[kWaves];
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, kWave * kWaves);
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  LDS RenderWave* w = (LDS RenderWave*)&rw[wv];
  LDS uint8_t* my_line = w->line + lane * kLStride;
  LDS uint8_t* my_qw = w->qw + lane * kQStride;
  const bool skip = A.skip_codan != 0;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;

  uint64_t c = (uint64_t)blockIdx.x * kWaves + wv;
  if (c >= W.n_chunks) return;
  Hot h;
  QInfo qn = {0u, 0};
  {
    const HotRaw<kH16> h0 = load_hot<kH16>(W, c, lane);
    if constexpr (kH16) qn = load_qinfo(A, W, h0);
    h = decode_hot<kH16>(W, h0, qn, true);
  }
  HotRaw<kH16> hn = load_hot<kH16>(W, c + nw, lane);
  int n_long = 0;  // entries in the wave's long-line list (uniform)
  RenderPre pre;
  render_pre<kH16>(A, W, h, c * kWave + (uint64_t)lane, skip, pre);
  {  // (six dropped stores: the loop is entered with the same count of memory operations after the
     // render_pre loads as each iteration leaves — hipcc's wait at the loop head takes the smaller)
    const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc((void*)A.text, (short)0, 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < 6; j++) __builtin_amdgcn_raw_buffer_store_b32(0u, rs0, kDropOff + 16u * (uint32_t)j, 0, 0);
  }
  for (; c < W.n_chunks; c += nw) {
    const uint64_t s = c * kWave + (uint64_t)lane;
    const bool act = h.fn != kNoEv;
    render_pre_ready<kH16>(pre);
    if constexpr (kH16) {
      // the next chunk's query starts / lengths (its records came in with this chunk's inputs),
      // consumed when it is decoded after this chunk's lines; this chunk's first literal bytes
      qn = load_qinfo(A, W, hn);
      lit8(h.ls, pre.lw[0], pre.lw[1], pre.lw[2], h.l0, h.l1);
    }
    const v4u t0 = pre.t0, t1 = pre.t1;
    const int ns_pre = pre.ns_ok ? (int)pre.ns_raw : kNsNone;
    const int qlo = pre.qlo, n_cur = pre.n;
    const Hot& hc = h;
    // the fast instantiation when every active lane's reads are in its registers / window: A/C/G/T,
    // rloc >= 4 (r_trloc = 3 * (rloc / 3 - 1) >= 0 with rloc - r_trloc in 3..5, and the RCTX
    // window rloc - 4 unclipped; the window starts at max(rloc - 8, 0) rounded down to 16, so it
    // covers every query byte in [rloc - 8, rloc + 25]), S runs of <= 4, insertions of <= 8
    // bases, deletions of <= 12 (the largest read, the tail image at r_trloc + deletion, ends by
    // rloc + 25).  (An insertion's modseq tail image starts at r_trloc - n, up to 8 bytes before
    // the lane's window: those bytes are LDS of the wave's line buffers, read and masked off.)
    // (and numbers below 10^8: emit_fast's decimal conversion)
    const int rlc = event_rloc(hc.L, (hc.fn >> 29) & 1u, hc.fn >> 30, hc.qp, n_cur);
    bool fast;
    {
      const uint32_t typ = hc.fn >> 30;
      const int rt = rlc >= 3 ? 3 * (rlc / 3 - 1) : 0;
      fast = !act || ((hc.fn & kFnAcgt) && rlc >= 4 && hc.L >= 9 && hc.L < 100000000 && hc.tloc < 99999999 &&
                      (typ == PW_OP_SUB ? (n_cur <= 4 && rt + 9 <= hc.L) : n_cur <= (typ == PW_OP_INS ? 8 : 12)));
    }
    // (uniform) the wave's line buffers and windows lane-interleaved (emit_fast) or per lane
    // (emit_event's byte sinks)
    const bool ilv = __ballot(!fast) == 0;
    if (ilv) {
      LDS uint32_t* q4 = reinterpret_cast<LDS uint32_t*>(w->qw) + lane;
#pragma unroll
      for (int q = 0; q < kQWin / 16; q++) {
        q4[(4 * q) * kTS] = pre.q[q].x;
        q4[(4 * q + 1) * kTS] = pre.q[q].y;
        q4[(4 * q + 2) * kTS] = pre.q[q].z;
        q4[(4 * q + 3) * kTS] = pre.q[q].w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < kQWin / 16; q++) {
        *reinterpret_cast<LDS v2u*>(my_qw + 16 * q) = (v2u){pre.q[q].x, pre.q[q].y};
        *reinterpret_cast<LDS v2u*>(my_qw + 16 * q + 8) = (v2u){pre.q[q].z, pre.q[q].w};
      }
    }
    int linelen = 0;
    bool held = false;  // a long line of a fast wave that the copy-out stores (one lane at most)
    if (act) {
      const uint32_t typ = hc.fn >> 30;
      const bool rev = (hc.fn >> 29) & 1u;
      const int n = n_cur;
      const bool use_tx = !((hc.fn >> 28) & 1u);
      Rec r;
      r.lits = A.lits;
      r.R = A.qseq + ((uint64_t)hc.qb << 4);
      r.L = hc.L;
      r.NS = A.next_stop ? A.next_stop + ((uint64_t)hc.qb << 4) : nullptr;
      r.tab = tp;
      r.opw = nullptr;
      r.op_lo = 0;
      r.op_n = 0;
      r.lw = nullptr;
      r.l_lo = 0;
      r.l_n = 0;
      r.lit0 = hc.l0;
      r.lit1 = hc.l1;
      r.ls0 = hc.ls;
      r.ln = 8;
      r.rev = rev;
      r.acgt = (hc.fn & kFnAcgt) != 0;
      r.offset = 0;
      r.T = 0;
      r.ops = nullptr;
      r.n_ops = 0;
      r.qw = my_qw;
      r.qlo = qlo;
      r.qn = kQWin;
      EvIn in;
      in.typ = typ;
      in.n = n;
      in.qp = hc.qp;
      in.tloc = hc.tloc;
      in.ls = hc.ls;
      in.tmode = use_tx ? 1 : 0;
      in.ll = (int)((hc.fn >> 23) & 7u);
      in.rl = (int)((hc.fn >> 20) & 7u);
      in.tx[0] = t0.x, in.tx[1] = t0.y, in.tx[2] = t0.z, in.tx[3] = t0.w, in.tx[4] = t1.x, in.tx[5] = t1.y;
      in.ns_pre = ns_pre;
      LineSink k;
      k.line = my_line;
      k.pos = 0;
      k.lim = kLine;
      int rel = 0;
      int merr;
      if (ilv) {
        DLine dl;
        dl.buf = w->line + 4 * lane;
        dl.pos = 0;
        merr = emit_fast(dl, w->qw + 4 * lane, qlo, tp, in, rev, r.L, hc.l0, hc.l1, r.NS, skip, rel);
        linelen = dl.pos;
        const uint64_t lng = __ballot(linelen > kLine);
        if (lng && lane == (int)__builtin_ctzll(lng) && linelen <= kAppMax) held = true;
      } else {
        merr = emit_event(k, r, in, skip, rel);
        linelen = k.pos;
      }
      if (merr >= 0) {  // modseq error: first failing event of the record in output order
        const uint32_t ai = rec_of_slot(A.desc, A.n_alns, s);
        const pw_aln_desc d = A.desc[ai];
        const uint64_t evb = d.ev_begin;
        const uint64_t ev_next = (ai + 1 < A.n_alns) ? A.desc[ai + 1].ev_begin : A.n_ev_slots;
        const uint64_t nmax = ev_next - evb, nev = A.results[ai].n_events;
        const uint64_t first = rev ? evb + nmax - nev : evb;
        const uint64_t key = (s - first) << 40 | (uint64_t)((uint32_t)(rel + merr) & 0xFFFFFu) << 20 |
                             (uint64_t)((uint32_t)merr & 0xFFFFFu);
        atomicMin((unsigned long long*)&W.rec_mod[ai], (unsigned long long)key);
      }
    }
    const uint32_t fn_cur = h.fn;
    const uint32_t ai_cur = pre.ai;
    // the next chunk's inputs load behind this one's output
    if constexpr (kH16) pin(qn);
    h = decode_hot<kH16>(W, hn, qn, c + nw < W.n_chunks);
    hn = load_hot<kH16>(W, c + 2 * nw, lane);
    render_pre<kH16>(A, W, h, (c + nw) * kWave + (uint64_t)lane, skip, pre);
    const uint32_t incl = wave_incl_scan((uint32_t)linelen, lane);
    const uint32_t B = wave_last(incl);
    const uint32_t my_off = incl - (uint32_t)linelen;
    // the page: in place, or an arena allocation when the lines (+ kPageSlack) do not fit
    uint64_t P = c * (uint64_t)PW_PAGE_BYTES;
    bool ok = true;
    if (B > (uint32_t)PW_PAGE_BYTES - kPageSlack) {
      const uint32_t need = ((B + 15u) & ~15u) + kPageSlack;
      unsigned long long a = 0;
      if (lane == 0) a = atomicAdd(W.arena_used, (unsigned long long)need);
      a = (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a, 0) |
          (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a >> 32), 0) << 32;  // (uniform: SGPRs)
      P = W.arena0 + a;
      if (P + need > A.text_total) {  // capacity violated: report, never write outside
        ok = false;
        if (lane == 0) atomicOr(&W.ctr[2], 1u);
      }
    }
    // long lines not held -> the wave's list (kLongCap, lines up to kLong bytes) or fixup_kernel:
    // the chunk's lane mask (every chunk writes it) and the lines' destinations — plain stores: a
    // returning atomic here cost a round trip per chunk with a long line
    const uint64_t lone = __ballot(held);
    const bool later = ok && linelen > kLine && !held;
    bool need_fix = later && linelen > kLong - kLSlack;
    {
      const uint64_t lm2 = __ballot(later && linelen <= kLong - kLSlack);
      if (lm2) {  // (uniform)
        const int k = n_long + __popcll(lm2 & ((1ull << lane) - 1ull));
        if ((lm2 >> lane) & 1ull) {
          if (k < kLongCap) {
            w->lst[k].s = (uint32_t)s;
            w->lst[k].dst = P + my_off;
          } else {
            need_fix = true;
          }
        }
        n_long = min(n_long + __popcll(lm2), kLongCap);
      }
    }
    const uint64_t lm = __ballot(need_fix);
    if (lane == 0) {
      pw_page pg;
      pg.off = P;
      pg.len = ok ? B : 0u;
      pg.pad = 0;
      A.pages[c] = pg;
      W.lmask[c] = lm;
      if (lm) atomicAdd(&W.ctr[1], (uint32_t)__popcll(lm));  // (no return value: no wait)
    }
    const uint64_t g0 = P + my_off;
    if (act && (fn_cur & (3u << 26))) {  // first / last line of a record
      const uint32_t ai = ai_cur;
      if ((fn_cur >> 27) & 1u) {
        A.results[ai].text_off = g0;
        A.results[ai].page_first = (uint32_t)c;
      }
      if ((fn_cur >> 26) & 1u) {
        A.results[ai].text_end = g0 + (uint64_t)linelen;
        A.results[ai].page_last = (uint32_t)c;
      }
    }
    if (need_fix) {  // the line's destination for fixup_kernel
      Fixup f;
      f.s = (uint32_t)s;
      f.pad = 0;
      f.dst = g0;
      W.fix[s] = f;
    }
    {
      // copy-out: every lane places its own line at page offset my_off (a long line: its first
      // kLine bytes, fixup_kernel rewrites it) as dwords realigned to the page, 16 bytes per group,
      // its last group first.  A group's dwords past the line's end are overwritten later by the
      // next line's first group (written in the last round), and that group's first dword is the
      // shared one: the next line ORs this line's tail bytes into it (shuffled from the previous
      // non-empty lane).  The page's last line may write up to 12 bytes past B: the page keeps
      // kPageSlack bytes free.  The groups go to an LDS image of the page (then stored as
      // contiguous 1 KB rows), or, for an arena page, straight to global memory.
      // Every global store here is a buffer store issued by every lane: one with no bytes to write
      // gets an offset past the buffer's range and the hardware drops it (as branches, the next
      // iteration's first wait — for the render_pre loads, which precede these stores — would count
      // them as possibly absent and wait for them too: vmcnt is in order).
      const bool wr = ok && B > 0;  // (uniform)
      // (the descriptor's fields through readfirstlane: hipcc otherwise treats the arena path's
      // values as divergent and wraps each store in a waterfall loop)
      const uint64_t pa = (uint64_t)A.text + (wr ? P : 0ull);
      const uint64_t Pu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pa) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pa >> 32)) << 32;
      const int nrec = __builtin_amdgcn_readfirstlane(wr ? (int)(B + (uint32_t)kPageSlack) : 0);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)Pu, (short)0, nrec, 0x00020000);
      const uint64_t ne = __ballot(linelen > 0);
      const int ln = linelen > kLine ? kLine : linelen;
      const uint32_t sh = my_off & 3u, a0 = my_off & ~3u;
      // this line's bytes in the dword at floor4(my_off + linelen): [linelen - t, linelen), t of them
      const uint32_t t = (my_off + (uint32_t)linelen) & 3u;
      uint32_t Lw[28];
      if (ilv) {  // (uniform) lane-interleaved line buffers
        const LDS uint32_t* l4 = reinterpret_cast<const LDS uint32_t*>(w->line) + lane;
#pragma unroll
        for (int k = 0; k < 28; k++) Lw[k] = l4[k * kTS];
      } else {
        const LDS v4a4* lp4 = reinterpret_cast<const LDS v4a4*>(my_line);  // (4-byte aligned: 148-byte stride)
#pragma unroll
        for (int q = 0; q < 7; q++) {
          const v4u v = lp4[q];
          Lw[4 * q] = v.x, Lw[4 * q + 1] = v.y, Lw[4 * q + 2] = v.z, Lw[4 * q + 3] = v.w;
        }
      }
      uint32_t tail;
      {
        // (an empty line's tail is never used: tb < 0 reads dword 0)
        const int tb = min(linelen - (int)t, kLine);
        uint32_t d0, d1;
        if (ilv) {
          const LDS uint32_t* tp4 = reinterpret_cast<const LDS uint32_t*>(w->line) + lane + (max(tb, 0) >> 2) * kTS;
          d0 = tp4[0];
          d1 = tp4[kTS];
        } else {
          const LDS uint32_t* tp4 = reinterpret_cast<const LDS uint32_t*>(my_line + (tb & ~3));
          d0 = tp4[0];
          d1 = tp4[1];
        }
        tail = __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)tb & 3u) & (uint32_t)((1ull << (8 * t)) - 1ull);
      }
      const uint64_t below = ne & ((1ull << lane) - 1ull);
      const int prev = below ? 63 - __builtin_clzll(below) : lane;
      const uint32_t ptail = (uint32_t)__shfl((int)tail, prev, kWave) & (uint32_t)((1ull << (8 * sh)) - 1ull);
      const uint32_t sel = 0x07060504u - __builtin_amdgcn_perm(0u, sh, 0u);
      const int kmax = linelen > 0 ? ((int)sh + ln - 1) >> 2 : -1;  // last dword (from a0) holding a line byte
      const int jmax = kmax >> 2;
      auto group = [&](int j) -> v4u {  // the line's dwords [4j, 4j + 4) realigned to the page
        uint32_t v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int k = 4 * j + i;
          const uint32_t cur = k < 28 ? Lw[k] : 0u, prv = k == 0 ? 0u : Lw[k - 1];
          v[i] = __builtin_amdgcn_perm(cur, prv, sel);
        }
        if (j == 0) v[0] |= ptail;
        return (v4u){v[0], v[1], v[2], v[3]};
      };
      // the held line's column, contiguous, to the window rows past it (from row kLStride / 4,
      // column jl + 1: clear of the column's own dwords there), before the page image overwrites
      // the line rows
      LDS uint32_t* const hl = reinterpret_cast<LDS uint32_t*>(w->line) + (kLStride / 4) * kTS + 1;
      if (lone != 0) {  // (uniform)
        const int jl = (int)__builtin_ctzll(lone);
        const uint32_t v = reinterpret_cast<const LDS uint32_t*>(w->line)[(lane < kIlvRows ? lane : 0) * kTS + jl];
        if (lane < kIlvRows) hl[jl + lane] = v;
      }
      if (B + (uint32_t)kPageSlack <= (uint32_t)PW_PAGE_BYTES) {  // (uniform) the page in place:
        // every lane writes its groups into the wave's line buffer at its page offset (the page
        // image; the lines are in Lw already), then the image goes out as contiguous 1 KB stores —
        // one cache line per 8 lanes instead of one or two per lane
        wave_sync();
        LDS uint8_t* img = w->line;
#pragma unroll
        for (int j = 6; j >= 0; j--)
          if (j <= jmax) *reinterpret_cast<LDS v4a4*>(img + a0 + 16u * (uint32_t)j) = group(j);
        wave_sync();
#pragma unroll
        for (int q = 0; q < 8; q++) {  // (PW_PAGE_BYTES / 1024 rows; rows past B are dropped)
          const uint32_t o = 1024u * (uint32_t)q + 16u * (uint32_t)lane;
          __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const LDS v4u*>(img + o), rs, o < B ? o : kDropOff, 0, kTextPolicy);
        }
      } else {  // an arena page: every lane stores its own groups
#pragma unroll
        for (int j = 6; j >= 0; j--)
          __builtin_amdgcn_raw_buffer_store_b128(group(j), rs, j <= jmax ? a0 + 16u * (uint32_t)j : kDropOff, 0, kTextPolicy);
      }
      if (lone != 0 && wr) {  // (uniform) the held line, byte by byte over the wave, once the stores
        // above (its first kLine bytes; the next line's first dword, which ORs in this line's tail
        // from the clamped buffer) have completed
        const int jl = (int)__builtin_ctzll(lone);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)my_off, jl);
        const int ln2 = __builtin_amdgcn_readlane(linelen, jl);
        const uint32_t v = lane < kIlvRows ? hl[jl + lane] : 0u;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int o = 4 * lane + i;
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> (8 * i)), rs, o < ln2 ? lo + (uint32_t)o : kDropOff, 0, kTextPolicy);
        }
      }
    }
    wave_sync();
  }
  // epilogue: the listed long lines (out of line: a second emit_event instance inlined here
  // doubled the kernel's code)
  if (n_long > 0) {  // (the lane-derived addresses recomputed: kept live across the loop, one was spilled)
    int l2 = lane;
    asm volatile("" : "+v"(l2));
    render_long_lines(A, W, tp, w, w->qw + l2 * kQStride, n_long, l2, skip);
  }
}

// ------------------------------------------------------------------ tctx_kernel
// Target contexts that are not a plain copy of query bytes (another event within 5 bases, an
// S run, a long insertion; setTContext, pafreport.cpp:120-128, revCompl :631, abbreviation
// :918-927).  A wavefront scans its 256-slot groups' flag bytes (one group ahead), queues the
// flagged slots in LDS across groups and takes them 64 at a time, one event per lane: the lane stages its event's op words, forward
// query bytes and literal bytes in LDS windows (independent loads, one wait), then walks the op
// stream from the event's head op through the windows (tseq is never materialised; reads
// outside a window fall back to global memory) and stores the 32-byte record (length byte +
// field) for render_kernel.
constexpr int kTcOps = 12;   // op words staged per event, from head op - 6
constexpr int kTcQ = 48;     // forward-query bytes staged (16-byte aligned, from centre - 24)
struct TctxLane {
  uint32_t opw[kTcOps];
  uint8_t qw[kTcQ];
  uint8_t out[kTx + 4];      // record + junk
};
struct TctxWave {
  TctxLane ln[kWave];
  uint32_t list[5 * kWave];  // the wave's queue of flagged slots (carried + a 256-slot group: the
                             // carried entries are taken first when they would not fit)
};
// One flagged event's inputs, loaded in three dependent levels (tc_load1..3: the caller issues
// each level for all its events before the next)
struct TcIn {
  uint64_t s;
  v4u a;             // the event record's first 16 bytes
  v4u b;             // its second 16 bytes (32-byte records)
  Cold cd;           // the walk's start: record, head op, query / target position (index_kernel)
  uint32_t qi_off_lo, qi_off_hi;
  int32_t L;
  uint32_t lw0, lw1, lw2;  // literal dwords from ls & ~3 (16-byte records)
  uint32_t op_begin, n_ops;
  int32_t offset, t_len;
  v4u qv[kTcQ / 16];
  uint32_t ow[kTcOps];
  int x0a, o0;
};
__device__ __forceinline__ void tc_load1(const Work& W, uint64_t s, TcIn& x) {
  x.s = s;
  const v4u* p = reinterpret_cast<const v4u*>(W.hotw + (s << W.hot_sh));
  x.a = p[0];
  x.b = W.hot_pbits ? (v4u){0u, 0u, 0u, 0u} : p[1];
  x.cd = W.cold[s];
}
__device__ __forceinline__ void tc_load2(const pw_report_args& A, const Work& W, TcIn& x) {
  const pw_aln_desc d = A.desc[x.cd.ai];
  x.op_begin = d.op_begin;
  x.n_ops = d.n_ops;
  x.offset = d.offset;
  x.t_len = d.t_len;
  if (W.hot_pbits) {
    const uint32_t qi = hot16_qi(W, x.a.x, x.a.y);
    const uint64_t qo = A.qoff[qi];
    x.qi_off_lo = (uint32_t)(qo >> 4);
    x.qi_off_hi = 0;
    x.L = A.qlen[qi];
    const uint32_t ls = x.a.x == kNoEv ? 0u : x.a.w;
    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(A.lits) + (ls >> 2);
    x.lw0 = l32[0];
    x.lw1 = l32[1];
    x.lw2 = l32[2];
  } else {
    x.qi_off_lo = x.b.x;
    x.qi_off_hi = 0;
    x.L = (int32_t)x.b.y;
    x.lw0 = x.lw1 = x.lw2 = 0u;
  }
}
__device__ __forceinline__ int tc_qp(const Work& W, const TcIn& x) {
  return W.hot_pbits ? (int32_t)hot16_qp(W, x.a.y) : (int32_t)x.a.y;
}
__device__ __forceinline__ void tc_load3(const pw_report_args& A, TcIn& x, const Work& W) {
  // forward query bytes of the context: [fc - 5, fc + n + 5) for a '+' record, [fc - n - 5,
  // fc + 5] for a '-' record (n <= 12 unless abbreviated), fc = the event's forward position
  const bool rev = (x.a.x >> 29) & 1u;
  const int qp = tc_qp(W, x);
  const int fc = rev ? x.L - 1 - qp : qp;
  int x0 = fc - (rev ? kTcQ / 2 : 8);
  if (x0 < 0) x0 = 0;
  x.x0a = x0 & ~15;  // (the query is 16-byte aligned)
  const GV4* a0 = reinterpret_cast<const GV4*>((GU8)(A.qseq + ((uint64_t)x.qi_off_lo << 4)) + x.x0a);
#pragma unroll
  for (int q = 0; q < kTcQ / 16; q++) x.qv[q] = a0[q];
  // op words [j - 6, j + 6) (indices clamped to the record's last op, values masked after: a
  // guarded load would be a branch and a vmcnt(0) per word)
  const int j = (int)x.cd.j;
  x.o0 = j - kTcOps / 2 < 0 ? 0 : j - kTcOps / 2;
  const uint32_t* ops = A.ops + x.op_begin;
  const uint32_t olast = x.n_ops ? x.n_ops - 1 : 0u;
#pragma unroll
  for (int q = 0; q < kTcOps; q++) x.ow[q] = ops[(uint32_t)(x.o0 + q) < olast ? (uint32_t)(x.o0 + q) : olast];
}
// the event's target context, walked over the staged windows, stored as its 32-byte tx record
__device__ __forceinline__ void tc_event(const pw_report_args& A, const Work& W, const LDS SmallTables* tp,
                                         LDS TctxLane* me, const TcIn& x) {
  Rec r;
  r.R = A.qseq + ((uint64_t)x.qi_off_lo << 4);
  r.L = x.L;
  const uint32_t fn = x.a.x;
  r.rev = (fn >> 29) & 1u;
  r.ops = A.ops + x.op_begin;
  r.lits = A.lits;
  r.NS = nullptr;
  r.tab = tp;
  r.offset = x.offset;
  r.T = x.t_len;
  r.n_ops = x.n_ops;
  r.acgt = false;
  // the event's first 8 literal bytes are in registers; op words and forward query bytes
  // around the event are staged in LDS
  const uint32_t ls = fn == kNoEv ? 0u : x.a.w;
  uint32_t l0, l1;
  if (W.hot_pbits) {
    lit8(ls, x.lw0, x.lw1, x.lw2, l0, l1);
  } else {
    l0 = x.b.z;
    l1 = x.b.w;
  }
  r.lit0 = l0;
  r.lit1 = l1;
  r.ls0 = ls;
  r.ln = 8;
  r.lw = nullptr;
  r.l_lo = 0;
  r.l_n = 0;
  const int j = (int)x.cd.j;
#pragma unroll
  for (int q = 0; q < kTcOps; q++) me->opw[q] = (uint32_t)(x.o0 + q) < r.n_ops ? x.ow[q] : 0u;
#pragma unroll
  for (int q = 0; q < kTcQ / 16; q++) *reinterpret_cast<LDS v4u*>(me->qw + 16 * q) = x.qv[q];
  r.opw = me->opw;
  r.op_lo = x.o0;
  r.op_n = (uint32_t)kTcOps;
  r.qw = me->qw;
  r.qlo = x.x0a;
  r.qn = kTcQ;
  const uint32_t wd = opword(r, (uint32_t)j);
  int ne = (int)(fn & kNBig);
  if ((uint32_t)ne == kNBig) ne = event_len(r, (uint32_t)j, wd);
  LdsSink<kTx - 1> ks;
  ks.buf = me->out + 1;
  ks.junk = me->out + kTx;
  ks.pos = 0;
  emit_tctx_walk(ks, r, wd >> 30, ne, (uint32_t)j, wd, x.cd.qs, x.cd.ts, ls);
  me->out[0] = (uint8_t)ks.pos;
  const LDS uint32_t* t32 = reinterpret_cast<const LDS uint32_t*>(me->out);
  v4u t0, t1;
  t0.x = t32[0];
  t0.y = t32[1];
  t0.z = t32[2];
  t0.w = t32[3];
  t1.x = t32[4];
  t1.y = t32[5];
  t1.z = t32[6];
  t1.w = t32[7];
  v4u* dtx = reinterpret_cast<v4u*>(W.tx + (uint64_t)kTx * x.s);
  dtx[0] = t0;
  dtx[1] = t1;
}
__global__ __launch_bounds__(kWave* kWaves) void tctx_kernel(pw_report_args A, Work W) {
  __shared__ SmallTables tab;
  __shared__ __attribute__((aligned(16))) TctxWave tw[kWaves];
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, kWave * kWaves);
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  LDS TctxWave* w = (LDS TctxWave*)&tw[wv];
  LDS TctxLane* me = &w->ln[lane];
  const uint64_t n_groups = (W.n_chunks * kWave + 255) / 256;
  const uint32_t* f32 = reinterpret_cast<const uint32_t*>(W.sflag);
  const uint64_t nf32 = W.n_chunks * kWave / 4;
  // the next group's flag words load one group ahead (clamped index, masked when consumed)
  const uint64_t gstride = (uint64_t)gridDim.x * kWaves;
  uint64_t gi = (uint64_t)blockIdx.x * kWaves + wv;
  const uint64_t flast = nf32 ? nf32 - 1 : 0;
  uint32_t fnext = nf32 ? f32[gi * kWave + lane < nf32 ? gi * kWave + lane : flast] : 0u;
  // flagged slots queue up in the wave's list across its groups and are processed 64 at a time
  // (every lane has an event except in the wave's last batch): the walk runs once per 64 events,
  // not once per group (~40 flagged slots per 256 at cfg2)
  uint32_t nl = 0;  // entries in the list (wave-uniform)
  // A batch takes up to 128 entries: lane l the events of entries l and 64 + l.  Both events'
  // records load together, level by level (Hot / Cold, then the query table / descriptor /
  // literal words); the second event's wait in registers while the first one is walked, so a
  // wave's second 64 events cost one level of loads (their windows) and a walk, not a whole chain.
  auto batch = [&](uint32_t nb) {
    const bool has1 = (uint32_t)lane < nb, has2 = (uint32_t)lane + kWave < nb;
    // (unconditional loads: a lane without an entry reads entry 0's records)
    const uint64_t s1 = w->list[has1 ? lane : 0], s2 = w->list[has2 ? kWave + lane : 0];
    TcIn x1, x2;
    tc_load1(W, s1, x1);
    tc_load1(W, s2, x2);
    tc_load2(A, W, x1);
    tc_load2(A, W, x2);
    tc_load3(A, x1, W);
    if (has1) tc_event(A, W, tp, me, x1);
    // (the second event's windows load after the first walk: held across it, they pushed the
    // kernel past 128 VGPRs)
    if (nb > (uint32_t)kWave) {  // (uniform)
      tc_load3(A, x2, W);
      if (has2) tc_event(A, W, tp, me, x2);
    }
  };
  for (; gi < n_groups; gi += gstride) {
    const uint64_t fi = gi * kWave + lane;
    uint32_t fcur = fnext;
    asm volatile("" : "+v"(fcur));
    const uint64_t fin = fi + gstride * kWave;
    fnext = nf32 ? f32[fin < nf32 ? fin : flast] : 0u;
    const uint32_t f4 = (fi < nf32 ? fcur : 0u) & 0x01010101u;
    const uint32_t cnt = (uint32_t)__popc(f4);
    const uint32_t incl = wave_incl_scan(cnt, lane);
    const uint32_t total = wave_last(incl);
    if (total == 0) continue;
    if (nl + total > 5u * kWave) {  // (uniform; only groups of > 192 flagged slots)
      batch(nl);
      nl = 0;
      wave_sync();
    }
    uint32_t o = nl + incl - cnt;
#pragma unroll
    for (int q = 0; q < 4; q++)
      if ((f4 >> (8 * q)) & 1u) w->list[o++] = (uint32_t)(gi * 256 + (uint64_t)(4 * lane + q));
    nl += total;
    wave_sync();
    while (nl >= (uint32_t)(2 * kWave)) {
      batch((uint32_t)(2 * kWave));
      // the entries after the batch move to the front (<= 4 per lane)
      const uint32_t rest = nl - (uint32_t)(2 * kWave);
      uint32_t mv[4];
      wave_sync();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = (uint32_t)(lane + kWave * k);
        mv[k] = i < rest ? w->list[2 * kWave + i] : 0u;
      }
      wave_sync();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = (uint32_t)(lane + kWave * k);
        if (i < rest) w->list[i] = mv[k];
      }
      nl = rest;
      wave_sync();
    }
  }
  if (nl) batch(nl);
}

// ------------------------------------------------------------------ fixup_kernel
__device__ __forceinline__ void finalize_record(const pw_report_args& A, const Work& W, uint32_t ai);
// Lines longer than the LDS line buffer, one per thread, rewritten in place (their bytes were
// reserved).  The thread stages the same windows as render_kernel (query bytes around the event,
// the tx record) plus 32 literal bytes in LDS, so only the line itself goes to global memory.
struct FixLane {
  uint8_t qw[kQWin];
  uint8_t lw[kFxLit];
};
__global__ __launch_bounds__(256) void fixup_kernel(pw_report_args A, Work W) {
  __shared__ SmallTables tab;
  __shared__ __attribute__((aligned(16))) FixLane fl[256];
  __shared__ uint64_t mk[kWaves][kWave];  // the long-line masks of the wave's 64 chunks
  __shared__ uint32_t ex[kWaves][kWave];  // exclusive prefix of their popcounts
  // workgroups [fix_wg, gridDim.x): the per-record results (finalize_kernel's work: one launch
  // less per pass; they do not depend on the long lines' bytes), one record per thread, beside
  // the long lines of workgroups [0, fix_wg) — the two dependent-load chains run side by side
  const uint32_t fix_wg = gridDim.x - (A.n_alns + 255) / 256;
  if (blockIdx.x >= fix_wg) {  // (the whole workgroup: before any barrier)
    const uint32_t ai = (blockIdx.x - fix_wg) * 256 + threadIdx.x;
    if (ai < A.n_alns) finalize_record(A, W, ai);
    return;
  }
  // no long lines (inputs without S runs of many codons / long indels): the workgroup ends here
  if (W.ctr[1] == 0) return;
  LDS SmallTables* tp = (LDS SmallTables*)&tab;
  stage_small_tables(tp, threadIdx.x, 256);
  __syncthreads();
  LDS FixLane* me = (LDS FixLane*)&fl[threadIdx.x];
  const bool skip = A.skip_codan != 0;
  if (W.ctr[2]) return;  // overflow: the results report it, nothing is rewritten
  // a wave takes 64 chunks at a time and spreads their long lines over its lanes (line j of the
  // group -> lane j % 64): the chunk of line j is the last one whose prefix is <= j
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint64_t nwt = (uint64_t)fix_wg * kWaves;
  for (uint64_t c0 = ((uint64_t)blockIdx.x * kWaves + wv) * kWave; c0 < W.n_chunks; c0 += nwt * kWave) {
    const uint64_t cl = c0 + (uint64_t)lane;
    const uint64_t m = cl < W.n_chunks ? W.lmask[cl] : 0ull;
    const uint32_t cnt = (uint32_t)__popcll(m);
    const uint32_t incl = wave_incl_scan(cnt, lane);
    const uint32_t T = wave_last(incl);
    if (T == 0) continue;
    mk[wv][lane] = m;
    ex[wv][lane] = incl - cnt;
    wave_sync();
  for (uint32_t jl = (uint32_t)lane; jl < T; jl += kWave) {
    int k = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1)
      if (k + step < kWave && ex[wv][k + step] <= jl) k += step;
    uint64_t mm = mk[wv][k];
    for (uint32_t r = jl - ex[wv][k]; r > 0; r--) mm &= mm - 1;
    const Fixup f = W.fix[(c0 + (uint64_t)k) * kWave + (uint64_t)__builtin_ctzll(mm)];
    GlobalSink g;
    g.p = (PW_GLOBAL uint8_t*)(A.text + f.dst);
    g.pos = 0;
    long_line(A, W, tp, f.s, me->qw, me->lw, g, skip);
  }
    wave_sync();
  }
}

// ------------------------------------------------------------------ finalize_kernel
__device__ __forceinline__ void finalize_record(const pw_report_args& A, const Work& W, uint32_t ai) {
  const bool planned = A.max_rec_ops == 0 || A.max_rec_ops > (uint32_t)kBlkOps;
  pw_aln_result r = A.results[ai];
  if (W.ctr[2]) {
    r.err = PW_REC_OVERFLOW;
  } else if (r.err == PW_REC_OK && planned && W.rec_blk[ai] != kNoBlk && W.rec_bad[ai] != kNoBlk) {
    // a long record's first block with a base mismatch (blocks decoded by other wavefronts)
    const v4u e = W.berr[W.rec_blk[ai] + W.rec_bad[ai]];
    r.err = (int32_t)e.x;
    r.err_a = (int32_t)e.y;
    r.err_b = (int32_t)e.z;
    r.err_c = (int32_t)e.w;
  } else if (r.err == PW_REC_OK) {
    if (r.n_events) {  // bytes of the lines, across the pages they span
      uint64_t len;
      if (r.page_first == r.page_last) {
        len = r.text_end - r.text_off;
      } else {
        const pw_page p0 = A.pages[r.page_first];
        len = p0.off + p0.len - r.text_off;
        // (eight independent page loads per step: a record of a Mb contig spans ~500 pages)
        uint32_t c = r.page_first + 1;
        for (; c + 8 <= r.page_last; c += 8) {
          uint32_t pl[8];
#pragma unroll
          for (int u = 0; u < 8; u++) pl[u] = A.pages[c + u].len;
#pragma unroll
          for (int u = 0; u < 8; u++) len += pl[u];
        }
        for (; c < r.page_last; c++) len += A.pages[c].len;
        len += r.text_end - A.pages[r.page_last].off;
      }
      r.text_len = (uint32_t)len;
    }
    const uint64_t key = W.rec_mod[ai];
    if (key != ~0ull) {
      r.err = PW_REC_MODSEQ;
      r.err_c = (int32_t)(key >> 40);
      r.err_a = (int32_t)((key >> 20) & 0xFFFFFu);
      r.err_b = (int32_t)(key & 0xFFFFFu);
    }
  }
  A.results[ai] = r;
}

__global__ __launch_bounds__(256) void finalize_kernel(pw_report_args A, Work W) {
  const uint32_t ai = blockIdx.x * 256 + threadIdx.x;
  if (ai < A.n_alns) finalize_record(A, W, ai);
}

// ------------------------------------------------------------------ per-genome tables
// One row per target sequence: alignments, event lines, aligned target bases (the tables the
// multi-GPU driver all-gathers).  A thread per record, atomics into the rows.
__global__ __launch_bounds__(256) void genome_table_kernel(const pw_aln_result* res, const uint32_t* gof,
                                                           const int32_t* taln, uint32_t n, pw_genome_row* rows,
                                                           uint32_t ng) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = gof[i];
  if (g >= ng) return;
  const int32_t tb = taln[i];
  atomicAdd(&rows[g].records, 1u);
  atomicAdd(&rows[g].events, res[i].n_events);
  atomicAdd((unsigned long long*)&rows[g].t_bases, (unsigned long long)(tb > 0 ? tb : 0));
}

}  // namespace pw

extern "C" int pw_genome_table(const pw_aln_result* results, const uint32_t* genome_of, const int32_t* t_aln,
                               uint32_t n_alns, pw_genome_row* rows, uint32_t n_genomes, void* stream) {
  if (n_genomes && !rows) return PW_E_ARG;
  if (n_alns && (!results || !genome_of || !t_aln)) return PW_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n_genomes && hipMemsetAsync(rows, 0, (size_t)n_genomes * sizeof(pw_genome_row), st) != hipSuccess)
    return PW_E_HIP;
  if (n_alns)
    hipLaunchKernelGGL(pw::genome_table_kernel, dim3((n_alns + 255) / 256), dim3(256), 0, st, results, genome_of,
                       t_aln, n_alns, rows, n_genomes);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

extern "C" uint32_t pw_report_hot_pbits(uint64_t max_qlen, uint64_t n_queries) {
  uint32_t pb = 1, qb = 0;
  while (pb < 32 && (1ull << pb) <= max_qlen) pb++;
  while (qb < 32 && (1ull << qb) < n_queries) qb++;
  return pb <= 31 && pb + qb <= 32 ? pb : 0u;
}
extern "C" uint64_t pw_report_workspace_bytes(uint64_t n_events_max, uint64_t n_alns) {
  return pw::work_layout(nullptr, n_events_max, n_alns, nullptr);
}
extern "C" uint64_t pw_report_page_count(uint64_t n_ev_slots) { return (n_ev_slots + PW_PAGE_EVENTS - 1) / PW_PAGE_EVENTS; }
extern "C" uint64_t pw_report_text_bytes(uint64_t n_ev_slots, uint64_t text_bound) {
  // (an arena allocation is its text rounded to 16 bytes + kPageSlack: at most one per page)
  return pw_report_page_count(n_ev_slots) * (PW_PAGE_BYTES + pw::kPageSlack) + pw::align_up(text_bound, 16) + 16;
}

extern "C" int pw_report_events_after(const pw_report_args* args, void* stream, void* next_stop_ready);
extern "C" int pw_report_events(const pw_report_args* args, void* stream) {
  return pw_report_events_after(args, stream, nullptr);
}
extern "C" int pw_report_events_after(const pw_report_args* args, void* stream, void* next_stop_ready) {
  if (!args || !args->desc || !args->ops || !args->qseq || !args->qoff || !args->qlen || !args->results ||
      (!args->text && args->text_total))
    return PW_E_ARG;
  if (!args->skip_codan && !args->next_stop) return PW_E_ARG;
  // (unknown flag bits or a nonzero pad: a caller that left fields unset, e.g. a stack struct)
  if ((args->flags & ~(uint32_t)PW_REPORT_BUILD_NEXT_STOP) || args->pad || args->skip_codan > 1) return PW_E_ARG;
  const bool build_ns = (args->flags & PW_REPORT_BUILD_NEXT_STOP) && !args->skip_codan;
  if (args->n_alns == 0) {  // (the table is still built when asked for)
    if (build_ns && args->n_queries)
      return pw_stop_table_build(args->qseq, args->qoff, args->qlen, args->n_queries, const_cast<int32_t*>(args->next_stop),
                                 stream);
    return PW_OK;
  }
  const uint64_t need = pw_report_workspace_bytes(args->n_ev_slots, args->n_alns);
  if (!args->workspace || args->workspace_bytes < need || ((uintptr_t)args->workspace & 255)) return PW_E_ARG;
  // per-lane windows are 16-byte loads, literal words 4-byte loads, pages 16-byte stores
  if (((uintptr_t)args->qseq & 15) || ((uintptr_t)args->lits & 3) || ((uintptr_t)args->text & 15)) return PW_E_ARG;
  if (args->n_ev_slots && (!args->pages || args->text_total < pw_report_page_count(args->n_ev_slots) * PW_PAGE_BYTES))
    return PW_E_ARG;
  // (event slots are 32-bit indices in the fixup records and tctx_kernel's queue: a batch holds
  // fewer than 2^32 - 2^16 slots; the hosts cut batches far below that)
  if (args->n_ev_slots >= (1ull << 32) - (1ull << 16)) return PW_E_ARG;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  if (args->hot_pbits > 31) return PW_E_ARG;
  pw::Work W;
  pw::work_layout(static_cast<uint8_t*>(args->workspace), args->n_ev_slots, args->n_alns, &W);
  W.hot_pbits = args->hot_pbits;
  W.hot_sh = args->hot_pbits ? 2u : 3u;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t nwave = pw::kWaves;
  uint64_t ig = (args->n_alns + nwave - 1) / nwave;
  const bool planned = args->max_rec_ops == 0 || args->max_rec_ops > (uint32_t)pw::kBlkOps;
  // the next-stop table by index's first workgroups (one per query, 4096 at most), and the
  // counters: a memset launch when plan_kernel runs first (it counts blocks in ctr[3]), else
  // cleared by index itself (round 5: the memset dispatch and the side stream's event wait before
  // render were ~11 us of the cfg2 pass)
  W.ns_grid = build_ns ? (args->n_queries < 4096u ? args->n_queries : 4096u) : 0u;
  W.clear_ctr = planned ? 0u : 1u;
  if (build_ns && args->n_queries && !args->qseq) return PW_E_ARG;
  if (planned && hipMemsetAsync(args->workspace, 0, 64, st) != hipSuccess) return PW_E_HIP;
  // (four rounds at 5 waves/SIMD — round-4 sweep on cfg2, same-box pairs: 10 / 15 / 20 / 30 per
  // CU 127.9-128.8 / 128.3 / 125.9-126.1 / 128.7 us; round 2 found 16 worse than 10 before the
  // segment and prefetch changes); with long records (planned) the blocks of 1.. are spread over a
  // grid of 10 per CU whatever the record count (the grid that was measured for cfg4)
  if (planned) ig = (uint64_t)ncu * 10u;
  else if (ig > (uint64_t)ncu * 20u) ig = (uint64_t)ncu * 20u;
  if (planned) {  // records of more than PW_BLOCK_OPS ops
    hipLaunchKernelGGL(pw::plan_kernel, dim3((args->n_alns + 255) / 256), dim3(256), 0, st, *args, W);
    hipLaunchKernelGGL(pw::carry_kernel, dim3((uint32_t)ncu * 8u), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
  }
  // mostly short records (a gene panel): two per wavefront (index_pair_kernel); its grid is two
  // full rounds at the 4 waves/SIMD it runs at (sweep on cfg3 at 0.2: 8 per CU 1,421-1,436 us,
  // 4 / 12 1,427 / 1,421, 10 — index_kernel's, 2.5 rounds here — 1,474-1,481, 16 1,458)
  if (args->n_short && (uint64_t)args->n_short * 4 >= (uint64_t)args->n_alns * 3)
    hipLaunchKernelGGL(pw::index_pair_kernel,
                       dim3((uint32_t)std::min<uint64_t>(((args->n_alns + 1) / 2 + nwave - 1) / nwave, (uint64_t)ncu * 8u) +
                            W.ns_grid),
                       dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
  else
    hipLaunchKernelGGL(pw::index_kernel, dim3((uint32_t)ig + W.ns_grid), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
  if (W.n_chunks) {
    uint64_t tg = (W.n_chunks * pw::kWave + 255) / 256 / pw::kWaves + 1;
    if (tg > (uint64_t)ncu * 4u) tg = (uint64_t)ncu * 4u;
    hipLaunchKernelGGL(pw::tctx_kernel, dim3((uint32_t)tg), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
    uint64_t rg = (W.n_chunks + nwave - 1) / nwave;
    // four rounds of the kRenderOcc resident workgroups per CU: later rounds fill the CUs whose
    // first workgroups finish early (round 2: 2 rounds 286.5 vs 288-290 us at one; round 4,
    // same-call pairs on cfg2: 4 rounds 214.1-216.3 us, 8 rounds 215.2, 2 rounds 220.8-221.5)
    if (rg > (uint64_t)ncu * 4u * pw::kRenderOcc) rg = (uint64_t)ncu * 4u * pw::kRenderOcc;
    // (render is the first kernel that reads next_stop)
    if (next_stop_ready && hipStreamWaitEvent(st, (hipEvent_t)next_stop_ready, 0) != hipSuccess) return PW_E_HIP;
    if (W.hot_pbits)
      hipLaunchKernelGGL(pw::render_kernel<true>, dim3((uint32_t)rg), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
    else
      hipLaunchKernelGGL(pw::render_kernel<false>, dim3((uint32_t)rg), dim3(pw::kWave * pw::kWaves), 0, st, *args, W);
    // (+ finalize: ncu workgroups for the long lines, then one thread per record)
    hipLaunchKernelGGL(pw::fixup_kernel, dim3((uint32_t)ncu + (uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0,
                       st, *args, W);
  } else {
    hipLaunchKernelGGL(pw::finalize_kernel, dim3((uint32_t)((args->n_alns + 255) / 256)), dim3(256), 0, st, *args, W);
  }
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
