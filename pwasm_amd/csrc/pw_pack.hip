// pw_pack.hip — cs-string tokenising on gfx950.
//
// Reference: the cs loop of PAFAlignment::PAFAlignment (pafreport.cpp:536-626), restated on the
// host by pw_pack_cs (pw_host.cpp).  This kernel packs a whole batch of cs strings at once into
// the same op words and literal bytes, one 64-lane wavefront per record at a time (persistent
// waves, the next record's head loaded ahead), 256 characters per window, 4 per lane:
//   * a lane's 4 characters come straight from two aligned dword loads and one alignbyte (no LDS
//     staging pass); the window is also stored in LDS once, for the next two lanes' characters
//     (an op's digits) — that is the only LDS traffic;
//   * in a well-formed cs string every op starts at one of ':', '*', '+', '-' and no other
//     character is one of them (digits follow ':', letters the others), so the op starts of a
//     window are a ballot, and an op runs to the next op start (the last one of a window that
//     does not reach the string end is carried into the next window); a lane holds at most two
//     op starts (every op has at least two characters);
//   * per op: the 8 characters after its start are a register image (two alignbytes of this and
//     the next two lanes' characters): a ':' run of 1-9 digits is checked and converted in SIMD
//     (two 4-digit halves, then the 9th); per character: its governing op (its own lane's, or the last start
//     below it: a DPP max-scan) says whether it is a literal ('*' pair, '-' bases) or must be a
//     letter ('+' / '-' content);
//   * DPP wave scans of the query / target / literal advances and of the packed op / event /
//     substitution counts place every op word and literal byte (byte stores, one per literal
//     character, from the lane that holds it) and give the positions of the reference's bounds
//     checks; the record totals are the scans' last lanes (no LDS reductions).
// Anything else — a character outside [0-9A-Za-z:*+-], a ':' run of 0 or more than 9 digits, a
// '*' not followed by exactly two characters, an empty indel or one holding a digit, '~' / '=', a
// bounds violation, one op longer than a window — flags the record PW_PACK_HOST: the caller packs
// it with pw_pack_cs, which produces the reference's exact error (such records are rare and end
// the report at their line anyway).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pwasm_amd.h"
#include "pw_wave.h"

namespace pw {

#define LDS __attribute__((address_space(3)))
constexpr int kPackWin = 256;  // characters per window (4 per lane)
constexpr uint32_t kPkBoundSub = 190, kPkBoundIndel = 140;  // = the host packer's text bounds

// per byte of a dword: 0x80 where the byte is (not) in a class
__device__ __forceinline__ uint32_t bytes_eq(uint32_t x, uint32_t c) {  // 0x80 where byte == c
  const uint32_t t = x ^ (c * 0x01010101u);
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
__device__ __forceinline__ uint32_t bytes_digit(uint32_t x) {  // 0x80 where '0'..'9'
  const uint32_t t = x ^ 0x30303030u;                          // digits -> 0..9
  return ~(((t & 0x7F7F7F7Fu) + 0x76767676u) | t) & 0x80808080u;
}
__device__ __forceinline__ uint32_t bytes_alpha(uint32_t x) {  // 0x80 where A-Z / a-z
  // per byte u = 0x80 + (c & 0xDF) - 'A' (every byte >= 0x80 before the subtraction: no borrow)
  const uint32_t u = ((x & 0xDFDFDFDFu) | 0x80808080u) - 0x41414141u;
  const uint32_t t = u ^ 0x80808080u;  // (c & 0xDF) - 'A' where that is >= 0, else a byte >= 0x80
  const uint32_t lt26 = ~(((t & 0x7F7F7F7Fu) + 0x66666666u) | t) & 0x80808080u;  // 0 <= t < 26
  return lt26 & ~(x & 0x80808080u);  // (bytes >= 0x80 are not letters)
}
__device__ __forceinline__ uint32_t msb_bits(uint32_t m) {  // 0x80 per byte -> bits 0..3
  return (m >> 7 & 1u) | (m >> 14 & 2u) | (m >> 21 & 4u) | (m >> 28 & 8u);
}
// value of a run of 4 decimal digits held as byte values 0..9, most significant in byte 0
__device__ __forceinline__ uint32_t dec4(uint32_t x) {
  const uint32_t y = (x * 10u + (x >> 8)) & 0x00FF00FFu;
  return (y * 100u + (y >> 16)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t up_bytes(uint32_t x) {  // a-z -> A-Z per byte (letters only)
  return x & ~(bytes_alpha(x) >> 2);                         // 0x80 >> 2 = 0x20: clear the case bit
}
__device__ __forceinline__ uint32_t dpp_max_incl(uint32_t v) {  // inclusive prefix max (v >= 0)
  v = max(v, dpp_or_zero<0x111>(v));
  v = max(v, dpp_or_zero<0x112>(v));
  v = max(v, dpp_or_zero<0x114>(v));
  v = max(v, dpp_or_zero<0x118>(v));
  v = max(v, dpp_or_zero<0x142, 0xA>(v));
  v = max(v, dpp_or_zero<0x143, 0xC>(v));
  return v;
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane l gets lane l-1's value (lane 0: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

// A record's head in two prefetch stages: its extent, offset and query length two records ahead
// (uniform: scalar loads — as per-lane vector loads every lane's copy went through the texture
// units: 4 of a record's 7 vector reads), then its first window's two aligned dwords per lane one
// record ahead (vector loads).  Addresses past the record are clamped to its last
// dword (the caller's text is only readable up to the last record's end + 16 bytes).
struct PkHead {
  uint64_t base, end;
  int off, ql;
};
__device__ __forceinline__ void pk_words(const uint8_t* text, uint64_t st, uint64_t last, int lane, uint32_t& d0,
                                         uint32_t& d1) {
  const uint64_t a0 = (st & ~3ull) + 4ull * (uint64_t)lane;
  d0 = *reinterpret_cast<const uint32_t*>(text + (a0 < last ? a0 : last));
  d1 = *reinterpret_cast<const uint32_t*>(text + (a0 + 4 < last ? a0 + 4 : last));
}
__device__ __forceinline__ uint64_t pk_last(const PkHead& h) {  // the record's last dword
  return h.end > h.base ? (h.end - 1) & ~3ull : h.base & ~3ull;
}
__device__ __forceinline__ void pk_head(const uint64_t* cs_off, const int32_t* offset, const int32_t* qlen, uint32_t ri,
                                        PkHead& h) {
  h.base = cs_off[ri];
  h.end = cs_off[ri + 1];
  h.off = offset[ri];
  h.ql = qlen[ri];
}
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }

__global__ __launch_bounds__(256) void pack_cs_kernel(const uint8_t* text, const uint64_t* __restrict__ cs_off,
                                                      const int32_t* __restrict__ offset,
                                                      const int32_t* __restrict__ qlen, uint32_t n, uint32_t* ops,
                                                      uint8_t* lits, pw_cs_rec* out) {
  __shared__ uint32_t win[4][kPackWin / 4 + 4];  // the window's characters, zeros past its end (lanes read 3 dwords on)
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: scalar loop)
  LDS uint32_t* w = (LDS uint32_t*)win[wv];
  const uint32_t nw = gridDim.x * 4;
  uint32_t ri = blockIdx.x * 4 + (uint32_t)wv;
  if (ri >= n) return;
  const uint32_t nl1 = n - 1;
  PkHead h1, h2;
  pk_head(cs_off, offset, qlen, ri, h1);
  pk_head(cs_off, offset, qlen, ri + nw < n ? ri + nw : nl1, h2);
  uint32_t d0n, d1n;
  pk_words(text, h1.base, pk_last(h1), lane, d0n, d1n);
  if (lane < 4) w[64 + lane] = 0u;
  for (; ri < n; ri += nw) {
    // this record's head (two stages loaded ahead); the next record's first window words and the
    // one after's head are issued before this record is decoded
    pin(d0n);
    pin(d1n);
    const PkHead cur = h1;
    const uint32_t w0 = d0n, w1 = d1n;
    pk_words(text, h2.base, pk_last(h2), lane, d0n, d1n);
    h1 = h2;
    pk_head(cs_off, offset, qlen, ri + 2 * nw < n ? ri + 2 * nw : nl1, h2);
    const uint64_t base = __builtin_amdgcn_readfirstlane((int)(uint32_t)cur.base) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(cur.base >> 32)) << 32;
    const uint64_t L = cur.end - cur.base;
    const uint64_t last = pk_last(cur);
    const int off = cur.off, ql = cur.ql;
    int qpos = 0, tpos = 0;
    uint32_t nops = 0, nlits = 0, nev = 0;
    uint64_t bound = 0;
    bool bad = false, acgt = true;
    uint64_t pos = 0;
    uint32_t* const ops_r = ops + base;  // (uniform: stores take 32-bit lane offsets)
    uint8_t* const lits_r = lits + base;
    // one 256-character window at pos (the first from the prefetched words; later ones load theirs)
    auto window = [&](uint32_t d0, uint32_t d1) -> bool {
      const int wl = (int)(L - pos < (uint64_t)kPackWin ? L - pos : (uint64_t)kPackWin);
      const bool last_win = pos + (uint64_t)wl == L;
      // this lane's 4 characters (zeros past the window)
      const uint32_t sh = (uint32_t)((base + pos) & 3ull);
      uint32_t c4 = __builtin_amdgcn_alignbyte(d1, d0, sh);
      const int have = min(max(wl - 4 * lane, 0), 4);  // characters of this lane in the window
      c4 = have >= 4 ? c4 : (c4 & ((1u << (8 * have)) - 1u));
      w[lane] = c4;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t n1 = w[lane + 1], n2 = w[lane + 2], n3 = w[lane + 3];  // the next 12 characters
      // classes (per byte 0x80), restricted to the lane's characters
      const uint32_t vmask = have >= 4 ? 0x80808080u : ((0x80808080u << (8 * have)) ^ 0x80808080u) & 0x80808080u;
      const uint32_t m_col = bytes_eq(c4, ':'), m_sub = bytes_eq(c4, '*'), m_ins = bytes_eq(c4, '-'),
                     m_del = bytes_eq(c4, '+');
      const uint32_t m_op = (m_col | m_sub | m_ins | m_del) & vmask;
      const uint32_t m_dig = bytes_digit(c4), m_alp = bytes_alpha(c4);
      bool lbad = (vmask & ~(m_op | m_dig | m_alp)) != 0;
      const uint32_t smask = msb_bits(m_op);  // op starts among this lane's characters (bit j)
      // every window starts at an op start (the string's first character, or an op carried over)
      const bool starts = (__builtin_amdgcn_readfirstlane(smask) & 1u) != 0;
      const uint64_t any = __ballot(smask != 0);
      const int ll = 63 - __builtin_clzll(any | 1ull);
      const uint32_t lmask = (uint32_t)__builtin_amdgcn_readlane((int)smask, ll);
      const int last_start = 4 * ll + (31 - __builtin_clz(lmask | 1u));
      const int lim = last_win ? wl : last_start;  // ops starting before lim are decoded now
      // the first op start after this lane's characters (an op ends there)
      const uint64_t above = lane == 63 ? 0ull : any & ~((2ull << lane) - 1ull);
      const int nl = above ? __builtin_ctzll(above) : 64;
      const uint32_t nl_mask = (uint32_t)__shfl((int)smask, nl < 64 ? nl : 0, 64);
      const int next_start = nl < 64 ? 4 * nl + __builtin_ctz(nl_mask) : wl;
      // this lane's op starts before lim: at most two
      const int lim_l = min(max(lim - 4 * lane, 0), 4);
      const uint32_t sm = smask & ((1u << lim_l) - 1u);
      const int ns = __popc(sm);
      lbad = lbad || ns > 2;
      // the (at most two) ops of this lane, without branches: every quantity is computed for both
      // slots and selected by the op kind (a divergent branch per kind costs every wave all kinds)
      int q_a = 0, t_a = 0;                  // query / target advance of this lane's ops
      // ops emitted | events << 8 | substitutions << 16 | literals << 23: a window of 256 characters
      // has at most 128 ops / events, 85 substitutions and 255 literals, so the fields of one
      // scan's prefixes never carry into each other
      uint32_t cnt = 0;
      uint32_t opw[2];
      bool emit[2];
      int qb[2], qn[2];                      // bounds checks: query advance before the op, its length
      int kind[2];                           // 0 ':' 1 '*' 2 '-' 3 '+' (PW_OP_* order), -1 none
      const uint32_t sm1 = sm & (sm - 1u);
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const uint32_t rest = t == 0 ? sm : sm1;
        const bool valid = rest != 0;
        const int j = __builtin_ctz(rest | 8u);  // (3 when none: any in-range value)
        const uint32_t after = smask & ~((2u << j) - 1u);  // this lane's next start (a carried op's too)
        const int e = after ? 4 * lane + __builtin_ctz(after) : next_start;
        const int len = e - (4 * lane + j) - 1;
        const uint32_t c = __builtin_amdgcn_ubfe(c4, 8u * (uint32_t)j, 8u);
        // the 9 characters after the op start (zeros past the window)
        const uint32_t k1 = (uint32_t)j + 1u;
        const bool k4 = k1 >= 4;
        const uint32_t lo = k4 ? n1 : __builtin_amdgcn_alignbyte(n1, c4, k1);
        const uint32_t hi = k4 ? n2 : __builtin_amdgcn_alignbyte(n2, n1, k1);
        const uint32_t c9 = (k4 ? n3 : __builtin_amdgcn_alignbyte(n3, n2, k1)) & 0xFFu;
        const bool is_col = valid && c == ':', is_sub = valid && c == '*', is_ins = valid && c == '-',
                   is_del = valid && c == '+';
        kind[t] = is_col ? PW_OP_MATCH : (is_sub ? PW_OP_SUB : (is_ins ? PW_OP_INS : (is_del ? PW_OP_DEL : -1)));
        // ':' - 1..9 digits, checked and converted in SIMD (8 as two 4-digit halves, then the 9th)
        const uint64_t d = (uint64_t)(lo ^ 0x30303030u) | (uint64_t)(hi ^ 0x30303030u) << 32;
        const uint64_t have_d = (uint64_t)bytes_digit(lo) | (uint64_t)bytes_digit(hi) << 32;
        const int ln = min(max(len, 1), 8);
        const uint64_t lmask = ln >= 8 ? ~0ull : ((1ull << (8 * ln)) - 1ull);
        const bool dig_bad = ((uint32_t)(len - 1) > 8u) | ((lmask & 0x8080808080808080ull & ~have_d) != 0) |
                             ((len == 9) & (c9 - '0' > 9u));
        const uint64_t al = (d & lmask) << (8 * (8 - ln));  // right-aligned
        const uint32_t v8 = dec4((uint32_t)al) * 10000u + dec4((uint32_t)(al >> 32));
        const uint32_t v = len == 9 ? v8 * 10u + (c9 - '0') : v8;
        lbad = lbad | (is_col & dig_bad) | (is_sub & (len != 2)) | ((is_ins | is_del) & (len < 1));
        const int n_op = is_col ? (int)v : (is_sub ? 1 : max(len, 0));
        qb[t] = q_a;
        qn[t] = is_sub ? 0 : n_op;
        q_a += (is_col || is_sub || is_del) ? n_op : 0;
        t_a += (is_col || is_sub || is_ins) ? n_op : 0;
        emit[t] = valid && (!is_col || v > 0);
        opw[t] = PW_OP((uint32_t)(kind[t] & 3), (uint32_t)n_op);
        cnt += (emit[t] ? 1u : 0u) | (valid && !is_col ? 1u << 8 : 0u) | (is_sub ? 1u << 16 : 0u);
      }
      // per character: its governing op (this lane's last start at or before it, else the last
      // one below the lane) -> literal ('*' pair, '-' bases) or letter required ('+' / '-')
      const int klast = sm1 ? kind[1] : kind[0];
      const uint32_t key_own = sm ? ((uint32_t)(4 * lane + 31 - __builtin_clz(sm)) << 2 | (uint32_t)(klast & 3)) + 1u : 0u;
      const uint32_t key_below = wave_shr1(dpp_max_incl(key_own));
      const int g_below = (int)((key_below - 1u) >> 2), ty_below = key_below ? (int)((key_below - 1u) & 3u) : -1;
      const int j0 = __builtin_ctz(sm | 16u), j1 = __builtin_ctz(sm1 | 16u);  // (4: none)
      uint32_t litm = 0;  // literal characters of this lane (bit j)
      uint32_t need_letter = 0;  // characters of this lane inside a '+' / '-' op (bit j)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int i = 4 * lane + j;
        const uint32_t in = (uint32_t)(i < lim) & ~(sm >> j) & 1u;
        // governing start: the lane's second start if before j, else its first, else the one below
        const int g = j1 < j ? 4 * lane + j1 : (j0 < j ? 4 * lane + j0 : g_below);
        const int ty = j1 < j ? kind[1] : (j0 < j ? kind[0] : ty_below);
        const uint32_t indel = (uint32_t)(ty == PW_OP_INS) | (uint32_t)(ty == PW_OP_DEL);
        const uint32_t lit = (uint32_t)(ty == PW_OP_INS) | ((uint32_t)(ty == PW_OP_SUB) & (uint32_t)(i - g - 1 < 2));
        need_letter |= (in & indel) << j;
        litm |= (in & lit) << j;
      }
      lbad = lbad | ((need_letter & ~msb_bits(m_alp)) != 0);
      // exclusive prefixes over the lanes (ops and characters are in lane order)
      const uint32_t nlit = (uint32_t)__popc(litm);
      cnt += nlit << 23;
      const int iq = wave_scan_incl(q_a), it = wave_scan_incl(t_a);
      const uint32_t ic = wave_scan_incl(cnt), il = ic >> 23;
      // bounds checks (pafreport.cpp:542-626 as restated by pw_pack_cs)
      const int q0 = qpos + iq - q_a;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const int qp = off + q0 + qb[t];
        const bool chk = kind[t] == PW_OP_MATCH || kind[t] == PW_OP_SUB || kind[t] == PW_OP_DEL;
        // (qp >= 0 and qn < 2^30: the 32-bit unsigned sum does not wrap)
        lbad = lbad | (chk & ((qp < 0) | ((uint32_t)qp + (uint32_t)qn[t] > (uint32_t)ql)));
      }
      if (__ballot(lbad) || !starts || (!last_win && last_start == 0)) {
        bad = true;  // (one op filling a window also lands here)
        return false;
      }
      // op words and literal bytes at their places (32-bit offsets from the record's bases)
      const uint32_t op_i = nops + ((ic - cnt) & 0xFFu);
      if (emit[0]) ops_r[op_i] = opw[0];
      if (emit[1]) ops_r[op_i + (emit[0] ? 1u : 0u)] = opw[1];
      const uint32_t u4 = up_bytes(c4);
      uint32_t lp = nlits + il - nlit;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if ((litm >> j) & 1u) lits_r[lp] = (uint8_t)(u4 >> (8 * j));
        lp += (litm >> j) & 1u;
      }
      // A/C/G/T literals: per byte of the upper-cased characters
      const uint32_t m_acgt = bytes_eq(u4, 'A') | bytes_eq(u4, 'C') | bytes_eq(u4, 'G') | bytes_eq(u4, 'T');
      acgt = acgt && (msb_bits(m_acgt) & litm) == litm;
      // ':' values up to 999,999,999: sums stay in range for queries below 2^31
      qpos += wave_last(iq);
      tpos += wave_last(it);
      const uint32_t ctot = wave_last(ic);
      nlits += ctot >> 23;
      nops += ctot & 0xFFu;
      const uint32_t wev = (ctot >> 8) & 0xFFu, nsub = (ctot >> 16) & 0x7Fu;
      nev += wev;
      bound += (uint64_t)kPkBoundIndel * (wev - nsub) + (uint64_t)kPkBoundSub * nsub;
      pos += (uint64_t)lim;
      __builtin_amdgcn_wave_barrier();
      return true;
    };
    if (L > 0 && window(w0, w1)) {
      while (pos < L) {  // (records longer than one window: their later windows load on the spot)
        uint32_t d0, d1;
        pk_words(text, base + pos, last, lane, d0, d1);
        if (!window(d0, d1)) break;
      }
    }
    const bool all_acgt = __ballot(!acgt) == 0;
    if (lane == 0) {
      pw_cs_rec r;
      r.q_total = qpos;
      r.t_total = tpos;
      r.n_ops = nops;
      r.n_lits = nlits;
      r.n_events_max = nev;
      r.flags = (bad ? PW_PACK_HOST : 0u) | (!bad && all_acgt ? PW_PACK_ACGT : 0u);
      r.text_bound = bound;
      out[ri] = r;
    }
  }
}

}  // namespace pw

extern "C" int pw_pack_cs_batch(const uint8_t* cs_text, const uint64_t* cs_off, const int32_t* offset,
                                const int32_t* qlen, uint32_t n, uint32_t* ops, uint8_t* lits, pw_cs_rec* out,
                                void* stream) {
  if (!cs_text || !cs_off || !offset || !qlen || !ops || !lits || !out) return PW_E_ARG;
  if (n == 0) return PW_OK;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  // persistent wavefronts, 64 workgroups per CU (~8 rounds of resident workgroups: fewer records
  // per wave, a shorter tail — round-4 sweep on cfg2's 100k records: 8 / 16 / 32 / 64 / 1000 per CU
  // 145.9 / 132.0 / 124.7-125.4 / 123.1-123.8 / 126.0 us)
  const uint32_t cap = (uint32_t)ncu * 64u;
  const uint32_t grid = (n + 3) / 4 < cap ? (n + 3) / 4 : cap;
  hipLaunchKernelGGL(pw::pack_cs_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, cs_text, cs_off, offset, qlen,
                     n, ops, lits, out);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}
