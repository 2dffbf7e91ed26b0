// pw_pack.hip — cs-string tokenising on gfx950.
//
// Reference: the cs loop of PAFAlignment::PAFAlignment (pafreport.cpp:536-626), restated on the
// host by pw_pack_cs (pw_host.cpp).  This kernel packs a whole batch of cs strings at once into
// the same op words and literal bytes, one 64-lane wavefront per record:
//   * the string is read in windows of 256 characters (4 per lane, staged in LDS);
//   * in a well-formed cs string every op starts at one of ':', '*', '+', '-' and no other
//     character is one of them (digits follow ':', letters the others), so the op starts of a
//     window are a ballot; an op runs to the next op start (the last one of a window that does
//     not reach the string end is carried into the next window);
//   * each lane decodes the (at most two) ops starting in its 4 characters; wave scans of the
//     query / target / literal advances and of the emitted-op counts place every op word and
//     literal byte and give the positions of the reference's bounds checks.
// Anything else — a character outside [0-9A-Za-z:*+-], a ':' run of more than 9 digits, a '*'
// not followed by exactly two characters, an empty indel or one holding a digit, '~' / '=', a
// bounds violation, one op longer than a window — flags the record PW_PACK_HOST: the caller packs it with pw_pack_cs, which produces
// the reference's exact error (such records are rare and end the report at their line anyway).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pwasm_amd.h"
#include "pw_wave.h"

namespace pw {

#define LDS __attribute__((address_space(3)))
constexpr int kPackWin = 256;  // characters per window (4 per lane)
constexpr uint64_t kPkBoundSub = 190, kPkBoundIndel = 140;  // = the host packer's text bounds

__device__ __forceinline__ bool pk_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ bool pk_alpha(uint32_t c) { return (c | 0x20u) - 'a' < 26u; }
__device__ __forceinline__ bool pk_opc(uint32_t c) { return c == ':' || c == '*' || c == '+' || c == '-'; }
__device__ __forceinline__ uint32_t pk_up(uint32_t c) { return c - 'a' < 26u ? c - 32u : c; }
__device__ __forceinline__ bool pk_acgt(uint32_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }

struct PkOp {
  uint32_t type;  // 0 ':', 1 '*', 2 '-' (INS), 3 '+' (DEL); PW_OP_* order
  int n;          // ':' value / indel length
  int s, e;       // content [s, e) in the window
  bool emit;      // an op word is written (':0' is dropped)
};

// A record's head, loaded one record ahead: its extent, offset / query length and the first
// window as aligned dwords (lane l: bytes [a0 + 4l, a0 + 4l + 4); lane 0 also the dword after the
// window, which an unaligned start needs).  Addresses past the record are clamped to its last
// dword: the caller's text is only readable up to the last record's end (+16 bytes).
struct PkHead {
  uint64_t base, L;
  int off, ql;
  uint32_t d0, d1;
};
__device__ __forceinline__ void pk_head(const uint8_t* text, const uint64_t* cs_off, const int32_t* offset,
                                        const int32_t* qlen, uint32_t ri, int lane, PkHead& h) {
  h.base = cs_off[ri];
  h.L = cs_off[ri + 1] - h.base;
  h.off = offset[ri];
  h.ql = qlen[ri];
  const uint64_t a0 = h.base & ~3ull, last = h.L ? (h.base + h.L - 1) & ~3ull : a0;
  const uint64_t x0 = a0 + 4ull * (uint64_t)lane, x1 = a0 + 256ull;
  h.d0 = *reinterpret_cast<const uint32_t*>(text + (x0 < last ? x0 : last));
  h.d1 = *reinterpret_cast<const uint32_t*>(text + (x1 < last ? x1 : last));
}
// stage window bytes [pos, pos + 256) of the record into w (from the dwords of pk_head when pos
// is 0, else loaded here); returns the window's shift inside the staging buffer
__device__ __forceinline__ int pk_stage(const uint8_t* text, const PkHead& h, uint64_t pos, int lane, LDS uint8_t* wr,
                                        bool first) {
  const uint64_t st = h.base + pos, a0 = st & ~3ull, last = (h.base + h.L - 1) & ~3ull;
  uint32_t d0 = h.d0, d1 = h.d1;
  if (!first) {
    const uint64_t x0 = a0 + 4ull * (uint64_t)lane, x1 = a0 + 256ull;
    d0 = *reinterpret_cast<const uint32_t*>(text + (x0 < last ? x0 : last));
    d1 = *reinterpret_cast<const uint32_t*>(text + (x1 < last ? x1 : last));
  }
  *reinterpret_cast<LDS uint32_t*>(wr + 4 * lane) = d0;
  if (lane == 0) *reinterpret_cast<LDS uint32_t*>(wr + 256) = d1;
  return (int)(st & 3ull);
}

// Persistent wavefronts: wave g takes records g, g + NW, ...; the next record's head and first
// window are loaded before this one is decoded, so their latency hides behind the decode (the
// per-record work is a short dependent chain: load -> classify -> scans -> stores).
__global__ __launch_bounds__(256) void pack_cs_kernel(const uint8_t* text, const uint64_t* cs_off, const int32_t* offset,
                                                      const int32_t* qlen, uint32_t n, uint32_t* ops, uint8_t* lits,
                                                      pw_cs_rec* out) {
  __shared__ uint8_t win[4][kPackWin + 8];   // staged window (shifted by the start's alignment)
  __shared__ uint8_t wz[4][kPackWin + 8];    // the window from its first character, zeros past its end
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform: scalar loop)
  // (address-space-3 pointers: through a generic one every window read would be a flat load,
  // which also waits for the wave's outstanding global stores)
  LDS uint8_t* wr = (LDS uint8_t*)win[wv];
  LDS uint8_t* w = (LDS uint8_t*)wz[wv];
  const uint32_t nw = gridDim.x * 4;
  uint32_t ri = blockIdx.x * 4 + (uint32_t)wv;
  if (ri >= n) return;
  PkHead nxt;
  pk_head(text, cs_off, offset, qlen, ri, lane, nxt);
  for (; ri < n; ri += nw) {
    const PkHead cur = nxt;
    if (ri + nw < n) pk_head(text, cs_off, offset, qlen, ri + nw, lane, nxt);
    const uint64_t base = cur.base, L = cur.L;
    const int off = cur.off, ql = cur.ql;
    int qpos = 0, tpos = 0;
    uint32_t nops = 0, nlits = 0, nev = 0;
    uint64_t bound = 0;
    bool bad = false, acgt = true;
    uint64_t pos = 0;
    while (pos < L && !bad) {
      const int wl = (int)(L - pos < (uint64_t)kPackWin ? L - pos : (uint64_t)kPackWin);
      const bool last_win = pos + (uint64_t)wl == L;
      // stage the window (aligned dword loads, then this lane's 4 characters re-read at the
      // window's shift; zeros past its end)
      const int sh = pk_stage(text, cur, pos, lane, wr, pos == 0);
      __builtin_amdgcn_wave_barrier();
      uint32_t c4 = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int i = 4 * lane + j;
        const uint32_t c = i < wl ? (uint32_t)wr[sh + i] : 0u;
        c4 |= c << (8 * j);
      }
      __builtin_amdgcn_wave_barrier();
      *reinterpret_cast<LDS uint32_t*>(w + 4 * lane) = c4;
      if (lane == 0) *reinterpret_cast<LDS uint32_t*>(w + kPackWin) = 0u;
      __builtin_amdgcn_wave_barrier();
      // character classes; op starts
      bool lbad = false;
      uint32_t smask = 0;  // op starts among this lane's 4 characters (bit j)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int i = 4 * lane + j;
        const uint32_t c = (c4 >> (8 * j)) & 0xFFu;
        if (i < wl) {
          if (pk_opc(c)) smask |= 1u << j;
          else if (!pk_digit(c) && !pk_alpha(c)) lbad = true;
        }
      }
      // every window starts at an op start (the string's first character, or an op carried over)
      if (!((uint32_t)__shfl((int)smask, 0, 64) & 1u)) {
        bad = true;
        break;
      }
      // the window's last op start (it runs past the window unless the string ends here)
      const uint64_t any = __ballot(smask != 0);
      const int ll = 63 - __builtin_clzll(any);
      const uint32_t lmask = (uint32_t)__shfl((int)smask, ll, 64);
      const int last_start = 4 * ll + (31 - __builtin_clz(lmask));
      const int lim = last_win ? wl : last_start;  // ops starting before lim are decoded now
      if (!last_win && last_start == 0) {
        bad = true;  // one op fills the window
        break;
      }
      // decode this lane's ops (one per op start among its 4 characters, in registers: j is a
      // constant after unrolling).  An op ends at the next op start: the next set bit of this
      // lane's starts, else the first start of the next lane that has one, else the window end.
      const uint64_t nxt_l = lane == 63 ? 0ull : any & ~((2ull << lane) - 1ull);  // op-start lanes above
      const int nl = nxt_l ? __builtin_ctzll(nxt_l) : 64;
      const uint32_t nl_mask = (uint32_t)__shfl((int)smask, nl < 64 ? nl : 0, 64);
      const int next_start = nl < 64 ? 4 * nl + __builtin_ctz(nl_mask) : wl;
      PkOp op[4];
      bool has[4];
      int la_q = 0, la_t = 0, la_l = 0, la_e = 0, la_v = 0;
      uint64_t la_b = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int s = 4 * lane + j;
        has[j] = ((smask >> j) & 1u) && s < lim;
        PkOp& o = op[j];
        o.type = PW_OP_MATCH;
        o.n = 0;
        o.s = s + 1;
        o.emit = false;
        const uint32_t later = (smask >> (j + 1)) << (j + 1);  // this lane's starts after j
        const int e = later ? 4 * lane + __builtin_ctz(later) : next_start;
        o.e = e;
        if (has[j]) {
          const uint32_t c = (c4 >> (8 * j)) & 0xFFu;
          const int len = e - s - 1;
          o.n = len;
          o.emit = true;
          if (c == ':') {
            o.type = PW_OP_MATCH;
            if (len < 1 || len > 9) lbad = true;
            int v = 0;
            for (int k = s + 1; k < e && k < s + 10; k++) {
              const uint32_t d = w[k];
              if (!pk_digit(d)) lbad = true;
              v = v * 10 + (int)(d - '0');
            }
            o.n = v;
            o.emit = v > 0;
            la_q += v;
            la_t += v;
          } else if (c == '*') {
            o.type = PW_OP_SUB;
            if (len != 2) lbad = true;  // (any two characters, as the host packer takes them)
            o.n = 1;
            la_q += 1;
            la_t += 1;
            la_l += 2;
            la_v += 1;
            la_b += kPkBoundSub;
          } else {
            o.type = c == '-' ? PW_OP_INS : PW_OP_DEL;
            if (len < 1) lbad = true;
            for (int k = s + 1; k < e; k++)  // (the host's is_alpha run ends at a digit: UNHANDLED)
              if (!pk_alpha(w[k])) lbad = true;
            if (c == '-') {
              la_t += len;
              la_l += len;
            } else {
              la_q += len;
            }
            la_v += 1;
            la_b += kPkBoundIndel;
          }
          la_e += o.emit ? 1 : 0;
        }
      }
      if (__ballot(lbad)) {
        bad = true;
        break;
      }
      // exclusive prefixes over the lanes (ops are in lane order)
      const int iq = wave_scan_incl(la_q), it = wave_scan_incl(la_t), il = wave_scan_incl(la_l),
                ie = wave_scan_incl(la_e);
      int q = qpos + iq - la_q;
      uint32_t lp = nlits + (uint32_t)(il - la_l), op_i = nops + (uint32_t)(ie - la_e);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!has[k]) continue;
        const PkOp& o = op[k];
        const int qp = off + q;
        if (o.type == PW_OP_MATCH) {
          if (qp < 0 || (int64_t)qp + o.n > ql) lbad = true;
          q += o.n;
        } else if (o.type == PW_OP_SUB) {
          if (qp < 0 || qp > ql) lbad = true;
          const uint32_t a = pk_up(w[o.s]), b = pk_up(w[o.s + 1]);
          lits[base + lp] = (uint8_t)a;
          lits[base + lp + 1] = (uint8_t)b;
          acgt = acgt && pk_acgt(a) && pk_acgt(b);
          lp += 2;
          q += 1;
        } else if (o.type == PW_OP_INS) {
          for (int x = o.s; x < o.e; x++) {
            const uint32_t a = pk_up(w[x]);
            lits[base + lp++] = (uint8_t)a;
            acgt = acgt && pk_acgt(a);
          }
        } else {
          if (qp < 0 || (int64_t)qp + o.n > ql) lbad = true;
          q += o.n;
        }
        if (o.emit) ops[base + op_i++] = PW_OP(o.type, (uint32_t)o.n);
      }
      if (__ballot(lbad)) {
        bad = true;
        break;
      }
      // ':' values up to 999,999,999: sums stay in range for queries below 2^31
      qpos += wave_last(iq);
      tpos += wave_last(it);
      nlits += (uint32_t)wave_last(il);
      nops += (uint32_t)wave_last(ie);
      {
        uint32_t v = (uint32_t)la_v;
        uint64_t bb = la_b;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          v += (uint32_t)__shfl_xor((int)v, d, 64);
          bb += (uint64_t)__shfl_xor((long long)bb, d, 64);
        }
        nev += v;
        bound += bb;
      }
      pos += (uint64_t)lim;
      __builtin_amdgcn_wave_barrier();
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
  // persistent wavefronts, two rounds of 8 resident workgroups per CU
  const uint32_t cap = (uint32_t)ncu * 16u;
  const uint32_t grid = (n + 3) / 4 < cap ? (n + 3) / 4 : cap;
  hipLaunchKernelGGL(pw::pack_cs_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, cs_text, cs_off, offset, qlen,
                     n, ops, lits, out);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}
