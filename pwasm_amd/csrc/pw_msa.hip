// pw_msa.hip — GapAssem column consensus on gfx950.
//
// Reference (gpertea/pwasm GapAssem):
//   GASeq::toMSA            GapAssem.cpp:551-591   row -> columns (gap runs + bases, clipping)
//   GAlnColumn::addGap/Nuc  GapAssem.h:295-337     6 counters A,C,G,T,N,- (+ layers)
//   GAlnColumn::bestChar    GapAssem.cpp:1048-1069 stable qsort + N/- tie rule
//   GSeqAlign::buildMSA     GapAssem.cpp:1088-1106
// The reference scatters row by row (one NucOri allocation per base).  Here ofs and seq are each
// read once per pass from HBM:
//   K0 slot_rows:      row of every chunk slot (no per-chunk binary search later)
//   K1 row_chunk_sums: per 256-base chunk of a row (16 lanes, 16 bases each), sum of
//                      (1 + max(ofs,0)) and the chunk's gap runs in layout order as
//                      (column offset in the chunk, length) — 32 B per chunk instead of 512 B of ofs
//   K2 row_prefix:     per row, exclusive scan of the chunk sums -> checkpoints (layout column at
//                      which each chunk's first gap run starts), row end column, bounds check, the
//                      counted extent, mincol / maxcol, and for every 2048-column tile that starts
//                      inside the row its first chunk and first base (the tile start table)
//   K3 tile_counts:    one 8-wave workgroup per 2048-column tile; lane l of a wave owns the tile's
//                      columns [32l, 32l + 32) for every row the wave takes.  Per row: a 2 KB window
//                      of the row's bases is staged in LDS (loaded a row ahead), the tile's gap-column
//                      bitmap is built from the runs of the <= 9 chunks that reach the tile, and each
//                      lane expands its bases into its columns 4 at a time (the bitmap's popcounts
//                      give the source offset, a v_perm inserts the gap characters) and adds them to
//                      32 packed 5-bit register counters — no scatter, no atomic per base.
//                      (pw_msa_count stops here: with rows sharded over GPUs the partial counts are
//                      summed by an all-reduce before the call)
//   K4 call_columns:   bestChar of every column (pw_msa_call) and the first zero-coverage column
//                      in [mincol, maxcol] (ErrZeroCov, :1121-1131)
// Column-closed form of bestChar: max count wins, ties resolved A<C<G<T; a tie between only N
// and '-' gives '-' (glibc qsort of 6 elements is a stable merge sort).
//
// refineMSA's consensus loop (GapAssem.cpp:1143-1162) and, with MSAColumns::removeConsGaps,
// its row edits (removeColumn :755-779 -> GASeq::removeBase :122-131, then removeClipGaps
// :522-549) in closed form (pw_msa_refine).  With G(c) = consensus-gap columns in
// [mincol, c] (gap columns are removed in increasing order, each at column - cols_removed, so
// the k-th removal hits exactly the layout column it was in before any removal), a row with
// first column O and base columns col(i) ends with
//   offset' = offset - G(O)                           (removeColumn's "offset--" branch)
//   ofs'[0] = ofs[0] - (G(col(0)) - G(O))
//   ofs'[i] = ofs[i] - (G(col(i)) - G(col(i-1)))      (removeBase of the first base at or
//                                                      after the removed column)
// for ofs >= 0 (the walk of :766-771 sees raw ofs values; negative input gaps are refused).
//   K6 gap_tiles / K7 gap_scan: G per column (tile counts + in-tile scan) and the consensus
//                      string ('-' -> '*', or gap columns dropped)
//   K8 row_edit:       ofs' of every base (one wave per chunk, columns from the checkpoints)
//   K9 row_finish:     offset', numgaps', then removeClipGaps on ofs' (i <= clipL and
//                      i >= seqlen - clipR) unless keep_clip_gaps (refineClipping first, host)
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include <type_traits>

#include "pwasm_amd.h"
#include "pw_wave.h"

namespace pw {

#define LDS __attribute__((address_space(3)))
constexpr int kChunk = 256;   // bases per checkpoint chunk
constexpr int kTileW = 2048;  // columns per refine tile
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

// GAlnColumn::addNuc / addGap bin (GapAssem.h:295-337): toupper(c) A,C,G,T -> 0..3, '-' / '*' ->
// 5 (gap), anything else -> 4 (N).  Branch-free: a switch compiles to a divergent compare tree.
__device__ __forceinline__ int bin_of(uint32_t c) {
  const uint32_t u = c & 0xDFu;  // clears bit 5 only: u == 'A' iff c is 'A' or 'a' (same for C, G, T)
  int b = (c == '-' || c == '*') ? 5 : 4;
  b = u == 'A' ? 0 : b;
  b = u == 'C' ? 1 : b;
  b = u == 'G' ? 2 : b;
  b = u == 'T' ? 3 : b;
  return b;
}

// a value the compiler must treat as per-lane (a load through it stays a vector load kept in
// VGPRs instead of a scalar load whose lgkmcnt wait would also hold every LDS wait after it)
__device__ __forceinline__ int64_t vary(int64_t v) {
  asm volatile("" : "+v"(v));
  return v;
}

// (orders a wave's LDS stores before its later LDS reads by other lanes)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// K0: the row of every slot (slot_row) and K1's chunk descriptor (sdesc: the chunk's first ofs
// element | its base count << 48 | 16-byte aligned << 63), gridDim.y workgroups per row (a few
// long rows still fill the chip), coalesced
constexpr uint64_t kDescVec = 1ull << 63;
__global__ __launch_bounds__(256) void slot_rows(const pw_msa_args A, int32_t* slot_row, uint64_t* sdesc) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 4)  // minmax sentinels (no host copy on the stream)
    A.minmax[threadIdx.x] = threadIdx.x == 1 ? -1 : INT_MAX;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int64_t b = A.slot_base[r], e = A.slot_base[r + 1];
    const uint64_t roff = A.row_off[r];
    const int len = A.row_len[r];
    for (int64_t k = b + (int64_t)blockIdx.y * 256 + threadIdx.x; k < e; k += (int64_t)gridDim.y * 256) {
      slot_row[k] = (int32_t)r;
      const int i0 = (int)(k - b) * kChunk;
      const uint64_t nv = (uint64_t)min(max(len - i0, 0), kChunk);
      sdesc[k] = ((roff + (uint64_t)i0) & ((1ull << 48) - 1)) | nv << 48 | ((roff & 7) == 0 ? kDescVec : 0ull);
    }
  }
}

// K1: per 256-base chunk, sum of (1 + max(ofs, 0)) and its gap runs.  A run is the gap before a
// base with ofs > 0 (~1 % of bases in an assembly layout): entry = (column offset of the run in
// the chunk, from the chunk's checkpoint) << 6 | length, 16 bits, in layout order, at most kRunCap
// per chunk, 0 = unused; kRunOverflow in entry 0 when a chunk has more runs, a run longer than 63
// or more than kRunCols columns
// (K2 / K3 then read that chunk's ofs).  A wavefront takes 4 consecutive slots at a time, 16 lanes
// per slot, 16 bases per lane (two 16-byte loads when the row starts 8-base aligned); the loads of
// the next three groups are in flight while a group is reduced.
constexpr int kRunCap = 16;  // (one per lane of the chunk's 16; > 16 runs in 256 bases: ~1e-7 at 1 % gaps)
constexpr uint32_t kRunOverflow = 0xFFFFu;
constexpr int kRunCols = 1000;  // (so no real entry is kRunOverflow)
// K1's inputs per lane: the slot's descriptor four groups ahead, its 16 gaps three groups ahead
struct SumPre {
  v4u q0, q1;
  uint64_t off;  // first ofs element of this lane's 16
  int nv;        // bases of this lane (0..16)
  int tv;        // bases of the chunk
  bool vec;
};
// (the descriptor load is unconditional and its value is not touched until sums_load: a select
// next to the load would make hipcc wait for it there)
// (chunk and group indices are 32-bit: pw_msa_count takes fewer than 2^27 slots)
__device__ __forceinline__ uint64_t sums_desc(const pw_msa_args& A, const uint64_t* sdesc, uint32_t g, int lane) {
  const uint32_t c = g * 4u + (uint32_t)(lane >> 4);
  return sdesc[c < A.n_slots ? c : A.n_slots - 1];
}
__device__ __forceinline__ void sums_load(const pw_msa_args& A, uint64_t d, uint32_t g, int lane, SumPre& p) {
  const int sub = lane & 15;
  const uint32_t c = g * 4u + (uint32_t)(lane >> 4);
  if (c >= A.n_slots) d &= (1ull << 48) - 1;  // past the end: no bases
  p.off = (d & ((1ull << 48) - 1)) + 16ull * (uint64_t)sub;
  p.tv = (int)((d >> 48) & 0x1FFu);
  p.nv = min(max(p.tv - 16 * sub, 0), 16);
  p.vec = (d & kDescVec) && p.nv == 16;
  // (unconditional loads: a row tail or unaligned row reads the scratch instead and takes the
  // element path when consumed)
  const v4u* src = p.vec ? reinterpret_cast<const v4u*>(A.ofs + p.off) : reinterpret_cast<const v4u*>(A.scratch);
  p.q0 = src[0];
  p.q1 = src[1];
}
__device__ __forceinline__ uint32_t row16_scan_incl(uint32_t v) {  // inclusive prefix within each 16-lane row
  v += dpp_or_zero<0x111>(v);
  v += dpp_or_zero<0x112>(v);
  v += dpp_or_zero<0x114>(v);
  v += dpp_or_zero<0x118>(v);
  return v;
}
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// one group of 4 chunks: the 16 gaps of this lane (two per dword, packed int16 math: per dword a
// max, a dot2 into the sum, a min into the nonzero mask, a max into the "long gap" check).  The
// chunk's run entries go to the wave's LDS strip (lr: 16 entries of this lane's chunk); returns the
// chunk sum (valid in every lane of the chunk)
__device__ __forceinline__ int sums_group(const pw_msa_args& A, const SumPre& cur, int lane, LDS uint16_t* lr) {
  const int sub = lane & 15;
  uint32_t w[8];  // 16 int16 gaps, two per dword
  if (cur.vec) {
    w[0] = cur.q0.x, w[1] = cur.q0.y, w[2] = cur.q0.z, w[3] = cur.q0.w;
    w[4] = cur.q1.x, w[5] = cur.q1.y, w[6] = cur.q1.z, w[7] = cur.q1.w;
  } else {  // row tail / unaligned row
#pragma unroll
    for (int d = 0; d < 8; d++) w[d] = 0;
    for (int i = 0; i < cur.nv; i++) w[i >> 1] |= (uint32_t)(uint16_t)A.ofs[cur.off + i] << (16 * (i & 1));
  }
  const i16x2 zero = {0, 0};
  const u16x2 one = {1, 1};
  uint32_t s = 0, pmw = 0;
  i16x2 bg = zero;
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const i16x2 v = __builtin_bit_cast(i16x2, w[d]);
    const u16x2 m = __builtin_bit_cast(u16x2, __builtin_elementwise_max(v, zero));
    s = __builtin_amdgcn_udot2(m, one, s, false);
    // gap > 0 per half: bit 15 of m + 0x7FFF (m <= 0x7FFF: no carry into the other half) ->
    // element 2d: bit d, 2d + 1: bit 16 + d (integer SWAR: a packed min here compiles to
    // per-half compares and selects)
    const uint32_t t = __builtin_bit_cast(uint32_t, m) + 0x7FFF7FFFu;
    pmw |= (t >> (15 - d)) & (0x00010001u << d);
    bg = __builtin_elementwise_max(bg, v);
  }
  // interleave: bit t of pm = element t has a gap
  uint32_t x = pmw;
  x = (x | x << 4) & 0x0F0F0F0Fu;
  x = (x | x << 2) & 0x33333333u;
  x = (x | x << 1) & 0x55555555u;
  uint32_t pm = (x & 0xFFFFu) | (x >> 15);
  const int big = max((int)bg.x, (int)bg.y) > 63 ? 1 : 0;  // a gap longer than a 6-bit run length
  const int n = __popc(pm);
  const uint32_t is = row16_scan_incl(s), in = row16_scan_incl((uint32_t)n | (uint32_t)big << 8);
  const int ts = __shfl((int)is, lane | 15, 64), tnb = __shfl((int)in, lane | 15, 64);
  const int tn = tnb & 0xFF, tv = cur.tv;
  const bool ovf = tn > kRunCap || (tnb >> 8) || tv + ts > kRunCols;
  // entries [0, tn) from the lanes with runs, [tn, 16) zero, or kRunOverflow in entry 0 (the rest
  // is then never read)
  if (sub >= tn && !(ovf && sub == 0)) lr[sub] = 0;
  if (ovf) {
    if (sub == 0) lr[0] = (uint16_t)kRunOverflow;
  } else {
    int slot = (int)(in & 0xFFu) - n;
    int col = 16 * sub + ((int)is - (int)s);  // column offset of this lane's first base's gap run
    int prev = 0;                             // base index (in the lane) the column offset refers to
    while (pm) {                              // (~0.15 runs per lane)
      const int t = __builtin_ctz(pm);
      pm &= pm - 1;
      const int d = t >> 1;
      const uint32_t dw = (d & 4) ? ((d & 2) ? ((d & 1) ? w[7] : w[6]) : ((d & 1) ? w[5] : w[4]))
                                  : ((d & 2) ? ((d & 1) ? w[3] : w[2]) : ((d & 1) ? w[1] : w[0]));
      const uint32_t gg = (t & 1) ? dw >> 16 : dw & 0xFFFFu;
      col += t - prev;
      prev = t;
      lr[slot++] = (uint16_t)((uint32_t)col << 6 | gg);
      col += (int)gg;
    }
  }
  return tv + ts;
}
__global__ __launch_bounds__(256) void row_chunk_sums(const pw_msa_args A, int32_t* chunk_sum, const uint64_t* sdesc,
                                                      uint16_t* runs) {
  __shared__ uint32_t lruns[4][4][kRunCap / 2];  // [wave][chunk of the group][entry pairs]
  const int lane = threadIdx.x & 63, sub = lane & 15, wv = threadIdx.x >> 6;
  LDS uint32_t* lr32 = (LDS uint32_t*)&lruns[wv][lane >> 4][0];
  const uint32_t ng = (uint32_t)((A.n_slots + 3) / 4);
  const uint32_t nw = gridDim.x * 4u;
  uint32_t g = blockIdx.x * 4u + (uint32_t)wv;
  if (g >= ng) return;
  // (pw_msa_count checks that 32 * n_slots fits a 32-bit offset)
  const __amdgpu_buffer_rsrc_t rs_runs =
      __builtin_amdgcn_make_buffer_rsrc(runs, (short)0, (int)((uint32_t)A.n_slots * (uint32_t)(2 * kRunCap)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_cs = __builtin_amdgcn_make_buffer_rsrc(chunk_sum, (short)0, (int)((uint32_t)A.n_slots * 4u), 0x00020000);
  constexpr uint32_t kOut = 0xFFFFFFF0u;
  // three groups' loads in flight (p0, p1, p2: unrolled by three, so no register copy waits for a
  // load issued one group earlier), the descriptor of the group after them.  vmcnt counts stores
  // too: a step issues its loads first and then a fixed two stores (chunk sum, run entries from the
  // LDS strip), so a wait for a load never waits for a younger load behind a variable number of
  // stores.
  SumPre p0, p1;
  sums_load(A, sums_desc(A, sdesc, g, lane), g, lane, p0);
  sums_load(A, sums_desc(A, sdesc, g + nw, lane), g + nw, lane, p1);
  uint64_t dn = sums_desc(A, sdesc, g + 2 * nw, lane);
  auto step = [&](SumPre& p) {
    asm volatile("" : "+v"(p.q0), "+v"(p.q1));
    const int cs = sums_group(A, p, lane, (LDS uint16_t*)lr32);
    const uint64_t dnn = sums_desc(A, sdesc, g + 3 * nw, lane);
    asm volatile("" : "+v"(dn)::"memory");
    sums_load(A, dn, g + 2 * nw, lane, p);
    dn = dnn;
    wave_sync();
    const uint32_t rw = lr32[sub & 7];
    const uint32_t c = g * 4u + (uint32_t)(lane >> 4);
    __builtin_amdgcn_raw_buffer_store_b32(rw, rs_runs, sub < 8 ? c * (uint32_t)(2 * kRunCap) + 4u * (uint32_t)sub : kOut, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)cs, rs_cs, sub == 0 ? 4u * c : kOut, 0, 0);
    wave_sync();
    g += nw;
  };
  const uint32_t n_mine = (ng - g + nw - 1) / nw;
  for (uint32_t k = 2; k <= n_mine; k += 2) {
    step(p0);
    step(p1);
  }
  if (n_mine & 1) step(p0);
}

// K2: one 1024-thread workgroup per row: chunk checkpoints (column where chunk k's first gap run
// starts) = col0 + exclusive scan of the chunk sums, row extent, bounds check
// (MSAColumns::operator[], GapAssem.h:366-370).  Thread t owns a contiguous run of chunks.
// K3's row record rinfo[8r..8r+7] = {ext_lo, ext_hi, first column, end column + 1, length,
// chunks | (no tile table) << 31, first slot (2 words)}, where [ext_lo, ext_hi] = [first column of
// the gap run before base lo, column of base hi - 1] is the counted extent of the unclipped bases
// [lo, hi) (empty: ext_lo > ext_hi), and mincol / maxcol (minmax[0] / [1]: GSeqAlign's
// minoffset/length bookkeeping over the bases toMSA counts): waves 0 / 1 scan the chunk holding
// lo / hi - 1.  The tile start table: for every tile t whose first column c0 lies in the row
// (first column < c0 < end column), tstart[first slot + t - floor(first column / kCntW)] =
// {chunk holding c0, first base at or after c0} (the row has room for it in its slots unless its
// gaps inflate it more than 8-fold: then the row is flagged and K3 searches).
constexpr int kCntW = 2048;  // K3 tile width
// A chunk's runs, all kRunCap entries loaded at once (one round trip, no dependent loads)
struct Runs {
  uint32_t v[kRunCap];
};
__device__ __forceinline__ Runs load_runs(const uint16_t* rl) {  // (rl 16-byte aligned: two 16-byte loads)
  Runs R;
  const v4u* p = reinterpret_cast<const v4u*>(rl);
#pragma unroll
  for (int e = 0; e < kRunCap / 8; e++) {
    const v4u v = p[e];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; q++) R.v[8 * e + 2 * q] = d[q] & 0xFFFFu, R.v[8 * e + 2 * q + 1] = d[q] >> 16;
  }
  return R;
}
// first base of chunk k (row-relative index) whose column is >= column x of the chunk (x from its
// checkpoint, 0 <= x < its column span): from the runs, or (overflowed chunk) by walking its ofs
__device__ __forceinline__ int first_base_at(const pw_msa_args& A, const Runs& R, uint64_t roff, int k, int len, int x) {
  if (R.v[0] != kRunOverflow) {
    int G = 0, ib = -1;
#pragma unroll
    for (int e = 0; e < kRunCap; e++) {
      const uint32_t v = R.v[e];
      const int co = (int)(v >> 6), gg = (int)(v & 63u);
      if (ib < 0 && v != 0 && x >= co) {
        if (x < co + gg) ib = co - G;  // inside the run: the base after it
        else G += gg;
      } else if (ib < 0) {
        ib = x - G;  // (a run at or after x, or none left: x is a base column)
      }
    }
    return k * kChunk + (ib < 0 ? x - G : ib);
  }
  int col = 0;
  const int i1 = min(k * kChunk + kChunk, len);
#pragma unroll 1
  for (int i8 = k * kChunk; i8 < i1; i8 += 16) {  // (16 loads issued together per step)
    int16_t g[16];
#pragma unroll
    for (int j = 0; j < 16; j++) g[j] = A.ofs[roff + (uint64_t)min(i8 + j, i1 - 1)];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (i8 + j >= i1) break;
      col += max((int)g[j], 0);
      if (col >= x) return i8 + j;
      col++;
    }
  }
  return i1;
}
// column offset (from the chunk's checkpoint) of base i of chunk k (i chunk-relative): its gap
// run's first column (run_start) or the base's own column
__device__ __forceinline__ int base_col(const pw_msa_args& A, const Runs& R, uint64_t roff, int k, int i, bool run_start) {
  if (R.v[0] != kRunOverflow) {
    int G = 0;
    bool done = false;
#pragma unroll
    for (int e = 0; e < kRunCap; e++) {
      const uint32_t v = R.v[e];
      const int co = (int)(v >> 6), gg = (int)(v & 63u);
      const int idx = co - G;  // the base this run precedes
      if (!done && v != 0 && (run_start ? idx < i : idx <= i)) G += gg;
      else done = true;
    }
    return i + G;
  }
  int col = 0;
  const uint64_t o = roff + (uint64_t)k * kChunk;
#pragma unroll 1
  for (int b8 = 0; b8 <= i; b8 += 16) {  // (16 loads issued together per step; reads stay inside the chunk)
    int16_t g[16];
#pragma unroll
    for (int j = 0; j < 16; j++) g[j] = A.ofs[o + (uint64_t)min(b8 + j, i)];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (b8 + j < i) col += 1 + max((int)g[j], 0);
      else if (b8 + j == i && !run_start) col += max((int)g[j], 0);
    }
  }
  return col;
}
constexpr int kRowInfo = 8;  // int32 words per row record
constexpr uint32_t kNoTable = 0x80000000u;
constexpr int kPfxUnroll = 4;  // chunk sums a thread keeps in registers (rows of <= 4096 chunks)
__global__ __launch_bounds__(1024) void row_prefix(const pw_msa_args A, const int32_t* chunk_sum, int32_t* ckpt,
                                                   int32_t* rinfo, const uint16_t* runs, int32_t* tstart) {
  __shared__ int wsum[16];
  __shared__ uint32_t notab;
  const int64_t* chunk_base = A.slot_base;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1];
    const int64_t n = e - b, per = (n + 1023) / 1024;
    const int64_t k0 = b + (int64_t)t * per, k1 = k0 + per < e ? k0 + per : e;
    const int len = A.row_len[r];
    const int lo = max(A.clip_l[r], 0), hi = min(len - A.clip_r[r], len);  // counted bases [lo, hi)
    const int64_t klo = b + lo / kChunk, khi = b + (hi - 1) / kChunk;
    const uint64_t roff = A.row_off[r];
    const int rs = A.col0[r];
    const int t_first = rs >> 11;  // floor(rs / kCntW)
    if (t == 0) notab = 0;
    // the thread's chunk sums: the first kPfxUnroll kept in registers (loads issued together)
    int cs[kPfxUnroll];
#pragma unroll
    for (int u = 0; u < kPfxUnroll; u++) cs[u] = k0 + u < k1 ? chunk_sum[k0 + u] : 0;
    int mine = 0;
#pragma unroll
    for (int u = 0; u < kPfxUnroll; u++) mine += cs[u];
    for (int64_t k = k0 + kPfxUnroll; k < k1; k++) mine += chunk_sum[k];
    const int incl = wave_scan_incl(mine);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = rs, end = rs;
#pragma unroll
    for (int w = 0; w < 16; w++) {
      const int v = wsum[w];
      base += w < wv ? v : 0;
      end += v;
    }
    int run = base + incl - mine;
    int32_t* ri = rinfo + (int64_t)kRowInfo * r;
    auto chunk = [&](int64_t k, int c) {
      ckpt[k] = run;
      const int kk = (int)(k - b);
      // tiles whose first column lies in this chunk's columns [run, run + c) and after rs, and the
      // counted extent's ends; both need the chunk's runs
      const int lo_c = max(run == rs ? run + 1 : run, 0), hi_c = run + c - 1;
      const bool tiles = c > 0 && lo_c <= hi_c && ((lo_c + kCntW - 1) >> 11) <= (hi_c >> 11);
      const bool ends = hi > lo && (k == klo || k == khi);
      if (tiles || ends) {
        const Runs R = load_runs(runs + (uint64_t)k * kRunCap);
        if (tiles)
          for (int tt = (lo_c + kCntW - 1) >> 11; tt <= (hi_c >> 11); tt++) {
            const int64_t idx = (int64_t)tt - t_first;
            if (idx > n - 1) {
              atomicOr(&notab, 1u);
              break;
            }
            tstart[2 * (b + idx)] = kk;
            tstart[2 * (b + idx) + 1] = first_base_at(A, R, roff, kk, len, tt * kCntW - run);
          }
        if (ends && k == klo) {  // gap-run start of base lo
          const int x = run + base_col(A, R, roff, kk, lo - kk * kChunk, true);
          ri[0] = x;
          if (A.clip_l[r] >= 0) atomicMin(&A.minmax[0], x);
        }
        if (ends && k == khi) {  // column of base hi - 1
          const int x = run + base_col(A, R, roff, kk, hi - 1 - kk * kChunk, false);
          ri[1] = x;
          if (A.clip_r[r] >= 0) atomicMax(&A.minmax[1], x);
        }
      }
      run += c;
    };
#pragma unroll
    for (int u = 0; u < kPfxUnroll; u++)
      if (k0 + u < k1) chunk(k0 + u, cs[u]);
    for (int64_t k = k0 + kPfxUnroll; k < k1; k++) chunk(k, chunk_sum[k]);
    if (t == 1023 && len > 0 && (rs < 0 || end - 1 >= A.n_cols)) atomicMin(&A.minmax[2], (int)r);  // (end - 1: last column)
    if (t == 0 && hi <= lo) {  // empty counted extent
      ri[0] = 1;
      ri[1] = 0;
    }
    __syncthreads();
    if (t == 0) {
      ri[2] = rs;
      ri[3] = end;
      ri[4] = len;
      ri[5] = (int)((uint32_t)(e - 1 - b) | (notab ? kNoTable : 0u));
      ri[6] = (int)(uint32_t)(uint64_t)b;
      ri[7] = (int)(uint32_t)((uint64_t)b >> 32);
    }
    __syncthreads();  // (wsum / notab are reused by the next row)
  }
}

// K3: counts for one 2048-column tile, no atomic per base.  The 8 waves share the rows
// overlapping the tile (row r -> wave r % 8).  Lane l owns the tile's columns [32l, 32l + 32).
// Per row, three dependent loads are pipelined over the wave's rows: the row's slot range, first
// column and offset (3 rows ahead); its record and tile-start entry (2 rows ahead); then its
// batch (a row ahead): the checkpoints and runs of the <= 9 chunks that reach the tile (a chunk
// spans >= 256 columns) and a 2176-byte window of its bases from the tile's first base (buffer
// loads: past the row's padded end they read 0).  For the row itself:
//   * the gap-column bitmap of the tile (one dword per lane) starts as the columns outside the
//     row's [first, end) columns, then every run of the batch ORs its columns in: the columns
//     left clear are exactly the row's base columns, in base order (the closed form of toMSA,
//     GapAssem.cpp:568-590);
//   * the base in lane l's first clear column is first + 32l - (set bits before lane l) — a
//     wave scan of the popcounts — so for each group of 4 columns the lane reads 4 bytes of the
//     window from there (two LDS dwords + alignbyte), and v_perm puts a '-' into each set column
//     and the next base into each clear one;
//   * bin codes for the 4 characters (GAlnColumn::addNuc / addGap, bin_codes5) shift a 1 into
//     the column's packed counter: six 5-bit fields A,C,G,T,N,- in a u32 (a "none" code for the
//     columns outside the row's counted extent lands in bits 30-31 and is discarded);
//   * the counters move to the workgroup's LDS table every 31 rows of the wave and at the end;
//     the table is written out coalesced.
// A row whose tile start is not in the table, or whose batch holds an overflowed chunk, builds
// the same bitmap from ofs (a wave scan per chunk) and loads its window after that.
constexpr int kCntWaves = 8;
constexpr int kWin = 2176;     // bytes of the per-wave base window

constexpr int kFlushRows = 31; // 5-bit packed counters
constexpr uint32_t kCodeNone = 30u;
struct TileLds {
  uint32_t tab[6 * kCntW];                 // [field][swizzled column]
  uint32_t win[kCntWaves][kWin / 4];       // per-wave base windows
  uint32_t bmap[kCntWaves][64];            // per-wave gap-column bitmaps
  uint32_t sel[16];                        // v_perm selectors: 4-bit gap mask -> byte picks
};
// LDS slot of column c: rotated within its 32 columns by its 32-column block index, so the adds
// of one counter index m of the 32 lanes of an LDS access group (lane l: column 32 l + m) fall
// into distinct banks ((m + l) & 31)
__device__ __forceinline__ int cnt_swz(int c) { return (c & ~31) | ((c + (c >> 5)) & 31); }
// the bin shifts (5 x GAlnColumn::addNuc/addGap bin, as bin_of) of 4 characters in a dword:
// h = (c >> 1) & 7 picks, per byte, the only characters that can have each bin (A/a 0, C/c 1,
// T/t 2, G/g 3, '*' 5, '-' 6; 4 and 7 none) and v_perm looks up the code, the expected
// character and its case mask; a byte that is not its h's character is N (20)
__device__ __forceinline__ uint32_t bin_codes5(uint32_t s4) {
  const uint32_t h = (s4 >> 1) & 0x07070707u;
  const uint32_t code = __builtin_amdgcn_perm(0x14191914u, 0x0A0F0500u, h);  // 0 5 15 10 | 20 25 25 20
  const uint32_t ex = __builtin_amdgcn_perm(0x002D2A00u, 0x47544341u, h);    // A C T G | - * - -
  const uint32_t mk = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xDFDFDFDFu, h);    // letters: either case
  const uint32_t x = (s4 & mk) ^ ex;                                         // 0 byte: the character
  const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // 0x80: not it
  const uint32_t m = (nz << 1) - (nz >> 7);                                  // 0xFF per such byte
  return (m & 0x14141414u) | (~m & code);
}
// the same codes when every byte is one of A C T G H * - N (the one character of each h): the
// byte's h's character XOR the byte goes to d (nonzero: redo with bin_codes5)
__device__ __forceinline__ uint32_t bin_codes_fast(uint32_t s4, uint32_t& d) {
  const uint32_t h = (s4 >> 1) & 0x07070707u;
  const uint32_t code = __builtin_amdgcn_perm(0x14191914u, 0x0A0F0500u, h);  // 0 5 15 10 | 20 25 25 20
  const uint32_t ex = __builtin_amdgcn_perm(0x4E2D2A48u, 0x47544341u, h);    // A C T G | H * - N
  d = s4 ^ ex;
  return code;
}
// bits of columns [32 lane, 32 lane + 32) that are < lo or >= hi (tile-relative)
__device__ __forceinline__ uint32_t outside_mask(int lane, int lo, int hi) {
  const int a = min(max(lo - 32 * lane, 0), 32), b = min(max(hi - 32 * lane, 0), 32);
  const uint32_t below = a >= 32 ? 0xFFFFFFFFu : ((1u << a) - 1u);
  const uint32_t above = b >= 32 ? 0u : ~((1u << b) - 1u);
  return below | above;
}
// Per-row values loaded ahead are spread over the lanes of one VGPR (a lane per dword, read
// back with readlane): vector loads, so their waits are vmcnt waits in issue order, not lgkmcnt
// waits that every LDS wait of the row body would share.
//   RowA (3 rows ahead): slot_base[r], slot_base[r + 1] (x, lanes 0-3), row_off (y, 0-1), col0 (z)
//   RowB (2 rows ahead): the row record (x, lanes 0-7), its tile-start entry (y, lanes 0-1)
struct RowA {
  int64_t sb, sbn;
  uint64_t roff;
  int rs;
};
// (no select between the loads: a select would wait for all of them where it is computed, and
// hipcc turns a lane select of loads into branches that wait vmcnt(0) — every later prefetch then
// waits too.  Each value stays in the VGPR it was loaded into; readlane picks lanes at use.)
struct AV {
  uint32_t x, y, z;
};
struct BV {
  uint32_t x, y;
};
__device__ __forceinline__ AV load_a(const pw_msa_args& A, uint32_t r, int lane) {
  // (three loads from uniform bases with small lane offsets: no per-lane pointers)
  const uint64_t rr = r < A.n_rows ? r : A.n_rows - 1;
  AV v;
  v.x = reinterpret_cast<const uint32_t*>(A.slot_base + rr)[lane & 3];
  v.y = reinterpret_cast<const uint32_t*>(A.row_off + rr)[lane & 1];
  v.z = (uint32_t)A.col0[rr];
  return v;
}
__device__ __forceinline__ uint32_t rd(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ RowA get_a(const AV& v) {
  RowA a;
  a.sb = (int64_t)((uint64_t)rd(v.x, 0) | (uint64_t)rd(v.x, 1) << 32);
  a.sbn = (int64_t)((uint64_t)rd(v.x, 2) | (uint64_t)rd(v.x, 3) << 32);
  a.roff = (uint64_t)rd(v.y, 0) | (uint64_t)rd(v.y, 1) << 32;
  a.rs = (int)rd(v.z, 0);
  return a;
}
__device__ __forceinline__ BV load_b(const pw_msa_args& A, const int32_t* rinfo, const int32_t* tstart, uint32_t r,
                                     const RowA& a, int c0, int lane) {
  const uint64_t rr = r < A.n_rows ? r : A.n_rows - 1;
  int64_t idx = (int64_t)(c0 >> 11) - (int64_t)(a.rs >> 11);
  idx = idx < 0 ? 0 : (idx > a.sbn - a.sb - 1 ? a.sbn - a.sb - 1 : idx);
  BV v;
  v.x = (uint32_t)(rinfo + kRowInfo * rr)[lane & 7];
  v.y = (uint32_t)(tstart + 2 * (a.sb + idx))[lane & 1];
  return v;
}
// word l of the row record (0-7) or of its tile-start entry (8-9)
__device__ __forceinline__ uint32_t rd(const BV& b, int l) { return l < 8 ? rd(b.x, l) : rd(b.y, l - 8); }
__device__ __forceinline__ void tile_start(const RowA& a, const BV& b, int c0, int& kt, int& ib) {
  if (c0 <= a.rs) {
    kt = 0;
    ib = 0;
  } else if (rd(b, 5) & kNoTable) {
    kt = -1;
    ib = 0;
  } else {
    kt = (int)rd(b, 8);
    ib = (int)rd(b, 9);
  }
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const pw_msa_args& A, uint64_t roff, int len) {
  // base 16-byte aligned at or before the row; the range ends at the row's readable end (len < 0:
  // an empty range — every load returns 0 without a memory access)
  const uint64_t b0 = roff & ~(uint64_t)15;
  const uint32_t nrec = len < 0 ? 0u : (uint32_t)(roff - b0) + (((uint32_t)len + 3u) & ~3u);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(A.seq + b0), (short)0, (int)nrec, 0x00020000);
}
__device__ __forceinline__ void load_win(const pw_msa_args& A, uint64_t roff, int len, int ib, int lane, v4u& w0, v4u& w1,
                                         v4u& w2) {
  const __amdgpu_buffer_rsrc_t rs = row_rsrc(A, roff, len);
  const uint32_t o = (uint32_t)(((roff + (uint64_t)ib) & ~(uint64_t)15) - (roff & ~(uint64_t)15));
  w0 = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16u * (uint32_t)lane, 0, 0);
  w1 = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 1024u + 16u * (uint32_t)lane, 0, 0);
  w2 = __builtin_amdgcn_raw_buffer_load_b128(rs, o + 2048u + 16u * (uint32_t)(lane & 7), 0, 0);
}
struct RowC {  // 1 row ahead
  int ckv;
  uint32_t gv[2];  // runs (two per dword) of chunks kt + (lane >> 3) (h = 0) and kt + 8 (h = 1, lanes 0-7)
  v4u w0, w1, w2;
};
__device__ __forceinline__ void load_c(const pw_msa_args& A, const int32_t* ckpt, const uint16_t* runs, const RowA& a,
                                       const BV& b, int c0, int c1, int lane, RowC& c) {
  int kt, ib;
  tile_start(a, b, c0, kt, ib);
  const int nch = (int)(rd(b, 5) & ~kNoTable);
  const int len = (int)rd(b, 4);
  kt = min(max(kt, 0), nch);  // (a row that does not reach the tile reads a stale entry: clamped)
  // (uniform row bases, 32-bit lane offsets)
  const int32_t* ck_r = ckpt + a.sb;
  const uint32_t* ru_r = reinterpret_cast<const uint32_t*>(runs + (uint64_t)a.sb * kRunCap);
  c.ckv = ck_r[min(kt + lane, nch)];
  c.gv[0] = ru_r[min(kt + (lane >> 3), nch) * (kRunCap / 2) + (lane & 7)];
  c.gv[1] = ru_r[min(kt + 8, nch) * (kRunCap / 2) + (lane & 7)];
  // (a row whose counted extent misses the tile loads no window: ~1/4 of a tile's rows at cfg5)
  const bool ov = max((int)rd(b, 0), c0) <= min((int)rd(b, 1), c1 - 1);
  load_win(A, a.roff, ov ? len : -1, ib, lane, c.w0, c.w1, c.w2);
}
__device__ __forceinline__ void pin(v4u& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(v2u& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(int& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void cnt_flush(uint32_t (&acc)[32], LDS uint32_t* tab, int lane) {
#pragma unroll
  for (int m = 0; m < 32; m++) {
    const int x = cnt_swz(32 * lane + m);  // (acc[m] = column 32 lane + m)
#pragma unroll
    for (int f = 0; f < 6; f++) {
      atomicAdd((uint32_t*)&tab[f * kCntW + x], (acc[m] >> (5 * f)) & 31u);
    }
    acc[m] = 0;
  }
}
// the gap bitmap of a row in this tile from ofs (rows without a tile-start entry, or with an
// overflowed chunk in the batch): ORs the gap runs of chunks kt.. into bm, returns the first
// base at or after column c0 (kt = -1: found by a search of the checkpoints first)
__device__ int slow_bitmap(const pw_msa_args& A, const int32_t* ckpt, int64_t sb, int nch, uint64_t roff, int len, int c0,
                           int c1, int kt, int lane, LDS uint32_t* bm) {
  if (kt < 0) {  // last chunk whose checkpoint is <= c0
    int lo = 0, hi = nch - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (ckpt[sb + mid] <= c0) lo = mid;
      else hi = mid - 1;
    }
    kt = lo;
  }
  int ib = INT_MAX;
  for (int k = kt; k < nch; k++) {
    int col = ckpt[sb + k];
    if (col >= c1) break;
    const int i0 = k * kChunk + 4 * lane;
    int gp[4], tot = 0;
    int16_t raw[4];
#pragma unroll
    for (int j = 0; j < 4; j++) raw[j] = A.ofs[roff + (uint64_t)min(i0 + j, len - 1)];  // (unconditional: one round trip)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const bool ok = i0 + j < len;
      gp[j] = ok ? max((int)raw[j], 0) : 0;
      tot += ok ? 1 + gp[j] : 0;
    }
    const int incl = wave_scan_incl(tot);
    int run = col + incl - tot;
    int first = INT_MAX;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i0 + j >= len) break;
      const int g0 = run, bc = run + gp[j];  // gap run [g0, bc), base column bc
      for (int x = max(g0, c0); x < bc && x < c1; x++) atomicOr((uint32_t*)&bm[(x - c0) >> 5], 1u << ((x - c0) & 31));
      if (bc >= c0 && first == INT_MAX) first = i0 + j;
      run = bc + 1;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) first = min(first, __shfl_xor(first, d, 64));
    ib = min(ib, first);
  }
  return ib == INT_MAX ? len : ib;
}
// bestChar of one column's six counts (GapAssem.cpp:1048-1069 in closed form; 0 = no coverage)
__device__ __forceinline__ uint8_t best_char(const int (&v)[6]) {
  const int layers = v[0] + v[1] + v[2] + v[3] + v[4] + v[5];
  if (layers <= 0) return 0;
  int m = v[0], bi = 0;
#pragma unroll
  for (int q = 1; q < 6; q++)
    if (v[q] > m) {
      m = v[q];
      bi = q;
    }
  uint8_t best = (uint8_t)"ACGTN-"[bi];
  if (bi == 4 && v[5] == m) best = '-';
  return best;
}
__global__ __launch_bounds__(64 * kCntWaves, 4) void tile_counts(const pw_msa_args A, const int32_t* __restrict__ ckpt,
                                                              const uint16_t* __restrict__ runs,
                                                              const int32_t* __restrict__ rinfo,
                                                              const int32_t* __restrict__ tstart, int call,
                                                              uint8_t* __restrict__ cons_star, int32_t* cons_len) {
  __shared__ __attribute__((aligned(16))) TileLds L;
  LDS TileLds* lp = (LDS TileLds*)&L;
  const int tid = threadIdx.x, lane0 = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.x * kCntW;
  const int c1 = min(c0 + kCntW, A.n_cols);
  for (int i = tid; i < 6 * kCntW; i += 64 * kCntWaves) lp->tab[i] = 0;
  if (tid < 16) {  // byte p: a gap column -> 4 (a '-' of src0), else the next source byte
    uint32_t s = 0;
    int k = 0;
    for (int p = 0; p < 4; p++) {
      s |= (uint32_t)(((tid >> p) & 1) ? 4 : k) << (8 * p);
      k += ((tid >> p) & 1) ? 0 : 1;
    }
    lp->sel[tid] = s;
  }
  __syncthreads();
  LDS uint32_t* win = lp->win[wv];
  LDS uint32_t* bm = lp->bmap[wv];
  LDS uint32_t* tab = lp->tab;
  uint32_t acc[32];
#pragma unroll
  for (int m = 0; m < 32; m++) acc[m] = 0;
  int nrow = 0;
  const uint32_t W = kCntWaves;
  uint32_t r = wv;
  if (r < A.n_rows) {
    // prologue: rows r (A, B, C), r + W (A, B), r + 2W (A)
    AV av1 = load_a(A, r, lane0), av2 = load_a(A, r + W, lane0), av3 = load_a(A, r + 2 * W, lane0);
    RowA a1 = get_a(av1);
    BV bv1 = load_b(A, rinfo, tstart, r, a1, c0, lane0);
    RowA a2 = get_a(av2);
    BV bv2 = load_b(A, rinfo, tstart, r + W, a2, c0, lane0);
    RowC cc;
    load_c(A, ckpt, runs, a1, bv1, c0, c1, lane0, cc);
    for (;; r += W) {
      // (lane-derived values are recomputed per row from a lane index the compiler cannot hoist:
      // left alone it keeps 64-bit per-lane pointers live across the loop and spills them)
      int lane = lane0;
      asm volatile("" : "+v"(lane));
      // the next rows' loads (each waits only for what the previous iteration issued), then this
      // row, whose batch was issued a row earlier
      // this row's window into LDS first (its registers are then free for the next row's)
      pin(cc.w0);
      pin(cc.w1);
      pin(cc.w2);
      {
        LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
        w4[lane] = cc.w0;
        w4[64 + lane] = cc.w1;
        if (lane < 8) w4[128 + lane] = cc.w2;
      }
      RowC cn;
      load_c(A, ckpt, runs, a2, bv2, c0, c1, lane, cn);
      const RowA a3 = get_a(av3);
      const BV bv3 = load_b(A, rinfo, tstart, r + 2 * W, a3, c0, lane);
      const AV av4 = load_a(A, r + 3 * W, lane);
      pin(cc.ckv);
      pin(cc.gv[0]);
      pin(cc.gv[1]);
      const int elo = (int)rd(bv1, 0), ehi = (int)rd(bv1, 1);
      const int a = max(elo, c0), z = min(ehi, c1 - 1);  // counted columns of this row here
      if (a <= z) {
        nrow++;
        const int rs = (int)rd(bv1, 2), re = (int)rd(bv1, 3);
        const int len = (int)rd(bv1, 4);
        const int nch = (int)(rd(bv1, 5) & ~kNoTable);
        const int64_t sb = a1.sb;
        const uint64_t roff = a1.roff;
        int kt, ib;
        tile_start(a1, bv1, c0, kt, ib);
        // gap bitmap: the columns outside [rs, re), then the runs of the batch's chunks
        bm[lane] = outside_mask(lane, rs - c0, re - c0);
        // the batch's chunks kt .. kt + 8 (chunk kt holds c0; each later one spans >= 256 columns)
        bool cv[2], ovl = false;
#pragma unroll
        for (int h = 0; h < 2; h++) {
          cv[h] = kt >= 0 && (h == 0 ? kt + (lane >> 3) < nch : (kt + 8 < nch && lane < 8));
          ovl = ovl || (cv[h] && (lane & 7) == 0 && (cc.gv[h] & 0xFFFFu) == kRunOverflow);
        }
        const bool ovf = kt < 0 || __ballot(ovl) != 0;
        wave_sync();
        if (!ovf) {
#pragma unroll
          for (int h = 0; h < 4; h++) {  // (h >> 1: which dword, h & 1: which half)
            const uint32_t v = cv[h >> 1] ? (cc.gv[h >> 1] >> (16 * (h & 1))) & 0xFFFFu : 0u;
            const int ck = (h >> 1) == 0 ? __shfl(cc.ckv, lane >> 3, 64) : __builtin_amdgcn_readlane(cc.ckv, 8);
            if (v != 0u) {
              const int s = max(ck + (int)(v >> 6) - c0, 0), e = min(ck + (int)(v >> 6) + (int)(v & 63u) - c0, kCntW);
              for (int x = s; x < e; x = (x | 31) + 1) {
                const int xe = min(e, (x | 31) + 1);
                const uint32_t m = (xe - x >= 32 ? 0xFFFFFFFFu : ((1u << (xe - x)) - 1u)) << (x & 31);
                atomicOr((uint32_t*)&bm[x >> 5], m);
              }
            }
          }
        } else {
          ib = slow_bitmap(A, ckpt, sb, nch, roff, len, c0, c1, kt, lane, bm);
          v4u w0, w1, w2;
          load_win(A, roff, len, ib, lane, w0, w1, w2);
          LDS v4u* w4 = reinterpret_cast<LDS v4u*>(win);
          w4[lane] = w0;
          w4[64 + lane] = w1;
          if (lane < 8) w4[128 + lane] = w2;
        }
        wave_sync();
        const uint32_t bmv = bm[lane];
        const int pc = __popc(bmv);
        const int excl = wave_scan_incl(pc) - pc;
        // byte offset in the window of the base in this lane's first clear column
        const int so = (int)((uint32_t)(roff + (uint64_t)ib) & 15u) + 32 * lane - excl;
        const LDS uint8_t* wb = reinterpret_cast<const LDS uint8_t*>(win);
        // step q: this lane's column group q (columns 32 lane + 4q ..), its source offset so + 4q -
        // popc(bitmap bits below 4q).  (Rounds 3-4 rotated each lane's group order so that the 32
        // lanes of an LDS access group read 32 distinct banks when the row has no gaps; the
        // rotation's offset and wrap arithmetic cost more than the conflicts it removed: round 5,
        // tools/exp_msa_variants.py norot, tile_counts 90.5 -> 87.1 us.)
        uint32_t codes[8];
        auto groups = [&](auto edge_c, auto fast_c) {
          constexpr bool kEdge = decltype(edge_c)::value, kFast = decltype(fast_c)::value;
          uint32_t rom = 0, bad = 0;
          if constexpr (kEdge) {
            const uint32_t om = outside_mask(lane, a - c0, z - c0 + 1);
            rom = om;
          }
#pragma unroll
          for (int q = 0; q < 8; q++) {
            const uint32_t nb = (bmv >> (4 * q)) & 15u;
            const int src = so + 4 * q - (q == 0 ? 0 : __popc(bmv & ((1u << (4 * q)) - 1u)));
            const LDS uint32_t* p = reinterpret_cast<const LDS uint32_t*>(wb + (src & ~3));
            const uint32_t s4 = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)src & 3u);
            const uint32_t e4 = __builtin_amdgcn_perm(0x2D2D2D2Du, s4, lp->sel[nb]);
            uint32_t d = 0;
            uint32_t cq = kFast ? bin_codes_fast(e4, d) : bin_codes5(e4);
            if constexpr (kEdge) {  // (columns outside the extent: code none, never "bad")
              const uint32_t on = (rom >> (4 * q)) & 15u;
              const uint32_t b1 = (on * 0x00204081u) & 0x01010101u;  // 4 bits -> 4 bytes
              const uint32_t bmask = (b1 << 8) - b1;
              cq = (cq & ~bmask) | (bmask & (kCodeNone * 0x01010101u));
              d &= ~bmask;
            }
            bad |= d;
            codes[q] = cq;
          }
          return bad;
        };
        const bool edge = a > c0 || z < c1 - 1;  // the row's counted extent starts / ends here
        const uint32_t bad = edge ? groups(std::true_type{}, std::true_type{}) : groups(std::false_type{}, std::true_type{});
        if (__ballot(bad != 0u)) {  // lower case, or a character outside A C G T N - * H
          if (edge) groups(std::true_type{}, std::false_type{});
          else groups(std::false_type{}, std::false_type{});
        }
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
          for (int j = 0; j < 4; j++) acc[4 * q + j] += 1u << ((codes[q] >> (8 * j)) & 31u);
        wave_sync();
      }
      a1 = a2;
      a2 = a3;
      av3 = av4;
      bv1 = bv2;
      bv2 = bv3;
      cc = cn;
      const bool last = r + W >= A.n_rows;
      if (last || nrow == kFlushRows) {  // (the counters' one flush site)
        cnt_flush(acc, tab, lane);
        nrow = 0;
      }
      if (last) break;
    }
  }
  __syncthreads();
  // the tile's counters: [col][6] rows in memory, coalesced — non-temporal stores, as the
  // consensus below: no later kernel of the step reads them (round 5: tile_counts -1 us,
  // row_chunk_sums of the next step -1 us)
  const int cw = c1 - c0;
  int32_t* dst = A.counts + (int64_t)c0 * 6;
  for (int i = tid; i < cw * 6; i += 64 * kCntWaves) {
    const int c = i / 6, f = i - 6 * c;
    __builtin_nontemporal_store((int32_t)tab[f * kCntW + cnt_swz(c)], dst + i);
  }
  if (call) {  // pw_msa_columns (all rows in this launch): the call step from the same table
    const int zlo = A.minmax[0], zhi = A.minmax[1];
    // (pw_msa_columns_refine without removeConsGaps: refineMSA's consensus string too, as K6')
    if (cons_star && blockIdx.x == 0 && tid == 0) *cons_len = zhi >= 0 && zhi < A.n_cols && zhi >= zlo ? zhi - zlo + 1 : 0;
    for (int c = tid; c < cw; c += 64 * kCntWaves) {
      int v[6];
#pragma unroll
      for (int f = 0; f < 6; f++) v[f] = (int)tab[f * kCntW + cnt_swz(c)];
      const uint8_t best = best_char(v);
      __builtin_nontemporal_store(best, A.consensus + c0 + c);
      if (cons_star && c0 + c >= zlo && c0 + c <= zhi)
        __builtin_nontemporal_store(best == '-' ? (uint8_t)'*' : best, cons_star + c0 + c - zlo);
      if (best == 0 && c0 + c >= zlo && c0 + c <= zhi) atomicMin(&A.minmax[3], c0 + c);
    }
  }
}

// bestChar of each column (GapAssem.cpp:1048-1069 in closed form); 0 = no coverage, and the
// first such column in [mincol, maxcol] (ErrZeroCov, :1121-1131) into minmax[3]
__global__ __launch_bounds__(256) void call_columns(const pw_msa_args A, int32_t lo, int32_t hi) {
  const int zlo = A.minmax[0], zhi = A.minmax[1];
  for (int64_t c = lo + (int64_t)blockIdx.x * 256 + threadIdx.x; c < hi; c += (int64_t)gridDim.x * 256) {
    int v[6];
    const int32_t* src = A.counts + c * 6;
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = src[q];
    const uint8_t best = best_char(v);
    A.consensus[c] = best;
    if (best == 0 && c >= zlo && c <= zhi) atomicMin(&A.minmax[3], (int)c);
  }
}

// ---------------------------------------------------------------- refineMSA (pw_msa_refine)
__device__ __forceinline__ bool cons_gap(const pw_msa_args& A, int lo, int hi, int c) {
  return c >= lo && c <= hi && A.consensus[c] == '-';
}

// K6: consensus-gap columns per 2048-column tile
__global__ __launch_bounds__(256) void gap_tiles(const pw_msa_args A, pw_msa_refine_args R) {
  __shared__ int part[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) *R.cons_len = 0;  // (gap_scan sets it when maxcol is a column)
  const int lo = A.minmax[0], hi = A.minmax[1];
  const int c0 = blockIdx.x * kTileW;
  int n = 0;
  for (int c = c0 + threadIdx.x; c < c0 + kTileW && c < A.n_cols; c += 256) n += cons_gap(A, lo, hi, c) ? 1 : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) R.tile_gaps[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// K7: G(c) (inclusive) for every column of the tile and the consensus string
__global__ __launch_bounds__(256) void gap_scan(const pw_msa_args A, pw_msa_refine_args R) {
  __shared__ int part[4];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lo = A.minmax[0], hi = A.minmax[1];
  const int t = blockIdx.x;
  // gap columns of the tiles before this one
  int b = 0;
  for (int i = tid; i < t; i += 256) b += R.tile_gaps[i];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
  if (lane == 0) part[wv] = b;
  __syncthreads();
  if (tid == 0) base_s = part[0] + part[1] + part[2] + part[3];
  __syncthreads();
  // each thread owns 8 consecutive columns
  const int c0 = t * kTileW + tid * 8;
  uint32_t gm = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) gm |= cons_gap(A, lo, hi, c0 + q) && c0 + q < A.n_cols ? (1u << q) : 0u;
  const int mine = __popc(gm);
  int incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  __syncthreads();
  if (lane == 63) part[wv] = incl;
  __syncthreads();
  int g = base_s + incl - mine;
  for (int w = 0; w < wv; w++) g += part[w];
  const bool rm = R.remove_gaps != 0;
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const int c = c0 + q;
    if (c >= A.n_cols) break;
    const bool isg = (gm >> q) & 1u;
    g += isg ? 1 : 0;
    R.gap_prefix[c] = g;
    if (c >= lo && c <= hi) {
      const uint8_t ch = A.consensus[c];
      if (!rm) R.cons_out[c - lo] = isg ? (uint8_t)'*' : ch;
      else if (!isg) R.cons_out[c - lo - g] = ch;
      if (c == hi) *R.cons_len = (hi - lo + 1) - (rm ? g : 0);
    }
  }
}

// K6' (refineMSA without removeConsGaps, GapAssem.cpp:1143-1162): no column moves, so no G(c) —
// the consensus string is the called columns [mincol, maxcol] with '-' printed as '*', one
// elementwise pass (K6 + K7 are two launches and a scan for the same bytes)
__global__ __launch_bounds__(256) void cons_mark(const pw_msa_args A, pw_msa_refine_args R) {
  const int lo = A.minmax[0], hi = A.minmax[1];
  if (blockIdx.x == 0 && threadIdx.x == 0)  // (= K7: set when maxcol is a column of the layout)
    *R.cons_len = hi >= 0 && hi < A.n_cols && hi >= lo ? hi - lo + 1 : 0;
  const int a = max(lo, 0), z = min(hi, A.n_cols - 1);
  for (int c = a + (int)(blockIdx.x * 256 + threadIdx.x); c <= z; c += (int)(gridDim.x * 256)) {
    const uint8_t ch = A.consensus[c];
    R.cons_out[c - lo] = ch == '-' ? (uint8_t)'*' : ch;
  }
}

__device__ __forceinline__ int gx(const pw_msa_refine_args& R, int n_cols, int c) {
  return c < 0 ? 0 : R.gap_prefix[c < n_cols ? c : n_cols - 1];
}

// K8: ofs' of every base, one wave per 256-base chunk (columns re-derived as in K3)
__global__ __launch_bounds__(256) void row_edit(const pw_msa_args A, pw_msa_refine_args R, const int32_t* ckpt,
                                                const int32_t* slot_row) {
  const int64_t* chunk_base = A.slot_base;
  const int lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (uint64_t c = wid; c < A.n_slots; c += (uint64_t)gridDim.x * 4) {
    const uint32_t r = (uint32_t)slot_row[c];
    const int64_t k = (int64_t)c - chunk_base[r];
    const int len = A.row_len[r];
    const int64_t ib = k * kChunk;
    if (ib >= len) continue;  // the row's end slot
    const uint64_t roff = A.row_off[r];
    int col = ckpt[c];
    long long dsum = 0;
#pragma unroll
    for (int j = 0; j < kChunk / 64; j++) {
      const int64_t i = ib + j * 64 + lane;
      const bool ok = i < len;
      const int g = ok ? A.ofs[roff + i] : 0;  // >= 0 (checked by the host)
      const int adv = ok ? 1 + g : 0;
      int incl = adv;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
      }
      const int bcol = col + incl - 1;
      if (ok) {
        const int prev = i == 0 ? bcol - g : bcol - g - 1;  // O for the first base
        const int dec = gx(R, A.n_cols, bcol) - gx(R, A.n_cols, prev);
        R.ofs_out[roff + i] = (int16_t)(g - dec);
        dsum += dec;
      }
      col += __shfl(incl, 63, 64);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dsum += __shfl_xor(dsum, d, 64);
    if (lane == 0 && dsum) atomicAdd((unsigned long long*)&R.numgaps_out[r], (unsigned long long)(-dsum));
  }
}

// K9: per row (one wave): offset', then removeClipGaps on ofs'
__global__ __launch_bounds__(64) void row_finish(const pw_msa_args A, pw_msa_refine_args R) {
  const int lane = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int len = A.row_len[r];
    const uint64_t roff = A.row_off[r];
    const int cl = R.keep_clip_gaps ? -1 : A.clip_l[r], cr = R.keep_clip_gaps ? 0 : A.clip_r[r];
    long long dl = 0, dr = 0;
    for (int i = lane; i < len && i <= cl; i += 64) {
      dl += R.ofs_out[roff + i];
      R.ofs_out[roff + i] = 0;
    }
    const int r0 = (len - cr > cl + 1) ? len - cr : cl + 1;  // (keep_clip_gaps: r0 = len, nothing)
    for (int i = r0 + lane; i < len; i += 64) {
      dr += R.ofs_out[roff + i];
      R.ofs_out[roff + i] = 0;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      dl += __shfl_xor(dl, d, 64);
      dr += __shfl_xor(dr, d, 64);
    }
    if (lane == 0) {
      R.offset_out[r] = R.row_offset[r] - gx(R, A.n_cols, A.col0[r]) + (int32_t)dl;
      R.numgaps_out[r] -= dl + dr;
    }
  }
}

// scratch word of the row records (16-byte aligned: K3 reads them as uint4)
// scratch words: chunk sums | checkpoints | slot -> row | runs (kRunCap per slot) | tile starts (2 per slot) | row records
inline uint64_t runs_word(uint64_t n_slots) { return (3 * n_slots + 3) & ~(uint64_t)3; }  // (16-byte aligned)
inline uint64_t tstart_word(uint64_t n_slots) { return runs_word(n_slots) + (uint64_t)kRunCap / 2 * n_slots; }
inline uint64_t rinfo_word(uint64_t n_slots) { return (tstart_word(n_slots) + 2 * n_slots + 3) & ~(uint64_t)3; }

}  // namespace pw

extern "C" uint64_t pw_msa_slots(const int32_t* row_len_host, uint32_t n_rows, int64_t* slot_base_host) {
  int64_t acc = 0;
  for (uint32_t r = 0; r < n_rows; r++) {
    slot_base_host[r] = acc;
    acc += ((int64_t)(row_len_host[r] > 0 ? row_len_host[r] : 0) + pw::kChunk - 1) / pw::kChunk + 1;
  }
  slot_base_host[n_rows] = acc;
  return (uint64_t)acc;
}

extern "C" uint64_t pw_msa_scratch_words(uint64_t n_slots, uint32_t n_rows) {
  return pw::rinfo_word(n_slots) + (uint64_t)pw::kRowInfo * n_rows;
}

static bool msa_args_ok(const pw_msa_args* a) {
  return a && a->seq && a->ofs && a->row_off && a->row_len && a->col0 && a->clip_l && a->clip_r && a->slot_base &&
         a->scratch && a->counts && a->consensus && a->minmax && a->n_rows > 0 && a->n_cols > 0 &&
         a->n_slots >= a->n_rows;
}

// count (+ with call, the bestChar step in tile_counts' epilogue: every row is in this launch)
static int msa_count(const pw_msa_args* a, void* stream, bool call, uint8_t* cons_star = nullptr,
                     int32_t* cons_len = nullptr) {
  if (!msa_args_ok(a)) return PW_E_ARG;
  if (a->n_slots >= (1ull << 27)) return PW_E_ARG;  // (K1's 32-bit buffer offsets: < 34 G bases)
  hipStream_t s = (hipStream_t)stream;
  // scratch: chunk sums | checkpoints | slot -> row | gap runs (kRunCap per slot) | tile starts |
  // row records
  int32_t* chunk_sum = a->scratch;
  int32_t* ckpt = a->scratch + a->n_slots;
  int32_t* slot_row = a->scratch + 2 * a->n_slots;
  uint16_t* runs = reinterpret_cast<uint16_t*>(a->scratch + pw::runs_word(a->n_slots));
  int32_t* tstart = a->scratch + pw::tstart_word(a->n_slots);
  int32_t* rinfo = a->scratch + pw::rinfo_word(a->n_slots);
  uint64_t* sdesc = reinterpret_cast<uint64_t*>(tstart);  // (K1's input; K2 then writes the tile starts there)
  const unsigned sy = a->n_rows >= 2048 ? 1u : (2048u / a->n_rows < 64u ? 2048u / a->n_rows : 64u);
  hipLaunchKernelGGL(pw::slot_rows, dim3(a->n_rows < 8192 ? a->n_rows : 8192, sy), dim3(256), 0, s, *a, slot_row, sdesc);
  const uint64_t nb1 = ((a->n_slots + 3) / 4 + 3) / 4;  // 4 slots per wave, 4 waves per workgroup
  // (persistent: 8192 workgroups, ~4 rounds of resident waves, each streaming a few groups — the
  // round-4 sweep on cfg5: 2048 68.6-69.2 us, 4096 65.3-65.5, 6144 63.8, 8192 62.1-62.3, uncapped
  // (36 k) 62.6: fewer groups per wave end the kernel with less of a tail)
  hipLaunchKernelGGL(pw::row_chunk_sums, dim3((unsigned)(nb1 < 8192 ? nb1 : 8192)), dim3(256), 0, s, *a,
                     chunk_sum, sdesc, runs);
  hipLaunchKernelGGL(pw::row_prefix, dim3(a->n_rows < 4096 ? a->n_rows : 4096), dim3(1024), 0, s, *a, chunk_sum, ckpt,
                     rinfo, runs, tstart);
  const unsigned ntiles = (unsigned)((a->n_cols + pw::kCntW - 1) / pw::kCntW);
  hipLaunchKernelGGL(pw::tile_counts, dim3(ntiles), dim3(64 * pw::kCntWaves), 0, s, *a, ckpt, runs, rinfo, tstart,
                     call ? 1 : 0, cons_star, cons_len);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

extern "C" int pw_msa_call_cols(const pw_msa_args* a, int32_t col_lo, int32_t col_hi, const int32_t* counts_lo,
                                void* stream) {
  if (!msa_args_ok(a) || col_lo < 0 || col_hi > a->n_cols || col_lo > col_hi) return PW_E_ARG;
  if (col_lo == col_hi) return PW_OK;
  hipStream_t s = (hipStream_t)stream;
  pw_msa_args b = *a;
  if (counts_lo) b.counts = const_cast<int32_t*>(counts_lo) - (int64_t)col_lo * 6;  // column c at counts_lo[(c - lo) * 6]
  const uint64_t nb = ((uint64_t)(col_hi - col_lo) + 255) / 256;
  hipLaunchKernelGGL(pw::call_columns, dim3((unsigned)(nb < 8192 ? nb : 8192)), dim3(256), 0, s, b, col_lo, col_hi);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

extern "C" int pw_msa_call(const pw_msa_args* a, void* stream) {
  if (!msa_args_ok(a)) return PW_E_ARG;
  return pw_msa_call_cols(a, 0, a->n_cols, nullptr, stream);
}

extern "C" int pw_msa_count(const pw_msa_args* a, void* stream) { return msa_count(a, stream, false); }

// count + call in one pass: tile_counts holds a tile's complete counts (all rows) in LDS, so it
// writes bestChar and the zero-coverage column too (no call_columns launch, no counts re-read)
extern "C" int pw_msa_columns(const pw_msa_args* a, void* stream) { return msa_count(a, stream, true); }

extern "C" uint64_t pw_msa_refine_tiles(int32_t n_cols) { return n_cols > 0 ? ((uint64_t)n_cols + pw::kTileW - 1) / pw::kTileW : 0; }

extern "C" int pw_msa_refine(const pw_msa_args* a, const pw_msa_refine_args* r, void* stream) {
  if (!msa_args_ok(a) || !r || !r->gap_prefix || !r->tile_gaps || !r->cons_out || !r->cons_len) return PW_E_ARG;
  if (r->remove_gaps && (!r->row_offset || !r->ofs_out || !r->offset_out || !r->numgaps_out)) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const unsigned ntiles = (unsigned)pw_msa_refine_tiles(a->n_cols);
  if (!r->remove_gaps) {  // (gap_prefix / tile_gaps are not written: nothing reads them)
    const unsigned nb = (unsigned)(((uint64_t)a->n_cols + 255) / 256);
    hipLaunchKernelGGL(pw::cons_mark, dim3(nb < 4096 ? nb : 4096), dim3(256), 0, s, *a, *r);
    return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
  }
  hipLaunchKernelGGL(pw::gap_tiles, dim3(ntiles), dim3(256), 0, s, *a, *r);
  hipLaunchKernelGGL(pw::gap_scan, dim3(ntiles), dim3(256), 0, s, *a, *r);
  if (r->remove_gaps) {
    const int32_t* ckpt = a->scratch + a->n_slots;  // from pw_msa_count
    const int32_t* slot_row = a->scratch + 2 * a->n_slots;
    const uint64_t nb = (a->n_slots + 3) / 4;
    hipLaunchKernelGGL(pw::row_edit, dim3((unsigned)(nb < 65536 ? nb : 65536)), dim3(256), 0, s, *a, *r, ckpt,
                       slot_row);
    hipLaunchKernelGGL(pw::row_finish, dim3(a->n_rows < 4096 ? a->n_rows : 4096), dim3(64), 0, s, *a, *r);
  }
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

// pw_msa_columns + pw_msa_refine; without removeConsGaps the consensus string comes out of
// tile_counts' call epilogue (no column moves: no G(c) scan, one launch less)
extern "C" int pw_msa_columns_refine(const pw_msa_args* a, const pw_msa_refine_args* r, void* stream) {
  if (!msa_args_ok(a) || !r || !r->cons_out || !r->cons_len) return PW_E_ARG;
  if (!r->remove_gaps) return msa_count(a, stream, true, r->cons_out, r->cons_len);
  const int rc = msa_count(a, stream, true);
  return rc != PW_OK ? rc : pw_msa_refine(a, r, stream);
}
