// pw_msa.hip — GapAssem column consensus on gfx950.
//
// Reference (gpertea/pwasm GapAssem):
//   GASeq::toMSA            GapAssem.cpp:551-591   row -> columns (gap runs + bases, clipping)
//   GAlnColumn::addGap/Nuc  GapAssem.h:295-337     6 counters A,C,G,T,N,- (+ layers)
//   GAlnColumn::bestChar    GapAssem.cpp:1048-1069 stable qsort + N/- tie rule
//   GSeqAlign::buildMSA     GapAssem.cpp:1088-1106
// The reference scatters row by row (one NucOri allocation per base).  Here the layout is
// read once, column tile by column tile:
//   K0 slot_rows:      row of every chunk slot (no per-chunk binary search later)
//   K1 row_chunk_sums: per 256-base chunk of a row, sum of (1 + max(ofs,0))   (1 wave / chunk)
//   K2 row_prefix:     per row, exclusive scan of the chunk sums -> layout column at which each
//                      chunk's first gap run starts (checkpoints), row end column, bounds check
//   K3 tile_counts:    one 1024-thread workgroup per 2048-column tile keeps the tile's 6 x 2048
//                      counters in LDS; its 16 waves walk the chunks of every row that overlaps
//                      the tile (first chunk interpolated from the checkpoints; the next chunk
//                      loads while one is scanned), re-derive columns with a wave scan and add
//                      into LDS; then the tile writes its counts coalesced and folds mincol /
//                      maxcol.
//                      (pw_msa_count stops here: with rows sharded over GPUs the partial
//                      counts are summed by an all-reduce before the call)
//   K4 call_columns:   bestChar of every column (pw_msa_call)
//   K5 zero_scan:      first zero-coverage column in [mincol, maxcol] (ErrZeroCov, :1121-1131).
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
//   K8 row_edit:       ofs' of every base (chunked like K3)
//   K9 row_finish:     offset', numgaps', then removeClipGaps on ofs' (i <= clipL and
//                      i >= seqlen - clipR) unless keep_clip_gaps (refineClipping first, host)
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "pwasm_amd.h"
#include "pw_wave.h"

namespace pw {

constexpr int kChunk = 256;   // bases per checkpoint chunk
constexpr int kTileW = 2048;  // columns per workgroup
typedef int v4i __attribute__((ext_vector_type(4)));
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

// K0: the row of every slot (slot_row), one workgroup per row, coalesced
__global__ __launch_bounds__(256) void slot_rows(const pw_msa_args A, int32_t* slot_row) {
  if (blockIdx.x == 0 && threadIdx.x < 4)  // minmax sentinels (no host copy on the stream)
    A.minmax[threadIdx.x] = threadIdx.x == 1 ? -1 : INT_MAX;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x)
    for (int64_t k = A.slot_base[r] + threadIdx.x; k < A.slot_base[r + 1]; k += 256) slot_row[k] = (int32_t)r;
}

// K1: per 256-base chunk of a row, sum of (1 + max(ofs, 0)).  A wavefront takes 8 consecutive
// slots at a time, 8 lanes per slot, 32 bases per lane (four 16-byte loads when the row starts
// 8-base aligned); the next group's loads are issued before this group is reduced.
__device__ __forceinline__ int adv_sum8(v4i q) {  // 8 int16 gaps packed in 16 bytes
  int s = 8;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int lo = (int16_t)(q[w] & 0xFFFF), hi = (int16_t)((uint32_t)q[w] >> 16);
    s += (lo > 0 ? lo : 0) + (hi > 0 ? hi : 0);
  }
  return s;
}
struct SumPre {
  v4i q[4];
  int len, i0;
  uint32_t r;
  bool vec;
};
__device__ __forceinline__ void sums_load(const pw_msa_args& A, const int32_t* slot_row, uint64_t g, int lane, SumPre& p) {
  const uint64_t c = g * 8 + (uint64_t)(lane >> 3);
  p.len = 0;
  p.vec = false;
  if (c >= A.n_slots) return;
  p.r = (uint32_t)slot_row[c];
  const int64_t k = (int64_t)c - A.slot_base[p.r];
  p.len = A.row_len[p.r];
  p.i0 = (int)(k * kChunk) + 32 * (lane & 7);
  const uint64_t roff = A.row_off[p.r];
  p.vec = (roff & 7) == 0 && p.i0 + 32 <= p.len;
  if (p.vec) {
    const v4i* src = reinterpret_cast<const v4i*>(A.ofs + roff + p.i0);
#pragma unroll
    for (int w = 0; w < 4; w++) p.q[w] = src[w];
  } else {
    int s = 0;  // (row tail / unaligned row: element loads, folded into q[0].x)
    for (int i = p.i0; i < p.i0 + 32 && i < p.len; i++) {
      const int gg = A.ofs[roff + i];
      s += 1 + (gg > 0 ? gg : 0);
    }
    p.q[0] = (v4i){s, 0, 0, 0};
  }
}
__global__ __launch_bounds__(256) void row_chunk_sums(const pw_msa_args A, int32_t* chunk_sum, const int32_t* slot_row) {
  const int lane = threadIdx.x & 63;
  const uint64_t ng = (A.n_slots + 7) / 8;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  SumPre cur;
  if (g < ng) sums_load(A, slot_row, g, lane, cur);
  for (; g < ng; g += nw) {
    SumPre nxt;
    if (g + nw < ng) sums_load(A, slot_row, g + nw, lane, nxt);
    int s = 0;
    if (cur.vec) {
#pragma unroll
      for (int w = 0; w < 4; w++) s += adv_sum8(cur.q[w]);
    } else if (cur.len > 0) {
      s = cur.q[0].x;
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    const uint64_t c = g * 8 + (uint64_t)(lane >> 3);
    if ((lane & 7) == 0 && c < A.n_slots) chunk_sum[c] = s;
    cur = nxt;
  }
}

// K2: one 1024-thread workgroup per row: chunk checkpoints (column where chunk k's first gap run
// starts) = col0 + exclusive scan of the chunk sums, row extent, bounds check
// (MSAColumns::operator[], GapAssem.h:366-370).  Thread t owns a contiguous run of chunks.
__global__ __launch_bounds__(1024) void row_prefix(const pw_msa_args A, const int32_t* chunk_sum, int32_t* ckpt) {
  __shared__ int wsum[16];
  const int64_t* chunk_base = A.slot_base;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1];
    const int64_t n = e - b, per = (n + 1023) / 1024;
    const int64_t k0 = b + (int64_t)t * per, k1 = k0 + per < e ? k0 + per : e;
    int mine = 0;
    for (int64_t k = k0; k < k1; k++) mine += chunk_sum[k];
    int incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d, 64);
      if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = A.col0[r];
    for (int w = 0; w < wv; w++) base += wsum[w];
    int run = base + incl - mine;
    for (int64_t k = k0; k < k1; k++) {
      ckpt[k] = run;
      run += chunk_sum[k];
    }
    if (t == 1023) {  // the row's last slot (chunk sum 0) now holds its end column + 1
      const int last = run - 1;
      if (A.row_len[r] > 0 && (A.col0[r] < 0 || last >= A.n_cols)) atomicMin(&A.minmax[2], (int)r);
    }
    __syncthreads();
  }
}

// K3: counts for one column tile.  16 waves share the rows overlapping the tile; a wave walks its
// row's 256-base chunks from the one holding the tile's first column: each lane takes 4
// consecutive bases (one 4-byte + one 8-byte load when the row starts 4-base aligned; the next
// chunk is loaded while this one is counted), a single wave scan of the lanes' column advances
// gives every base its column (the closed form of toMSA, GapAssem.cpp:568-590), and the bases are
// added to the LDS counters (bin from a 256-entry LDS table).  Gap runs (ofs > 0, ~1 % of bases)
// take a ballot-guarded per-lane loop; mincol / maxcol are only evaluated in the chunks holding
// the row's first / last unclipped base.
struct Quad {
  uint32_t s4;  // 4 bases
  v2u g4;       // 4 int16 gaps
};
__device__ __forceinline__ int16_t gap_of(const Quad& q, int j) {
  return (int16_t)((j < 2 ? q.g4.x : q.g4.y) >> (16 * (j & 1)));
}
__device__ __forceinline__ void quad_load(const pw_msa_args& A, uint64_t roff, bool vec, int i, int len, Quad& q) {
  if (vec && i + 3 < len) {
    q.s4 = *reinterpret_cast<const uint32_t*>(A.seq + roff + i);
    q.g4 = *reinterpret_cast<const v2u*>(A.ofs + roff + i);
  } else {
    q.s4 = 0;
    q.g4 = (v2u){0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (i + j < len) {
        q.s4 |= (uint32_t)A.seq[roff + i + j] << (8 * j);
        const uint32_t g = (uint16_t)A.ofs[roff + i + j];
        if (j < 2) q.g4.x |= g << (16 * j);
        else q.g4.y |= g << (16 * (j - 2));
      }
  }
}
constexpr int kTileWaves = 16;
__global__ __launch_bounds__(64 * kTileWaves) void tile_counts(const pw_msa_args A, const int32_t* ckpt) {
  const int64_t* chunk_base = A.slot_base;
  __shared__ int32_t cnt[6 * kTileW];
  __shared__ uint8_t bin_lut[256];  // GAlnColumn::addNuc/addGap bin of every byte, x kTileW
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.x * kTileW;
  const int c1 = min(c0 + kTileW, A.n_cols);
  const uint32_t tw = (uint32_t)(c1 - c0);
  for (int i = tid; i < 6 * kTileW; i += 64 * kTileWaves) cnt[i] = 0;
  if (tid < 256) bin_lut[tid] = (uint8_t)bin_of((uint32_t)tid);
  __syncthreads();
  int my_min = INT_MAX, my_max = -1;
  for (uint32_t r = wv; r < A.n_rows; r += kTileWaves) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1] - 1;  // [b, e) chunks, e = end slot
    if (b == e) continue;
    const int rs = ckpt[b], re = ckpt[e];  // row columns [rs, re)
    if (re <= c0 || rs >= c1) continue;
    const int len = A.row_len[r];
    const int lo = A.clip_l[r], hi = len - A.clip_r[r];  // bases [lo, hi) are counted (unclipped)
    const uint32_t span = hi > lo ? (uint32_t)(hi - lo) : 0u;
    // first chunk whose columns reach c0 (last k with ckpt[k] <= c0): interpolate, then step
    int64_t k = b;
    if (c0 > rs) {
      k = b + (int64_t)((double)(c0 - rs) * (double)(e - b) / (double)(re - rs));
      if (k > e - 1) k = e - 1;
      while (k > b && ckpt[k] > c0) k--;
      while (k + 1 < e && ckpt[k + 1] <= c0) k++;
    }
    const uint64_t roff = A.row_off[r];
    const bool vec = (roff & 3) == 0;
    int col = ckpt[k];
    int i0 = (int)(k - b) * kChunk + 4 * lane;  // this lane's first base of the chunk
    Quad nx;
    quad_load(A, roff, vec, i0, len, nx);
    for (; k < e && col < c1; k++, i0 += kChunk) {
      const Quad q = nx;
      if (k + 1 < e) quad_load(A, roff, vec, i0 + kChunk, len, nx);
      int adv[4], gp[4];
      int tot = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int g = gap_of(q, j);
        gp[j] = g > 0 ? g : 0;
        adv[j] = (i0 + j < len) ? 1 + gp[j] : 0;
        tot += adv[j];
      }
      const int incl = wave_scan_incl(tot);
      int run = col + incl - tot;
      int bcol[4];
      bool take[4];
      bool gaps = false;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        run += adv[j];
        bcol[j] = run - 1;  // this base's column; its gap run is [bcol - gp, bcol)
        take[j] = (uint32_t)(i0 + j - lo) < span;
        gaps = gaps || (take[j] && gp[j] > 0);
        const uint32_t o = (uint32_t)(bcol[j] - c0);
        if (take[j] && o < tw) atomicAdd(&cnt[bin_lut[(q.s4 >> (8 * j)) & 0xFFu] * kTileW + o], 1);
      }
      // mincol / maxcol: only the chunks holding the first / last unclipped base
      const int cb = (int)(k - b) * kChunk;
      if ((uint32_t)(lo - cb) < (uint32_t)kChunk || (uint32_t)(hi - 1 - cb) < (uint32_t)kChunk) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (take[j] && i0 + j == lo) my_min = min(my_min, bcol[j] - gp[j]);
          if (take[j] && i0 + j == hi - 1) my_max = max(my_max, bcol[j]);
        }
      }
      if (__ballot(gaps)) {
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (take[j] && gp[j] > 0)
            for (int c = max(bcol[j] - gp[j], c0); c < bcol[j] && c < c1; c++) atomicAdd(&cnt[5 * kTileW + c - c0], 1);
      }
      col += wave_last(incl);
    }
  }
  // fold mincol / maxcol
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    my_min = min(my_min, __shfl_xor(my_min, d, 64));
    my_max = max(my_max, __shfl_xor(my_max, d, 64));
  }
  if (lane == 0) {
    if (my_min != INT_MAX) atomicMin(&A.minmax[0], my_min);
    if (my_max >= 0) atomicMax(&A.minmax[1], my_max);
  }
  __syncthreads();
  // the tile's counters, coalesced: column-major in LDS -> [col][6] rows in memory
  int32_t* dst = A.counts + (int64_t)c0 * 6;
  for (int i = tid; i < (c1 - c0) * 6; i += 64 * kTileWaves) dst[i] = cnt[(i % 6) * kTileW + i / 6];
}

// bestChar of each column (GapAssem.cpp:1048-1069 in closed form); 0 = no coverage
__global__ __launch_bounds__(256) void call_columns(const pw_msa_args A, int32_t lo, int32_t hi) {
  for (int64_t c = lo + (int64_t)blockIdx.x * 256 + threadIdx.x; c < hi; c += (int64_t)gridDim.x * 256) {
    int v[6];
    const int32_t* src = A.counts + c * 6;
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = src[q];
    const int layers = v[0] + v[1] + v[2] + v[3] + v[4] + v[5];
    uint8_t best = 0;
    if (layers > 0) {
      int m = v[0], bi = 0;
#pragma unroll
      for (int q = 1; q < 6; q++)
        if (v[q] > m) {
          m = v[q];
          bi = q;
        }
      best = (uint8_t)"ACGTN-"[bi];
      if (bi == 4 && v[5] == m) best = '-';
    }
    A.consensus[c] = best;
  }
}

// (columns [c_lo, c_hi) of the consensus are this call's: the whole layout, or a rank's range)
__global__ __launch_bounds__(256) void zero_scan(const pw_msa_args A, int32_t c_lo, int32_t c_hi) {
  const int lo = max(A.minmax[0], c_lo), hi = min(A.minmax[1], c_hi - 1);
  for (int c = lo + blockIdx.x * 256 + threadIdx.x; c <= hi; c += gridDim.x * 256)
    if (c >= 0 && c < A.n_cols && A.consensus[c] == 0) atomicMin(&A.minmax[3], c);
}

// ---------------------------------------------------------------- refineMSA (pw_msa_refine)
__device__ __forceinline__ bool cons_gap(const pw_msa_args& A, int lo, int hi, int c) {
  return c >= lo && c <= hi && A.consensus[c] == '-';
}

// K6: consensus-gap columns per 2048-column tile
__global__ __launch_bounds__(256) void gap_tiles(const pw_msa_args A, pw_msa_refine_args R) {
  __shared__ int part[4];
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

static bool msa_args_ok(const pw_msa_args* a) {
  return a && a->seq && a->ofs && a->row_off && a->row_len && a->col0 && a->clip_l && a->clip_r && a->slot_base &&
         a->scratch && a->counts && a->consensus && a->minmax && a->n_rows > 0 && a->n_cols > 0 &&
         a->n_slots >= a->n_rows;
}

extern "C" int pw_msa_count(const pw_msa_args* a, void* stream) {
  if (!msa_args_ok(a)) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  int32_t* chunk_sum = a->scratch;
  int32_t* ckpt = a->scratch + a->n_slots;
  int32_t* slot_row = a->scratch + 2 * a->n_slots;
  hipLaunchKernelGGL(pw::slot_rows, dim3(a->n_rows < 8192 ? a->n_rows : 8192), dim3(256), 0, s, *a, slot_row);
  const uint64_t nb1 = ((a->n_slots + 7) / 8 + 3) / 4;  // 8 slots per wave, 4 waves per workgroup
  hipLaunchKernelGGL(pw::row_chunk_sums, dim3((unsigned)(nb1 < 4096 ? nb1 : 4096)), dim3(256), 0, s, *a,
                     chunk_sum, slot_row);
  hipLaunchKernelGGL(pw::row_prefix, dim3(a->n_rows < 4096 ? a->n_rows : 4096), dim3(1024), 0, s, *a, chunk_sum, ckpt);
  const unsigned ntiles = (unsigned)((a->n_cols + pw::kTileW - 1) / pw::kTileW);
  hipLaunchKernelGGL(pw::tile_counts, dim3(ntiles), dim3(64 * pw::kTileWaves), 0, s, *a, ckpt);
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
  hipLaunchKernelGGL(pw::zero_scan, dim3(256), dim3(256), 0, s, b, col_lo, col_hi);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}

extern "C" int pw_msa_call(const pw_msa_args* a, void* stream) {
  if (!msa_args_ok(a)) return PW_E_ARG;
  return pw_msa_call_cols(a, 0, a->n_cols, nullptr, stream);
}

extern "C" int pw_msa_columns(const pw_msa_args* a, void* stream) {
  const int rc = pw_msa_count(a, stream);
  return rc != PW_OK ? rc : pw_msa_call(a, stream);
}

extern "C" uint64_t pw_msa_refine_tiles(int32_t n_cols) { return n_cols > 0 ? ((uint64_t)n_cols + pw::kTileW - 1) / pw::kTileW : 0; }

extern "C" int pw_msa_refine(const pw_msa_args* a, const pw_msa_refine_args* r, void* stream) {
  if (!msa_args_ok(a) || !r || !r->gap_prefix || !r->tile_gaps || !r->cons_out || !r->cons_len) return PW_E_ARG;
  if (r->remove_gaps && (!r->row_offset || !r->ofs_out || !r->offset_out || !r->numgaps_out)) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(r->cons_len, 0, sizeof(int32_t), s) != hipSuccess) return PW_E_HIP;
  const unsigned ntiles = (unsigned)pw_msa_refine_tiles(a->n_cols);
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
