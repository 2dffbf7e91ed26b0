// pw_msa.hip — GapAssem column consensus on gfx950.
//
// Reference (gpertea/pwasm GapAssem):
//   GASeq::toMSA            GapAssem.cpp:551-591   row -> columns (gap runs + bases, clipping)
//   GAlnColumn::addGap/Nuc  GapAssem.h:295-337     6 counters A,C,G,T,N,- (+ layers)
//   GAlnColumn::bestChar    GapAssem.cpp:1048-1069 stable qsort + N/- tie rule
//   GSeqAlign::buildMSA     GapAssem.cpp:1088-1106
// The reference scatters row by row (one NucOri allocation per base).  Here the layout is
// read once, column tile by column tile:
//   K1 row_chunk_sums: per 256-base chunk of a row, sum of (1 + max(ofs,0))   (1 wave / chunk)
//   K2 row_prefix:     per row, exclusive scan of the chunk sums -> layout column at which each
//                      chunk's first gap run starts (checkpoints), row end column, bounds check
//   K3 tile_counts:    one 256-thread workgroup per 2048-column tile keeps the tile's 6 x 2048
//                      counters in LDS; its 4 waves walk the chunks of every row that overlaps
//                      the tile (binary search on the checkpoints), re-derive columns with a
//                      wave scan and add into LDS; then the tile writes counts + bestChar
//                      coalesced and folds mincol / maxcol.
//   K4 zero_scan:      first zero-coverage column in [mincol, maxcol] (ErrZeroCov, :1121-1131).
// Column-closed form of bestChar: max count wins, ties resolved A<C<G<T; a tie between only N
// and '-' gives '-' (glibc qsort of 6 elements is a stable merge sort).
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "pwasm_amd.h"

namespace pw {

constexpr int kChunk = 256;   // bases per checkpoint chunk
constexpr int kTileW = 2048;  // columns per workgroup

__device__ __forceinline__ int bin_of(uint8_t c) {
  if (c >= 'a' && c <= 'z') c -= 32;
  switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case '-':
    case '*': return 5;
    default: return 4;
  }
}

// per row: number of chunks = ceil(len / 256); chunk index space = prefix over rows
__global__ __launch_bounds__(256) void row_chunk_sums(const pw_msa_args A, int32_t* chunk_sum) {
  const int64_t* chunk_base = A.slot_base;
  const uint64_t n_chunks = A.n_slots;
  const int lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (uint64_t c = wid; c < n_chunks; c += (uint64_t)gridDim.x * 4) {
    // find the row of chunk c (binary search in chunk_base[0..n_rows])
    uint32_t lo = 0, hi = A.n_rows;
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if ((uint64_t)chunk_base[mid] <= c) lo = mid;
      else hi = mid;
    }
    const uint32_t r = lo;
    const int64_t k = (int64_t)c - chunk_base[r];
    const int len = A.row_len[r];
    const int64_t i0 = k * kChunk;
    int s = 0;
#pragma unroll
    for (int j = 0; j < kChunk / 64; j++) {
      const int64_t i = i0 + j * 64 + lane;
      if (i < len) {
        const int g = A.ofs[A.row_off[r] + i];
        s += 1 + (g > 0 ? g : 0);
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if (lane == 0) chunk_sum[c] = s;
  }
}

// one 64-thread workgroup per row: chunk checkpoints (column where chunk k's first gap run
// starts), row extent, bounds check (MSAColumns::operator[], GapAssem.h:366-370)
__global__ __launch_bounds__(64) void row_prefix(const pw_msa_args A, const int32_t* chunk_sum, int32_t* ckpt) {
  const int64_t* chunk_base = A.slot_base;
  const int lane = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1];
    int carry = A.col0[r];
    for (int64_t k0 = b; k0 < e; k0 += 64) {
      const int64_t k = k0 + lane;
      const int v = (k < e) ? chunk_sum[k] : 0;
      int incl = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
      }
      if (k < e) ckpt[k] = carry + incl - v;
      carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) {  // the row's last slot (chunk sum 0) now holds its end column + 1
      const int last = carry - 1;
      if (A.row_len[r] > 0 && (A.col0[r] < 0 || last >= A.n_cols)) {
        atomicMin(&A.minmax[2], (int)r);  // first offending row; host reports the column
      }
    }
  }
}

// counts for one column tile
__global__ __launch_bounds__(256) void tile_counts(const pw_msa_args A, const int32_t* ckpt) {
  const int64_t* chunk_base = A.slot_base;
  __shared__ int32_t cnt[6][kTileW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c0 = blockIdx.x * kTileW;
  const int c1 = min(c0 + kTileW, A.n_cols);
  for (int i = tid; i < 6 * kTileW; i += 256) (&cnt[0][0])[i] = 0;
  __syncthreads();
  int my_min = INT_MAX, my_max = -1;
  for (uint32_t r = wv; r < A.n_rows; r += 4) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1] - 1;  // [b, e) chunks, e = end slot
    if (b == e) continue;
    const int rs = ckpt[b], re = ckpt[e];  // row columns [rs, re)
    if (re <= c0 || rs >= c1) continue;
    const int len = A.row_len[r];
    const int cl = A.clip_l[r], cr = A.clip_r[r];
    // first chunk whose columns reach c0: last k with ckpt[k] <= c0
    int64_t lo = b, hi = e;
    while (hi - lo > 1) {
      int64_t mid = (lo + hi) >> 1;
      if (ckpt[mid] <= c0) lo = mid;
      else hi = mid;
    }
    const uint64_t roff = A.row_off[r];
    for (int64_t k = lo; k < e && ckpt[k] < c1; k++) {
      const int64_t ib = (k - b) * kChunk;
      int col = ckpt[k];
#pragma unroll
      for (int j = 0; j < kChunk / 64; j++) {
        const int64_t i = ib + j * 64 + lane;
        const bool ok = i < len;
        const int g0 = ok ? A.ofs[roff + i] : 0;
        const int g = g0 > 0 ? g0 : 0;
        const uint8_t ch = ok ? A.seq[roff + i] : 0;
        const int adv = ok ? 1 + g : 0;
        int incl = adv;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          int t = __shfl_up(incl, d, 64);
          if (lane >= d) incl += t;
        }
        const int bcol = col + incl - 1;  // this base's column
        const int gstart = bcol - g;      // its gap run starts here
        if (ok) {
          const bool clipped = (i < cl) || (i >= len - cr);
          if (!clipped) {
            for (int c = gstart > c0 ? gstart : c0; c < bcol && c < c1; c++) atomicAdd(&cnt[5][c - c0], 1);
            if (bcol >= c0 && bcol < c1) atomicAdd(&cnt[bin_of(ch)][bcol - c0], 1);
            if (i == cl) my_min = min(my_min, gstart);
            if (i == len - cr - 1) my_max = max(my_max, bcol);
          }
        }
        col += __shfl(incl, 63, 64);
      }
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
  for (int c = c0 + tid; c < c1; c += 256) {
    int v[6];
#pragma unroll
    for (int q = 0; q < 6; q++) v[q] = cnt[q][c - c0];
    int32_t* dst = A.counts + (int64_t)c * 6;
#pragma unroll
    for (int q = 0; q < 6; q++) dst[q] = v[q];
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

__global__ __launch_bounds__(256) void zero_scan(const pw_msa_args A) {
  const int lo = A.minmax[0], hi = A.minmax[1];
  for (int c = lo + blockIdx.x * 256 + threadIdx.x; c <= hi; c += gridDim.x * 256)
    if (c >= 0 && c < A.n_cols && A.consensus[c] == 0) atomicMin(&A.minmax[3], c);
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

extern "C" int pw_msa_columns(const pw_msa_args* a, void* stream) {
  if (!a || !a->seq || !a->ofs || !a->row_off || !a->row_len || !a->col0 || !a->clip_l || !a->clip_r ||
      !a->slot_base || !a->scratch || !a->counts || !a->consensus || !a->minmax)
    return PW_E_ARG;
  if (a->n_rows == 0 || a->n_cols <= 0 || a->n_slots < a->n_rows) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  int32_t* chunk_sum = a->scratch;
  int32_t* ckpt = a->scratch + a->n_slots;
  static const int32_t init[4] = {INT_MAX, -1, INT_MAX, INT_MAX};
  if (hipMemcpyAsync(a->minmax, init, sizeof init, hipMemcpyHostToDevice, s) != hipSuccess) return PW_E_HIP;
  const uint64_t nb1 = (a->n_slots + 3) / 4;
  hipLaunchKernelGGL(pw::row_chunk_sums, dim3((unsigned)(nb1 < 65536 ? nb1 : 65536)), dim3(256), 0, s, *a,
                     chunk_sum);
  hipLaunchKernelGGL(pw::row_prefix, dim3(a->n_rows < 4096 ? a->n_rows : 4096), dim3(64), 0, s, *a, chunk_sum, ckpt);
  const unsigned ntiles = (unsigned)((a->n_cols + pw::kTileW - 1) / pw::kTileW);
  hipLaunchKernelGGL(pw::tile_counts, dim3(ntiles), dim3(256), 0, s, *a, ckpt);
  hipLaunchKernelGGL(pw::zero_scan, dim3(256), dim3(256), 0, s, *a);
  return hipGetLastError() == hipSuccess ? PW_OK : PW_E_HIP;
}
