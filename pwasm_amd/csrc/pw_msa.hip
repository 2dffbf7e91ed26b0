// pw_msa.hip — GapAssem column consensus on gfx950.
//
// Reference (gpertea/pwasm GapAssem):
//   GASeq::toMSA            GapAssem.cpp:551-591   row -> columns (gap runs + bases, clipping)
//   GAlnColumn::addGap/Nuc  GapAssem.h:295-337     6 counters A,C,G,T,N,- (+ layers)
//   GAlnColumn::bestChar    GapAssem.cpp:1048-1069 stable qsort + N/- tie rule
//   GSeqAlign::buildMSA     GapAssem.cpp:1088-1106
// The reference scatters row by row (one NucOri allocation per base).  Here ofs is read once and
// seq once per pass, column tile by column tile:
//   K0 slot_rows:      row of every chunk slot (no per-chunk binary search later)
//   K1 row_chunk_sums: per 256-base chunk of a row, sum of (1 + max(ofs,0)) and the chunk's list
//                      of positive gaps (<= 8 entries, 32 B per 256 bases)
//   K2 row_prefix:     per row, exclusive scan of the chunk sums -> layout column at which each
//                      chunk's first gap run starts (checkpoints), row end column, bounds check,
//                      the row's counted column extent, mincol / maxcol
//   K3 tile_counts:    one 1024-thread workgroup per 2048-column tile; its 16 waves walk the
//                      chunks of every row that overlaps the tile, place each base's bin code in
//                      a per-wave LDS column strip (columns from the checkpoint + gap list, no
//                      scan), then count the strip into packed register counters; no LDS atomic
//                      per base.  The tile writes its counts coalesced.
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

// K1: per 256-base chunk of a row, sum of (1 + max(ofs, 0)) and the chunk's gap list: the
// (base index in chunk, gap) of every ofs > 0 (~1 % of bases in an assembly layout), at most
// kGapCap per chunk, unordered, 0 = unused, kGapOverflow in entry 0 when a chunk has more (K3
// then re-reads that chunk's ofs).  K3 reads these 32 bytes per chunk instead of 512 bytes of
// ofs, so the layout's ofs is read once per pass.  A wavefront takes 8 consecutive slots at a
// time, 8 lanes per slot, 32 bases per lane (four 16-byte loads when the row starts 8-base
// aligned); the next group's loads are issued before this group is reduced.
constexpr int kGapCap = 8;
constexpr uint32_t kGapOverflow = 0xFFFFFFFFu;
struct SumPre {
  v4i q[4];
  uint64_t roff;
  int len, i0;
  int s;        // (element path) the sum
  uint32_t pm;  // (element path) bit t: base i0 + t has ofs > 0
  bool vec;
};
__device__ __forceinline__ void sums_load(const pw_msa_args& A, const int32_t* slot_row, uint64_t g, int lane, SumPre& p) {
  const uint64_t c = g * 8 + (uint64_t)(lane >> 3);
  p.len = 0;
  p.vec = false;
  p.s = 0;
  p.pm = 0;
  if (c >= A.n_slots) return;
  const uint32_t r = (uint32_t)slot_row[c];
  const int64_t k = (int64_t)c - A.slot_base[r];
  p.len = A.row_len[r];
  p.i0 = (int)(k * kChunk) + 32 * (lane & 7);
  p.roff = A.row_off[r];
  p.vec = (p.roff & 7) == 0 && p.i0 + 32 <= p.len;
  if (p.vec) {
    const v4i* src = reinterpret_cast<const v4i*>(A.ofs + p.roff + p.i0);
#pragma unroll
    for (int w = 0; w < 4; w++) p.q[w] = src[w];
  } else {
    for (int i = p.i0; i < p.i0 + 32 && i < p.len; i++) {  // row tail / unaligned row
      const int gg = A.ofs[p.roff + i];
      p.s += 1 + (gg > 0 ? gg : 0);
      p.pm |= gg > 0 ? 1u << (i - p.i0) : 0u;
    }
  }
}
__global__ __launch_bounds__(256) void row_chunk_sums(const pw_msa_args A, int32_t* chunk_sum, const int32_t* slot_row,
                                                      uint32_t* glist) {
  const int lane = threadIdx.x & 63, sub = lane & 7;
  const uint64_t ng = (A.n_slots + 7) / 8;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  SumPre cur;
  if (g < ng) sums_load(A, slot_row, g, lane, cur);
  for (; g < ng; g += nw) {
    SumPre nxt;
    if (g + nw < ng) sums_load(A, slot_row, g + nw, lane, nxt);
    int s = cur.s;
    uint32_t pm = cur.pm;
    if (cur.vec) {
      s = 32;
#pragma unroll
      for (int w = 0; w < 16; w++) {
        const uint32_t d = (uint32_t)cur.q[w >> 2][w & 3];
        const int lo = max((int)(int16_t)(d & 0xFFFFu), 0), hi = max((int)(int16_t)(d >> 16), 0);
        s += lo + hi;
        pm |= (uint32_t)min(lo, 1) << (2 * w) | (uint32_t)min(hi, 1) << (2 * w + 1);
      }
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    // gap-list slots: exclusive prefix of the 8 lanes' counts
    const int n = __popc(pm);
    int incl = n;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      const int t = __shfl_up(incl, d, 64);
      if (sub >= d) incl += t;
    }
    const int total = __shfl(incl, lane | 7, 64);
    const uint64_t c = g * 8 + (uint64_t)(lane >> 3);
    if (c < A.n_slots) {
      if (sub == 0) chunk_sum[c] = s;
      uint32_t* gl = glist + c * kGapCap;
      if (total > kGapCap) {
        if (sub == 0) gl[0] = kGapOverflow;
      } else {
        if (sub >= total) gl[sub] = 0u;
        int slot = incl - n;
        const uint32_t base = (uint32_t)(32 * sub);
        while (pm) {  // (~0.3 per lane)
          const int t = __builtin_ctz(pm);
          pm &= pm - 1;
          uint32_t gg;
          if (cur.vec) {  // from the registers: dword t / 2 of the 16 (a select tree, no reload)
            const int d = t >> 1;
            uint32_t w4[4];
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const v4i& v = cur.q[w];
              w4[w] = (uint32_t)((d & 2) ? ((d & 1) ? v.w : v.z) : ((d & 1) ? v.y : v.x));
            }
            const uint32_t dw = (d & 8) ? ((d & 4) ? w4[3] : w4[2]) : ((d & 4) ? w4[1] : w4[0]);
            gg = (t & 1) ? dw >> 16 : dw & 0xFFFFu;
          } else {
            gg = (uint32_t)(uint16_t)A.ofs[cur.roff + cur.i0 + t];
          }
          gl[slot++] = (base + (uint32_t)t) << 16 | gg;
        }
      }
    }
    cur = nxt;
  }
}

// K2: one 1024-thread workgroup per row: chunk checkpoints (column where chunk k's first gap run
// starts) = col0 + exclusive scan of the chunk sums, row extent, bounds check
// (MSAColumns::operator[], GapAssem.h:366-370).  Thread t owns a contiguous run of chunks.
// Also K3's row record rinfo[8r..8r+7] = {ext_lo, ext_hi, first column, end column + 1, length,
// chunks, first slot (2 words)}, where [ext_lo, ext_hi] = [first column of the gap run before
// base lo, column of base hi - 1] is the counted extent of the unclipped bases [lo, hi) (empty:
// ext_lo > ext_hi), and mincol / maxcol (minmax[0] / [1]: GSeqAlign's minoffset/length
// bookkeeping over the bases toMSA counts): waves 0 / 1 scan the chunk holding lo / hi - 1.
__device__ __forceinline__ int chunk_cols_upto(const pw_msa_args& A, uint64_t roff, int i0, int i_end, int lane) {
  // sum over bases [i0, i_end) of 1 + max(ofs, 0) (i_end - i0 <= kChunk), wave-uniform result
  int s = 0;
#pragma unroll
  for (int j = 0; j < kChunk / 64; j++) {
    const int i = i0 + j * 64 + lane;
    if (i < i_end) s += 1 + max((int)A.ofs[roff + i], 0);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  return s;
}
constexpr int kRowInfo = 8;  // int32 words per row record
__global__ __launch_bounds__(1024) void row_prefix(const pw_msa_args A, const int32_t* chunk_sum, int32_t* ckpt,
                                                   int32_t* rinfo) {
  __shared__ int wsum[16];
  __shared__ int ck_s[2];
  const int64_t* chunk_base = A.slot_base;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (uint32_t r = blockIdx.x; r < A.n_rows; r += gridDim.x) {
    const int64_t b = chunk_base[r], e = chunk_base[r + 1];
    const int64_t n = e - b, per = (n + 1023) / 1024;
    const int64_t k0 = b + (int64_t)t * per, k1 = k0 + per < e ? k0 + per : e;
    const int len = A.row_len[r];
    const int lo = max(A.clip_l[r], 0), hi = min(len - A.clip_r[r], len);  // counted bases [lo, hi)
    const int64_t klo = b + lo / kChunk, khi = b + (hi - 1) / kChunk;
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
    int32_t* ri = rinfo + (int64_t)kRowInfo * r;
    if (t == 0) {
      int end = A.col0[r];
      for (int w = 0; w < 16; w++) end += wsum[w];
      ri[2] = A.col0[r];
      ri[3] = end;
      ri[4] = len;
      ri[5] = (int)(e - 1 - b);
      ri[6] = (int)(uint32_t)(uint64_t)b;
      ri[7] = (int)(uint32_t)((uint64_t)b >> 32);
    }
    for (int64_t k = k0; k < k1; k++) {
      if (k == klo) ck_s[0] = run;
      if (k == khi) ck_s[1] = run;
      ckpt[k] = run;
      run += chunk_sum[k];
    }
    if (t == 1023) {  // the row's last slot (chunk sum 0) now holds its end column + 1
      const int last = run - 1;
      if (len > 0 && (A.col0[r] < 0 || last >= A.n_cols)) atomicMin(&A.minmax[2], (int)r);
    }
    __syncthreads();
    if (wv < 2) {
      const uint64_t roff = A.row_off[r];
      if (hi <= lo) {
        if (lane == 0) ri[wv] = wv == 0 ? 1 : 0;
      } else if (wv == 0) {  // gap-run start of base lo
        const int i0 = (lo / kChunk) * kChunk;
        const int x = ck_s[0] + chunk_cols_upto(A, roff, i0, lo, lane);
        if (lane == 0) {
          ri[0] = x;
          if (A.clip_l[r] >= 0) atomicMin(&A.minmax[0], x);
        }
      } else {  // column of base hi - 1
        const int i0 = ((hi - 1) / kChunk) * kChunk;
        const int x = ck_s[1] + chunk_cols_upto(A, roff, i0, hi, lane) - 1;
        if (lane == 0) {
          ri[1] = x;
          if (A.clip_r[r] >= 0) atomicMax(&A.minmax[1], x);
        }
      }
    }
    __syncthreads();
  }
}

// K3: counts for one 2048-column tile, with no LDS atomic per base.  16 waves share the rows
// overlapping the tile (row r -> wave r % 16; the next row's K2 record is prefetched).  For one
// row a wave fetches, in one round trip, a batch of up to kBatch chunks starting 2 before the
// chunk its mean column density predicts for the tile's first counted column (checkpoints into
// one VGPR, gap lists into two, 4 bases per lane per chunk into registers), finds the true first
// chunk with a ballot over the checkpoints, and walks the chunks: each lane's 4 consecutive
// bases get their columns from the chunk's checkpoint (K2) plus its gap list (K1): an entry
// (i, g) moves every base from i on by g columns — the closed form of toMSA,
// GapAssem.cpp:568-590.  A batch holding a chunk whose list overflowed, or a row not 4-base
// aligned, takes a general loop that re-reads ofs and scans instead.  Each base writes its bin code (GAlnColumn::addNuc, bin_codes4: in
// registers, 4 bases at a time) into the wave's 2 KB column strip, one byte per column.  The strip's reset value is
// the gap code: the columns of the row's counted extent that receive no base are exactly its
// gap runs (GAlnColumn::addGap); columns outside the extent (K2's ext) are set to "none" in the
// tiles where the extent starts or ends.  Then each lane reads the 32 columns it owns (two
// 16-byte LDS reads), adds them to 32 packed register counters (six 10-bit fields in a u64: one
// shift-add per column) and resets the strip.  The counters move to the workgroup's LDS table
// every 1023 rows and at the end (packed u64 adds when the layout has at most 1023 rows); the
// tile is then written coalesced.  mincol / maxcol come from K2.
constexpr int kCntW = 2048;
constexpr int kCntWaves = 16;
constexpr uint32_t kCodeGap = 50u, kCodeNone = 60u;  // bit offsets: A,C,G,T,N,- at 0,10,..,50
constexpr int kPackRows = 1023;                       // 10-bit fields
// LDS index of column c in the tile table: conflict-free both for the flush (lanes l own
// columns 16l + m) and for the read-out (consecutive columns)
__device__ __forceinline__ int cnt_swz(int c) { return (c & 15) * (kCntW / 16) + (((c >> 4) + 2 * (c & 15)) & (kCntW / 16 - 1)); }
__device__ __forceinline__ uint32_t seq4(const pw_msa_args& A, uint64_t roff, bool vec, int i, int len) {
  if (vec && i + 3 < len) return *reinterpret_cast<const uint32_t*>(A.seq + roff + i);
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 4; j++)
    if (i + j < len) s |= (uint32_t)A.seq[roff + i + j] << (8 * j);
  return s;
}
// lane's columns: m < 16 -> 16 * lane + m, m >= 16 -> 1024 + 16 * lane + m - 16
__device__ __forceinline__ int acc_col(int lane, int m) { return (m < 16 ? 0 : kCntW / 2) + 16 * lane + (m & 15); }
__device__ __forceinline__ void cnt_flush(uint64_t (&acc)[32], uint32_t* tab, bool packed, int lane) {
  if (packed) {
    unsigned long long* pk = reinterpret_cast<unsigned long long*>(tab);
#pragma unroll
    for (int m = 0; m < 32; m++) {
      atomicAdd(&pk[cnt_swz(acc_col(lane, m))], (unsigned long long)(acc[m] & ((1ull << 60) - 1)));
      acc[m] = 0;
    }
  } else {
#pragma unroll
    for (int m = 0; m < 32; m++) {
      const int x = cnt_swz(acc_col(lane, m));
#pragma unroll
      for (int f = 0; f < 6; f++) atomicAdd(&tab[f * kCntW + x], (uint32_t)(acc[m] >> (10 * f)) & 1023u);
      acc[m] = 0;
    }
  }
}
// the bin codes (10 x GAlnColumn::addNuc/addGap bin, as bin_of) of 4 bases in a dword, in
// registers: h = (c >> 1) & 7 picks, per byte, the only characters that can have each bin
// (A/a 0, C/c 1, T/t 2, G/g 3, '*' 5, '-' 6; 4 and 7 none) and v_perm looks up the code, the
// expected character and its case mask; a byte that is not its h's character is N (40)
__device__ __forceinline__ uint32_t bin_codes4(uint32_t s4) {
  const uint32_t h = (s4 >> 1) & 0x07070707u;
  const uint32_t code = __builtin_amdgcn_perm(0x28323228u, 0x141E0A00u, h);  // 0 10 30 20 | 40 50 50 40
  const uint32_t ex = __builtin_amdgcn_perm(0x002D2A00u, 0x47544341u, h);    // A C T G | - * - -
  const uint32_t mk = __builtin_amdgcn_perm(0xFFFFFFFFu, 0xDFDFDFDFu, h);    // letters: either case
  const uint32_t x = (s4 & mk) ^ ex;                                         // 0 byte: the character
  const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // 0x80: not it
  const uint32_t m = (nz << 1) - (nz >> 7);                                  // 0xFF per such byte
  return (m & 0x28282828u) | (~m & code);
}
// one chunk: the columns of this lane's 4 bases (relative to the tile) from the chunk's start
// column and gap list (entries gl(x), x < kGapCap; 0 = unused), or from ofs and a scan
template <bool kAny, class GL>
__device__ __forceinline__ void place_chunk(const pw_msa_args& A, uint64_t roff, bool fast, GL gl, uint32_t s4,
                                            int colr, int cnr, int kb, int len, int ar, int zr, int lane,
                                            uint8_t* myb) {
  const int i0 = kb + 4 * lane;
  int p[4];
  if (!kAny || fast) {
    // gb: entries at or before this lane's first base; i1..i3: entries inside its quad (lane qe)
    int gb = 0, i1 = 0, i2 = 0, i3 = 0;
#pragma unroll
    for (int x = 0; x < kGapCap; x++) {
      const uint32_t v = gl(x);
      if (v == 0) break;
      const int idx = (int)(v >> 16), gg = (int)(v & 0xFFFFu);
      gb += 4 * lane >= idx ? gg : 0;
      const int qe = idx >> 2, je = idx & 3;
      if (je != 0) {
        const int add = lane == qe ? gg : 0;
        if (je <= 1) i1 += add;
        if (je <= 2) i2 += add;
        i3 += add;
      }
    }
    p[0] = colr + 4 * lane + gb;
    p[1] = p[0] + 1 + i1;
    p[2] = p[0] + 2 + i2;
    p[3] = p[0] + 3 + i3;
  } else {  // overflowed gap list / unaligned row: ofs and a wave scan
    int gp[4], tot = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const bool ok = i0 + j < len;
      gp[j] = ok ? max((int)A.ofs[roff + i0 + j], 0) : 0;
      tot += ok ? 1 + gp[j] : 0;
    }
    const int incl = wave_scan_incl(tot);
    int run = colr + incl - tot;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      run += (i0 + j < len) ? 1 + gp[j] : 0;
      p[j] = run - 1;
    }
  }
  const bool all = kb + kChunk <= len && colr >= ar && cnr - 1 <= zr;  // (wave-uniform)
  const uint32_t code4 = bin_codes4(s4);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (all || (i0 + j < len && p[j] >= ar && p[j] <= zr)) myb[p[j]] = (uint8_t)(code4 >> (8 * j));
  }
}
constexpr int kBatch = 14;  // chunks fetched per round trip (a 2048-column tile spans ~8-9)
__global__ __launch_bounds__(64 * kCntWaves) void tile_counts(const pw_msa_args A, const int32_t* __restrict__ ckpt,
                                                              const uint32_t* __restrict__ glist,
                                                              const int32_t* __restrict__ rinfo) {
  __shared__ uint32_t strip[kCntWaves * kCntW / 4];
  __shared__ uint32_t tab[6 * kCntW];  // u32 counters [field][swz col], or packed u64 [swz col]
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.x * kCntW;
  const int c1 = min(c0 + kCntW, A.n_cols);
  const bool packed = A.n_rows <= (uint32_t)kPackRows;
  for (int i = tid; i < 6 * kCntW; i += 64 * kCntWaves) tab[i] = 0;
  for (int i = tid; i < kCntWaves * kCntW / 4; i += 64 * kCntWaves) strip[i] = kCodeGap * 0x01010101u;
  __syncthreads();
  uint32_t* my = strip + wv * (kCntW / 4);
  uint8_t* myb = reinterpret_cast<uint8_t*>(my);  // myb[c - c0]: column c
  uint64_t acc[32];
#pragma unroll
  for (int m = 0; m < 32; m++) acc[m] = 0;
  int nrow = 0;
  const uint4* ri4 = reinterpret_cast<const uint4*>(rinfo);
  uint4 nx0 = make_uint4(0, 0, 0, 0), nx1 = nx0;  // the next row's record (prefetched)
  uint64_t nroff = 0;
  if ((uint32_t)wv < A.n_rows) {
    nx0 = ri4[2 * wv];
    nx1 = ri4[2 * wv + 1];
    nroff = A.row_off[wv];
  }
  for (uint32_t r = wv;; r += kCntWaves) {
    const bool end = r >= A.n_rows;
    if (end || nrow == kPackRows) {  // the counters' one flush site: every kPackRows rows, and the end
      if (nrow) cnt_flush(acc, tab, packed, lane);
      nrow = 0;
      if (end) break;
    }
    const int elo = __builtin_amdgcn_readfirstlane((int)nx0.x), ehi = __builtin_amdgcn_readfirstlane((int)nx0.y);
    const int rs = __builtin_amdgcn_readfirstlane((int)nx0.z), re = __builtin_amdgcn_readfirstlane((int)nx0.w);
    const int len = __builtin_amdgcn_readfirstlane((int)nx1.x), nch = __builtin_amdgcn_readfirstlane((int)nx1.y);
    const int64_t b = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)nx1.z) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)nx1.w) << 32);
    const uint64_t roff = nroff;
    if (r + kCntWaves < A.n_rows) {
      nx0 = ri4[2 * (r + kCntWaves)];
      nx1 = ri4[2 * (r + kCntWaves) + 1];
      nroff = A.row_off[r + kCntWaves];
    }
    const int a = max(elo, c0), z = min(ehi, c1 - 1);  // counted columns of this row here
    if (a > z) continue;
    const int ar = a - c0, zr = z - c0;
    if (a > c0 || z < c1 - 1) {  // the extent starts or ends in this tile
      for (int x = lane; x < kCntW / 4; x += 64) {
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int c = c0 + 4 * x + q;
          w |= ((c < a || c > z) ? kCodeNone : kCodeGap) << (8 * q);
        }
        my[x] = w;
      }
    }
    const bool vec = (roff & 3) == 0;
    // first chunk reaching column a (the last with start column <= a), guessed from the row's mean
    // column density; a batch starts 2 chunks before the guess
    const double dens = (double)nch / (double)(re - rs);  // chunks per column
    int ks = a > rs ? (int)((double)(a - rs) * dens) - 2 : 0;
    ks = min(max(ks, 0), nch - 1);
    bool exact = false;  // ks is the first chunk
    for (;;) {
      const int nb = min(min(kBatch, (int)((double)(z - a + 1) * dens) + (exact ? 2 : 4)), nch - ks);
      // one round trip: checkpoints [ks, ks + nb], gap lists and seq of chunks [ks, ks + nb)
      const int ckv = lane <= nb ? ckpt[b + ks + lane] : INT_MAX;
      const uint32_t* glb = glist + (uint64_t)(b + ks) * kGapCap;
      const uint32_t gv0 = lane < kGapCap * nb ? glb[lane] : 0u;
      const uint32_t gv1 = 64 + lane < kGapCap * nb ? glb[64 + lane] : 0u;
      uint32_t sq[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; j++) sq[j] = j < nb ? seq4(A, roff, vec, (ks + j) * kChunk + 4 * lane, len) : 0u;
      int j0 = 0;
      if (!exact) {
        const uint64_t m = __ballot(lane < nb && ckv <= a);
        if (m == 0 || (m >> (nb - 1)) != 0) {
          // guess off by more than the margin (or the batch ends before a): step from the guess
          int k = ks;
          while (k > 0 && ckpt[b + k] > a) k--;
          while (k + 1 < nch && ckpt[b + k + 1] <= a) k++;
          if (k + 1 < nch || ckpt[b + k] <= a) {
            ks = k;
            exact = true;
            continue;
          }
        }
        j0 = 63 - __builtin_clzll(m);
      }
      bool done = false;
      // a chunk whose gap list overflowed, or an unaligned row: the whole batch takes the general
      // loop (per chunk: gap list or ofs), else the unrolled gap-list loop over the registers
      const bool slow = !vec || __ballot((lane & 7) == 0 && (gv0 == kGapOverflow || gv1 == kGapOverflow)) != 0;
      if (!slow) {
#pragma unroll
        for (int j = 0; j < kBatch; j++) {
          if (j < j0) continue;
          if (j >= nb) break;
          const int colr = __builtin_amdgcn_readlane(ckv, j) - c0;
          if (colr > zr) {
            done = true;
            break;
          }
          const int cnr = __builtin_amdgcn_readlane(ckv, j + 1) - c0;
          auto gl = [&](int x) -> uint32_t {
            const int q = kGapCap * j + x;
            return (uint32_t)__builtin_amdgcn_readlane((int)(q < 64 ? gv0 : gv1), q & 63);
          };
          place_chunk<false>(A, roff, true, gl, sq[j], colr, cnr, (ks + j) * kChunk, len, ar, zr, lane, myb);
        }
      } else {
#pragma unroll 1
        for (int j = j0; j < nb; j++) {
          const int colr = __builtin_amdgcn_readlane(ckv, j) - c0;
          if (colr > zr) {
            done = true;
            break;
          }
          const int cnr = __builtin_amdgcn_readlane(ckv, j + 1) - c0;
          auto gl = [&](int x) -> uint32_t {
            const int q = kGapCap * j + x;
            const int lo = __builtin_amdgcn_readlane((int)gv0, q & 63), hi = __builtin_amdgcn_readlane((int)gv1, q & 63);
            return (uint32_t)(q < 64 ? lo : hi);
          };
          const bool fast = vec && gl(0) != kGapOverflow;
          const uint32_t s4 = seq4(A, roff, vec, (ks + j) * kChunk + 4 * lane, len);
          place_chunk<true>(A, roff, fast, gl, s4, colr, cnr, (ks + j) * kChunk, len, ar, zr, lane, myb);
        }
      }
      ks += nb;
      if (done || ks >= nch || __builtin_amdgcn_readlane(ckv, nb) > z) break;
      exact = true;  // the next batch starts right after this one
    }
    // the strip is read back by other lanes of this wave (LDS is in order within a wave)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4* w4 = reinterpret_cast<uint4*>(my);
    const uint4 wa = w4[lane], wb = w4[64 + lane];
    const uint32_t wd[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
    for (int m = 0; m < 32; m++) acc[m] += 1ull << ((wd[m >> 2] >> (8 * (m & 3))) & 0xFFu);
    const uint32_t g4 = kCodeGap * 0x01010101u;
    w4[lane] = make_uint4(g4, g4, g4, g4);
    w4[64 + lane] = make_uint4(g4, g4, g4, g4);
    nrow++;
  }
  __syncthreads();
  // the tile's counters: [col][6] rows in memory, one column per thread at a time
  for (int c = tid; c < c1 - c0; c += 64 * kCntWaves) {
    const int x = cnt_swz(c);
    uint32_t v[6];
    if (packed) {
      const uint64_t pv = reinterpret_cast<const unsigned long long*>(tab)[x];
#pragma unroll
      for (int f = 0; f < 6; f++) v[f] = (uint32_t)(pv >> (10 * f)) & 1023u;
    } else {
#pragma unroll
      for (int f = 0; f < 6; f++) v[f] = tab[f * kCntW + x];
    }
    int32_t* dst = A.counts + ((int64_t)c0 + c) * 6;
#pragma unroll
    for (int f = 0; f < 6; f++) dst[f] = (int32_t)v[f];
  }
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

// scratch word of the row records (16-byte aligned: K3 reads them as uint4)
inline uint64_t rinfo_word(uint64_t n_slots) { return ((3 + (uint64_t)kGapCap) * n_slots + 3) & ~(uint64_t)3; }

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

extern "C" int pw_msa_count(const pw_msa_args* a, void* stream) {
  if (!msa_args_ok(a)) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  // scratch: chunk sums | checkpoints | slot -> row | gap lists (kGapCap per slot) | row extents
  int32_t* chunk_sum = a->scratch;
  int32_t* ckpt = a->scratch + a->n_slots;
  int32_t* slot_row = a->scratch + 2 * a->n_slots;
  uint32_t* glist = reinterpret_cast<uint32_t*>(a->scratch + 3 * a->n_slots);
  int32_t* rinfo = a->scratch + pw::rinfo_word(a->n_slots);
  hipLaunchKernelGGL(pw::slot_rows, dim3(a->n_rows < 8192 ? a->n_rows : 8192), dim3(256), 0, s, *a, slot_row);
  const uint64_t nb1 = ((a->n_slots + 7) / 8 + 3) / 4;  // 8 slots per wave, 4 waves per workgroup
  hipLaunchKernelGGL(pw::row_chunk_sums, dim3((unsigned)(nb1 < 4096 ? nb1 : 4096)), dim3(256), 0, s, *a,
                     chunk_sum, slot_row, glist);
  hipLaunchKernelGGL(pw::row_prefix, dim3(a->n_rows < 4096 ? a->n_rows : 4096), dim3(1024), 0, s, *a, chunk_sum, ckpt,
                     rinfo);
  const unsigned ntiles = (unsigned)((a->n_cols + pw::kCntW - 1) / pw::kCntW);
  hipLaunchKernelGGL(pw::tile_counts, dim3(ntiles), dim3(64 * pw::kCntWaves), 0, s, *a, ckpt, glist, rinfo);
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
