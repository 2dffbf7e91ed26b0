// pw_gapassem.cpp — GapAssem consensus driver on the HIP path: a packed layout (PWL1 rows,
// tests/pwl_format.md) -> pw_msa_columns on the GPU -> GSeqAlign::refineMSA's consensus
// (GapAssem.cpp:1133-1162) -> PWC1 result file.  Messages and exit codes follow the reference:
//   "Warning: sequence %s (length %d) was trimmed too badly ..."  GapAssem.cpp:1096-1101
//   "MSAColumns op[]: bad index %d (size=%d)"  exit 1            GapAssem.h:366-370
//   "WARNING: 0 coverage column ..." + row ids, exit 5           GapAssem.cpp:1121-1131
// removeConsGaps=true (GapAssem.cpp:1152-1158, 1174-1175) runs on the GPU too (pw_msa_refine);
// it needs gap values >= 0.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "pwasm_amd.h"

namespace {

struct Row {
  int32_t offset, seqlen, clp5, clp3, revcompl;
  uint64_t base;  // first base in the packed arrays
  int64_t numgaps;
};

template <class T>
struct Dev {
  T* p = nullptr;
  bool alloc(size_t n) { return hipMalloc((void**)&p, (n ? n : 1) * sizeof(T)) == hipSuccess; }
  ~Dev() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

// flags: bit0 removeConsGaps, bit1 disable refineClipping (MSAColumns statics, GapAssem.cpp:5-6)
extern "C" int pw_gapassem_run(const char* layout_path, const char* out_path, uint32_t flags) {
  const bool remove_gaps = flags & 1u, refine_clip = !(flags & 2u);
  FILE* f = fopen(layout_path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open layout\n");
    return 2;
  }
  char magic[4];
  uint32_t nrows = 0;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PWL1", 4) || fread(&nrows, 4, 1, f) != 1 || nrows == 0) {
    fclose(f);
    fprintf(stderr, "bad layout header\n");
    return 2;
  }
  std::vector<Row> rows(nrows);
  std::vector<uint8_t> seq;
  std::vector<int16_t> ofs;
  for (uint32_t r = 0; r < nrows; r++) {
    int32_t h[5];
    if (fread(h, sizeof h, 1, f) != 1 || h[1] < 0) {
      fclose(f);
      fprintf(stderr, "bad row header\n");
      return 2;
    }
    Row& w = rows[r];
    w.offset = h[0];
    w.seqlen = h[1];
    w.clp5 = h[2];
    w.clp3 = h[3];
    w.revcompl = h[4];
    w.base = (seq.size() + 7) / 8 * 8;  // rows start 8-base aligned: the count kernels' vector loads
    seq.resize(w.base + (size_t)w.seqlen);
    ofs.resize(w.base + (size_t)w.seqlen);
    if (fread(seq.data() + w.base, 1, (size_t)w.seqlen, f) != (size_t)w.seqlen ||
        fread(ofs.data() + w.base, 2, (size_t)w.seqlen, f) != (size_t)w.seqlen) {
      fclose(f);
      fprintf(stderr, "truncated row\n");
      return 2;
    }
    w.numgaps = 0;
    for (int i = 0; i < w.seqlen; i++) w.numgaps += ofs[w.base + i];
    if (refine_clip && (w.clp5 || w.clp3)) {
      fclose(f);
      fprintf(stderr, "refineClipping is not implemented on the HIP path yet: disable it\n");
      return 2;
    }
  }
  fclose(f);
  if (remove_gaps)
    for (int16_t g : ofs)
      if (g < 0) {
        fprintf(stderr, "removeConsGaps with negative gap values is not supported on the HIP path\n");
        return 2;
      }
  // GSeqAlign bookkeeping (GapAssem.cpp:605-641, 694-716)
  int64_t minoffset = INT64_MAX, maxend = INT64_MIN;
  for (const Row& w : rows) {
    minoffset = std::min<int64_t>(minoffset, w.offset);
    maxend = std::max<int64_t>(maxend, (int64_t)w.offset + w.seqlen + w.numgaps);
  }
  const int64_t length = std::max<int64_t>(maxend - minoffset, 0);
  if (length <= 0 || length > INT32_MAX) {
    fprintf(stderr, "MSAColumns op[]: bad index %d (size=%d)\n", 0, (int)length);
    return 1;
  }
  const int ncols = (int)length;
  std::vector<uint64_t> row_off(nrows);
  std::vector<int32_t> row_len(nrows), col0(nrows), cl(nrows), cr(nrows);
  for (uint32_t r = 0; r < nrows; r++) {
    row_off[r] = rows[r].base;
    row_len[r] = rows[r].seqlen;
    col0[r] = (int32_t)(rows[r].offset - minoffset);
    cl[r] = rows[r].revcompl ? rows[r].clp3 : rows[r].clp5;
    cr[r] = rows[r].revcompl ? rows[r].clp5 : rows[r].clp3;
  }
  std::vector<int64_t> slot_base(nrows + 1);
  const uint64_t nslots = pw_msa_slots(row_len.data(), nrows, slot_base.data());
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fprintf(stderr, "gapassem: no HIP device available (this build has no CPU path)\n");
    return 2;
  }
  hipStream_t st;
  if (hipStreamCreate(&st) != hipSuccess) return 2;
  Dev<uint8_t> d_seq, d_cons;
  Dev<int16_t> d_ofs;
  Dev<uint64_t> d_roff;
  Dev<int32_t> d_len, d_col0, d_cl, d_cr, d_scr, d_cnt, d_mm, d_gp, d_tg, d_clen, d_roffs, d_offo;
  Dev<int64_t> d_slot, d_ngo;
  Dev<uint8_t> d_cout;
  Dev<int16_t> d_ofso;
  const uint64_t ntg = pw_msa_refine_tiles(ncols);
  bool ok = d_seq.alloc(seq.size()) && d_ofs.alloc(ofs.size()) && d_roff.alloc(nrows) && d_len.alloc(nrows) &&
            d_col0.alloc(nrows) && d_cl.alloc(nrows) && d_cr.alloc(nrows) && d_slot.alloc(nrows + 1) &&
            d_scr.alloc(3 * nslots) && d_cnt.alloc((size_t)ncols * 6) && d_cons.alloc((size_t)ncols) && d_mm.alloc(4) &&
            d_gp.alloc((size_t)ncols) && d_tg.alloc(ntg) && d_clen.alloc(1) && d_cout.alloc((size_t)ncols) &&
            (!remove_gaps || (d_roffs.alloc(nrows) && d_offo.alloc(nrows) && d_ngo.alloc(nrows) && d_ofso.alloc(ofs.size())));
  if (!ok) {
    fprintf(stderr, "gapassem: device allocation failed\n");
    return 2;
  }
  (void)hipMemcpyAsync(d_seq.p, seq.data(), seq.size(), hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_ofs.p, ofs.data(), ofs.size() * 2, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_roff.p, row_off.data(), nrows * 8, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_len.p, row_len.data(), nrows * 4, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_col0.p, col0.data(), nrows * 4, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_cl.p, cl.data(), nrows * 4, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_cr.p, cr.data(), nrows * 4, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_slot.p, slot_base.data(), (nrows + 1) * 8, hipMemcpyHostToDevice, st);
  pw_msa_args a;
  a.seq = d_seq.p;
  a.ofs = d_ofs.p;
  a.row_off = d_roff.p;
  a.row_len = d_len.p;
  a.col0 = d_col0.p;
  a.clip_l = d_cl.p;
  a.clip_r = d_cr.p;
  a.slot_base = d_slot.p;
  a.scratch = d_scr.p;
  a.counts = d_cnt.p;
  a.consensus = d_cons.p;
  a.minmax = d_mm.p;
  a.n_slots = nslots;
  a.n_rows = nrows;
  a.n_cols = ncols;
  if (pw_msa_columns(&a, st) != PW_OK) {
    fprintf(stderr, "gapassem: kernel launch failed\n");
    return 2;
  }
  std::vector<int32_t> counts((size_t)ncols * 6);
  std::vector<uint8_t> cons((size_t)ncols);
  int32_t mm[4];
  (void)hipMemcpyAsync(counts.data(), d_cnt.p, counts.size() * 4, hipMemcpyDeviceToHost, st);
  (void)hipMemcpyAsync(cons.data(), d_cons.p, cons.size(), hipMemcpyDeviceToHost, st);
  (void)hipMemcpyAsync(mm, d_mm.p, sizeof mm, hipMemcpyDeviceToHost, st);
  if (hipStreamSynchronize(st) != hipSuccess) {
    fprintf(stderr, "gapassem: device error\n");
    return 2;
  }
  // buildMSA messages in row order, stopping at the first out-of-range access
  const uint32_t bad_row = mm[2] == INT_MAX ? nrows : (uint32_t)mm[2];
  for (uint32_t r = 0; r < nrows && r <= bad_row; r++) {
    const Row& w = rows[r];
    if (w.seqlen - w.clp3 - w.clp5 < 1)
      fprintf(stderr,
              "Warning: sequence row%u (length %d) was trimmed too badly (%d,%d) -- should be removed from MSA w/ "
              "row0!\n",
              r, w.seqlen, w.clp5, w.clp3);
    if (r == bad_row) {  // find the first column toMSA would touch out of range (GapAssem.cpp:568-588)
      int64_t col = col0[r];
      for (int i = 0; i < w.seqlen; i++) {
        const bool clipped = i < cl[r] || i >= w.seqlen - cr[r];
        const int g = ofs[w.base + i];
        for (int j = 0; j < g; j++) {
          if (!clipped && (col < 0 || col >= ncols)) {
            fprintf(stderr, "MSAColumns op[]: bad index %d (size=%d)\n", (int)col, ncols);
            return 1;
          }
          col++;
        }
        if (col < 0 || col >= ncols) {
          fprintf(stderr, "MSAColumns op[]: bad index %d (size=%d)\n", (int)col, ncols);
          return 1;
        }
        col++;
      }
    }
  }
  const int mincol = mm[0];
  const int maxcol = mm[1] < 0 ? 0 : mm[1];
  if (mm[3] != INT_MAX) {
    fprintf(stderr, "WARNING: 0 coverage column %d (mincol=%d) found within alignment of %d seqs!\n", mm[3], mincol,
            (int)nrows);
    for (uint32_t r = 0; r < nrows; r++) fprintf(stderr, "row%u\n", r);
    return 5;
  }
  // refineMSA's consensus loop and (removeConsGaps) row edits on the GPU
  std::string consensus;
  std::vector<int32_t> off_out(nrows);
  std::vector<int64_t> ng_out(nrows);
  int32_t n_removed = 0;
  if (mincol != INT_MAX) {
    std::vector<int32_t> roffs(nrows);
    for (uint32_t r = 0; r < nrows; r++) {
      roffs[r] = rows[r].offset;
      ng_out[r] = rows[r].numgaps;
    }
    pw_msa_refine_args ra;
    memset(&ra, 0, sizeof ra);
    ra.gap_prefix = d_gp.p;
    ra.tile_gaps = d_tg.p;
    ra.cons_out = d_cout.p;
    ra.cons_len = d_clen.p;
    ra.remove_gaps = remove_gaps ? 1u : 0u;
    if (remove_gaps) {
      (void)hipMemcpyAsync(d_roffs.p, roffs.data(), nrows * 4, hipMemcpyHostToDevice, st);
      (void)hipMemcpyAsync(d_ngo.p, ng_out.data(), nrows * 8, hipMemcpyHostToDevice, st);
      ra.row_offset = d_roffs.p;
      ra.ofs_out = d_ofso.p;
      ra.offset_out = d_offo.p;
      ra.numgaps_out = d_ngo.p;
    }
    int32_t clen = 0;
    if (pw_msa_refine(&a, &ra, st) != PW_OK ||
        hipMemcpyAsync(&clen, d_clen.p, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      fprintf(stderr, "gapassem: refine failed\n");
      return 2;
    }
    consensus.resize((size_t)clen);
    (void)hipMemcpyAsync(&consensus[0], d_cout.p, (size_t)clen, hipMemcpyDeviceToHost, st);
    if (remove_gaps) {
      (void)hipMemcpyAsync(off_out.data(), d_offo.p, nrows * 4, hipMemcpyDeviceToHost, st);
      (void)hipMemcpyAsync(ng_out.data(), d_ngo.p, nrows * 8, hipMemcpyDeviceToHost, st);
      (void)hipMemcpyAsync(ofs.data(), d_ofso.p, ofs.size() * 2, hipMemcpyDeviceToHost, st);
      n_removed = (int32_t)(maxcol - mincol + 1) - clen;
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
      fprintf(stderr, "gapassem: device error\n");
      return 2;
    }
  }
  (void)hipStreamDestroy(st);
  if (!remove_gaps || mincol == INT_MAX)
    for (uint32_t r = 0; r < nrows; r++) {
      off_out[r] = rows[r].offset;
      ng_out[r] = rows[r].numgaps;
    }
  FILE* o = fopen(out_path, "wb");
  if (!o) return 2;
  int32_t h[6] = {ncols, (int32_t)minoffset, mincol == INT_MAX ? -1 : mincol, maxcol, (int32_t)consensus.size(),
                  n_removed};
  fwrite("PWC1", 1, 4, o);
  fwrite(h, sizeof h, 1, o);
  fwrite(consensus.data(), 1, consensus.size(), o);
  fwrite(counts.data(), 4, counts.size(), o);
  fwrite(&nrows, 4, 1, o);
  for (uint32_t r = 0; r < nrows; r++) {
    int32_t rh[2] = {off_out[r], (int32_t)ng_out[r]};
    fwrite(rh, sizeof rh, 1, o);
    fwrite(ofs.data() + rows[r].base, 2, (size_t)rows[r].seqlen, o);
  }
  fclose(o);
  return 0;
}
