// pw_gapassem.cpp — `gapassem_consensus`: GSeqAlign::refineMSA of a packed layout file (PWL1 rows,
// tests/pwl_format.md) through the GapAssem C++ API (pwasm_gapassem.hpp: buildMSA / refineMSA on
// the GPU, per-row refineClipping / removeClipGaps on the host), written as a PWC1 result.
// Messages and exit codes are the reference's, raised inside the API:
//   "Warning: sequence %s (length %d) was trimmed too badly ..."  GapAssem.cpp:1096-1101
//   "MSAColumns op[]: bad index %d (size=%d)"  exit 1            GapAssem.h:366-370
//   "WARNING: 0 coverage column ..." + row ids, exit 5           GapAssem.cpp:1121-1131
//   "Warning: reached clipL/clipR trying to find an initial match on %s!"  :266-272, :315-321
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <string>
#include <vector>

#include "pwasm_amd.h"
#include "pwasm_gapassem.hpp"

// flags: bit0 removeConsGaps, bit1 disable refineClipping (MSAColumns statics, GapAssem.cpp:5-6)
extern "C" int pw_gapassem_run_ex(const char* layout_path, const char* out_path, uint32_t flags, const char* ace_path,
                                  const char* info_path, const char* msa_path) {
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
  std::vector<GASeq*> rows;
  rows.reserve(nrows);
  std::vector<int16_t> ofs;
  std::string seq;
  for (uint32_t r = 0; r < nrows; r++) {
    int32_t h[5];
    if (fread(h, sizeof h, 1, f) != 1 || h[1] < 0) {
      fclose(f);
      for (GASeq* s : rows) delete s;
      fprintf(stderr, "bad row header\n");
      return 2;
    }
    seq.resize((size_t)h[1]);
    ofs.resize((size_t)h[1]);
    if (fread(&seq[0], 1, seq.size(), f) != seq.size() || fread(ofs.data(), 2, ofs.size(), f) != ofs.size()) {
      fclose(f);
      for (GASeq* s : rows) delete s;
      fprintf(stderr, "truncated row\n");
      return 2;
    }
    char id[24];
    snprintf(id, sizeof id, "row%u", r);
    GASeq* s = new GASeq(id, h[0], h[1], h[2], h[3], (char)h[4]);
    s->seq = seq;
    s->len = h[1];
    for (int i = 0; i < h[1]; i++)
      if (ofs[(size_t)i]) s->setGap(i, ofs[(size_t)i]);
    rows.push_back(s);
  }
  fclose(f);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    for (GASeq* s : rows) delete s;
    fprintf(stderr, "gapassem: no HIP device available (this build has no CPU path)\n");
    return 2;
  }
  MSAColumns::removeConsGaps = (flags & 1u) != 0;
  MSAColumns::refineClipping = (flags & 2u) == 0;
  std::unique_ptr<GSeqAlign> msa(new GSeqAlign(rows));
  const int length0 = msa->len();
  int n_removed = 0;
  try {
    pw_ga_exit_scope scope;
    msa->refineMSA();
    n_removed = length0 - msa->len();
  } catch (const pw_ga_exit& e) {
    return e.code;
  }
  FILE* o = fopen(out_path, "wb");
  if (!o) return 2;
  const MSAColumns& mc = *msa->msacolumns;
  const bool covered = mc.mincol != INT_MAX;
  int32_t h[6] = {length0, msa->minOffset(), covered ? mc.mincol : -1, mc.maxcol,
                  msa->consensus_len, n_removed};
  fwrite("PWC1", 1, 4, o);
  fwrite(h, sizeof h, 1, o);
  fwrite(msa->consensus.data(), 1, (size_t)msa->consensus_len, o);
  for (const GAlnColumn& c : mc.columns) fwrite(c.counts, 4, 6, o);
  fwrite(&nrows, 4, 1, o);
  for (uint32_t r = 0; r < nrows; r++) {
    const GASeq* s = msa->Get((int)r);
    int32_t rh[4] = {s->offset, s->getNumGaps(), s->clp5, s->clp3};
    fwrite(rh, sizeof rh, 1, o);
    fwrite(s->gaps(), 2, (size_t)s->seqlen, o);
  }
  fclose(o);
  // writeACE / writeInfo (contig "contig1") after refineMSA, then writeMSA (its finalize
  // reverse-complements the rows' bases, so it comes last)
  try {
    pw_ga_exit_scope scope;
    const char* paths[3] = {ace_path, info_path, msa_path};
    for (int k = 0; k < 3; k++) {
      if (!paths[k]) continue;
      FILE* w = fopen(paths[k], "w");
      if (!w) {
        fprintf(stderr, "cannot open %s\n", paths[k]);
        return 2;
      }
      if (k == 0) msa->writeACE(w, "contig1");
      else if (k == 1) msa->writeInfo(w, "contig1");
      else msa->writeMSA(w);
      fclose(w);
    }
  } catch (const pw_ga_exit& e) {
    return e.code;
  }
  return 0;
}

extern "C" int pw_gapassem_run(const char* layout_path, const char* out_path, uint32_t flags) {
  return pw_gapassem_run_ex(layout_path, out_path, flags, nullptr, nullptr, nullptr);
}
