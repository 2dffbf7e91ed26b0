// pw_msa_layout.cpp — `pafreport -w`: the progressive MSA of the last query run and its
// multi-FASTA (pafreport.cpp:382-421, 447-450; GapAssem.cpp:104-120, 605-753, 1006-1046, 482-520).
//
// The reference merges every pairwise alignment into the query's MSA with GSeqAlign::addAlign,
// which walks the query position by position and propagates each extra gap through every row
// (injectGap: O(rows x L) per gap).  The final layout has a closed form, used here:
//   * the query row's gap before base i is G[i] = max over the run's alignments of that
//     alignment's query gap R_a[i] ("once a gap, always a gap": addAlign keeps the larger of the
//     two gap values at every position);
//   * every injection at query position i lands in row a before its first base whose column is
//     at or after the column of query base i, and injections never reorder columns, so row a
//     ends with ofs[b] = T_a[b] + sum over i with b*(i) = b of (G[i] - R_a[i]), where b*(i) is
//     that base in the pairwise layout of alignment a (T_a: its own target gaps) — the target
//     bases inserted before query base i stay left-packed in the query's gap run.
// One pass over the gap positions per row: O(L + rows x row length) in total.  Inputs the closed
// form does not model (gap lengths outside 1..32767, gap sums overflowing GASeq's short ofs)
// take the literal replay of addAlign/injectGap instead.
#include "pw_msa_layout.h"

#include <ctype.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>

#include "pw_tables.h"
#include "pwasm_gapassem.hpp"

namespace pw {
namespace {

struct Comp {
  uint8_t c[256];
  Comp() {
    for (int i = 0; i < 256; i++) c[i] = (uint8_t)i;
    for (int i = 0; kIupacDefs[i]; i++) c[(uint8_t)kIupacDefs[i]] = (uint8_t)kIupacComp[i];
  }
};
const Comp& comp() {
  static const Comp t;
  return t;
}

// tseq of one alignment (PAFAlignment's cs loop, pafreport.cpp:536-626): query bases of ':' runs
// (aligned strand), lower-case target bases of '*' and '-' ops, nothing for '+'.
void build_tseq(const uint8_t* q, int qlen, const MsaRun& run, const MsaRec& r, std::string& out) {
  out.clear();
  out.reserve((size_t)r.t_len);
  const uint8_t* cm = comp().c;
  int qpos = 0;
  uint32_t li = r.lit_begin;
  for (uint32_t k = 0; k < r.n_ops; k++) {
    const uint32_t w = run.ops[r.op_begin + k];
    const uint32_t t = w >> 30, n = w & 0x3FFFFFFFu;
    if (t == 0) {  // match
      for (uint32_t j = 0; j < n; j++) {
        const int x = r.offset + qpos + (int)j;
        out.push_back((char)(r.reverse ? cm[q[qlen - 1 - x]] : q[x]));
      }
      qpos += (int)n;
    } else if (t == 1) {  // substitution
      out.push_back((char)tolower(run.lits[li]));
      li += 2;
      qpos++;
    } else if (t == 2) {  // target-only bases
      for (uint32_t j = 0; j < n; j++) out.push_back((char)tolower(run.lits[li + j]));
      li += n;
    } else {  // query-only bases
      qpos += (int)n;
    }
  }
}

// GASeq::printMFasta (GapAssem.cpp:482-520): offset dashes, then per base its gap dashes and the
// base, llen columns per line; a last line is closed even when empty.
struct Printer {
  std::string buf;
  int printed = 0;
  static constexpr int kLlen = 60;
  void put(char c) {
    buf.push_back(c);
    if (++printed == kLlen) {
      buf.push_back('\n');
      printed = 0;
    }
  }
  void dashes(long n) {
    while (n > 0) {
      const long room = kLlen - printed;
      const long k = n < room ? n : room;
      buf.append((size_t)k, '-');
      printed += (int)k;
      n -= k;
      if (printed == kLlen) {
        buf.push_back('\n');
        printed = 0;
      }
    }
  }
  void row(FILE* f, const std::string& id, const char* seq, int seqlen, long offset, const int32_t* ofs) {
    buf.clear();
    printed = 0;
    buf.push_back('>');
    buf += id;
    buf.push_back('\n');
    dashes(offset);
    for (int i = 0; i < seqlen; i++) {
      if (ofs[i] < 0) continue;  // deleted base
      dashes(ofs[i]);
      put(seq[i]);
    }
    if (printed < kLlen) buf.push_back('\n');
    fwrite(buf.data(), 1, buf.size(), f);
  }
};

// gap list of an alignment -> position-sorted, last setGap at a position wins (GASeq::setGap)
void gap_set(const int32_t* g, uint32_t n, std::vector<std::pair<int, int>>& out) {
  out.clear();
  for (uint32_t k = 0; k < n; k++) out.emplace_back(g[2 * k], g[2 * k + 1]);
  std::stable_sort(out.begin(), out.end(), [](auto& a, auto& b) { return a.first < b.first; });
  size_t w = 0;
  for (size_t k = 0; k < out.size(); k++) {
    if (w > 0 && out[w - 1].first == out[k].first) out[w - 1] = out[k];
    else out[w++] = out[k];
  }
  out.resize(w);
}

bool closed_form_ok(const MsaRun& run) {
  for (int32_t i = 1; i < (int32_t)run.gaps.size(); i += 2)
    if (run.gaps[i] < 1 || run.gaps[i] > 32767) return false;
  return true;
}

// ---------------------------------------------------------------- literal replay (fallback)
// pafreport's own construction (pafreport.cpp:382-421) through the GapAssem C++ API: the first
// alignment's GSeqAlign(refseq, taseq) becomes refMSA, every later one is a GSeqAlign(rseq,
// taseq) merged into it by addAlign (injectGap both ways, addSeq), then writeMSA.
int replay(FILE* f, FILE* dbg, const char* qid, const uint8_t* q, int qlen, const MsaRun& run) {
  GASeq* refseq = new GASeq(qid, nullptr, (const char*)q, qlen);  // (upper case already: allupper)
  refseq->setFlag(GA_FLAG_IS_REF);
  GSeqAlign* refMSA = nullptr;
  std::string tseq;
  for (size_t a = 0; a < run.recs.size(); a++) {
    const MsaRec& r = run.recs[a];
    build_tseq(q, qlen, run, r, tseq);
    const std::string label = run.labels.substr(r.lab_off, r.lab_len);
    GASeq* taseq = new GASeq(label.c_str(), "", tseq.c_str(), (int)tseq.size(), r.r_alnstart);
    taseq->revcompl = r.reverse != 0;
    GASeq* rseq = refseq->msa != nullptr ? new GASeq(qid, 0, qlen) : refseq;
    const int32_t* g = &run.gaps[r.gap_off];
    for (uint32_t k = 0; k < r.n_rg; k++) rseq->setGap(g[2 * k], (short)g[2 * k + 1]);
    for (uint32_t k = 0; k < r.n_tg; k++) taseq->setGap(g[2 * (r.n_rg + k)], (short)g[2 * (r.n_rg + k) + 1]);
    GSeqAlign* newmsa = new GSeqAlign(rseq, taseq);
    if (rseq == refseq) {
      refMSA = newmsa;
    } else {
      refseq->msa->addAlign(refseq, newmsa, rseq);
      refMSA = refseq->msa;
      delete newmsa;  // its rows now belong to refMSA (addAlign cleared its free flag)
    }
  }
  if (refMSA && dbg) {  // -D (pafreport.cpp:443-446)
    fprintf(dbg, ">MSA (%d)\n", refMSA->Count());
    refMSA->print(dbg, 'v');
  }
  if (refMSA) refMSA->writeMSA(f);
  delete refMSA;  // frees refseq and every taseq
  return 0;
}

}  // namespace

int write_run_msa(FILE* f, FILE* dbg, const char* qid, const uint8_t* q, int qlen, const MsaRun& run) {
  if (run.recs.empty()) return 0;  // no alignment: the reference dereferences NULL
  // PW_MSA_PATH (tests): "replay" forces the literal merge, "closed" refuses to fall back to it
  const char* path = getenv("PW_MSA_PATH");
  const bool force_replay = path && !strcmp(path, "replay"), no_replay = path && !strcmp(path, "closed");
  auto fallback = [&]() {
    if (no_replay) {
      fprintf(stderr, "pw msa: the closed form does not apply to this run (PW_MSA_PATH=closed)\n");
      return 2;
    }
    return replay(f, dbg, qid, q, qlen, run);
  };
  if (force_replay) return replay(f, dbg, qid, q, qlen, run);
  if (!closed_form_ok(run)) return fallback();
  // G = elementwise max of the alignments' query gaps (setGap semantics per alignment)
  std::vector<int32_t> G((size_t)qlen, 0);
  std::vector<std::pair<int, int>> rg, tg;
  for (const MsaRec& r : run.recs) {
    gap_set(&run.gaps[r.gap_off], r.n_rg, rg);
    for (auto& p : rg) G[(size_t)p.first] = std::max(G[(size_t)p.first], p.second);
  }
  std::vector<int> gpos;  // query positions with a gap in the final layout
  for (int i = 0; i < qlen; i++)
    if (G[(size_t)i] > 0) gpos.push_back(i);
  for (int32_t g : G)
    if (g > 32767) return fallback();
  std::string tseq;
  std::vector<int32_t> ofs, extra;
  long shift = 0;  // columns injected before the row's offset (injectGap moves the offset itself)
  // The row of alignment r in the final layout: its pairwise gaps plus, for every query gap
  // column i where the query row gained G[i] - R_a[i] columns, that many before the first target
  // base b placed at or after column i (injectGap, GapAssem.cpp:720-753) — or, when the row starts
  // at or after that column (`salpos >= alpos`, :733-737), added to the row's offset instead.  The
  // relation "row offset >= column of query base i" never changes under injections, so it is
  // decided on the pairwise layout.  False: a gap length outside the 16-bit range the reference
  // stores (the literal merge handles that).
  auto row_layout = [&](const MsaRec& r) {
    build_tseq(q, qlen, run, r, tseq);
    const int tl = (int)tseq.size();
    const int32_t* g = &run.gaps[r.gap_off];
    gap_set(g, r.n_rg, rg);
    gap_set(g + 2 * r.n_rg, r.n_tg, tg);
    ofs.assign((size_t)tl, 0);
    for (auto& p : tg) ofs[(size_t)p.first] = p.second;
    // walk the gap positions i of the final query row against this row's pairwise layout:
    // rc(i) = column of query base i, pc(b) = column of target base b (both pairwise)
    size_t ri = 0;   // next entry of rg
    long rsum = 0;   // sum of R_a over positions <= i
    int b = 0;
    long pc = tl > 0 ? r.r_alnstart + ofs[0] : 0;  // column of base b (pairwise: own gaps only)
    extra.clear();
    shift = 0;
    for (int i : gpos) {
      while (ri < rg.size() && rg[ri].first <= i) rsum += rg[ri++].second;
      const int Ra = (ri > 0 && rg[ri - 1].first == i) ? rg[ri - 1].second : 0;
      const int d = G[(size_t)i] - Ra;
      if (d <= 0) continue;
      const long rc = (long)i + rsum;
      if (r.r_alnstart >= rc) {  // the row starts at or after the column: its offset moves
        shift += d;
        continue;
      }
      while (b < tl && pc < rc) {
        b++;
        if (b < tl) pc += 1 + ofs[(size_t)b];
      }
      if (b >= tl) break;  // the row ends before this column: not affected
      if (extra.empty()) extra.assign((size_t)tl, 0);
      extra[(size_t)b] += d;
    }
    if (!extra.empty())
      for (int k = 0; k < tl; k++) {
        ofs[(size_t)k] += extra[(size_t)k];
        if (ofs[(size_t)k] > 32767) return false;
      }
    return true;
  };
  for (const MsaRec& r : run.recs)  // decide before anything is printed
    if (!row_layout(r)) return fallback();
  const uint8_t* cm = comp().c;
  auto prepped = [&](const MsaRec& r) {  // finalize -> prepSeq: the sequence, not its gaps
    if (r.reverse) {
      std::reverse(tseq.begin(), tseq.end());
      for (char& c : tseq) c = (char)cm[(uint8_t)c];
    }
  };
  if (dbg) {  // -D: refMSA->print(stderr, 'v') (pafreport.cpp:443-446, GapAssem.cpp:1013-1037)
    // minoffset / length as GSeqAlign keeps them: the smallest row offset, the largest row end
    long minoff = 0, end = (long)qlen;
    size_t namew = strlen(qid);
    for (int32_t g : G) end += g;
    for (const MsaRec& r : run.recs) {
      row_layout(r);
      long e = r.r_alnstart + shift + (long)tseq.size();
      for (int32_t o : ofs) e += o;
      minoff = std::min(minoff, (long)r.r_alnstart + shift);
      end = std::max(end, e);
      namew = std::max(namew, (size_t)r.lab_len);
    }
    const int w = (int)namew;
    std::string out;
    auto row = [&](const char* name, size_t nlen, char orient, long offset, const char* seq, int n, const int32_t* o) {
      out.assign((size_t)w - std::min(nlen, (size_t)w), ' ');
      out.append(name, nlen);
      out.push_back(' ');
      out.push_back(orient);
      out.push_back(' ');
      out.append((size_t)std::max(0L, offset - minoff), ' ');
      for (int k = 0; k < n; k++) {
        if (o[k] < 0) continue;
        out.append((size_t)o[k], '-');
        out.push_back(seq[k]);
      }
      out.push_back('\n');
      fwrite(out.data(), 1, out.size(), dbg);
    };
    fprintf(dbg, ">MSA (%d)\n", (int)run.recs.size() + 1);
    out.assign((size_t)w + 3, ' ');
    out.append((size_t)(end - minoff), 'v');
    out.push_back('\n');
    fwrite(out.data(), 1, out.size(), dbg);
    row(qid, strlen(qid), '+', 0, (const char*)q, qlen, G.data());
    for (const MsaRec& r : run.recs) {
      row_layout(r);
      prepped(r);
      row(run.labels.data() + r.lab_off, r.lab_len, r.reverse ? '-' : '+', r.r_alnstart + shift, tseq.data(),
          (int)tseq.size(), ofs.data());
    }
  }
  Printer pr;
  pr.row(f, qid, (const char*)q, qlen, 0, G.data());
  for (const MsaRec& r : run.recs) {
    row_layout(r);
    prepped(r);
    pr.row(f, run.labels.substr(r.lab_off, r.lab_len), tseq.data(), (int)tseq.size(), r.r_alnstart + shift, ofs.data());
  }
  return 0;
}

}  // namespace pw
