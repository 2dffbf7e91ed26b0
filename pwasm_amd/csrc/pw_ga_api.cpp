// pw_ga_api.cpp — the GapAssem C++ API (include/pwasm_gapassem.hpp) and the host per-row C-ABI
// (pw_ga_row_* in pwasm_amd.h).
//
// Row bookkeeping (setGap, injectGap, addAlign, removeColumn, …) is host code on the row
// objects, as in the reference.  GSeqAlign::buildMSA / refineMSA stage every row in HBM and run
// the column work on the GPU (pw_msa_count + pw_msa_call: toMSA's scatter and bestChar;
// pw_msa_refine: the consensus and, with removeConsGaps, every row's removeColumn edits in
// closed form).  What stays per row on the host is what the reference does per row after the
// consensus exists: refineClipping's X-drop at the two clip boundaries, removeClipGaps, and the
// removeColumn edits of rows that hold deleted bases (ofs < 0), replayed in one linear pass.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <string.h>

#include <algorithm>

#include "pw_tables.h"
#include "pwasm_amd.h"
#include "pwasm_gapassem.hpp"

bool MSAColumns::removeConsGaps = true;  // GapAssem.cpp:5-6
bool MSAColumns::refineClipping = true;

namespace {

pw_ga_error_fn g_error_fn = nullptr;
hipStream_t g_stream = nullptr;
thread_local int g_catch_exit = 0;  // > 0: pw_gapassem_run turns the reference's exits into a return

// the reference's exit(code) after a GError / ErrZeroCov
[[noreturn]] void ga_exit(int code) {
  if (g_catch_exit > 0) throw pw_ga_exit{code};
  exit(code);
}

std::string vfmt(const char* fmt, va_list ap) {
  char buf[512];
  va_list aq;
  va_copy(aq, ap);
  const int n = vsnprintf(buf, sizeof buf, fmt, ap);
  std::string s;
  if (n >= (int)sizeof buf) {
    s.resize((size_t)n);
    vsnprintf(&s[0], (size_t)n + 1, fmt, aq);
  } else if (n > 0) {
    s.assign(buf, (size_t)n);
  }
  va_end(aq);
  return s;
}

// GError: the handler (or stderr), then exit(1) — a handler that returns does not resume
[[noreturn]] void gerror(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  const std::string m = vfmt(fmt, ap);
  va_end(ap);
  if (g_error_fn) {
    g_error_fn(m.c_str());
  } else {
    fflush(stdout);
    fputs(m.c_str(), stderr);
  }
  ga_exit(1);
}

void gmessage(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}

const uint8_t* comp_table() {
  struct T {
    uint8_t c[256];
    T() {
      for (int i = 0; i < 256; i++) c[i] = (uint8_t)i;
      for (int i = 0; pw::kIupacDefs[i]; i++) c[(uint8_t)pw::kIupacDefs[i]] = (uint8_t)pw::kIupacComp[i];
    }
  };
  static const T t;
  return t.c;
}

int iround(double x) { return (int)floor(x + 0.5); }  // gclib GBase iround

// One row as the per-row steps see it (GASeq fields or a pw_ga_row).
struct RowView {
  const char* seq;
  int16_t* ofs;
  int seqlen;
  int* numgaps;
  int* offset;
  int* clp5;
  int* clp3;
  bool revcompl;
  const char* id;
};

// GASeq::refineClipping (GapAssem.cpp:182-349).  Reads outside gseq / cons give 0 (the reference
// reads out of bounds there); an empty consensus changes nothing (the reference dereferences its
// NULL consensus) — DESIGN.md D11.  Returns false after a GError (message in *err).
// Warnings go to *msgs when given, else to stderr.
void warn_to(std::string* msgs, const char* fmt, const char* id) {
  char b[512];
  snprintf(b, sizeof b, fmt, id);
  if (msgs) *msgs += b;
  else gmessage("%s", b);
}
bool refine_clipping(RowView r, const char* cons, int cons_len, int cpos, bool skipDels, std::string* err,
                     std::string* msgs = nullptr) {
  if (*r.clp3 == 0 && *r.clp5 == 0) return true;
  if (cons_len == 0) return true;
  int& clipL = r.revcompl ? *r.clp3 : *r.clp5;
  int& clipR = r.revcompl ? *r.clp5 : *r.clp3;
  const int seqlen = r.seqlen;
  auto O = [&](int i) -> int { return (i >= 0 && i < seqlen) ? r.ofs[i] : 0; };
  int glen = seqlen + *r.numgaps;
  int allocsize = glen;
  int gclipR = clipR, gclipL = clipL;
  if (skipDels) {
    for (int i = 1; i <= clipR; i++) {
      if (O(seqlen - i) < 0) allocsize++;
      else gclipR += O(seqlen - i);
    }
    for (int i = 0; i < clipL; i++) {
      if (O(i) < 0) allocsize++;
      else gclipL += O(i);
    }
  } else {
    for (int i = 1; i <= clipR; i++) gclipR += O(seqlen - i);
    for (int i = 0; i < clipL; i++) gclipL += O(i);
  }
  // the gapped row ('*' per gap) and its base index map
  const int cap = allocsize > 0 ? allocsize : 0;
  std::string gseq((size_t)cap, '\0');
  std::vector<int> gxpos((size_t)cap + 1, 0);
  int gp = 0;
  for (int i = 0; i < seqlen; i++) {
    if (r.ofs[i] < 0) {
      if (!skipDels) continue;
      if (i >= clipL && i < seqlen - clipR) continue;
      glen++;
    }
    for (int j = 0; j < r.ofs[i]; j++) {
      if (gp < cap) gseq[(size_t)gp] = '*';
      gp++;
    }
    if (gp < cap) {
      gseq[(size_t)gp] = r.seq[i];
      gxpos[(size_t)gp] = i;
    }
    gp++;
  }
  if (glen != allocsize) {
    char b[256];
    snprintf(b, sizeof b, "Length mismatch (allocsize %d vs. glen %d) while refineClipping for seq %s !\n", allocsize,
             glen, r.id);
    *err = b;
    return false;
  }
  auto G = [&](int i) -> char { return (i >= 0 && i < cap) ? gseq[(size_t)i] : '\0'; };
  auto C = [&](int i) -> char { return (i >= 0 && i < cons_len) ? cons[i] : '\0'; };
  constexpr int kXDrop = -16, kMatch = 1, kMismatch = -3;
  if (clipR > 0) {
    // right end: back to the last match at or before the clip boundary, then extend forward
    int cp = cpos + glen - gclipR - 1;
    int sp = glen - gclipR - 1;
    while (G(sp) != C(cp) || G(sp) == '*') {
      if (G(sp) != '*') clipR++;
      sp--;
      cp--;
      if (sp < gclipL) {
        warn_to(msgs, "Warning: reached clipL trying to find an initial match on %s!\n", r.id);
        return true;
      }
    }
    int score = kMatch, maxscore = kMatch;
    const int startpos = sp;
    int bestpos = sp;
    while (score > kXDrop && ++cp < cons_len && ++sp < glen) {
      if (G(sp) == C(cp)) {
        if (G(sp) != '*') {
          score += kMatch;
          if (score > maxscore) {
            bestpos = sp;
            maxscore = score;
          }
        }
      } else if (G(sp) != '*') {
        score += kMismatch;
      }
    }
    if (bestpos > startpos) clipR = seqlen - gxpos[(size_t)bestpos] - 1;
  }
  if (clipL > 0) {
    // left end: forward to the first match at or after the clip boundary, then extend backward
    int cp = cpos + gclipL;
    int sp = gclipL;
    while (G(sp) != C(cp) || G(sp) == '*') {
      if (G(sp) != '*') clipL++;
      sp++;
      cp++;
      if (sp >= glen - gclipR) {
        warn_to(msgs, "Warning: reached clipR trying to find an initial match on %s!\n", r.id);
        return true;
      }
    }
    int score = kMatch, maxscore = kMatch;
    const int startpos = sp;
    int bestpos = sp;
    while (score > kXDrop && --cp >= 0 && --sp >= 0) {
      if (G(sp) == C(cp)) {
        if (G(sp) != '*') {
          score += kMatch;
          if (score > maxscore) {
            bestpos = sp;
            maxscore = score;
          }
        }
      } else if (G(sp) != '*') {
        score += kMismatch;
      }
    }
    if (bestpos < startpos) clipL = gxpos[(size_t)bestpos];
  }
  return true;
}

// GASeq::removeClipGaps (GapAssem.cpp:522-549): only the clipped ends are touched
int remove_clip_gaps(RowView r) {
  const int clipL = r.revcompl ? *r.clp3 : *r.clp5;
  const int clipR = r.revcompl ? *r.clp5 : *r.clp3;
  int dl = 0, dr = 0;
  const int lend = std::min(clipL, r.seqlen - 1);
  for (int i = 0; i <= lend; i++) {
    dl += r.ofs[i];
    r.ofs[i] = 0;
  }
  for (int i = std::max(std::max(r.seqlen - clipR, lend + 1), 0); i < r.seqlen; i++) {
    dr += r.ofs[i];
    r.ofs[i] = 0;
  }
  *r.offset += dl;
  *r.numgaps -= (dl + dr);
  return dl + dr;
}

// removeColumn(alpos_k) for non-decreasing alpos_k (GapAssem.cpp:755-779).  The walk of one
// removal stops at the first base p with offset + sum_{k<=p}(1 + ofs[k]) > alpos; every base
// before it stays at or before alpos <= the next alpos after the edit (ofs[p]-- only moves p and
// later bases; offset only moves while offset >= alpos), so the next walk resumes at p.
void remove_columns(RowView r, const int32_t* alpos, uint64_t n) {
  int p = 0;
  long long acc = 0;  // sum_{k<p} (1 + ofs[k])
  for (uint64_t k = 0; k < n; k++) {
    const long long a = alpos[k];
    if (*r.offset >= a) {  // the row starts after the column: it moves left
      (*r.offset)--;
      continue;
    }
    while (p < r.seqlen && *r.offset + acc + 1 + r.ofs[p] <= a) {
      acc += 1 + r.ofs[p];
      p++;
    }
    if (p >= r.seqlen) break;  // past the row's end: neither this nor any later column touches it
    r.ofs[p]--;                // removeBase (GapAssem.cpp:122-131)
    (*r.numgaps)--;
  }
}

RowView view_of(GASeq* s, int* numgaps, int16_t* ofs) {
  RowView v;
  v.seq = s->seq.data();
  v.ofs = ofs;
  v.seqlen = s->seqlen;
  v.numgaps = numgaps;
  v.offset = &s->offset;
  v.clp5 = &s->clp5;
  v.clp3 = &s->clp3;
  v.revcompl = s->revcompl != 0;
  v.id = s->id.c_str();
  return v;
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t k) {
    if (hipMalloc((void**)&p, (k ? k : 1) * sizeof(T)) != hipSuccess) gerror("GSeqAlign: device allocation failed\n");
    n = k;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) gerror("GSeqAlign: %s failed (%s)\n", what, hipGetErrorString(e));
}

// The rows of one GSeqAlign staged in HBM by buildMSA (kept for refineMSA)
struct DevLayout {
  DevBuf<uint8_t> seq, cons, cout;
  DevBuf<int16_t> ofs, ofso;
  DevBuf<uint64_t> row_off;
  DevBuf<int32_t> len, col0, cl, cr, scr, counts, mm, gp, tg, clen, roffs, offo;
  DevBuf<int64_t> slot, ngo;
  std::vector<uint64_t> h_row_off;
  pw_msa_args a{};
  uint32_t nrows = 0;
  int32_t zero_col = INT_MAX;  // first zero-coverage column in [mincol, maxcol] (pw_msa_call)
};

}  // namespace

void pw_ga_set_error_handler(pw_ga_error_fn fn) { g_error_fn = fn; }
pw_ga_exit_scope::pw_ga_exit_scope() { g_catch_exit++; }
pw_ga_exit_scope::~pw_ga_exit_scope() { g_catch_exit--; }
void pw_ga_set_stream(void* stream) { g_stream = (hipStream_t)stream; }

// ================================================================== GASeq
GASeq::GASeq(const char* sname, int slen)
    : numgaps(0), ofs((size_t)(slen > 0 ? slen : 0), 0), id(sname ? sname : ""), len(0), flags(0), msa(nullptr),
      msaidx(-1), seqlen(slen), offset(0), ng_ofs(0), revcompl(0), ext5(0), ext3(0), clp5(0), clp3(0) {}

GASeq::GASeq(const char* sname, const char* sdescr, const char* sseq, int slen, int soffset)
    : numgaps(0), id(sname ? sname : ""), descr(sdescr ? sdescr : ""), len(0), flags(0), msa(nullptr), msaidx(-1),
      seqlen(0), offset(soffset), ng_ofs(soffset), revcompl(0), ext5(0), ext3(0), clp5(0), clp3(0) {
  if (sseq) seq.assign(sseq, (size_t)(slen > 0 ? slen : (int)strlen(sseq)));  // FastaSeq(sname, sdescr, sseq, slen)
  len = (int)seq.size();
  seqlen = len;
  ofs.assign((size_t)seqlen, 0);
}

GASeq::GASeq(const char* sname, int soffset, int slen, int sclipL, int sclipR, char rev)
    : numgaps(0), ofs((size_t)(slen > 0 ? slen : 0), 0), id(sname ? sname : ""), len(0), flags(0), msa(nullptr),
      msaidx(-1), seqlen(slen), offset(soffset), ng_ofs(soffset), revcompl(rev), ext5(0), ext3(0), clp5(sclipL),
      clp3(sclipR) {}

GASeq::GASeq(GASeq& a)
    : numgaps(0), ofs((size_t)a.len, 0), id(a.id), descr(a.descr), seq(a.seq), len(a.len), flags(0), msa(nullptr),
      msaidx(-1), seqlen(a.len), offset(0), ng_ofs(0), revcompl(0), ext5(0), ext3(0), clp5(0), clp3(0) {}

void GASeq::allupper() {
  for (char& c : seq) c = (char)toupper((unsigned char)c);
}
void GASeq::lowercase() {
  for (char& c : seq) c = (char)tolower((unsigned char)c);
}
void GASeq::reverseComplement() {
  if (len == 0) return;
  std::reverse(seq.begin(), seq.end());
  const uint8_t* cm = comp_table();
  for (char& c : seq) c = (char)cm[(uint8_t)c];
}

void GASeq::prepSeq() {  // GapAssem.cpp:89-101 (delops: never filled, removeBase only edits ofs)
  if (revcompl == 1) reverseComplement();
  setFlag(GA_FLAG_PREPPED);
}

void GASeq::setGap(int pos, short gaplen) {  // GapAssem.cpp:104-111
  if (pos < 0 || pos >= seqlen) gerror("Error: invalid gap position (%d) given for sequence %s\n", pos + 1, id.c_str());
  numgaps -= ofs[(size_t)pos];
  ofs[(size_t)pos] = gaplen;
  numgaps += gaplen;
}

void GASeq::addGap(int pos, short gapadd) {  // GapAssem.cpp:114-120
  if (pos < 0 || pos >= seqlen) gerror("Error: invalid gap position (%d) given for sequence %s\n", pos + 1, id.c_str());
  numgaps += gapadd;
  ofs[(size_t)pos] = (int16_t)(ofs[(size_t)pos] + gapadd);
}

void GASeq::removeBase(int pos) {  // GapAssem.cpp:122-131
  if (pos < 0 || pos >= seqlen) gerror("Error: invalid gap position (%d) given for sequence %s\n", pos + 1, id.c_str());
  ofs[(size_t)pos]--;
  numgaps--;
}

void GASeq::refineClipping(const char* cons, int cons_len, int cpos, bool skipDels) {
  std::string err;
  if (!refine_clipping(view_of(this, &numgaps, ofs.data()), cons, cons_len, cpos, skipDels, &err))
    gerror("%s", err.c_str());
}

int GASeq::removeClipGaps() { return remove_clip_gaps(view_of(this, &numgaps, ofs.data())); }

void GASeq::reverseGaps() {  // GapAssem.cpp:351-364 (ofs[0] stays)
  int l = 1, r = seqlen - 1;
  while (l < r) std::swap(ofs[(size_t)l++], ofs[(size_t)r--]);
}

void GASeq::revComplement(int alignlen) {  // GapAssem.cpp:366-392
  if (alignlen > 0) {
    offset = alignlen - endOffset();
    if (msa != nullptr) {
      ng_ofs = msa->ng_len - endNgOffset();
      if (msa->minoffset > offset) msa->minoffset = offset;
      if (msa->ng_minofs > ng_ofs) msa->ng_minofs = ng_ofs;
    }
  }
  revcompl = !revcompl;
  if (len == seqlen) reverseComplement();
  reverseGaps();
}

void GASeq::printGappedSeq(FILE* f, int baseoffs) {  // GapAssem.cpp:412-440
  if (len == 0 || len != seqlen)
    gerror("GASeq print Error: invalid sequence data '%s' (len=%d, seqlen=%d)\n", id.c_str(), len, seqlen);
  const int clipL = revcompl ? clp3 : clp5, clipR = revcompl ? clp5 : clp3;
  for (int i = 0; i < offset - baseoffs; i++) fputc(' ', f);
  for (int i = 0; i < seqlen; i++) {
    if (ofs[(size_t)i] < 0) continue;
    for (int j = 0; j < ofs[(size_t)i]; j++) fputc('-', f);
    char c = seq[(size_t)i];
    if (i < clipL || i >= seqlen - clipR) c = (char)tolower((unsigned char)c);
    fputc(c, f);
  }
  fputc('\n', f);
}

void GASeq::printGappedFasta(FILE* f) {  // GapAssem.cpp:442-480
  if (len == 0 || len != seqlen)
    gerror("GASeq print Error: invalid sequence data '%s' (len=%d, seqlen=%d)\n", id.c_str(), len, seqlen);
  int printed = 0;
  for (int i = 0; i < seqlen; i++) {
    if (ofs[(size_t)i] < 0) continue;
    for (int j = 0; j < ofs[(size_t)i]; j++) {
      fputc('*', f);
      if (++printed == 60) {
        fputc('\n', f);
        printed = 0;
      }
    }
    fputc(seq[(size_t)i], f);
    if (++printed == 60) {
      fputc('\n', f);
      printed = 0;
    }
  }
  if (printed < 60) fputc('\n', f);
}

void GASeq::printMFasta(FILE* f, int llen) {  // GapAssem.cpp:482-520
  if (len == 0 || len != seqlen)
    gerror("GASeq print Error: invalid sequence data '%s' (len=%d, seqlen=%d)\n", id.c_str(), len, seqlen);
  if (!descr.empty()) fprintf(f, ">%s %s\n", id.c_str(), descr.c_str());
  else fprintf(f, ">%s\n", id.c_str());
  int printed = 0;
  auto put = [&](char c) {
    fputc(c, f);
    if (++printed == llen) {
      fputc('\n', f);
      printed = 0;
    }
  };
  for (int i = 0; i < offset; i++) put('-');
  for (int i = 0; i < seqlen; i++) {
    if (ofs[(size_t)i] < 0) continue;
    for (int j = 0; j < ofs[(size_t)i]; j++) put('-');
    put(seq[(size_t)i]);
  }
  if (printed < llen) fputc('\n', f);
}

void GASeq::toMSA(MSAColumns& msacols) {  // GapAssem.cpp:551-591 (host scatter)
  if (len == 0 || len != seqlen)
    gerror("GASeq::toMSA Error: invalid sequence data '%s' (len=%d, seqlen=%d)\n", id.c_str(), len, seqlen);
  const int clipL = revcompl ? clp3 : clp5, clipR = revcompl ? clp5 : clp3;
  int mincol = INT_MAX, maxcol = 0;
  int col = offset - msa->minoffset;
  for (int i = 0; i < seqlen; i++) {
    const bool clipped = i < clipL || i >= seqlen - clipR;
    if (!clipped && mincol == INT_MAX) mincol = col;
    for (int j = 0; j < ofs[(size_t)i]; j++) {
      if (!clipped) msacols[col].addGap();
      col++;
    }
    msacols[col].addNuc(this, i, clipped);
    if (!clipped) maxcol = col;
    col++;
  }
  msacols.updateMinMax(mincol, maxcol);
}

// ================================================================== columns
void GAlnColumn::addNuc(GASeq* s, int pos, bool clipped) {  // GapAssem.h:299-337
  if (clipped) {
    hasClip = true;
    return;
  }
  switch (toupper((unsigned char)s->seq[(size_t)pos])) {
    case 'A': counts[ncA]++; break;
    case 'C': counts[ncC]++; break;
    case 'G': counts[ncG]++; break;
    case 'T': counts[ncT]++; break;
    case '-':
    case '*': counts[ncGap]++; break;
    default: counts[ncN]++;
  }
  layers++;
}

char GAlnColumn::bestChar() {  // GapAssem.cpp:1048-1069: stable order by count, N/- tie rule
  if (layers == 0) return 0;
  if (consensus != 0) return consensus;
  static const char kc[6] = {'A', 'C', 'G', 'T', 'N', '-'};
  int idx[6] = {0, 1, 2, 3, 4, 5};
  std::stable_sort(idx, idx + 6, [&](int a, int b) { return counts[a] > counts[b]; });
  int r = 0;
  char best = kc[idx[0]];
  while ((best == '-' || best == 'N') && r + 1 < 6 && counts[idx[r]] == counts[idx[r + 1]]) {
    r++;
    best = kc[idx[r]];
  }
  consensus = best;
  return best;
}

GAlnColumn& MSAColumns::operator[](int idx) {  // GapAssem.h:366-370
  if (idx < 0 || idx >= size) gerror("MSAColumns op[]: bad index %d (size=%d)\n", idx, size);
  return columns[(size_t)idx];
}

// ================================================================== AlnClipOps (GapAssem.h:196-252)
static int max_overhang(GASeq* s, float clipmax) {
  return clipmax > 1 ? (int)clipmax : iround(clipmax * (float)s->seqlen);
}
bool AlnClipOps::add5(GASeq* s, int clp, float clipmax) {
  if (s->clp5 < clp) {
    if (clipmax > 0 && clp > max_overhang(s, clipmax)) return false;
    if (s->seqlen - s->clp3 - clp < (s->seqlen >> 2)) return false;
    total += 10000 + clp - s->clp5;
    Add(SeqClipOp(s, clp, -1));
  }
  return true;
}
bool AlnClipOps::add3(GASeq* s, int clp, float clipmax) {
  if (s->clp3 < clp) {
    if (clipmax > 0 && clp > max_overhang(s, clipmax)) return false;
    if (s->seqlen - s->clp5 - clp < (s->seqlen >> 2)) return false;
    total += 10000 + clp - s->clp3;
    Add(SeqClipOp(s, -1, clp));
  }
  return true;
}
bool AlnClipOps::add(GASeq* s, int clp5, int clp3, float clipmax) {
  int newclp5 = -1, newclp3 = -1, a = 0;
  if (s->clp5 < clp5) {
    if (clipmax > 0 && clp5 > max_overhang(s, clipmax)) return false;
    if (s->seqlen - s->clp3 - clp5 < (s->seqlen >> 2)) return false;
    a += 10000 + clp5 - s->clp5;
    newclp5 = clp5;
  } else {
    clp5 = s->clp5;
  }
  if (s->clp3 < clp3) {
    if (clipmax > 0 && clp3 > max_overhang(s, clipmax)) return false;
    if (s->seqlen - clp5 - clp3 < (s->seqlen >> 2)) return false;
    a += 10000 + clp3 - s->clp3;
    newclp3 = clp3;
  }
  if (a > 0) {
    total += a;
    Add(SeqClipOp(s, newclp5, newclp3));
  }
  return true;
}

// ================================================================== GSeqAlign
// offset - minoffset - mincol as the reference's int arithmetic gives it (mincol is INT_MAX when
// no column is covered: wraps there, without undefined behaviour here)
static int rel_col(int offset, int minoffset, int mincol) {
  return (int)(uint32_t)((uint32_t)offset - (uint32_t)minoffset - (uint32_t)mincol);
}

GSeqAlign::GSeqAlign()
    : free_items_(true), dev_(nullptr), length(0), minoffset(0), refinedMSA(false), msacolumns(nullptr), ordnum(0),
      ng_len(0), ng_minofs(0), badseqs(0), consensus_len(0) {}

GSeqAlign::GSeqAlign(bool, bool free_elements, bool) : GSeqAlign() { free_items_ = free_elements; }

GSeqAlign::GSeqAlign(GASeq* s1, GASeq* s2) : GSeqAlign() {  // GapAssem.cpp:605-641
  s1->msa = this;
  s2->msa = this;
  Add(s1);
  Add(s2);
  minoffset = std::min(s1->offset, s2->offset);
  ng_minofs = minoffset;
  length = std::max(s1->endOffset(), s2->endOffset()) - minoffset;
  ng_len = std::max(s1->endNgOffset(), s2->endNgOffset()) - ng_minofs;
}

GSeqAlign::GSeqAlign(const std::vector<GASeq*>& rows) : GSeqAlign() {
  if (rows.empty()) return;
  int mo = INT_MAX, me = INT_MIN, ngo = INT_MAX, nge = INT_MIN;
  for (GASeq* s : rows) {
    s->msa = this;
    Add(s);
    mo = std::min(mo, s->offset);
    me = std::max(me, s->endOffset());
    ngo = std::min(ngo, s->ng_ofs);
    nge = std::max(nge, s->endNgOffset());
  }
  minoffset = mo;
  length = std::max(me - mo, 0);
  ng_minofs = ngo;
  ng_len = std::max(nge - ngo, 0);
}

GSeqAlign::~GSeqAlign() {
  delete msacolumns;
  delete (DevLayout*)dev_;
  if (free_items_)
    for (GASeq* s : rows_) delete s;
}

void GSeqAlign::Sort() {
  std::stable_sort(rows_.begin(), rows_.end(), [](const GASeq* a, const GASeq* b) { return a->offset < b->offset; });
}

void GSeqAlign::revComplement() {  // GapAssem.cpp:998-1004
  for (GASeq* s : rows_) s->revComplement(length);
  Sort();
}

void GSeqAlign::addSeq(GASeq* s, int soffs, int ngofs) {  // GapAssem.cpp:694-716
  s->offset = soffs;
  s->ng_ofs = ngofs;
  s->msa = this;
  Add(s);
  if (soffs < minoffset) {
    length += minoffset - soffs;
    minoffset = soffs;
  }
  if (ngofs < ng_minofs) {
    ng_len += ng_minofs - ngofs;
    ng_minofs = ngofs;
  }
  if (s->endOffset() - minoffset > length) length = s->endOffset() - minoffset;
  if (s->endNgOffset() - ng_minofs > ng_len) ng_len = s->endNgOffset() - ng_minofs;
}

void GSeqAlign::injectGap(GASeq* seq, int pos, int xgap) {  // GapAssem.cpp:720-753
  int alpos = seq->offset + pos;
  for (int i = 0; i <= pos; i++) alpos += seq->gap(i);
  for (GASeq* s : rows_) {
    int spos = 0;
    if (s == seq) {
      spos = pos;
    } else {
      int salpos = s->offset;
      if (salpos >= alpos) {
        s->offset += xgap;
        continue;
      }
      while (spos < s->seqlen) {
        salpos += 1 + s->gap(spos);
        if (salpos > alpos) break;
        spos++;
      }
      if (spos >= s->seqlen) continue;
    }
    s->addGap(spos, (short)xgap);
  }
  length += xgap;
}

void GSeqAlign::removeColumn(int column) {  // GapAssem.cpp:755-779
  const int32_t alpos = column + minoffset;
  for (GASeq* s : rows_) {
    RowView v = view_of(s, &s->numgaps, s->ofs.data());
    remove_columns(v, &alpos, 1);
  }
  length--;
}

void GSeqAlign::removeBase(GASeq* seq, int pos) {  // GapAssem.cpp:781-812
  int alpos = seq->offset + pos;
  for (int i = 0; i <= pos; i++) alpos += seq->gap(i);
  for (GASeq* s : rows_) {
    int spos = 0;
    if (s == seq) {
      spos = pos;
    } else {
      int salpos = s->offset;
      if (salpos >= alpos) {
        s->offset--;
        continue;
      }
      while (spos < s->seqlen) {
        salpos += 1 + s->gap(spos);
        if (salpos > alpos) break;
        spos++;
      }
      if (spos >= s->seqlen) continue;
    }
    s->removeBase(spos);
  }
  length--;
}

void GSeqAlign::applyClipping(AlnClipOps& clipops) {  // GapAssem.cpp:814-822
  for (int i = 0; i < clipops.Count(); i++) {
    SeqClipOp& c = *clipops.Get(i);
    if (c.clp[0] >= 0) c.seq->clp5 = c.clp[0];
    if (c.clp[1] >= 0) c.seq->clp3 = c.clp[1];
  }
}

bool GSeqAlign::evalClipping(GASeq* seq, int c5, int c3, float clipmax, AlnClipOps& clipops) {  // :823-996
  // position of seq[pos] in the layout, and the base of s at or after it (or -1 / seqlen)
  auto layout_pos = [](GASeq* q, int pos) {
    int alpos = q->offset + pos;
    for (int i = 0; i <= pos; i++) alpos += q->gap(i);
    return alpos;
  };
  auto walk = [](GASeq* s, int alpos, bool& starts_after) {
    starts_after = false;
    int spos = 0, salpos = s->offset;
    if (salpos >= alpos) {
      starts_after = true;
      return 0;
    }
    while (spos < s->seqlen) {
      salpos += 1 + s->gap(spos);
      if (salpos > alpos) break;
      spos++;
    }
    return spos;
  };
  const bool rev = seq->revcompl != 0;
  if (c5 >= 0) {
    const int alpos = layout_pos(seq, rev ? seq->seqlen - c5 - 1 : c5);
    for (GASeq* s : rows_) {
      if (s == seq) {
        if (!clipops.add5(s, c5, clipmax)) return false;
        continue;
      }
      bool after;
      const int spos = walk(s, alpos, after);
      if (after) {
        if (rev) return false;
        continue;
      }
      if (spos >= s->seqlen) {
        if (!rev) return false;
        continue;
      }
      const bool srev = s->revcompl != 0;
      bool ok;
      if (rev) ok = srev ? clipops.add5(s, s->seqlen - spos - 1, clipmax) : clipops.add3(s, s->seqlen - spos - 1, clipmax);
      else ok = srev ? clipops.add3(s, spos, clipmax) : clipops.add5(s, spos, clipmax);
      if (!ok) return false;
    }
  }
  if (c3 >= 0) {
    const int alpos = layout_pos(seq, rev ? c3 : seq->seqlen - c3 - 1);
    for (GASeq* s : rows_) {
      if (s == seq) {
        if (!clipops.add3(s, c3, clipmax)) return false;
        continue;
      }
      bool after;
      const int spos = walk(s, alpos, after);
      if (after) {
        if (!rev) return false;
        continue;
      }
      if (spos >= s->seqlen) {
        if (rev) return false;
        continue;
      }
      const bool srev = s->revcompl != 0;
      bool ok;
      if (rev) ok = srev ? clipops.add3(s, spos, clipmax) : clipops.add5(s, spos, clipmax);
      else ok = srev ? clipops.add5(s, s->seqlen - spos - 1, clipmax) : clipops.add3(s, s->seqlen - spos - 1, clipmax);
      if (!ok) return false;
    }
  }
  return true;
}

bool GSeqAlign::addAlign(GASeq* seq, GSeqAlign* omsa, GASeq* oseq) {  // GapAssem.cpp:645-690
  if (seq->seqlen != oseq->seqlen)
    gerror("GSeqAlign Error: invalid merge %s(len %d) vs %s(len %d)\n", seq->getName(), seq->seqlen, oseq->getName(),
           oseq->seqlen);
  if (seq->revcompl != oseq->revcompl) omsa->revComplement();
  for (int i = 0; i < seq->seqlen; i++) {
    const int d = seq->gap(i) - oseq->gap(i);
    if (d > 0) omsa->injectGap(oseq, i, d);
    else if (d < 0) injectGap(seq, i, -d);
  }
  for (int i = 0; i < omsa->Count(); i++) {
    GASeq* s = omsa->Get(i);
    if (s == oseq) continue;
    addSeq(s, seq->offset + s->offset - oseq->offset, seq->ng_ofs + s->ng_ofs - oseq->ng_ofs);
  }
  omsa->setFreeItem(false);
  delete oseq;
  return true;
}

void GSeqAlign::finalize() {  // GapAssem.cpp:1006-1012
  for (GASeq* s : rows_) {
    if (s->len == 0) gerror("Error: sequence for %s not loaded!\n", s->getId());
    if (!s->hasFlag(GA_FLAG_PREPPED)) s->prepSeq();
  }
}

void GSeqAlign::print(FILE* f, char c) {  // GapAssem.cpp:1013-1037
  finalize();
  int mx = 0;
  for (GASeq* s : rows_) mx = std::max(mx, s->getNameLen());
  if (c != 0) {
    fprintf(f, "%*s %c ", mx, " ", ' ');
    for (int k = 0; k < length; k++) fputc(c, f);
    fputc('\n', f);
  }
  for (GASeq* s : rows_) {
    fprintf(f, "%*s %c ", mx, s->name(), s->revcompl == 1 ? '-' : '+');
    s->printGappedSeq(f, minoffset);
  }
}

void GSeqAlign::writeMSA(FILE* f, int linelen) {  // GapAssem.cpp:1039-1046
  finalize();
  for (GASeq* s : rows_) s->printMFasta(f, linelen);
}

void GSeqAlign::extendConsensus(char c) {  // GapAssem.cpp:1185-1198
  consensus.push_back(c);
  consensus_len++;
}

void GSeqAlign::freeMSA() {  // GapAssem.cpp:1108-1119
  delete msacolumns;
  msacolumns = nullptr;
  delete (DevLayout*)dev_;
  dev_ = nullptr;
  for (GASeq* s : rows_) {
    s->seq.clear();
    s->seq.shrink_to_fit();
    s->len = 0;
  }
}

void GSeqAlign::ErrZeroCov(int col) {  // GapAssem.cpp:1121-1131
  fflush(stdout);
  fprintf(stderr, "WARNING: 0 coverage column %d (mincol=%d) found within alignment of %d seqs!\n", col,
          msacolumns->mincol, Count());
  for (GASeq* s : rows_) fprintf(stderr, "%s\n", s->id.c_str());
  ga_exit(5);
}

// buildMSA (GapAssem.cpp:1088-1106) on the GPU: the rows go to HBM once, pw_msa_count scatters
// them into the column histograms, pw_msa_call picks bestChar per column.  The reference's
// messages come out in row order up to the first row whose toMSA fails (a row without loaded
// bases, or a column outside [0, length)), which then GErrors as toMSA would.
void GSeqAlign::buildMSA() {
  if (msacolumns != nullptr) gerror("Error: cannot call buildMSA() twice!\n");
  msacolumns = new MSAColumns(length, minoffset);
  const uint32_t nrows = (uint32_t)Count();
  uint32_t n_stage = nrows;  // rows before the first one without loaded bases
  for (uint32_t i = 0; i < nrows; i++)
    if (rows_[i]->len == 0 || rows_[i]->len != rows_[i]->seqlen) {
      n_stage = i;
      break;
    }
  // first row whose toMSA touches a column outside [0, length): on the GPU (minmax[2]) when the
  // layout has columns, else every row with a base does
  uint32_t bad_row = UINT32_MAX;
  std::vector<int32_t> counts;
  std::vector<uint8_t> bestc;
  int32_t mm[4] = {INT_MAX, -1, INT_MAX, INT_MAX};
  DevLayout* D = nullptr;
  if (length > 0 && n_stage > 0) {
    D = new DevLayout();
    delete (DevLayout*)dev_;
    dev_ = D;
    D->nrows = n_stage;
    std::vector<int32_t> row_len(n_stage), col0(n_stage), cl(n_stage), cr(n_stage);
    D->h_row_off.resize(n_stage);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n_stage; i++) {
      GASeq* s = rows_[i];
      D->h_row_off[i] = total;
      total += ((uint64_t)s->seqlen + 7) / 8 * 8;  // rows start 8-base aligned (count kernels' vector loads)
      row_len[i] = s->seqlen;
      col0[i] = s->offset - minoffset;
      cl[i] = s->revcompl ? s->clp3 : s->clp5;
      cr[i] = s->revcompl ? s->clp5 : s->clp3;
    }
    std::vector<uint8_t> hseq((size_t)std::max<uint64_t>(total, 1), 0);
    std::vector<int16_t> hofs((size_t)std::max<uint64_t>(total, 1), 0);
    for (uint32_t i = 0; i < n_stage; i++) {
      GASeq* s = rows_[i];
      memcpy(hseq.data() + D->h_row_off[i], s->seq.data(), (size_t)s->seqlen);
      memcpy(hofs.data() + D->h_row_off[i], s->ofs.data(), (size_t)s->seqlen * 2);
    }
    std::vector<int64_t> slot_base(n_stage + 1);
    const uint64_t nslots = pw_msa_slots(row_len.data(), n_stage, slot_base.data());
    const size_t ncols = (size_t)length;
    D->seq.alloc(hseq.size());
    D->ofs.alloc(hofs.size());
    D->row_off.alloc(n_stage);
    D->len.alloc(n_stage);
    D->col0.alloc(n_stage);
    D->cl.alloc(n_stage);
    D->cr.alloc(n_stage);
    D->slot.alloc(n_stage + 1);
    D->scr.alloc(pw_msa_scratch_words(nslots, n_stage));
    D->counts.alloc(ncols * 6);
    D->cons.alloc(ncols);
    D->mm.alloc(4);
    hipStream_t st = g_stream;
    hip_check(hipMemcpyAsync(D->seq.p, hseq.data(), hseq.size(), hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->ofs.p, hofs.data(), hofs.size() * 2, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->row_off.p, D->h_row_off.data(), n_stage * 8, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->len.p, row_len.data(), n_stage * 4, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->col0.p, col0.data(), n_stage * 4, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->cl.p, cl.data(), n_stage * 4, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->cr.p, cr.data(), n_stage * 4, hipMemcpyHostToDevice, st), "copy");
    hip_check(hipMemcpyAsync(D->slot.p, slot_base.data(), (n_stage + 1) * 8, hipMemcpyHostToDevice, st), "copy");
    pw_msa_args& a = D->a;
    a.seq = D->seq.p;
    a.ofs = D->ofs.p;
    a.row_off = D->row_off.p;
    a.row_len = D->len.p;
    a.col0 = D->col0.p;
    a.clip_l = D->cl.p;
    a.clip_r = D->cr.p;
    a.slot_base = D->slot.p;
    a.scratch = D->scr.p;
    a.counts = D->counts.p;
    a.consensus = D->cons.p;
    a.minmax = D->mm.p;
    a.n_slots = nslots;
    a.n_rows = n_stage;
    a.n_cols = length;
    if (pw_msa_columns(&a, st) != PW_OK) gerror("GSeqAlign::buildMSA: kernel launch failed\n");
    counts.resize(ncols * 6);
    bestc.resize(ncols);
    hip_check(hipMemcpyAsync(counts.data(), D->counts.p, counts.size() * 4, hipMemcpyDeviceToHost, st), "copy");
    hip_check(hipMemcpyAsync(bestc.data(), D->cons.p, ncols, hipMemcpyDeviceToHost, st), "copy");
    hip_check(hipMemcpyAsync(mm, D->mm.p, sizeof mm, hipMemcpyDeviceToHost, st), "copy");
    hip_check(hipStreamSynchronize(st), "buildMSA");
    if (mm[2] != INT_MAX) bad_row = (uint32_t)mm[2];
  } else if (length <= 0) {
    for (uint32_t i = 0; i < n_stage; i++)
      if (rows_[i]->seqlen > 0) {
        bad_row = i;
        break;
      }
  }
  const uint32_t stop = std::min(bad_row, n_stage);  // the row whose toMSA fails (nrows: none)
  for (uint32_t i = 0; i < nrows && i <= stop; i++) {
    GASeq* seq = rows_[i];
    seq->msaidx = (int)i;
    if (seq->seqlen - seq->clp3 - seq->clp5 < 1) {
      gmessage("Warning: sequence %s (length %d) was trimmed too badly (%d,%d) -- should be removed from MSA w/ %s!\n",
               seq->id.c_str(), seq->seqlen, seq->clp5, seq->clp3, rows_[0]->id.c_str());
      seq->setFlag(GA_FLAG_BAD_ALN);
      badseqs++;
    }
    if (i == stop && stop < nrows) {
      if (stop == n_stage && bad_row != stop) seq->toMSA(*msacolumns);  // GErrors: bases not loaded
      // the first out-of-range column, as toMSA meets it (GapAssem.cpp:568-588)
      const int clipL = seq->revcompl ? seq->clp3 : seq->clp5, clipR = seq->revcompl ? seq->clp5 : seq->clp3;
      int col = seq->offset - minoffset;
      for (int k = 0; k < seq->seqlen; k++) {
        const bool clipped = k < clipL || k >= seq->seqlen - clipR;
        for (int j = 0; j < seq->gap(k); j++) {
          if (!clipped) (*msacolumns)[col];
          col++;
        }
        (*msacolumns)[col];
        col++;
      }
      gerror("GSeqAlign::buildMSA: row %u reported out of range\n", i);  // (not reached)
    }
  }
  // the column histograms and bestChar of the GPU into MSAColumns
  for (size_t c = 0; c < bestc.size(); c++) {
    GAlnColumn& col = msacolumns->columns[c];
    int lay = 0;
    for (int k = 0; k < 6; k++) {
      col.counts[k] = counts[6 * c + (size_t)k];
      lay += col.counts[k];
    }
    col.layers = lay;
    col.consensus = (char)bestc[c];
  }
  if (mm[0] != INT_MAX) msacolumns->updateMinMax(mm[0], mm[1] < 0 ? 0 : mm[1]);
  if (D) D->zero_col = mm[3];
}

// refineMSA (GapAssem.cpp:1133-1183).  The column loop (bestChar, ErrZeroCov, removeColumn of
// every consensus-gap column, extendConsensus) is pw_msa_refine on the GPU: the consensus string
// and, with removeConsGaps, every row's offset / ofs / numgaps after all removeColumn calls (closed
// form; rows holding deleted bases are replayed on the host instead, pw_ga_row_remove_columns).
// Then, per row as the reference does: refineClipping, removeClipGaps, refineClipping(skipDels).
void GSeqAlign::refineMSA(bool redo_ends) {
  if (!redo_ends || msacolumns == nullptr) buildMSA();  // (redo_ends: the reference's TODO branch)
  DevLayout* D = (DevLayout*)dev_;
  const int mincol = msacolumns->mincol, maxcol = msacolumns->maxcol;
  if (D && D->zero_col != INT_MAX) ErrZeroCov(D->zero_col);
  const bool rm = MSAColumns::removeConsGaps;
  consensus.clear();
  consensus_len = 0;
  if (D && mincol != INT_MAX && mincol <= maxcol) {
    hipStream_t st = g_stream;
    const pw_msa_args& a = D->a;
    const uint32_t nr = D->nrows;
    const size_t ncols = (size_t)a.n_cols;
    D->gp.alloc(ncols);
    D->tg.alloc(pw_msa_refine_tiles(a.n_cols));
    D->cout.alloc(ncols);
    D->clen.alloc(1);
    pw_msa_refine_args ra;
    memset(&ra, 0, sizeof ra);
    ra.gap_prefix = D->gp.p;
    ra.tile_gaps = D->tg.p;
    ra.cons_out = D->cout.p;
    ra.cons_len = D->clen.p;
    ra.remove_gaps = rm ? 1u : 0u;
    ra.keep_clip_gaps = 1u;  // refineClipping comes first, on the host
    std::vector<int32_t> off_in(nr), off_out(nr);
    std::vector<int64_t> ng(nr);
    if (rm) {
      D->roffs.alloc(nr);
      D->offo.alloc(nr);
      D->ngo.alloc(nr);
      D->ofso.alloc(D->ofs.n);
      for (uint32_t i = 0; i < nr; i++) {
        off_in[i] = rows_[i]->offset;
        ng[i] = rows_[i]->numgaps;
      }
      hip_check(hipMemcpyAsync(D->roffs.p, off_in.data(), nr * 4, hipMemcpyHostToDevice, st), "copy");
      hip_check(hipMemcpyAsync(D->ngo.p, ng.data(), nr * 8, hipMemcpyHostToDevice, st), "copy");
      ra.row_offset = D->roffs.p;
      ra.ofs_out = D->ofso.p;
      ra.offset_out = D->offo.p;
      ra.numgaps_out = D->ngo.p;
    }
    int32_t clen = 0;
    if (pw_msa_refine(&a, &ra, st) != PW_OK) gerror("GSeqAlign::refineMSA: kernel launch failed\n");
    hip_check(hipMemcpyAsync(&clen, D->clen.p, 4, hipMemcpyDeviceToHost, st), "copy");
    hip_check(hipStreamSynchronize(st), "refineMSA");
    consensus.resize((size_t)clen);
    std::vector<uint8_t> bestc;
    std::vector<int16_t> ofs_out;
    if (clen > 0) hip_check(hipMemcpyAsync(&consensus[0], D->cout.p, (size_t)clen, hipMemcpyDeviceToHost, st), "copy");
    if (rm) {
      ofs_out.resize(D->ofs.n);
      hip_check(hipMemcpyAsync(off_out.data(), D->offo.p, nr * 4, hipMemcpyDeviceToHost, st), "copy");
      hip_check(hipMemcpyAsync(ng.data(), D->ngo.p, nr * 8, hipMemcpyDeviceToHost, st), "copy");
      hip_check(hipMemcpyAsync(ofs_out.data(), D->ofso.p, ofs_out.size() * 2, hipMemcpyDeviceToHost, st), "copy");
    }
    hip_check(hipStreamSynchronize(st), "refineMSA");
    consensus_len = clen;
    if (rm) {
      // the layout positions of the removed columns, in removal order (alpos = col - removed + minoffset)
      std::vector<int32_t> alpos;
      for (int c = mincol; c <= maxcol; c++)
        if (msacolumns->columns[(size_t)c].consensus == '-') alpos.push_back(c - (int32_t)alpos.size() + minoffset);
      for (uint32_t i = 0; i < nr; i++) {
        GASeq* s = rows_[i];
        bool neg = false;
        for (int16_t g : s->ofs) neg = neg || g < 0;
        if (neg) {  // deleted bases: the raw-ofs walk of removeColumn, replayed exactly
          RowView v = view_of(s, &s->numgaps, s->ofs.data());
          remove_columns(v, alpos.data(), alpos.size());
        } else {
          memcpy(s->ofs.data(), ofs_out.data() + D->h_row_off[i], (size_t)s->seqlen * 2);
          s->offset = off_out[i];
          s->numgaps = (int)ng[i];
        }
      }
      length -= (int)alpos.size();
    }
  }
  // refine clipping and remove gaps propagated in the clipping regions (GapAssem.cpp:1163-1181)
  for (GASeq* seq : rows_) {
    if (MSAColumns::refineClipping)
      seq->refineClipping(consensus.data(), consensus_len, rel_col(seq->offset, minoffset, msacolumns->mincol));
    int grem = 0;
    if (rm) grem = seq->removeClipGaps();
    if (grem != 0 && MSAColumns::refineClipping)
      seq->refineClipping(consensus.data(), consensus_len, rel_col(seq->offset, minoffset, msacolumns->mincol), true);
  }
  refinedMSA = true;
}

// FastaSeq::write(f, NULL, NULL, seq, linelen, len) (gclib GFastaFile.h): no header, linelen
// characters per line, a newline after the last one
static void write_fasta_lines(FILE* f, const char* s, int n, int linelen) {
  for (int i = 0, col = 0; i < n; i++, col++) {
    if (col == linelen) {
      fputc('\n', f);
      col = 0;
    }
    fputc(s[i], f);
  }
  fputc('\n', f);
}

void GSeqAlign::writeACE(FILE* f, const char* name) {  // GapAssem.cpp:1200-1262
  if (!refinedMSA) refineMSA();
  int fwd = 0, rvs = 0;
  for (GASeq* s : rows_) (s->revcompl != 0 ? rvs : fwd)++;
  const char consDir = (rvs > fwd) ? 'C' : 'U';
  fprintf(f, "CO %s %d %d 0 %c\n", name, consensus_len, Count(), consDir);
  write_fasta_lines(f, consensus.data(), consensus_len, 60);
  fprintf(f, "\nBQ \n\n");
  for (GASeq* s : rows_)
    fprintf(f, "AF %s %c %d\n", s->id.c_str(), s->revcompl == 0 ? 'U' : 'C',
            rel_col(s->offset, minoffset, msacolumns->mincol) + 1);
  fprintf(f, "\n");
  for (GASeq* s : rows_) {
    const int gapped_len = s->seqlen + s->numgaps;
    fprintf(f, "RD %s %d 0 0\n", s->id.c_str(), gapped_len);
    s->printGappedFasta(f);
    int clpl = s->revcompl == 0 ? s->clp5 : s->clp3, clpr = s->revcompl == 0 ? s->clp3 : s->clp5;
    const int l = clpl, r = clpr;
    for (int j = 1; j <= r; j++) clpr += (s->seqlen - j >= 0 && s->seqlen - j < s->seqlen) ? s->ofs[(size_t)(s->seqlen - j)] : 0;
    for (int j = 0; j <= l; j++) clpl += (j < s->seqlen) ? s->ofs[(size_t)j] : 0;
    int seql = clpl + 1, seqr = gapped_len - clpr;
    if (seqr < seql) {
      fprintf(stderr, "Bad trimming for %s of gapped len %d (%d, %d)\n", s->id.c_str(), gapped_len, seql, seqr);
      seqr = seql + 1;
    }
    fprintf(f, "\nQA %d %d %d %d\nDS \n\n", seql, seqr, seql, seqr);
  }
}

void GSeqAlign::writeInfo(FILE* f, const char* name) {  // GapAssem.cpp:1264-1367
  if (!refinedMSA) refineMSA();
  fprintf(f, ">%s %d %s\n", name, Count(), consensus.c_str());
  for (GASeq* s : rows_) {
    std::string alndata;
    const int gapped_len = s->seqlen + s->numgaps;
    const int seqoffset = rel_col(s->offset, minoffset, msacolumns->mincol) + 1;
    const int asml = seqoffset + 1;
    int asmr = asml - 1;
    float pid = 0;
    const int clpl = s->revcompl == 0 ? s->clp5 : s->clp3, clpr = s->revcompl == 0 ? s->clp3 : s->clp5;
    int aligned_len = 0, indel_ofs = 0;
    for (int j = s->clp5; j < s->seqlen - s->clp3; j++) {
      int indel = (j >= 0) ? s->ofs[(size_t)j] : 0;
      char indel_type = 0;
      asmr += indel + 1;
      if (indel < 0) {
        indel_type = 'd';
        indel = -indel;
      } else {
        if (indel > 0) indel_type = 'g';
        else indel_ofs++;
        const int ci = asmr - 1;
        const char cc = (ci >= 0 && ci < consensus_len) ? consensus[(size_t)ci] : '\0';  // (D11)
        if (j >= 0 && toupper((unsigned char)s->seq[(size_t)j]) == toupper((unsigned char)cc)) pid++;
        aligned_len++;
      }
      if (indel_type) {
        if (indel > 2) {
          char b[48];
          snprintf(b, sizeof b, "%d%c%d-", indel_ofs, indel_type, indel);
          alndata += b;
        } else {
          alndata.append((size_t)indel, indel_type);
        }
        indel_ofs = 0;
      }
    }
    // 0/0 when no base is aligned: x86's default NaN (sign set, printed "-nan"), as the reference's
    // division produces it there, whatever this compiler folds the expression into
    pid = aligned_len ? (pid * 100.0f) / (float)aligned_len : -__builtin_nanf("");
    int seql = clpl + 1, seqr = s->len - clpr;
    if (seqr < seql) {
      fprintf(stderr, "WARNING: Bad trimming for %s of gapped len %d (%d, %d)\n", s->id.c_str(), gapped_len, seql,
              seqr);
      seqr = seql + 1;
    }
    if (s->revcompl) std::swap(seqr, seql);
    fprintf(f, "%s %d %d %d %d %d %d %4.2f %s\n", s->id.c_str(), s->len, seqoffset, asml, asmr, seql, seqr, pid,
            alndata.c_str());
  }
}

// ================================================================== C-ABI: host per-row steps
static RowView view_of_row(pw_ga_row* r) {
  RowView v;
  v.seq = (const char*)r->seq;
  v.ofs = r->ofs;
  v.seqlen = r->seqlen;
  v.numgaps = &r->numgaps;
  v.offset = &r->offset;
  v.clp5 = &r->clp5;
  v.clp3 = &r->clp3;
  v.revcompl = r->revcompl != 0;
  v.id = r->id ? r->id : "";
  return v;
}

extern "C" int pw_ga_row_remove_columns(pw_ga_row* row, const int32_t* alpos, uint64_t n) {
  if (!row || (row->seqlen > 0 && !row->ofs) || (n && !alpos)) return PW_E_ARG;
  remove_columns(view_of_row(row), alpos, n);
  return PW_OK;
}

// refineClipping / removeClipGaps / refineClipping(skipDels) of one row (refineMSA's tail,
// GapAssem.cpp:1163-1181); what the reference prints for the row is appended to msgs, uncut
static int row_finish(pw_ga_row* row, const uint8_t* cons, int32_t cons_len, int32_t cpos_base, uint32_t flags,
                      std::string& msgs) {
  RowView v = view_of_row(row);
  const bool rc = flags & PW_GA_REFINE_CLIP, rm = flags & PW_GA_REMOVE_GAPS;
  std::string err;
  const char* c = (const char*)cons;
  int status = PW_OK;
  if (rc && !refine_clipping(v, c, cons_len, rel_col(row->offset, cpos_base, 0), false, &err, &msgs)) {
    status = 1;
  } else if (rm && remove_clip_gaps(v) != 0 && rc &&
             !refine_clipping(v, c, cons_len, rel_col(row->offset, cpos_base, 0), true, &err, &msgs)) {
    status = 1;
  }
  msgs += err;
  return status;
}

extern "C" int pw_ga_row_finish(pw_ga_row* row, const uint8_t* cons, int32_t cons_len, int32_t cpos_base,
                                uint32_t flags, char* msgbuf, size_t msglen) {
  if (!row || (row->seqlen > 0 && (!row->ofs || !row->seq)) || (cons_len > 0 && !cons)) return PW_E_ARG;
  std::string msgs;
  const int status = row_finish(row, cons, cons_len, cpos_base, flags, msgs);
  if (msgbuf && msglen) snprintf(msgbuf, msglen, "%s", msgs.c_str());
  return status;
}

// The per-row tail for many rows in one call (the multi-GPU driver's own rows): rows with
// replay[k] != 0 first get removeColumn replayed for alpos (pw_ga_row_remove_columns), then every
// row pw_ga_row_finish.  Messages back to back in msgbuf (row k's are [msg_off[k], msg_off[k+1]));
// failed[k] = 1 after a GError.  Stops after the first failing row (the reference exits there);
// returns the number of rows processed.  When the messages do not fit in msg_cap, every row is
// restored to its input state (ofs, offset, numgaps, clips), msg_off still holds the full sizes
// (msg_off[k] > msg_cap): the caller calls again with a buffer of msg_off[k] bytes.
extern "C" int64_t pw_ga_rows_finish(pw_ga_row* rows, uint64_t n, const uint8_t* replay, const int32_t* alpos,
                                     uint64_t n_alpos, const uint8_t* cons, int32_t cons_len, int32_t cpos_base,
                                     uint32_t flags, char* msgbuf, uint64_t msg_cap, uint64_t* msg_off,
                                     int32_t* failed) {
  if ((n && (!rows || !msg_off || !failed)) || (n_alpos && !alpos)) return PW_E_ARG;
  for (uint64_t k = 0; k < n; k++)
    if (rows[k].seqlen < 0 || (rows[k].seqlen > 0 && (!rows[k].ofs || !rows[k].seq))) return PW_E_ARG;
  if (cons_len > 0 && !cons) return PW_E_ARG;
  struct Saved {
    int32_t offset, numgaps, clp5, clp3;
    std::vector<int16_t> ofs;
  };
  std::vector<Saved> saved(n);
  for (uint64_t k = 0; k < n; k++) {
    saved[k] = {rows[k].offset, rows[k].numgaps, rows[k].clp5, rows[k].clp3, {}};
    saved[k].ofs.assign(rows[k].ofs, rows[k].ofs + rows[k].seqlen);
  }
  std::string msgs;
  msg_off[0] = 0;
  uint64_t k = 0;
  for (; k < n; k++) {
    failed[k] = 0;
    if (replay && replay[k]) remove_columns(view_of_row(&rows[k]), alpos, n_alpos);
    const int rc = row_finish(&rows[k], cons, cons_len, cpos_base, flags, msgs);
    msg_off[k + 1] = msgs.size();
    if (rc == 1) {
      failed[k] = 1;
      k++;
      break;
    }
  }
  if (msgs.size() > msg_cap || (!msgbuf && !msgs.empty())) {
    for (uint64_t j = 0; j < n; j++) {
      rows[j].offset = saved[j].offset;
      rows[j].numgaps = saved[j].numgaps;
      rows[j].clp5 = saved[j].clp5;
      rows[j].clp3 = saved[j].clp3;
      std::copy(saved[j].ofs.begin(), saved[j].ofs.end(), rows[j].ofs);
    }
    return (int64_t)k;
  }
  if (!msgs.empty()) memcpy(msgbuf, msgs.data(), msgs.size());
  return (int64_t)k;
}
