/* pwasm_gapassem.hpp — the GapAssem C++ API (GASeq, GAlnColumn, MSAColumns, GSeqAlign) on the
 * MI355X path.  Drop-in for gpertea/pwasm GapAssem.h: the same class names, members, methods,
 * argument meaning, messages and exit behaviour, so a caller switches by including this header
 * instead of GapAssem.h and linking libpwasm_amd.so.
 *
 *   GASeq        GapAssem.h:35-138     setGap/addGap/removeBase, refineClipping (X-drop),
 *                                      removeClipGaps, revComplement, print*, toMSA
 *   GAlnColumn   GapAssem.h:255-342    the six counters + bestChar (GapAssem.cpp:1048-1069)
 *   MSAColumns   GapAssem.h:345-376    removeConsGaps / refineClipping statics (GapAssem.cpp:5-6)
 *   GSeqAlign    GapAssem.h:381-461    pairwise creation, addSeq, injectGap, addAlign,
 *                                      removeColumn, refineMSA, writeACE / writeMSA / writeInfo
 *
 * GSeqAlign::buildMSA() and refineMSA() run on the GPU: the rows are staged in HBM and the
 * column histograms, bestChar and the removeConsGaps column edits come from the pw_msa_* kernels
 * (pwasm_amd.h).  The per-row work the reference does after the consensus — refineClipping's
 * X-drop, removeClipGaps, and the removeColumn edits of rows holding deleted bases (ofs < 0) —
 * runs on the host per row (pw_ga_row_* in pwasm_amd.h), in the reference's order.
 *
 * Differences from GapAssem.h, all at the container level:
 *   - GASeq keeps its bases in `seq` / `len` like gclib's FastaSeq, without deriving from it;
 *   - GSeqAlign holds its rows in a vector (Count() / Get(i)); Sort() orders them by offset with
 *     a stable sort (gclib's GList sort is a quicksort: equal offsets may come out in another
 *     order there);
 *   - GAlnColumn keeps counts, not the per-base NucOri lists (remove() is not provided: nothing
 *     on refineMSA's path calls it);
 *   - GError (print + exit(1)) is the default error action; pw_ga_set_error_handler() may
 *     replace it (e.g. to throw).
 */
#ifndef PWASM_GAPASSEM_HPP
#define PWASM_GAPASSEM_HPP

#include <limits.h>
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

class GSeqAlign;
class MSAColumns;

#define GA_FLAG_IS_REF 0
#define GA_FLAG_HAS_PARENT 1
#define GA_FLAG_PREPPED 2
#define GA_FLAG_BAD_ALN 7

/* Called with the formatted message of a GError (GapAssem.cpp:105-107, 240-242, 648-649,
 * 1009, 1090; GapAssem.h:367-368).  The default prints it to stderr and exits with status 1. */
typedef void (*pw_ga_error_fn)(const char* msg);
void pw_ga_set_error_handler(pw_ga_error_fn fn);
/* While a pw_ga_exit_scope lives on this thread, the exits the reference takes (GError: 1,
 * ErrZeroCov: 5) throw pw_ga_exit{code} instead, after the same messages. */
struct pw_ga_exit {
  int code;
};
struct pw_ga_exit_scope {
  pw_ga_exit_scope();
  ~pw_ga_exit_scope();
};
/* HIP stream for GSeqAlign::buildMSA / refineMSA (NULL: the default stream). */
void pw_ga_set_stream(void* stream);

class GASeq {
 protected:
  int numgaps;               // total of ofs[]
  std::vector<int16_t> ofs;  // gap before each base; negative = deleted base
  void prepSeq();            // reverse-complement when revcompl (GapAssem.cpp:89-101)

 public:
  // FastaSeq part
  std::string id, descr;
  std::string seq;  // the bases
  int len;          // seq.size() once loaded, else 0
  // GASeq part (GapAssem.h:51-65)
  unsigned char flags;
  GSeqAlign* msa;
  int msaidx;
  int seqlen;   // size of ofs
  int offset;   // offset in the layout
  int ng_ofs;   // non-gapped offset (clipping constraints)
  char revcompl;
  int ext5, ext3;
  int clp5, clp3;

  GASeq(const char* sname = NULL, int slen = 0);
  GASeq(const char* sname, const char* sdescr, const char* sseq, int slen = 0, int soffset = 0);
  GASeq(const char* sname, int soffset, int slen, int sclipL = 0, int sclipR = 0, char rev = 0);
  GASeq(GASeq& aseq);  // copy constructor: id, descr, bases; no gaps, offset 0
  virtual ~GASeq() {}

  const char* getId() const { return id.c_str(); }
  const char* getName() const { return id.c_str(); }
  const char* name() const { return id.c_str(); }
  int getNameLen() const { return (int)id.size(); }
  void allupper();
  void lowercase();
  void reverseComplement();
  bool operator==(const GASeq& d) const { return offset == d.offset && id == d.id; }
  bool operator>(const GASeq& d) const { return offset > d.offset; }
  bool operator<(const GASeq& d) const { return offset < d.offset; }
  friend class GSeqAlign;

  void refineClipping(const char* cons, int cons_len, int cpos, bool skipDels = false);
  void setGap(int pos, short gaplen = 1);
  void addGap(int pos, short gapadd);
  void setFlag(unsigned char bitno) { flags |= (unsigned char)(1u << bitno); }
  void clearFlag(unsigned char bitno) { flags ^= (unsigned char)(1u << bitno); }
  bool hasFlag(unsigned char bitno) const { return ((1u << bitno) & flags) != 0; }
  int getNumGaps() const { return numgaps; }
  int gap(int pos) const { return ofs[(size_t)pos]; }
  const int16_t* gaps() const { return ofs.data(); }
  void removeBase(int pos);
  int endOffset() const { return offset + seqlen + numgaps; }
  int endNgOffset() const { return ng_ofs + seqlen; }
  int removeClipGaps();
  void printGappedSeq(FILE* f, int baseoffs = 0);
  void printGappedSeq(int baseoffs = 0) { printGappedSeq(stdout, baseoffs); }
  void printGappedFasta(FILE* f);
  void printMFasta(FILE* f, int llen = 60);
  void reverseGaps();
  void revComplement(int alignlen = 0);
  void toMSA(MSAColumns& msa);  // host scatter (small layouts; buildMSA uses the GPU)
};

/* Clipping propagation (GapAssem.h:163-253; GSeqAlign::evalClipping / applyClipping). */
struct SeqClipOp {
  GASeq* seq;
  int clp[2];
  SeqClipOp(GASeq* s, int newclp5, int newclp3 = -1) : seq(s), clp{newclp5, newclp3} {}
};
class AlnClipOps {
  std::vector<SeqClipOp> ops_;

 public:
  char q_rev;
  int d5, d3;
  int total;
  AlnClipOps() : q_rev(0), d5(0), d3(0), total(0) {}
  int Count() const { return (int)ops_.size(); }
  SeqClipOp* Get(int i) { return &ops_[(size_t)i]; }
  void Add(const SeqClipOp& op) { ops_.push_back(op); }
  bool add5(GASeq* s, int clp, float clipmax);
  bool add3(GASeq* s, int clp, float clipmax);
  bool add(GASeq* s, int clp5, int clp3, float clipmax);
};

class GAlnColumn {
 public:
  enum { ncA = 0, ncC, ncG, ncT, ncN, ncGap };
  int counts[6];  // A, C, G, T, N, - (GapAssem.h:263 order)
  bool hasClip;
  char consensus;
  int layers;
  GAlnColumn() : counts{0, 0, 0, 0, 0, 0}, hasClip(false), consensus(0), layers(0) {}
  void addGap() {
    counts[ncGap]++;
    layers++;
  }
  void addNuc(GASeq* seq, int pos, bool clipped = false);
  char bestChar();
};

class MSAColumns {
  int size;

 public:
  static bool removeConsGaps;
  static bool refineClipping;
  std::vector<GAlnColumn> columns;
  int baseoffset;
  int mincol;
  int maxcol;
  MSAColumns(int len, int baseofs = 0) : size(len), columns((size_t)(len > 0 ? len : 0)), baseoffset(baseofs),
                                         mincol(INT_MAX), maxcol(0) {}
  GAlnColumn& operator[](int idx);
  int len() const { return maxcol - mincol + 1; }
  int capacity() const { return size; }
  void updateMinMax(int minc, int maxc) {
    if (minc < mincol) mincol = minc;
    if (maxc > maxcol) maxcol = maxc;
  }
};

class GSeqAlign {
  std::vector<GASeq*> rows_;
  bool free_items_;
  void* dev_;  // device staging of buildMSA kept for refineMSA (pw_ga_api.cpp)
  int length;
  int minoffset;
  void buildMSA();
  void ErrZeroCov(int col);

 public:
  bool refinedMSA;
  MSAColumns* msacolumns;
  unsigned int ordnum;
  int ng_len;
  int ng_minofs;
  int badseqs;
  std::string consensus;  // built by refineMSA()
  int consensus_len;
  friend class GASeq;
  bool operator==(const GSeqAlign& d) const { return this == &d; }
  bool operator>(const GSeqAlign& d) const { return this > &d; }
  bool operator<(const GSeqAlign& d) const { return this < &d; }

  GSeqAlign();
  GSeqAlign(bool sorted, bool free_elements = true, bool beUnique = false);
  GSeqAlign(GASeq* s1, GASeq* s2);  // first creation from a pairwise alignment
  // pwasm: a layout of rows placed at their own offsets (= GSeqAlign(s1, s2) + addSeq(s, s->offset,
  // s->ng_ofs) for the rest; minoffset / length from all rows, also for a single row)
  explicit GSeqAlign(const std::vector<GASeq*>& rows);
  ~GSeqAlign();
  void incOrd() { ordnum++; }
  int len() const { return length; }
  int minOffset() const { return minoffset; }
  // GList part
  int Count() const { return (int)rows_.size(); }
  GASeq* Get(int i) const { return rows_[(size_t)i]; }
  void Add(GASeq* s) { rows_.push_back(s); }
  void setFreeItem(bool v) { free_items_ = v; }
  void Sort();

  void revComplement();
  void addSeq(GASeq* s, int soffs, int ngofs);
  void injectGap(GASeq* seq, int pos, int xgap);
  void removeBase(GASeq* seq, int pos);
  void extendConsensus(char c);
  bool addAlign(GASeq* seq, GSeqAlign* omsa, GASeq* oseq);
  void applyClipping(AlnClipOps& clipops);
  bool evalClipping(GASeq* seq, int c5, int c3, float clipmax, AlnClipOps& clipops);
  void finalize();
  void print(FILE* f, char c = 0);
  void print() { print(stdout); }
  void removeColumn(int column);
  void freeMSA();
  void refineMSA(bool redo_ends = false);
  void writeACE(FILE* f, const char* name);
  void writeMSA(FILE* f, int linelen = 60);
  void writeInfo(FILE* f, const char* name);
};

#endif
