// pw_host.cpp — host side of libpwasm_amd.so: the CPU pre-pass (PAF record -> packed cs op
// stream), batch staging on the GPU, and the `pafreport` CLI (pafreport.cpp:175-460) driving
// the HIP kernels of pw_report.hip.  Everything the reference prints is printed here, in the
// reference's order, from the per-record results the GPU returns; there is no CPU fallback:
// without a usable gfx950 device the CLI stops with an error.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "pwasm_amd.h"

namespace {

// ----------------------------------------------------------------- small helpers
std::string strf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
std::string strf(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  va_list ap2;
  va_copy(ap2, ap);
  int n = vsnprintf(nullptr, 0, fmt, ap);
  va_end(ap);
  std::string s((size_t)(n > 0 ? n : 0), '\0');
  if (n > 0) vsnprintf(&s[0], (size_t)n + 1, fmt, ap2);
  va_end(ap2);
  return s;
}

// gclib parseInt: skip blanks, optional sign, digits; false (p unchanged) if no digit.
bool parse_int(const char*& p, int& out) {
  const char* q = p;
  while (*q == ' ' || *q == '\t') q++;
  const char* start = q;
  if (*q == '-' || *q == '+') q++;
  const char* dig = q;
  while (*q >= '0' && *q <= '9') q++;
  if (q == dig) return false;
  out = (int)strtol(start, nullptr, 10);
  p = q;
  return true;
}

inline bool is_alpha(unsigned char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
inline unsigned char up(unsigned char c) { return (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c; }

// Device copies of the query and literal arrays carry this many readable bytes past their end:
// the report kernel stages them into LDS with 16-byte loads (pw_report.hip).
constexpr size_t kDevPad = 256;

// Per-event report-line byte bounds (see DESIGN.md §Text slots): the kernel never writes past them.
constexpr uint64_t kBoundSub = 190, kBoundIndel = 140;

}  // namespace

// ================================================================= cs packer (CPU pre-pass)
// Mirrors the cs loop of PAFAlignment::PAFAlignment (pafreport.cpp:536-626) without touching
// the query: only lengths, literal bytes and the positions needed for the reference's
// bounds-free reads are produced.
extern "C" int pw_pack_cs(const char* cs, int32_t offset, int32_t qlen, uint32_t* ops, size_t ops_cap,
                          uint8_t* lits, size_t lits_cap, pw_cs_totals* tot, int32_t* err_pos) {
  if (!cs || !tot) return PW_CS_PARSE;
  int qpos = 0, tpos = 0;
  uint32_t nops = 0, nlits = 0, nev = 0;
  uint64_t bound = 0;
  int rc = PW_CS_OK;
  const char* p = cs;
  auto fail = [&](int code, const char* at) {
    rc = code;
    if (err_pos) *err_pos = (int32_t)(at - cs);
  };
  auto push_op = [&](uint32_t w) -> bool {
    if (nops >= ops_cap) return false;
    ops[nops++] = w;
    return true;
  };
  while (*p != 0 && rc == PW_CS_OK) {
    const char op = *p;
    p++;
    switch (op) {
      case ':': {
        int cl = 0;
        if (!parse_int(p, cl)) {
          fail(PW_CS_PARSE, p);
          break;
        }
        if (cl < 0 || offset + qpos < 0 || (int64_t)offset + qpos + cl > qlen) {
          fail(PW_CS_BOUNDS, p);
          break;
        }
        if (cl > 0) {
          if (!push_op(PW_OP(PW_OP_MATCH, (uint32_t)cl))) {
            fail(PW_CS_NOSPACE, p);
            break;
          }
        }
        qpos += cl;
        tpos += cl;
        break;
      }
      case '*': {
        if (p[0] == 0 || p[1] == 0) {
          fail(PW_CS_PARSE, p);
          break;
        }
        const int q_pos = offset + qpos;
        if (q_pos < 0 || q_pos > qlen) {  // q_pos == qlen reads the NUL terminator: mismatch on GPU
          fail(PW_CS_BOUNDS, p);
          break;
        }
        if (nlits + 2 > lits_cap || !push_op(PW_OP(PW_OP_SUB, 1))) {
          fail(PW_CS_NOSPACE, p);
          break;
        }
        lits[nlits++] = up((unsigned char)p[0]);
        lits[nlits++] = up((unsigned char)p[1]);
        p += 2;
        qpos++;
        tpos++;
        nev++;
        bound += kBoundSub;
        break;
      }
      case '-': {
        const char* s0 = p;
        while (is_alpha((unsigned char)*p)) p++;
        const uint32_t n = (uint32_t)(p - s0);
        if (n == 0) {
          fail(PW_CS_EMPTY, p);
          break;
        }
        if (nlits + n > lits_cap || !push_op(PW_OP(PW_OP_INS, n))) {
          fail(PW_CS_NOSPACE, p);
          break;
        }
        for (uint32_t i = 0; i < n; i++) lits[nlits++] = up((unsigned char)s0[i]);
        tpos += (int)n;
        nev++;
        bound += kBoundIndel;
        break;
      }
      case '+': {
        const char* s0 = p;
        while (is_alpha((unsigned char)*p)) p++;
        const int n = (int)(p - s0);
        if (n == 0) {
          fail(PW_CS_EMPTY, p);
          break;
        }
        const int q_pos = offset + qpos;
        if (q_pos < 0 || (int64_t)q_pos + n > qlen) {
          fail(PW_CS_BOUNDS, p);
          break;
        }
        if (!push_op(PW_OP(PW_OP_DEL, (uint32_t)n))) {
          fail(PW_CS_NOSPACE, p);
          break;
        }
        qpos += n;
        nev++;
        bound += kBoundIndel;
        break;
      }
      case '~':
        fail(PW_CS_SPLICED, p);
        break;
      default:
        fail(PW_CS_UNHANDLED, p);
        break;
    }
  }
  tot->q_total = qpos;
  tot->t_total = tpos;
  tot->n_ops = nops;
  tot->n_lits = nlits;
  tot->n_events_max = nev;
  tot->text_bound = bound;
  return rc;
}

// ================================================================= batch structures
namespace {

struct QueryDb {
  std::vector<std::string> ids;
  std::vector<uint64_t> off;
  std::vector<int32_t> len;
  std::vector<uint8_t> seq;  // upper case (GASeq::allupper, pafreport.cpp:350)
  std::unordered_map<std::string, int> index;
  std::vector<uint8_t> acgt;  // per query: all bases in {A,C,G,T}
  bool all_acgt(int qi) const { return acgt[qi] != 0; }
  static bool is_acgt_byte(uint8_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }
  // Each sequence starts 16-byte aligned and is followed by >= 64 zero bytes: the kernels'
  // 16-byte-aligned LDS windows then read NUL past the end of a query, as the reference reads
  // the string terminator (never the next query's bases).
  void close_record() {
    len.back() = (int32_t)(seq.size() - off.back());
    bool ok = true;
    for (size_t i = off.back(); i < seq.size() && ok; i++) ok = is_acgt_byte(seq[i]);
    acgt.push_back(ok ? 1 : 0);
    seq.resize((seq.size() + 15) / 16 * 16 + 64, 0);
  }
  bool load(const char* path, std::string& err) {
    FILE* f = fopen(path, "rb");
    if (!f) {
      err = strf("Error: invalid FASTA file %s !\n", path);
      return false;
    }
    std::vector<char> buf(1 << 20);
    std::string line;
    bool have = false;
    auto flush_line = [&](std::string& l) {
      if (!l.empty() && l[0] == '>') {
        size_t e = 1;
        while (e < l.size() && !isspace((unsigned char)l[e])) e++;
        std::string id = l.substr(1, e - 1);
        if (have) close_record();
        ids.push_back(id);
        off.push_back(seq.size());
        len.push_back(0);
        if (!index.count(id)) index.emplace(id, (int)ids.size() - 1);
        have = true;
      } else if (have) {
        for (char c : l) seq.push_back(up((unsigned char)c));
      }
      l.clear();
    };
    size_t n;
    while ((n = fread(buf.data(), 1, buf.size(), f)) > 0) {
      for (size_t i = 0; i < n; i++) {
        char c = buf[i];
        if (c == '\n') flush_line(line);
        else if (c != '\r') line.push_back(c);
      }
    }
    if (!line.empty()) flush_line(line);
    if (have) close_record();
    fclose(f);
    return true;
  }
};

struct Options {
  bool fullgenome = false, skip_codan = false, verbose = false;
  bool single_query_gene = false;  // rlabel "" (pafreport.cpp:378-379)
};

struct RecHost {
  uint32_t line_off, line_len;  // original line in the batch text (for messages)
  uint32_t hdr_off, hdr_len;    // header line in the header pool
  int32_t pre_msg = -1;         // message index: fatal before the cs loop
  int32_t cs_msg = -1;          // fatal from the host cs parse (after GPU mismatch)
  int32_t post_msg = -1;        // fatal from the CIGAR loop / length checks
  uint16_t n_softclip = 0;
  int32_t qlen = 0;
};

// Ordered log of what a batch prints: messages, records, a terminating fatal.
struct LogItem {
  uint8_t kind;  // 0 message, 1 record, 2 fatal
  uint32_t idx;
  uint64_t line;  // 0-based input line it came from (shard merge order)
};

struct Batch {
  std::string text;     // raw lines of this batch (messages quote them)
  std::string hdr;      // report headers
  std::vector<std::string> msgs;
  std::vector<LogItem> log;
  std::vector<RecHost> recs;
  std::vector<pw_aln_desc> desc;
  std::vector<uint32_t> ops;
  std::vector<uint8_t> lits;
  uint64_t text_total = 0, n_events_max = 0;
  bool fatal = false;
  void clear() {
    text.clear();
    hdr.clear();
    msgs.clear();
    log.clear();
    recs.clear();
    desc.clear();
    ops.clear();
    lits.clear();
    text_total = n_events_max = 0;
    fatal = false;
  }
  uint32_t add_msg(std::string m) {
    msgs.push_back(std::move(m));
    return (uint32_t)msgs.size() - 1;
  }
  uint64_t cur_line = 0;  // input line being packed
  void log_msg(std::string m) { log.push_back({0, add_msg(std::move(m)), cur_line}); }
  void log_fatal(std::string m) {
    log.push_back({2, add_msg(std::move(m)), cur_line});
    fatal = true;
  }
};

const char* CIGAR_ERROR = "Error parsing cigar string from line: %s (cigar position: %s)\n";
const char* CS_ERROR = "Error parsing cs string from line: %s (cs position: %s)\n";

struct Packer {
  const QueryDb* qdb;
  Options opt;
  std::unordered_map<std::string, int> alnpairs;  // q~t (gene mode), persists across batches
  std::vector<char*> t;
  uint64_t n_lines = 0;  // input lines seen (across batches)

  // Handle one input line (pafreport.cpp:304-382).  Returns false after a fatal error.
  bool add_line(Batch& b, const char* line0, size_t n) {
    b.cur_line = n_lines++;
    if (n > 0 && line0[0] == '#') return true;
    const uint32_t loff = (uint32_t)b.text.size();
    b.text.append(line0, n);
    b.text.push_back('\0');
    const char* lstr = b.text.data() + loff;  // the untouched copy (lstr)
    std::string work(line0, n);               // split copy
    char* s = &work[0];
    t.clear();
    bool after = true;
    for (size_t i = 0; i < n; i++) {  // strsplit(line, t, '\t')
      if (after) t.push_back(s + i);
      after = false;
      if (s[i] == '\t') {
        s[i] = 0;
        after = true;
      }
    }
    const int numt = (int)t.size();
    if (numt < 15) {
      b.log_fatal(strf("Error: invalid PAF fline (num. fields=%d):\n%s\n", numt, lstr));
      return false;
    }
    const bool reverse = t[4][0] == '-';
    const char* r_id = t[0];
    const int r_len = atoi(t[1]), r_alnstart = atoi(t[2]), r_alnend = atoi(t[3]);
    const char* t_id = t[5];
    const int t_alnstart = atoi(t[7]), t_alnend = atoi(t[8]);
    if (strcmp(r_id, t_id) == 0) {
      if (opt.verbose) b.log_msg("Skipping alignment of qry seq to itself.\n");
      return true;
    }
    if (!opt.fullgenome) {
      std::string key(r_id);
      key.push_back('~');
      key.append(t_id);
      auto it = alnpairs.find(key);
      if (it == alnpairs.end()) alnpairs.emplace(std::move(key), 0);
      else {
        ++it->second;
        if (it->second == 1) b.log_msg(strf("Warning: alignment %s to %s already seen, ignoring \n", r_id, t_id));
        return true;
      }
    }
    auto qit = qdb->index.find(r_id);
    if (qit == qdb->index.end()) {
      b.log_fatal(strf("Error: could not retrieve sequence for %s !\n", r_id));
      return false;
    }
    const int qi = qit->second;
    const int L = qdb->len[qi];
    if (r_len != L) {
      b.log_fatal(strf("Error: ref seq len in this PAF line (%d) differs from loaded sequence length(%d)!\n%s\n",
                       r_len, L, lstr));
      return false;
    }
    // ---- record
    RecHost rh;
    rh.line_off = loff;
    rh.line_len = (uint32_t)n;
    rh.qlen = L;
    const int offset = reverse ? r_len - r_alnend : r_alnstart;
    const int eff_t_len = t_alnend - t_alnstart;
    int edist = -1, alnscore = 0;
    const char* cigar = nullptr;
    const char* cs = nullptr;
    int got = 0;
    for (int i = 12; i < numt; ++i) {  // tag scan, pafreport.cpp:495-520
      if (!strncmp(t[i], "NM:i:", 5)) {
        edist = atoi(t[i] + 5);
        got |= 1;
      } else if (!strncmp(t[i], "AS:i:", 5)) {
        alnscore = atoi(t[i] + 5);
        got |= 2;
      } else if (!strncmp(t[i], "cg:Z:", 5)) {
        cigar = t[i] + 5;
        got |= 4;
      } else if (!strncmp(t[i], "cs:Z:", 5)) {
        cs = t[i] + 5;
        got |= 8;
      } else continue;
      if (got == 15) break;
    }
    pw_aln_desc d;
    d.op_begin = (uint32_t)b.ops.size();
    d.n_ops = 0;
    d.lit_begin = (uint32_t)b.lits.size();
    d.ref = (uint32_t)qi | (reverse ? PW_REF_REVERSE : 0u);
    d.offset = offset;
    d.t_len = 0;
    d.ev_begin = b.n_events_max;
    if (cigar == nullptr || cigar[0] == 0) {
      rh.pre_msg = (int32_t)b.add_msg(strf(CIGAR_ERROR, lstr, "(null)"));
    } else if (cs == nullptr) {
      rh.pre_msg = (int32_t)b.add_msg(strf("Error: cs tag missing at line:\n%s\n", lstr));
    } else {
      // pack cs (grow the arrays to the worst case first: one op per cs byte)
      const size_t cslen = strlen(cs);
      b.ops.resize(d.op_begin + cslen + 1);
      b.lits.resize(d.lit_begin + cslen + 1);
      pw_cs_totals tot;
      int32_t epos = 0;
      int rc = pw_pack_cs(cs, offset, L, b.ops.data() + d.op_begin, cslen + 1, b.lits.data() + d.lit_begin,
                          cslen + 1, &tot, &epos);
      b.ops.resize(d.op_begin + tot.n_ops);
      b.lits.resize(d.lit_begin + tot.n_lits);
      d.n_ops = tot.n_ops;
      d.t_len = tot.t_total;
      // fast-path flag for the kernels: the query and this record's literal bytes are A/C/G/T
      bool acgt = rc == PW_CS_OK && qdb->all_acgt((int)qi);
      for (uint32_t i = 0; i < tot.n_lits && acgt; i++) acgt = QueryDb::is_acgt_byte(b.lits[d.lit_begin + i]);
      if (acgt) d.ref |= PW_REF_ACGT;
      b.text_total += tot.text_bound;
      b.n_events_max += tot.n_events_max;
      if (rc != PW_CS_OK) {
        const char* at = cs + epos;
        std::string m;
        switch (rc) {
          case PW_CS_PARSE: m = strf(CS_ERROR, lstr, at); break;
          case PW_CS_SPLICED: m = strf("Error: spliced alignments not supported! at line:\n%s\n", lstr); break;
          case PW_CS_UNHANDLED: m = strf("Error: unhandled event at %s in cs, line:\n%s\n", at, lstr); break;
          case PW_CS_EMPTY: m = strf("Error: empty indel in cs string at line:\n%s\n", lstr); break;
          case PW_CS_BOUNDS: m = strf("Error: cs string extends beyond query sequence at line:\n%s\n", lstr); break;
          default: m = strf("Error: cs string too long at line:\n%s\n", lstr); break;
        }
        rh.cs_msg = (int32_t)b.add_msg(std::move(m));
      } else {
        // CIGAR loop (pafreport.cpp:645-718): warnings and errors come after the cs loop
        const char* p = cigar;
        int qpos = 0, tpos = 0;
        std::string err;
        while (*p != '\0') {
          int cl = 0;
          if (!parse_int(p, cl)) {
            err = strf(CIGAR_ERROR, lstr, p);
            break;
          }
          const char cop = *p;
          if (cop == '\0') {
            err = strf(CIGAR_ERROR, lstr, p);
            break;
          }
          bool bad = false;
          switch (cop) {
            case 'X':
            case 'M':
            case '=':
              tpos += cl;
              qpos += cl;
              break;
            case 'P':
            case 'H': break;
            case 'S':
              qpos += cl;
              rh.n_softclip++;
              break;
            case 'I': qpos += cl; break;
            case 'D':
            case 'N': tpos += cl; break;
            default:
              err = strf("Error: unhandled cigar_op %c (len %d) in %s\n", cop, cl, lstr);
              bad = true;
          }
          if (bad) break;
          ++p;
        }
        if (err.empty()) {
          if (eff_t_len != tpos || tot.t_total != tpos)
            err = strf("Error: tseq alignment length mismatch (%d vs %d(%d-%d)) at line:%s\n", tpos, eff_t_len,
                       t_alnend, t_alnstart, lstr);
          else if (r_alnend - r_alnstart != qpos)
            err = strf("Error: ref alignment length mismatch (%d vs %d-%d) at line:%s\n", qpos, r_alnend,
                       r_alnstart, lstr);
        }
        if (!err.empty()) rh.post_msg = (int32_t)b.add_msg(std::move(err));
      }
    }
    // header (printDiffInfo, pafreport.cpp:886-892; labels :366-379)
    std::string tlabel = strf("%s:%d-%d%c", t_id, t_alnstart, t_alnend, reverse ? '-' : '+');
    std::string rlabel(r_id);
    if (opt.fullgenome) rlabel += strf(":%d-%d", r_alnstart, r_alnend);
    if (opt.single_query_gene) rlabel.clear();
    const double cov = ((r_alnend - r_alnstart) * 100.00) / r_len;
    std::string hdr = rlabel.empty()
                          ? strf(">%s coverage:%.2f score=%d edit_distance=%d\n", tlabel.c_str(), cov, alnscore, edist)
                          : strf(">%s--%s coverage:%.2f score=%d edit_distance=%d\n", rlabel.c_str(), tlabel.c_str(),
                                 cov, alnscore, edist);
    rh.hdr_off = (uint32_t)b.hdr.size();
    rh.hdr_len = (uint32_t)hdr.size();
    b.hdr += hdr;
    b.desc.push_back(d);
    b.recs.push_back(rh);
    b.log.push_back({1, (uint32_t)b.recs.size() - 1, b.cur_line});
    return true;
  }
};

// ----------------------------------------------------------------- device state
#define HIPCHK(x)                                                                             \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "pafreport (HIP): %s failed: %s\n", #x, hipGetErrorString(e_));         \
      return false;                                                                           \
    }                                                                                         \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    size_t c = n + n / 4 + 64;
    if (hipMalloc((void**)&p, c * sizeof(T)) != hipSuccess) {
      p = nullptr;
      cap = 0;
      return false;
    }
    cap = c;
    return true;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

struct Device {
  hipStream_t stream = nullptr;
  DevBuf<uint8_t> qseq;
  DevBuf<uint64_t> qoff;
  DevBuf<int32_t> qlen, next_stop;
  DevBuf<pw_aln_desc> desc;
  DevBuf<uint32_t> ops;
  DevBuf<uint8_t> lits, text, work;
  DevBuf<pw_aln_result> res;
  DevBuf<pw_page> pages;
  uint32_t nq = 0;
  bool init(const QueryDb& q, bool skip_codan) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      fprintf(stderr, "pafreport: no HIP device available (this build has no CPU path)\n");
      return false;
    }
    HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    nq = (uint32_t)q.len.size();
    if (!qseq.ensure(q.seq.size() + kDevPad) || !qoff.ensure(nq + 1) || !qlen.ensure(nq + 1) ||
        (!skip_codan && !next_stop.ensure(q.seq.size() + 1))) {
      fprintf(stderr, "pafreport: device allocation failed\n");
      return false;
    }
    if (!q.seq.empty()) HIPCHK(hipMemcpyAsync(qseq.p, q.seq.data(), q.seq.size(), hipMemcpyHostToDevice, stream));
    if (nq) {
      HIPCHK(hipMemcpyAsync(qoff.p, q.off.data(), nq * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
      HIPCHK(hipMemcpyAsync(qlen.p, q.len.data(), nq * sizeof(int32_t), hipMemcpyHostToDevice, stream));
      if (!skip_codan && pw_stop_table_build(qseq.p, qoff.p, qlen.p, nq, next_stop.p, stream) != PW_OK) {
        fprintf(stderr, "pafreport: stop table launch failed\n");
        return false;
      }
    }
    HIPCHK(hipStreamSynchronize(stream));
    return true;
  }
  // run the batch; fills text/results on the host
  bool run(const Batch& b, bool skip_codan, std::vector<uint8_t>& text_h, std::vector<pw_aln_result>& res_h,
           std::vector<pw_page>& pages_h) {
    const size_t na = b.desc.size();
    res_h.resize(na);
    const uint64_t np = pw_report_page_count(b.n_events_max);
    const uint64_t tcap = pw_report_text_bytes(b.n_events_max, b.text_total);
    pages_h.resize(np);
    if (na == 0) return true;
    if (!desc.ensure(na) || !ops.ensure(b.ops.size() + 1) || !lits.ensure(b.lits.size() + kDevPad) ||
        !text.ensure(tcap + 1) || !res.ensure(na) || !pages.ensure(np + 1) ||
        !work.ensure(pw_report_workspace_bytes(b.n_events_max, na))) {
      fprintf(stderr, "pafreport: device allocation failed\n");
      return false;
    }
    HIPCHK(hipMemcpyAsync(desc.p, b.desc.data(), na * sizeof(pw_aln_desc), hipMemcpyHostToDevice, stream));
    if (!b.ops.empty())
      HIPCHK(hipMemcpyAsync(ops.p, b.ops.data(), b.ops.size() * 4, hipMemcpyHostToDevice, stream));
    if (!b.lits.empty())
      HIPCHK(hipMemcpyAsync(lits.p, b.lits.data(), b.lits.size(), hipMemcpyHostToDevice, stream));
    pw_report_args a;
    a.desc = desc.p;
    a.ops = ops.p;
    a.lits = lits.p;
    a.qseq = qseq.p;
    a.qoff = qoff.p;
    a.qlen = qlen.p;
    a.next_stop = skip_codan ? nullptr : next_stop.p;
    a.text = text.p;
    a.results = res.p;
    a.text_total = tcap;
    a.n_alns = (uint32_t)na;
    a.skip_codan = skip_codan ? 1u : 0u;
    a.workspace = work.p;
    a.workspace_bytes = pw_report_workspace_bytes(b.n_events_max, na);
    a.n_ev_slots = b.n_events_max;
    a.pages = pages.p;
    if (pw_report_events(&a, stream) != PW_OK) {
      fprintf(stderr, "pafreport: kernel launch failed\n");
      return false;
    }
    HIPCHK(hipMemcpyAsync(res_h.data(), res.p, na * sizeof(pw_aln_result), hipMemcpyDeviceToHost, stream));
    if (np) HIPCHK(hipMemcpyAsync(pages_h.data(), pages.p, np * sizeof(pw_page), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    // copy back the used part of the text (pages + arena)
    uint64_t used = 0;
    for (const pw_page& pg : pages_h)
      if (pg.len && pg.off + pg.len > used) used = pg.off + pg.len;
    if (used > tcap) used = tcap;
    text_h.resize(used);
    if (used) HIPCHK(hipMemcpy(text_h.data(), text.p, used, hipMemcpyDeviceToHost));
    return true;
  }
  ~Device() {
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// Print what the reference prints for one log item; returns -1 to continue, else the exit code
// the reference ends with at this item.
// Write the first `nlines` event lines of a record (all of them when nlines == n_events): the
// bytes from text_off to text_end, crossing pages in chunk order (pwasm_amd.h, text pages).
void write_lines(const uint8_t* text, const pw_page* pages, const pw_aln_result& r, uint32_t nlines, FILE* out) {
  if (r.n_events == 0 || nlines == 0) return;
  uint32_t seen = 0;
  for (uint32_t c = r.page_first;; c++) {
    const uint64_t lo = c == r.page_first ? r.text_off : pages[c].off;
    const uint64_t hi = c == r.page_last ? r.text_end : pages[c].off + pages[c].len;
    const uint8_t* p = text + lo;
    size_t n = (size_t)(hi - lo);
    if (nlines != r.n_events) {  // stop after the nlines-th newline
      size_t k = 0;
      while (k < n && seen < nlines) {
        if (p[k] == '\n') seen++;
        k++;
      }
      n = k;
    }
    fwrite(p, 1, n, out);
    if (c == r.page_last || (nlines != r.n_events && seen >= nlines)) break;
  }
}

int emit_item(const Batch& b, const LogItem& it, const uint8_t* text, const pw_aln_result* res, const pw_page* pages,
              FILE* out, FILE* err) {
  if (it.kind == 0) {
    fputs(b.msgs[it.idx].c_str(), err);
    return -1;
  }
  if (it.kind == 2) {
    fflush(out);
    fputs(b.msgs[it.idx].c_str(), err);
    return 1;
  }
  const RecHost& rh = b.recs[it.idx];
  const pw_aln_result& r = res[it.idx];
  const char* lstr = b.text.data() + rh.line_off;
  if (rh.pre_msg >= 0) {
    fputs(b.msgs[rh.pre_msg].c_str(), err);
    return 1;
  }
  if (r.err == PW_REC_MISMATCH) {
    fprintf(err, "Error: base mismatch %c != qstr[%d] (%c) at line\n%s\n", (char)r.err_b, r.err_a, (char)r.err_c,
            lstr);
    return 1;
  }
  if (rh.cs_msg >= 0) {
    fputs(b.msgs[rh.cs_msg].c_str(), err);
    return 1;
  }
  for (int k = 0; k < rh.n_softclip; k++)
    fprintf(err, "Warning: soft clipping shouldn't be found in this application!\n%s\n", lstr);
  if (rh.post_msg >= 0) {
    fputs(b.msgs[rh.post_msg].c_str(), err);
    return 1;
  }
  if (r.err == PW_REC_OVERFLOW || r.err == PW_REC_LAYOUT) {
    fprintf(err, "pafreport: internal error: %s\n",
            r.err == PW_REC_OVERFLOW ? "report slot overflow" : "batch layout rejected by the device");
    return 2;
  }
  fwrite(b.hdr.data() + rh.hdr_off, 1, rh.hdr_len, out);
  uint32_t nlines = r.n_events;
  std::string post;
  if (rh.qlen < 9 && r.n_events > 0) {
    nlines = 0;
    post = "Error: query sequence too short for a 9-nt context\n";
  } else if (r.err == PW_REC_MODSEQ) {
    nlines = (uint32_t)r.err_c;
    post = strf("Error: modseq[%d] not matching di.evtsub[%d] !\n", r.err_a, r.err_b);
  }
  write_lines(text, pages, r, nlines, out);
  if (nlines == r.n_events) return -1;
  fflush(out);
  fputs(post.c_str(), err);
  return 1;
}

// Print what the reference prints for this batch; returns -1 to continue, else an exit code.
int emit(const Batch& b, const uint8_t* text, const pw_aln_result* res, const pw_page* pages, FILE* out) {
  for (const LogItem& it : b.log) {
    const int rc = emit_item(b, it, text, res, pages, out, stderr);
    if (rc >= 0) return rc;
  }
  return -1;
}

// ----------------------------------------------------------------- GLineReader
struct LineReader {
  FILE* f;
  std::vector<char> buf;
  size_t pos = 0, end = 0;
  bool eof = false;
  std::string line;
  explicit LineReader(FILE* ff) : f(ff), buf(1 << 22) {}
  int getc_() {
    if (pos == end) {
      if (eof) return EOF;
      end = fread(buf.data(), 1, buf.size(), f);
      pos = 0;
      if (end == 0) {
        eof = true;
        return EOF;
      }
    }
    return (unsigned char)buf[pos++];
  }
  // \n, \r or \r\n end a line (gclib GLineReader::getLine)
  bool next() {
    line.clear();
    int c;
    while ((c = getc_()) != EOF) {
      if (c == '\n') return true;
      if (c == '\r') {
        int d = getc_();
        if (d != '\n' && d != EOF) pos--;  // unget
        return true;
      }
      // fast path: copy a run of plain bytes
      line.push_back((char)c);
      while (pos < end) {
        char ch = buf[pos];
        if (ch == '\n' || ch == '\r') break;
        size_t e = pos;
        while (e < end && buf[e] != '\n' && buf[e] != '\r') e++;
        line.append(buf.data() + pos, e - pos);
        pos = e;
      }
    }
    return !line.empty();
  }
};

#define USAGE                                                             \
  "Usage:\n\
 pafreport <paf_with_cg_cs> -r <refseq.fa> [-s <summary.txt>]\n\
    [-o <diff_report.dfa>][-w <outfile.mfa>] [-G|-F|-C|-N]\n\
    \n\
   <paf_with_cg_cs> is the input PAF file with high quality query sequence(s)\n\
      aligned to many target sequences using minimap2 --cs\n\
   -r provide the fasta file with query sequence(s) (required)\n\
   -o write difference data for each alignment into <diff_report.dfa>\n\
   -s write event summary counts into <summary.txt>\n\
   -w write MSA as multifasta into <outfile.mfa>\n\
   -G gene CDS analysis mode (default for query<100K; assumes -C)\n\
   -F full genome alignment mode (default for query>100Kb; assumes -N)\n\
   -C perform codon impact analysis\n\
   -N skip codon impact analysis\n"

struct Args {
  const char* val[128] = {};
  bool set[128] = {};
  std::vector<const char*> nonopt;
  int err = 0;
  // GArgs(argc, argv, "DGFCNvd:p:r:o:m:w:c:s:")
  void parse(int argc, char** argv, const char* fmt) {
    for (int i = 1; i < argc; i++) {
      const char* p = argv[i];
      if (p[0] == '-' && p[1] != 0) {
        for (int k = 1; p[k]; k++) {
          unsigned char c = (unsigned char)p[k];
          const char* f = (c < 128 && c != ':') ? strchr(fmt, c) : nullptr;
          if (!f) {
            err = i;
            return;
          }
          if (f[1] == ':') {
            if (p[k + 1]) val[c] = p + k + 1;
            else if (i + 1 < argc) val[c] = argv[++i];
            else {
              err = i;
              return;
            }
            set[c] = true;
            break;
          }
          set[c] = true;
          val[c] = "";
        }
      } else {
        nonopt.push_back(p);
      }
    }
  }
};

struct FileCloser {
  FILE* f = nullptr;
  ~FileCloser() {
    if (f && f != stdout && f != stdin) fclose(f);
  }
};

uint64_t alg_bytes(const Batch& b, const QueryDb& q, bool skip_codan) {
  // descriptor + ops + literals + each distinct query once (+ its
  // next-stop table when the codon pass runs); output bytes are added from the results.
  uint64_t v = (uint64_t)b.desc.size() * (sizeof(pw_aln_desc) + sizeof(pw_aln_result)) + b.ops.size() * 4ull +
               b.lits.size();
  std::vector<char> seen(q.len.size(), 0);
  for (const auto& d : b.desc) {
    uint32_t qi = d.ref & PW_REF_QMASK;
    if (!seen[qi]) {
      seen[qi] = 1;
      v += (uint64_t)q.len[qi] * (skip_codan ? 1u : 5u);
    }
  }
  return v;
}

}  // namespace

// ================================================================= CLI
extern "C" int pw_pafreport_main(int argc, char** argv) {
  Args args;
  args.parse(argc, argv, "DGFCNvd:p:r:o:m:w:c:s:");
  if (args.err > 0) {
    fprintf(stderr, "%s\nInvalid argument: %s\n", USAGE, argv[args.err]);
    return 1;
  }
  const bool debug = args.set['D'];
  bool fullgenome = args.set['F'];
  const bool gene = args.set['G'];
  if (fullgenome && gene) {
    fprintf(stderr, "%s Error: cannot use both -G and -F!\n", USAGE);
    return 1;
  }
  const bool force_coding = args.set['C'], force_noncoding = args.set['N'];
  if (force_coding && force_noncoding) {
    fprintf(stderr, "%s Error: cannot use both -N and -C!\n", USAGE);
    return 1;
  }
  const bool verbose = args.set['v'] || debug;
  FileCloser in, out;
  in.f = stdin;
  if (!args.nonopt.empty() && args.nonopt[0][0]) {
    in.f = fopen(args.nonopt[0], "r");
    if (!in.f) {
      fprintf(stderr, "Cannot open input file %s!\n", args.nonopt[0]);
      return 1;
    }
  }
  if (args.set['c'] && args.val['c'][0]) {  // -c clipmax: parsed, never used (pafreport.cpp:217-240)
    std::string c(args.val['c']);
    const bool pct = !c.empty() && c.back() == '%';
    while (!c.empty() && c.back() == '%') c.pop_back();
    const int v = atoi(c.c_str());
    if (v <= 0) {
      fprintf(stderr, "Error: invalid -c <clipmax> (%d) option provided (must be a positive integer)!\n", v);
      return 1;
    }
    if (pct && v > 99) {
      fprintf(stderr, "Error: invalid percent value (%d) for -c option  (must be an integer between 1 and 99)!\n", v);
      return 1;
    }
    if (pct) {
      float clipmax = (float)v / 100;
      if (verbose) fprintf(stderr, "Percentual max clipping set to %d%%\n", (int)(100 * clipmax + 0.5f));
    } else if (verbose)
      fprintf(stderr, "Max clipping set to %d bases\n", v);
  }
  out.f = stdout;
  if (args.set['o'] && args.val['o'][0]) {
    out.f = fopen(args.val['o'], "w");
    if (!out.f) {
      fprintf(stderr, "Cannot open file %s for writing!\n", args.val['o']);
      return 1;
    }
  }
  const char* fa = args.set['r'] ? args.val['r'] : "";
  if (!fa[0]) {
    fprintf(stderr, "Error: query FASTA file (-r) is required!\n");
    return 1;
  }
  struct stat st;
  const long long fsize = (stat(fa, &st) == 0) ? (long long)st.st_size : -1;
  if (fsize <= 0) {
    fprintf(stderr, "Error: invalid FASTA file %s !\n", fa);
    return 1;
  }
  QueryDb qdb;
  std::string err;
  if (!qdb.load(fa, err)) {
    fputs(err.c_str(), stderr);
    return 1;
  }
  if (!fullgenome && !gene && fsize > 120000) fullgenome = true;
  bool skip_codan = fullgenome || force_noncoding;
  if (!skip_codan && !force_coding && fsize > 120000) skip_codan = true;
  if (args.set['w'] && args.val['w'][0]) {
    if (fullgenome) {
      fprintf(stderr, "%s Error: can only generate MSA for -G mode!\n", USAGE);
      return 1;
    }
    fprintf(stderr, "Error: -w (MSA output) is not supported by this build yet\n");
    return 1;
  }
  Device dev;
  if (!dev.init(qdb, skip_codan)) return 2;
  Packer pk;
  pk.qdb = &qdb;
  pk.opt.fullgenome = fullgenome;
  pk.opt.skip_codan = skip_codan;
  pk.opt.verbose = verbose;
  pk.opt.single_query_gene = (qdb.ids.size() == 1 && !fullgenome);
  LineReader lr(in.f);
  Batch b;
  std::vector<uint8_t> text_h;
  std::vector<pw_aln_result> res_h;
  std::vector<pw_page> pages_h;
  const size_t kBatchBytes = 256u << 20, kBatchRecs = 1u << 20;
  bool more = true;
  while (more) {
    b.clear();
    while (b.text.size() < kBatchBytes && b.desc.size() < kBatchRecs) {
      if (!lr.next()) {
        more = false;
        break;
      }
      if (!pk.add_line(b, lr.line.data(), lr.line.size())) {
        more = false;
        break;
      }
    }
    if (!dev.run(b, skip_codan, text_h, res_h, pages_h)) return 2;
    const int rc = emit(b, text_h.data(), res_h.data(), pages_h.data(), out.f);
    if (rc >= 0) {
      fflush(out.f);
      return rc;
    }
  }
  fflush(out.f);
  return 0;
}

// ================================================================= batch API (bench / tests)
struct pw_batch {
  QueryDb q;
  Batch b;
  Packer pk;
  bool skip_codan = false;
  uint64_t alg_in = 0;
};

extern "C" pw_batch* pw_batch_from_files(const char* fasta, const char* paf, uint32_t flags, char* errbuf,
                                         size_t errlen) {
  auto fail = [&](const std::string& m) -> pw_batch* {
    if (errbuf && errlen) snprintf(errbuf, errlen, "%s", m.c_str());
    return nullptr;
  };
  pw_batch* bt = new pw_batch();
  std::string err;
  if (!bt->q.load(fasta, err)) {
    delete bt;
    return fail(err);
  }
  struct stat st;
  const long long fsize = (stat(fasta, &st) == 0) ? (long long)st.st_size : -1;
  bool gene = flags & 1u, full = flags & 2u, fc = flags & 4u, fn = flags & 8u;
  if (!full && !gene && fsize > 120000) full = true;
  bool skip = full || fn;
  if (!skip && !fc && fsize > 120000) skip = true;
  bt->skip_codan = skip;
  bt->pk.qdb = &bt->q;
  bt->pk.opt.fullgenome = full;
  bt->pk.opt.skip_codan = skip;
  bt->pk.opt.single_query_gene = (bt->q.ids.size() == 1 && !full);
  FILE* f = fopen(paf, "r");
  if (!f) {
    delete bt;
    return fail(strf("cannot open %s", paf));
  }
  LineReader lr(f);
  while (lr.next())
    if (!bt->pk.add_line(bt->b, lr.line.data(), lr.line.size())) break;
  fclose(f);
  bt->alg_in = alg_bytes(bt->b, bt->q, skip);
  return bt;
}

extern "C" int pw_batch_view_get(const pw_batch* bt, pw_batch_view* v) {
  if (!bt || !v) return PW_E_ARG;
  v->desc = bt->b.desc.data();
  v->ops = bt->b.ops.data();
  v->lits = bt->b.lits.data();
  v->qseq = bt->q.seq.data();
  v->qoff = bt->q.off.data();
  v->qlen = bt->q.len.data();
  v->n_alns = bt->b.desc.size();
  v->n_ops = bt->b.ops.size();
  v->n_lits = bt->b.lits.size();
  v->qseq_len = bt->q.seq.size();
  v->n_queries = bt->q.len.size();
  v->text_total = bt->b.text_total;
  v->n_events_max = bt->b.n_events_max;
  v->alg_bytes_in = bt->alg_in;
  v->skip_codan = bt->skip_codan ? 1u : 0u;
  return PW_OK;
}

extern "C" int pw_batch_write_report(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                                     const pw_page* pages_host, const char* path) {
  if (!bt || !path) return PW_E_ARG;
  FILE* f = fopen(path, "wb");
  if (!f) return PW_E_IO;
  int rc = emit(bt->b, text_host, res_host, pages_host, f);
  fclose(f);
  return rc < 0 ? 0 : rc;
}

// Item stream of a shard (PWI1): per log item {u64 line, i32 status, u32 n_out,
// u32 n_err, stdout bytes, stderr bytes}; ends after the first item with status >= 0.
extern "C" int pw_batch_write_items(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                                    const pw_page* pages_host, const char* path) {
  if (!bt || !path) return PW_E_ARG;
  FILE* f = fopen(path, "wb");
  if (!f) return PW_E_IO;
  fwrite("PWI1", 1, 4, f);
  char *ob = nullptr, *eb = nullptr;
  size_t on = 0, en = 0;
  int ret = PW_OK;
  for (const LogItem& it : bt->b.log) {
    FILE* o = open_memstream(&ob, &on);
    FILE* e = open_memstream(&eb, &en);
    if (!o || !e) {
      ret = PW_E_NOMEM;
      if (o) fclose(o);
      if (e) fclose(e);
      break;
    }
    const int32_t st = emit_item(bt->b, it, text_host, res_host, pages_host, o, e);
    fclose(o);
    fclose(e);
    const uint32_t no = (uint32_t)on, ne = (uint32_t)en;
    fwrite(&it.line, 8, 1, f);
    fwrite(&st, 4, 1, f);
    fwrite(&no, 4, 1, f);
    fwrite(&ne, 4, 1, f);
    fwrite(ob, 1, on, f);
    fwrite(eb, 1, en, f);
    free(ob);
    free(eb);
    ob = eb = nullptr;
    if (st >= 0) break;
  }
  if (fclose(f) != 0 && ret == PW_OK) ret = PW_E_IO;
  return ret;
}

extern "C" void pw_batch_free(pw_batch* bt) { delete bt; }

extern "C" const char* pw_version(void) { return "pwasm_amd 0.1 (gfx950)"; }
