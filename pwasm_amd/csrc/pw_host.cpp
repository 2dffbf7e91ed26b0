// pw_host.cpp — host side of libpwasm_amd.so: the CPU pre-pass (PAF record -> packed cs op
// stream), batch staging on the GPU, and the `pafreport` CLI (pafreport.cpp:175-460) driving
// the HIP kernels of pw_report.hip.  Everything the reference prints is printed here, in the
// reference's order, from the per-record results the GPU returns; there is no CPU fallback:
// without a usable gfx950 device the CLI stops with an error.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <sched.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <future>
#include <memory>
#include <new>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "pw_msa_layout.h"
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

// gclib parseInt on the string [p, end): skip blanks, optional sign, digits; false (p
// unchanged) if no digit.
bool parse_int(const char*& p, const char* end, int& out) {
  const char* q = p;
  while (q < end && (*q == ' ' || *q == '\t')) q++;
  const char* start = q;
  if (q < end && (*q == '-' || *q == '+')) q++;
  const char* dig = q;
  while (q < end && *q >= '0' && *q <= '9') q++;
  if (q == dig) return false;
  if (q - dig <= 9) {  // cannot overflow: the value directly
    int v = 0;
    for (const char* d = dig; d < q; d++) v = v * 10 + (*d - '0');
    out = *start == '-' ? -v : v;
    p = q;
    return true;
  }
  char tmp[48];  // strtol on a bounded copy (same overflow behaviour as the reference's strtol)
  const size_t n = (size_t)(q - start);
  if (n < sizeof tmp) {
    memcpy(tmp, start, n);
    tmp[n] = 0;
    out = (int)strtol(tmp, nullptr, 10);
  } else {
    out = (int)(*start == '-' ? LONG_MIN : LONG_MAX);
  }
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
// cs = [cs, cs_end): the tag's field (the reference strdup's it out of the split line).
static int pack_cs_n(const char* cs, const char* cs_end, int32_t offset, int32_t qlen, uint32_t* ops, size_t ops_cap,
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
  while (p < cs_end && rc == PW_CS_OK) {
    const char op = *p;
    p++;
    switch (op) {
      case ':': {
        int cl = 0;
        if (!parse_int(p, cs_end, cl)) {
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
        if (p + 2 > cs_end || p[0] == 0 || p[1] == 0) {
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
        while (p < cs_end && is_alpha((unsigned char)*p)) p++;
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
        while (p < cs_end && is_alpha((unsigned char)*p)) p++;
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

extern "C" int pw_pack_cs(const char* cs, int32_t offset, int32_t qlen, uint32_t* ops, size_t ops_cap,
                          uint8_t* lits, size_t lits_cap, pw_cs_totals* tot, int32_t* err_pos) {
  return pack_cs_n(cs, cs ? cs + strlen(cs) : nullptr, offset, qlen, ops, ops_cap, lits, lits_cap, tot, err_pos);
}

// ================================================================= batch structures
namespace {

// Growable array of trivially copyable T without value-initialisation (the batch arrays are
// written once, in parallel, after being sized).
template <class T>
struct PodVec {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  PodVec() = default;
  PodVec(PodVec&& o) noexcept { swap(o); }
  PodVec(const PodVec&) = delete;
  PodVec& operator=(const PodVec&) = delete;
  ~PodVec() { free(p); }
  void reserve(size_t c) {
    if (c <= cap) return;
    size_t nc = std::max(c, cap + cap / 2 + 16);
    T* q = (T*)realloc(p, nc * sizeof(T));
    if (!q) {
      fprintf(stderr, "pafreport: host allocation failed\n");
      abort();
    }
    p = q;
    cap = nc;
  }
  void resize(size_t m) {
    reserve(m);
    n = m;
  }
  void clear() { n = 0; }
  void push_back(const T& v) {
    if (n == cap) reserve(n + 1);
    p[n++] = v;
  }
  void append(const T* v, size_t k) {
    reserve(n + k);
    if (k) memcpy(p + n, v, k * sizeof(T));
    n += k;
  }
  void swap(PodVec& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
  }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T* data() { return p; }
  const T* data() const { return p; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T& back() { return p[n - 1]; }
  T* begin() { return p; }
  T* end() { return p + n; }
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
};

struct QueryDb {
  std::vector<std::string> ids;
  std::vector<uint64_t> off;
  std::vector<int32_t> len;
  std::vector<uint8_t> seq;  // upper case (GASeq::allupper, pafreport.cpp:350)
  std::unordered_map<std::string_view, int> index;  // first record of each id (built after load)
  std::vector<uint8_t> acgt;  // per query: all bases in {A,C,G,T}
  bool all_acgt(int qi) const { return acgt[qi] != 0; }
  uint64_t max_len() const {
    int32_t m = 0;
    for (int32_t l : len) m = l > m ? l : m;
    return (uint64_t)m;
  }
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
        if (have) close_record();
        ids.push_back(l.substr(1, e - 1));
        off.push_back(seq.size());
        len.push_back(0);
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
    index.reserve(ids.size() * 2);
    for (size_t i = 0; i < ids.size(); i++) index.emplace(std::string_view(ids[i]), (int)i);
    return true;
  }
};

// Worker threads of the host pre-pass: PW_THREADS, else OMP_NUM_THREADS, else the CPUs this
// process may run on (at most 16: a GPU box gives each GPU a 16-CPU share).
int host_threads() {
  for (const char* v : {"PW_THREADS", "OMP_NUM_THREADS"}) {
    const char* e = getenv(v);
    if (e && atoi(e) > 0) return std::min(atoi(e), 256);
  }
  cpu_set_t cs;
  int n = 0;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 16));
}
// wall clock for the PW_PROFILE_HOST lines
static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static bool host_prof() {
  static const bool on = getenv("PW_PROFILE_HOST") && *getenv("PW_PROFILE_HOST") && strcmp(getenv("PW_PROFILE_HOST"), "0");
  return on;
}

template <class F>
void parallel_for(int nt, F&& f) {
  if (nt <= 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)nt - 1);
  for (int t = 1; t < nt; t++) th.emplace_back([&f, t] { f(t); });
  f(0);
  for (auto& x : th) x.join();
}

// CRC-32 (IEEE, as zlib.crc32): the shard of a PAF line is crc32(target name) % world
// (pwasm_amd/shard.py:shard_of).
uint32_t crc32_ieee(const char* p, size_t n) {
  static uint32_t tab[256];
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
  });
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = tab[(c ^ (uint8_t)p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

uint64_t fnv1a(const char* p, size_t n, uint64_t h = 1469598103934665603ull) {
  for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 1099511628211ull;
  return h;
}

struct Options {
  bool fullgenome = false, skip_codan = false, verbose = false;
  bool single_query_gene = false;  // rlabel "" (pafreport.cpp:378-379)
  uint32_t shard = 0, nshards = 1;  // multi-GPU: only lines whose target hashes to `shard`
  bool msa = false;                 // -w: gap lists, setGap checks and the query run are kept
  bool gpu_pack = false;            // cs strings packed on the GPU (pw_pack_cs_batch; the CLI)
};

struct RecHost {                // (trivial: lives in PodVec; pack_line sets every field)
  uint64_t line_off;            // original line in the batch buffer (NUL-terminated; messages)
  uint64_t hdr_off;             // header line in the header pool
  uint32_t hdr_len;
  int32_t pre_msg;              // message index: fatal before the cs loop (-1: none)
  int32_t cs_msg;               // fatal from the host cs parse (after GPU mismatch)
  int32_t post_msg;             // fatal from the CIGAR loop / length checks
  uint16_t n_softclip;
  int32_t qlen;
  uint32_t tname_off, tname_len;  // target name (per-genome tables of the multi-GPU driver)
  int32_t t_aln;                // aligned target bases (t_alnend - t_alnstart)
  // -w (Options::msa): the alignment's gap lists in Batch::gaps (rgaps then tgaps), its tlabel
  // in the header pool after the header, and the setGap error it ends with
  int32_t w_msg;
  int32_t r_alnstart, t_len;
  uint32_t gap_off, n_rg, n_tg, lab_len;
  // GPU packing (Options::gpu_pack): the cs field in Batch::cstext, and the CIGAR loop's outcome,
  // judged once the cs totals are back (finish_gpu_pack)
  uint64_t cs_off;
  uint32_t cs_len;
  int32_t cig_msg;              // CIGAR parse / op error (message index) or -1
  int32_t cig_tpos, cig_qpos;
  int32_t r_alnend, t_alnstart, t_alnend;
};

// Ordered log of what a batch prints: messages, records, a terminating fatal.
struct LogItem {
  uint8_t kind;  // 0 message, 1 record, 2 fatal
  uint32_t idx;
  uint64_t line;  // 0-based input line it came from (shard merge order)
};

struct LineRef {
  uint64_t off;  // into Batch::buf
  uint32_t len;
};

// One batch: its input lines (the buffer keeps them, NUL-terminated, for messages) and the
// packed device arrays.  A thread's share of a batch is packed into a Batch of its own
// (without buf) and then appended here (Batch::append).
struct Batch {
  PodVec<char> buf;
  PodVec<LineRef> lines;
  uint64_t line0 = 0;   // global input line of lines[0]
  PodVec<uint64_t> line_no;  // (multi-GPU exchange) the global input line of each line, when set
  PodVec<char> hdr;     // report headers
  std::vector<std::string> msgs;
  PodVec<LogItem> log;
  PodVec<RecHost> recs;
  PodVec<pw_aln_desc> desc;
  PodVec<uint32_t> ops;
  PodVec<uint8_t> lits;
  PodVec<int32_t> gaps;  // -w: (pos, len) pairs
  PodVec<char> cstext;   // GPU packing: the records' cs fields back to back
  bool gpu_packed = false;
  uint64_t text_total = 0, n_events_max = 0;
  bool fatal = false;
  void clear_out() {
    gaps.clear();
    cstext.clear();
    gpu_packed = false;
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
  void clear() {
    buf.clear();
    lines.clear();
    clear_out();
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

// Append parts (packed by threads over consecutive line ranges) to `b`, in order, up to and
// including the first part that ended in a fatal error; the offsets each part holds into its
// own arrays are rebased in parallel.
void append_parts(Batch& b, std::vector<Batch>& parts, int nt) {
  size_t np = parts.size();
  for (size_t i = 0; i < parts.size(); i++)
    if (parts[i].fatal) {
      np = i + 1;
      break;
    }
  std::vector<uint64_t> o_desc(np + 1), o_ops(np + 1), o_lits(np + 1), o_hdr(np + 1), o_msg(np + 1), o_log(np + 1),
      o_ev(np + 1), o_txt(np + 1), o_gap(np + 1), o_cs(np + 1);
  for (size_t i = 0; i < np; i++) {
    const Batch& p = parts[i];
    o_desc[i + 1] = o_desc[i] + p.desc.size();
    o_ops[i + 1] = o_ops[i] + p.ops.size();
    o_lits[i + 1] = o_lits[i] + p.lits.size();
    o_hdr[i + 1] = o_hdr[i] + p.hdr.size();
    o_msg[i + 1] = o_msg[i] + p.msgs.size();
    o_log[i + 1] = o_log[i] + p.log.size();
    o_ev[i + 1] = o_ev[i] + p.n_events_max;
    o_txt[i + 1] = o_txt[i] + p.text_total;
    o_gap[i + 1] = o_gap[i] + p.gaps.size();
    o_cs[i + 1] = o_cs[i] + p.cstext.size();
  }
  const size_t d0 = b.desc.size(), op0 = b.ops.size(), l0 = b.lits.size(), h0 = b.hdr.size(), m0 = b.msgs.size(),
               g0 = b.log.size();
  const uint64_t e0 = b.n_events_max;
  const size_t gp0 = b.gaps.size(), cs0 = b.cstext.size();
  b.gaps.resize(gp0 + o_gap[np]);
  b.cstext.resize(cs0 + o_cs[np]);
  b.desc.resize(d0 + o_desc[np]);
  b.recs.resize(d0 + o_desc[np]);
  b.ops.resize(op0 + o_ops[np]);
  b.lits.resize(l0 + o_lits[np]);
  b.hdr.resize(h0 + o_hdr[np]);
  b.msgs.resize(m0 + o_msg[np]);
  b.log.resize(g0 + o_log[np]);
  b.n_events_max += o_ev[np];
  b.text_total += o_txt[np];
  std::atomic<size_t> next{0};
  parallel_for(std::min<int>(nt, (int)np), [&](int) {
    for (size_t i; (i = next.fetch_add(1)) < np;) {
      Batch& p = parts[i];
      const uint32_t dop = (uint32_t)(op0 + o_ops[i]), dlit = (uint32_t)(l0 + o_lits[i]);
      const uint64_t dev = e0 + o_ev[i];
      for (size_t k = 0; k < p.desc.size(); k++) {
        pw_aln_desc d = p.desc[k];
        d.op_begin += dop;
        d.lit_begin += dlit;
        d.ev_begin += dev;
        b.desc[d0 + o_desc[i] + k] = d;
        RecHost r = p.recs[k];
        r.hdr_off += h0 + o_hdr[i];
        const int32_t dm = (int32_t)(m0 + o_msg[i]);
        if (r.pre_msg >= 0) r.pre_msg += dm;
        if (r.cs_msg >= 0) r.cs_msg += dm;
        if (r.post_msg >= 0) r.post_msg += dm;
        if (r.w_msg >= 0) r.w_msg += dm;
        r.gap_off += (uint32_t)(gp0 + o_gap[i]);
        r.cs_off += cs0 + o_cs[i];
        b.recs[d0 + o_desc[i] + k] = r;
      }
      if (!p.ops.empty()) memcpy(&b.ops[op0 + o_ops[i]], p.ops.data(), p.ops.size() * 4);
      if (!p.lits.empty()) memcpy(&b.lits[l0 + o_lits[i]], p.lits.data(), p.lits.size());
      if (!p.gaps.empty()) memcpy(&b.gaps[gp0 + o_gap[i]], p.gaps.data(), p.gaps.size() * 4);
      if (!p.cstext.empty()) memcpy(&b.cstext[cs0 + o_cs[i]], p.cstext.data(), p.cstext.size());
      if (!p.hdr.empty()) memcpy(&b.hdr[h0 + o_hdr[i]], p.hdr.data(), p.hdr.size());
      for (size_t k = 0; k < p.msgs.size(); k++) b.msgs[m0 + o_msg[i] + k] = std::move(p.msgs[k]);
      for (size_t k = 0; k < p.log.size(); k++) {
        LogItem it = p.log[k];
        it.idx += (uint32_t)(it.kind == 1 ? d0 + o_desc[i] : m0 + o_msg[i]);
        b.log[g0 + o_log[i] + k] = it;
      }
    }
  });
  b.fatal = b.fatal || parts[np - 1].fatal;
}

// The reference's message for a cs string that stops the record (pafreport.cpp:542, 620-624; D1,
// D2): rc from pw_pack_cs, `at` = the rest of the cs string from where it stopped.
std::string cs_error_msg(int rc, const char* s, const std::string& at) {
  switch (rc) {
    case PW_CS_PARSE: return strf("Error parsing cs string from line: %s (cs position: %s)\n", s, at.c_str());
    case PW_CS_SPLICED: return strf("Error: spliced alignments not supported! at line:\n%s\n", s);
    case PW_CS_UNHANDLED: return strf("Error: unhandled event at %s in cs, line:\n%s\n", at.c_str(), s);
    case PW_CS_EMPTY: return strf("Error: empty indel in cs string at line:\n%s\n", s);
    case PW_CS_BOUNDS: return strf("Error: cs string extends beyond query sequence at line:\n%s\n", s);
    default: return strf("Error: cs string too long at line:\n%s\n", s);
  }
}

const char* CIGAR_ERROR = "Error parsing cigar string from line: %s (cigar position: %s)\n";

// Line classes of the pre-scan (kind) and the gene-mode dedupe verdict (dup).
enum : uint8_t { kLineSkip = 0, kLineShort = 1, kLineSelf = 2, kLineRec = 3 };
enum : uint8_t { kDupNo = 0, kDupSilent = 1, kDupWarn = 2 };
struct LineInfo {
  uint8_t kind, dup;
  uint64_t khash;  // hash of "q~t" (gene mode)
};

// Pre-scan of one line: enough fields to classify it (pafreport.cpp:304-317); the shard filter.
// Field starts follow strsplit (a field starts after every tab that is not the last byte).
LineInfo classify(const char* s, uint32_t n, const Options& opt) {
  LineInfo li{kLineSkip, kDupNo, 0};
  if (n > 0 && s[0] == '#') return li;
  uint32_t fs[16];
  int nf = 0;
  bool after = true;
  for (uint32_t i = 0; i < n && nf < 16; i++) {
    if (after) fs[nf++] = i;
    after = s[i] == '\t';
  }
  if (opt.nshards > 1) {  // shard.py:shard_of — column 6 of a Python split on tabs, else rank 0
    const char* t5 = nullptr;
    size_t t5n = 0;
    int tabs = 0;
    for (uint32_t i = 0; i < n; i++)
      if (s[i] == '\t') {
        tabs++;
        if (tabs == 5) t5 = s + i + 1;
        if (tabs == 6) {
          t5n = (size_t)(s + i - t5);
          break;
        }
      }
    const uint32_t sh = tabs >= 6 ? crc32_ieee(t5, t5n) % opt.nshards : 0u;
    if (sh != opt.shard) return li;
  }
  if (nf < 15) {
    li.kind = kLineShort;
    return li;
  }
  auto fend = [&](int k) -> uint32_t {
    const char* e = (const char*)memchr(s + fs[k], '\t', n - fs[k]);
    return e ? (uint32_t)(e - s) : n;
  };
  const uint32_t q0 = fs[0], q1 = fend(0), t0 = fs[5], t1 = fend(5);
  if (q1 - q0 == t1 - t0 && memcmp(s + q0, s + t0, q1 - q0) == 0) {
    li.kind = kLineSelf;
    return li;
  }
  li.kind = kLineRec;
  if (!opt.fullgenome) li.khash = fnv1a(s + t0, t1 - t0, fnv1a("~", 1, fnv1a(s + q0, q1 - q0)));
  return li;
}

struct Packer {
  const QueryDb* qdb;
  Options opt;
  int nt = 1;
  // q~t pairs seen (gene mode), persisting across batches; partitioned by key hash so that the
  // threads dedupe in parallel while each partition still sees its keys in input order
  struct PairSet {
    std::unordered_map<uint64_t, uint32_t> by_hash;  // key hash -> first key with that hash
    PodVec<char> keys;                               // key bytes, back to back
    PodVec<uint64_t> koff;                           // [k, k+1): key k
    PodVec<int> count;                               // times seen after the first
    std::unordered_map<std::string, int> spill;      // keys whose hash another key owns
    // times `key` was seen before (0 = first occurrence, now recorded)
    int seen(const char* key, size_t n, uint64_t h) {
      auto it = by_hash.find(h);
      if (it == by_hash.end()) {
        by_hash.emplace(h, (uint32_t)count.size());
        if (koff.empty()) koff.push_back(0);
        keys.append(key, n);
        koff.push_back(keys.size());
        count.push_back(0);
        return 0;
      }
      const uint32_t k = it->second;
      if (koff[k + 1] - koff[k] == n && memcmp(keys.data() + koff[k], key, n) == 0) return ++count[k];
      auto jt = spill.find(std::string(key, n));
      if (jt == spill.end()) {
        spill.emplace(std::string(key, n), 0);
        return 0;
      }
      return ++jt->second;
    }
  };
  std::vector<PairSet> alnpairs;
  uint64_t n_lines = 0;  // input lines seen (across batches)

  // Pack the lines of b (b.lines, b.line0) into b's arrays (pafreport.cpp:304-382 per line).
  void pack(Batch& b) {
    static const bool prof = getenv("PW_PROFILE_HOST") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_0 = prof ? now() : 0;
    const size_t nl = b.lines.size();
    b.line0 = n_lines;
    n_lines += nl;
    if (nl == 0) return;
    if ((int)alnpairs.size() != nt) alnpairs.resize((size_t)nt);
    std::vector<LineInfo> info(nl);
    // ---- phase 0: classify (parallel)
    parallel_for(nt, [&](int t) {
      for (size_t i = nl * (size_t)t / (size_t)nt; i < nl * (size_t)(t + 1) / (size_t)nt; i++)
        info[i] = classify(b.buf.data() + b.lines[i].off, b.lines[i].len, opt);
    });
    const double t_1 = prof ? now() : 0;
    // ---- phase 1: gene-mode q~t dedupe, first occurrence in input order (pafreport.cpp:319-334)
    size_t stop = nl;  // lines after the first short line are never reached
    for (size_t i = 0; i < nl; i++)
      if (info[i].kind == kLineShort) {
        stop = i + 1;
        break;
      }
    if (!opt.fullgenome) {
      parallel_for(nt, [&](int t) {
        auto& m = alnpairs[(size_t)t];
        std::string key;
        for (size_t i = 0; i < stop; i++) {
          LineInfo& li = info[i];
          if (li.kind != kLineRec || li.khash % (uint64_t)nt != (uint64_t)t) continue;
          const char* s = b.buf.data() + b.lines[i].off;
          const char* q1 = strchr(s, '\t');
          const char* t0 = q1;  // field 5 starts after the 5th tab
          for (int k = 0; k < 4; k++) t0 = strchr(t0 + 1, '\t');
          t0++;
          const char* t1 = strchr(t0, '\t');
          key.assign(s, (size_t)(q1 - s));
          key.push_back('~');
          key.append(t0, (size_t)(t1 - t0));
          const int c = m.seen(key.data(), key.size(), li.khash);
          if (c > 0) li.dup = c == 1 ? kDupWarn : kDupSilent;
        }
      });
    }
    const double t_2 = prof ? now() : 0;
    // ---- phase 2: pack consecutive line ranges (balanced by bytes) in parallel
    const int np = (int)std::min<size_t>((size_t)nt * 4, std::max<size_t>(stop / 64, 1));
    std::vector<size_t> cut((size_t)np + 1, stop);
    cut[0] = 0;
    {
      const uint64_t tot = b.lines[stop - 1].off + b.lines[stop - 1].len - b.lines[0].off;
      size_t i = 0;
      for (int k = 1; k < np; k++) {
        const uint64_t target = b.lines[0].off + tot * (uint64_t)k / (uint64_t)np;
        while (i < stop && b.lines[i].off < target) i++;
        cut[(size_t)k] = std::max(i, cut[(size_t)k - 1]);
      }
    }
    std::vector<Batch> parts((size_t)np);
    std::atomic<int> next{0};
    parallel_for(std::min(nt, np), [&](int) {
      std::vector<uint32_t> fs;
      for (int k; (k = next.fetch_add(1)) < np;) {
        Batch& p = parts[(size_t)k];
        for (size_t i = cut[(size_t)k]; i < cut[(size_t)k + 1] && !p.fatal; i++) {
          p.cur_line = b.line_no.empty() ? b.line0 + i : b.line_no[i];
          pack_line(p, b.buf.data(), b.lines[i], info[i], fs);
        }
      }
    });
    const double t_3 = prof ? now() : 0;
    append_parts(b, parts, nt);
    b.gpu_packed = opt.gpu_pack;
    if (opt.msa) track_run(b);
    if (prof)
      fprintf(stderr, "[pack] %zu lines, %d threads: classify %.3f dedupe %.3f pack %.3f append %.3f s\n", nl, nt,
              t_1 - t_0, t_2 - t_1, t_3 - t_2, now() - t_3);
  }

  // -w: the alignments of the current query run, in input order (a record of another query
  // starts a new run: pafreport fetches a fresh refseq GASeq at every query switch, :338-351)
  pw::MsaRun run;
  void track_run(const Batch& b) {
    for (size_t k = 0; k < b.recs.size(); k++) {
      const RecHost& rh = b.recs[k];
      const pw_aln_desc& d = b.desc[k];
      if (rh.pre_msg >= 0 || rh.cs_msg >= 0 || rh.post_msg >= 0 || rh.w_msg >= 0) return;  // the run stops here
      const int qi = (int)(d.ref & PW_REF_QMASK);
      if (run.qi != qi) {
        run.clear();
        run.qi = qi;
      }
      pw::MsaRec m;
      m.offset = d.offset;
      m.r_alnstart = rh.r_alnstart;
      m.t_len = rh.t_len;
      m.reverse = (d.ref & PW_REF_REVERSE) ? 1 : 0;
      m.op_begin = (uint32_t)run.ops.size();
      m.n_ops = d.n_ops;
      uint32_t nl = 0;
      for (uint32_t j = 0; j < d.n_ops; j++) {
        const uint32_t w = b.ops[d.op_begin + j];
        run.ops.push_back(w);
        nl += (w >> 30) == PW_OP_SUB ? 2u : ((w >> 30) == PW_OP_INS ? (w & 0x3FFFFFFFu) : 0u);
      }
      m.lit_begin = (uint32_t)run.lits.size();
      m.n_lits = nl;
      run.lits.insert(run.lits.end(), b.lits.data() + d.lit_begin, b.lits.data() + d.lit_begin + nl);
      m.gap_off = (uint32_t)run.gaps.size();
      m.n_rg = rh.n_rg;
      m.n_tg = rh.n_tg;
      run.gaps.insert(run.gaps.end(), b.gaps.data() + rh.gap_off, b.gaps.data() + rh.gap_off + 2 * (rh.n_rg + rh.n_tg));
      m.lab_off = (uint32_t)run.labels.size();
      m.lab_len = rh.lab_len;
      run.labels.append(b.hdr.data() + rh.hdr_off + rh.hdr_len, rh.lab_len);
      run.recs.push_back(m);
    }
  }

  // One input line (pafreport.cpp:304-382).
  void pack_line(Batch& b, const char* base, const LineRef& lr, const LineInfo& li, std::vector<uint32_t>& fs) {
    thread_local std::vector<std::pair<int, int>> rgl, tgl;  // -w gap lists of this record
    const char* s = base + lr.off;  // the untouched, NUL-terminated line (lstr)
    const uint32_t n = lr.len;
    if (li.kind == kLineSkip) return;
    fs.clear();
    bool after = true;
    for (uint32_t i = 0; i < n; i++) {  // strsplit(line, t, '\t')
      if (after) fs.push_back(i);
      after = s[i] == '\t';
    }
    const int numt = (int)fs.size();
    if (li.kind == kLineShort) {
      b.log_fatal(strf("Error: invalid PAF fline (num. fields=%d):\n%s\n", numt, s));
      return;
    }
    if (li.kind == kLineSelf) {
      if (opt.verbose) b.log_msg("Skipping alignment of qry seq to itself.\n");
      return;
    }
    // field k = [fld(k), fend(k)) (strsplit turns the tab after it, or a trailing tab, into NUL)
    auto fend = [&](int k) -> const char* {
      return k + 1 < numt ? s + fs[(size_t)k + 1] - 1 : (n > 0 && s[n - 1] == '\t' ? s + n - 1 : s + n);
    };
    auto fld = [&](int k) { return s + fs[(size_t)k]; };
    auto fint = [&](const char* p, const char* e) {  // atoi of the field's own bytes
      char tmp[32];
      const size_t m = std::min<size_t>((size_t)(e - p), sizeof tmp - 1);
      memcpy(tmp, p, m);
      tmp[m] = 0;
      return atoi(tmp);
    };
    auto fi = [&](int k) { return fint(fld(k), fend(k)); };
    const bool reverse = fld(4)[0] == '-';
    const char* r_id = fld(0);
    const int r_idn = (int)(fend(0) - r_id);
    const int r_len = fi(1), r_alnstart = fi(2), r_alnend = fi(3);
    const char* t_id = fld(5);
    const int t_idn = (int)(fend(5) - t_id);
    const int t_alnstart = fi(7), t_alnend = fi(8);
    if (li.dup != kDupNo) {
      if (li.dup == kDupWarn)
        b.log_msg(strf("Warning: alignment %.*s to %.*s already seen, ignoring \n", r_idn, r_id, t_idn, t_id));
      return;
    }
    auto qit = qdb->index.find(std::string_view(r_id, (size_t)r_idn));
    if (qit == qdb->index.end()) {
      b.log_fatal(strf("Error: could not retrieve sequence for %.*s !\n", r_idn, r_id));
      return;
    }
    const int qi = qit->second;
    const int L = qdb->len[qi];
    if (r_len != L) {
      b.log_fatal(strf("Error: ref seq len in this PAF line (%d) differs from loaded sequence length(%d)!\n%s\n",
                       r_len, L, s));
      return;
    }
    // ---- record
    RecHost rh;
    rh.pre_msg = rh.cs_msg = rh.post_msg = rh.w_msg = -1;
    rh.n_softclip = 0;
    rh.r_alnstart = r_alnstart;
    rh.r_alnend = r_alnend;
    rh.t_alnstart = t_alnstart;
    rh.t_alnend = t_alnend;
    rh.cs_off = b.cstext.size();
    rh.cs_len = 0;
    rh.cig_msg = -1;
    rh.cig_tpos = rh.cig_qpos = 0;
    rh.t_len = 0;
    rh.gap_off = (uint32_t)b.gaps.size();
    rh.n_rg = rh.n_tg = rh.lab_len = 0;
    rh.line_off = lr.off;
    rh.qlen = L;
    rh.tname_off = (uint32_t)(t_id - s);
    rh.tname_len = (uint32_t)t_idn;
    rh.t_aln = t_alnend - t_alnstart;
    const int offset = reverse ? r_len - r_alnend : r_alnstart;
    const int eff_t_len = t_alnend - t_alnstart;
    int edist = -1, alnscore = 0;
    const char *cigar = nullptr, *cigar_end = nullptr, *cs = nullptr, *cs_end = nullptr;
    int got = 0;
    for (int i = 12; i < numt; ++i) {  // tag scan, pafreport.cpp:495-520
      const char* f = fld(i);
      if (!strncmp(f, "NM:i:", 5)) {
        edist = fint(f + 5, std::max(f + 5, fend(i)));
        got |= 1;
      } else if (!strncmp(f, "AS:i:", 5)) {
        alnscore = fint(f + 5, std::max(f + 5, fend(i)));
        got |= 2;
      } else if (!strncmp(f, "cg:Z:", 5)) {
        cigar = f + 5;
        cigar_end = fend(i);
        got |= 4;
      } else if (!strncmp(f, "cs:Z:", 5)) {
        cs = f + 5;
        cs_end = fend(i);
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
    if (cigar == nullptr || cigar == cigar_end) {
      rh.pre_msg = (int32_t)b.add_msg(strf(CIGAR_ERROR, s, "(null)"));
    } else if (cs == nullptr) {
      rh.pre_msg = (int32_t)b.add_msg(strf("Error: cs tag missing at line:\n%s\n", s));
    } else if (opt.gpu_pack) {
      // the cs field goes to the GPU packer; the CIGAR loop runs now, its verdict waits for the
      // cs totals (finish_gpu_pack)
      rh.cs_len = (uint32_t)(cs_end - cs);
      b.cstext.append(cs, rh.cs_len);
      const char* p = cigar;
      int qpos = 0, tpos = 0;
      std::string err;
      while (p < cigar_end) {
        int cl = 0;
        if (!parse_int(p, cigar_end, cl)) {
          err = strf(CIGAR_ERROR, s, std::string(p, cigar_end).c_str());
          break;
        }
        if (p >= cigar_end) {
          err = strf(CIGAR_ERROR, s, "");
          break;
        }
        const char cop = *p;
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
            err = strf("Error: unhandled cigar_op %c (len %d) in %s\n", cop, cl, s);
            bad = true;
        }
        if (bad) break;
        ++p;
      }
      if (!err.empty()) rh.cig_msg = (int32_t)b.add_msg(std::move(err));
      rh.cig_tpos = tpos;
      rh.cig_qpos = qpos;
    } else {
      // pack cs (grow the arrays to the worst case first: one op per cs byte)
      const size_t cslen = (size_t)(cs_end - cs);
      b.ops.resize(d.op_begin + cslen + 1);
      b.lits.resize(d.lit_begin + cslen + 1);
      pw_cs_totals tot;
      int32_t epos = 0;
      int rc = pack_cs_n(cs, cs_end, offset, L, b.ops.data() + d.op_begin, cslen + 1, b.lits.data() + d.lit_begin,
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
        rh.cs_msg = (int32_t)b.add_msg(cs_error_msg(rc, s, std::string(cs + epos, cs_end)));
      } else {
        // CIGAR loop (pafreport.cpp:645-718): warnings and errors come after the cs loop
        const char* p = cigar;
        int qpos = 0, tpos = 0;
        std::string err;
        rgl.clear();
        tgl.clear();
        while (p < cigar_end) {
          int cl = 0;
          if (!parse_int(p, cigar_end, cl)) {
            err = strf(CIGAR_ERROR, s, std::string(p, cigar_end).c_str());
            break;
          }
          if (p >= cigar_end) {
            err = strf(CIGAR_ERROR, s, "");
            break;
          }
          const char cop = *p;
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
            case 'I':  // gap in the target (pafreport.cpp:685-691)
              if (opt.msa) tgl.push_back({reverse ? eff_t_len - tpos : tpos, cl});
              qpos += cl;
              break;
            case 'D':  // gap in the query (:692-711)
            case 'N':
              if (opt.msa) rgl.push_back({reverse ? r_len - (offset + qpos) : offset + qpos, cl});
              tpos += cl;
              break;
            default:
              err = strf("Error: unhandled cigar_op %c (len %d) in %s\n", cop, cl, s);
              bad = true;
          }
          if (bad) break;
          ++p;
        }
        if (err.empty()) {
          if (eff_t_len != tpos || tot.t_total != tpos)
            err = strf("Error: tseq alignment length mismatch (%d vs %d(%d-%d)) at line:%s\n", tpos, eff_t_len,
                       t_alnend, t_alnstart, s);
          else if (r_alnend - r_alnstart != qpos)
            err = strf("Error: ref alignment length mismatch (%d vs %d-%d) at line:%s\n", qpos, r_alnend,
                       r_alnstart, s);
        }
        if (!err.empty()) {
          rh.post_msg = (int32_t)b.add_msg(std::move(err));
        } else if (opt.msa) {
          // -w: rseq->setGap / taseq->setGap after the report block (pafreport.cpp:394-404)
          rh.t_len = tot.t_total;
          for (auto& g : rgl) {
            b.gaps.push_back(g.first);
            b.gaps.push_back(g.second);
          }
          for (auto& g : tgl) {
            b.gaps.push_back(g.first);
            b.gaps.push_back(g.second);
          }
          rh.n_rg = (uint32_t)rgl.size();
          rh.n_tg = (uint32_t)tgl.size();
          for (auto& g : rgl)
            if (g.first < 0 || g.first >= r_len) {
              rh.w_msg = (int32_t)b.add_msg(strf("Error: invalid gap position (%d) given for sequence %.*s\n",
                                                 g.first + 1, r_idn, r_id));
              break;
            }
          if (rh.w_msg < 0)
            for (auto& g : tgl)
              if (g.first < 0 || g.first >= tot.t_total) {
                rh.w_msg = (int32_t)b.add_msg(strf("Error: invalid gap position (%d) given for sequence %.*s:%d-%d%c\n",
                                                   g.first + 1, t_idn, t_id, t_alnstart, t_alnend,
                                                   reverse ? '-' : '+'));
                break;
              }
        }
      }
    }
    // header (printDiffInfo, pafreport.cpp:886-892; labels :366-379)
    const double cov = ((r_alnend - r_alnstart) * 100.00) / r_len;
    char hb[512];
    // (the common full-length case prints "100.00" without the float formatter)
    int hn;
    if (opt.single_query_gene)
      hn = snprintf(hb, sizeof hb, ">%.*s:%d-%d%c coverage:%.2f score=%d edit_distance=%d\n", t_idn, t_id, t_alnstart,
                    t_alnend, reverse ? '-' : '+', cov, alnscore, edist);
    else if (opt.fullgenome)
      hn = snprintf(hb, sizeof hb, ">%.*s:%d-%d--%.*s:%d-%d%c coverage:%.2f score=%d edit_distance=%d\n", r_idn, r_id,
                    r_alnstart, r_alnend, t_idn, t_id, t_alnstart, t_alnend, reverse ? '-' : '+', cov, alnscore, edist);
    else
      hn = snprintf(hb, sizeof hb, ">%.*s--%.*s:%d-%d%c coverage:%.2f score=%d edit_distance=%d\n", r_idn, r_id, t_idn,
                    t_id, t_alnstart, t_alnend, reverse ? '-' : '+', cov, alnscore, edist);
    rh.hdr_off = b.hdr.size();
    if (hn >= 0 && (size_t)hn < sizeof hb) {
      b.hdr.append(hb, (size_t)hn);
    } else {  // long names
      std::string rl = opt.single_query_gene ? std::string() : std::string(r_id, (size_t)r_idn);
      if (!rl.empty() && opt.fullgenome) rl += strf(":%d-%d", r_alnstart, r_alnend);
      const std::string tl = strf("%.*s:%d-%d%c", t_idn, t_id, t_alnstart, t_alnend, reverse ? '-' : '+');
      const std::string h = rl.empty() ? strf(">%s coverage:%.2f score=%d edit_distance=%d\n", tl.c_str(), cov, alnscore, edist)
                                       : strf(">%s--%s coverage:%.2f score=%d edit_distance=%d\n", rl.c_str(), tl.c_str(),
                                              cov, alnscore, edist);
      b.hdr.append(h.data(), h.size());
    }
    rh.hdr_len = (uint32_t)(b.hdr.size() - rh.hdr_off);
    if (opt.msa) {  // the taseq name (tlabel) right after the header
      char lb[300];
      const int ln = snprintf(lb, sizeof lb, "%.*s:%d-%d%c", t_idn > 256 ? 256 : t_idn, t_id, t_alnstart, t_alnend,
                              reverse ? '-' : '+');
      b.hdr.append(lb, (size_t)ln);
      rh.lab_len = (uint32_t)ln;
    }
    b.desc.push_back(d);
    b.recs.push_back(rh);
    b.log.push_back({1, (uint32_t)b.recs.size() - 1, b.cur_line});
  }
};

// ----------------------------------------------------------------- input chunks (GLineReader)
// Reads the PAF in chunks of about `target` bytes that end on a line end; splits them into
// lines as GLineReader::getLine does (\n, \r or \r\n end a line; a last line without an end is
// a line when non-empty) and NUL-terminates every line in place.
struct ChunkReader {
  FILE* f;
  bool eof = false;
  PodVec<char> carry;
  explicit ChunkReader(FILE* ff) : f(ff) {
    struct stat st;  // a regular file: reserve it whole up front (no regrowth copies)
    if (fstat(fileno(f), &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) carry.reserve((size_t)st.st_size + 1);
  }
  bool next(Batch& b, size_t target) {
    b.buf.swap(carry);
    carry.clear();
    if (eof && b.buf.empty()) return false;
    size_t cut;
    for (;;) {
      if (!eof && b.buf.size() < target) {
        const size_t want = std::min<size_t>(std::max<size_t>(target - b.buf.size(), 1 << 20), 256u << 20);
        const size_t o = b.buf.size();
        b.buf.resize(o + want);
        const size_t got = fread(b.buf.data() + o, 1, want, f);
        b.buf.resize(o + got);
        if (got < want) eof = true;
        if (!eof && b.buf.size() < target) continue;
      }
      const size_t sz = b.buf.size();
      if (eof) {
        cut = sz;
        break;
      }
      const char* nl = (const char*)memrchr(b.buf.data(), '\n', sz);
      if (nl) {
        cut = (size_t)(nl - b.buf.data()) + 1;
        break;
      }
      const char* cr = (const char*)memrchr(b.buf.data(), '\r', sz);
      if (cr && (size_t)(cr - b.buf.data()) + 1 < sz) {
        cut = (size_t)(cr - b.buf.data()) + 1;
        break;
      }
      target += target / 2 + (1 << 20);  // one line longer than the chunk: read on
    }
    carry.append(b.buf.data() + cut, b.buf.size() - cut);
    b.buf.resize(cut);
    b.buf.push_back('\0');
    char* s = b.buf.data();
    const size_t n = cut;
    const bool has_cr = memchr(s, '\r', n) != nullptr;
    size_t p = 0;
    while (p < n) {
      size_t e;
      if (!has_cr) {
        const char* q = (const char*)memchr(s + p, '\n', n - p);
        e = q ? (size_t)(q - s) : n;
      } else {
        e = p;
        while (e < n && s[e] != '\n' && s[e] != '\r') e++;
      }
      if (e == n && e == p) break;  // nothing after the last line end
      b.lines.push_back({p, (uint32_t)(e - p)});
      size_t nx = e + 1;
      if (e < n && s[e] == '\r' && e + 1 < n && s[e + 1] == '\n') nx = e + 2;
      s[e] = '\0';
      p = nx;
    }
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
  DevBuf<uint8_t> cs_text;  // GPU packing
  DevBuf<uint64_t> cs_offs;
  DevBuf<int32_t> cs_o, cs_q;
  DevBuf<pw_cs_rec> cs_rec;
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
  // GPU packing of a batch whose records carry their cs fields (Options::gpu_pack): every cs
  // string through pw_pack_cs_batch into the device op / literal arrays (record k's ops and
  // literal bytes start at its cs field's offset), the per-record totals back to the host, and the
  // rest of the record's host work that needs them — descriptor (op count, tseq length, event
  // slots, A/C/G/T flag), the cs / CIGAR verdict in the reference's order (pafreport.cpp:536-718).
  // Records the kernel hands back (PW_PACK_HOST: not plain cs, or an op longer than a window) are
  // packed by pw_pack_cs here, which gives the exact error, or their ops are uploaded.
  bool gpu_pack(Batch& b, const QueryDb& q) {
    const size_t na = b.desc.size();
    const size_t ct = b.cstext.size();
    std::vector<uint64_t> off(na + 1);
    std::vector<int32_t> o(na), ql(na);
    for (size_t k = 0; k < na; k++) {
      off[k] = b.recs[k].cs_off;
      o[k] = b.desc[k].offset;
      ql[k] = b.recs[k].qlen;
    }
    off[na] = ct;
    if (ct >= (1ull << 32) - 64) {  // op_begin / lit_begin are 32-bit offsets into the batch's cs text
      fprintf(stderr, "pafreport: batch cs text of %zu bytes exceeds the 4 GiB a batch can address\n", ct);
      return false;
    }
    if (!cs_text.ensure(ct + 16) || !ops.ensure(ct + 16) || !lits.ensure(ct + kDevPad) || !cs_offs.ensure(na + 1) ||
        !cs_o.ensure(na + 1) || !cs_q.ensure(na + 1) || !cs_rec.ensure(na + 1)) {
      fprintf(stderr, "pafreport: device allocation failed\n");
      return false;
    }
    if (ct) HIPCHK(hipMemcpyAsync(cs_text.p, b.cstext.data(), ct, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemsetAsync(cs_text.p + ct, 0, 16, stream));
    HIPCHK(hipMemcpyAsync(cs_offs.p, off.data(), (na + 1) * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(cs_o.p, o.data(), na * 4, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(cs_q.p, ql.data(), na * 4, hipMemcpyHostToDevice, stream));
    if (pw_pack_cs_batch(cs_text.p, cs_offs.p, cs_o.p, cs_q.p, (uint32_t)na, ops.p, lits.p, cs_rec.p, stream) != PW_OK) {
      fprintf(stderr, "pafreport: cs packing launch failed\n");
      return false;
    }
    std::vector<pw_cs_rec> rec(na);
    HIPCHK(hipMemcpyAsync(rec.data(), cs_rec.p, na * sizeof(pw_cs_rec), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    uint64_t ev = 0, txt = 0;
    std::vector<uint32_t> hops;
    std::vector<uint8_t> hlits;
    // host-packed op / literal prefixes of handed-back records, uploaded after the loop on `stream`
    // whatever the packer's verdict: index_kernel decodes d.n_ops words of a failing record too
    // (a base mismatch before the cs error is the reference's first error, pafreport.cpp:545-548)
    std::vector<uint32_t> fb_ops;
    std::vector<uint8_t> fb_lits;
    std::vector<std::array<uint64_t, 4>> fb;  // dst offset, fb_ops start, n_ops, n_lits (lits at fb_lits start = [1])
    std::vector<uint64_t> fb_lit0;
    for (size_t k = 0; k < na; k++) {
      RecHost& rh = b.recs[k];
      pw_aln_desc& d = b.desc[k];
      d.op_begin = d.lit_begin = (uint32_t)rh.cs_off;
      d.ev_begin = ev;
      if (rh.pre_msg >= 0) continue;  // no cs loop (pafreport.cpp:521-524)
      const char* s = b.buf.data() + rh.line_off;
      const char* cs = b.cstext.data() + rh.cs_off;
      const int qi = (int)(d.ref & PW_REF_QMASK);
      pw_cs_totals tot;
      int rc = PW_CS_OK;
      int32_t epos = 0;
      bool acgt;
      if (rec[k].flags & PW_PACK_HOST) {
        hops.resize((size_t)rh.cs_len + 1);
        hlits.resize((size_t)rh.cs_len + 1);
        rc = pack_cs_n(cs, cs + rh.cs_len, d.offset, rh.qlen, hops.data(), hops.size(), hlits.data(), hlits.size(), &tot,
                       &epos);
        if (tot.n_ops || tot.n_lits) {
          fb.push_back({rh.cs_off, fb_ops.size(), tot.n_ops, tot.n_lits});
          fb_lit0.push_back(fb_lits.size());
          fb_ops.insert(fb_ops.end(), hops.begin(), hops.begin() + tot.n_ops);
          fb_lits.insert(fb_lits.end(), hlits.begin(), hlits.begin() + tot.n_lits);
        }
        acgt = rc == PW_CS_OK && q.all_acgt(qi);
        for (uint32_t i = 0; i < tot.n_lits && acgt; i++) acgt = QueryDb::is_acgt_byte(hlits[i]);
      } else {
        tot.q_total = rec[k].q_total;
        tot.t_total = rec[k].t_total;
        tot.n_ops = rec[k].n_ops;
        tot.n_lits = rec[k].n_lits;
        tot.n_events_max = rec[k].n_events_max;
        tot.text_bound = rec[k].text_bound;
        acgt = q.all_acgt(qi) && (rec[k].flags & PW_PACK_ACGT);
      }
      d.n_ops = tot.n_ops;
      d.t_len = tot.t_total;
      if (acgt) d.ref |= PW_REF_ACGT;
      ev += tot.n_events_max;
      txt += tot.text_bound;
      if (rc != PW_CS_OK) {
        rh.cs_msg = (int32_t)b.add_msg(cs_error_msg(rc, s, std::string(cs + epos, cs + rh.cs_len)));
      } else if (rh.cig_msg >= 0) {
        rh.post_msg = rh.cig_msg;
      } else {
        const int eff_t_len = rh.t_alnend - rh.t_alnstart, tpos = rh.cig_tpos, qpos = rh.cig_qpos;
        if (eff_t_len != tpos || tot.t_total != tpos)
          rh.post_msg = (int32_t)b.add_msg(strf("Error: tseq alignment length mismatch (%d vs %d(%d-%d)) at line:%s\n",
                                                tpos, eff_t_len, rh.t_alnend, rh.t_alnstart, s));
        else if (rh.r_alnend - rh.r_alnstart != qpos)
          rh.post_msg = (int32_t)b.add_msg(strf("Error: ref alignment length mismatch (%d vs %d-%d) at line:%s\n", qpos,
                                                rh.r_alnend, rh.r_alnstart, s));
      }
    }
    for (size_t j = 0; j < fb.size(); j++) {
      if (fb[j][2]) HIPCHK(hipMemcpyAsync(ops.p + fb[j][0], fb_ops.data() + fb[j][1], fb[j][2] * 4, hipMemcpyHostToDevice, stream));
      if (fb[j][3]) HIPCHK(hipMemcpyAsync(lits.p + fb[j][0], fb_lits.data() + fb_lit0[j], fb[j][3], hipMemcpyHostToDevice, stream));
    }
    if (!fb.empty()) HIPCHK(hipStreamSynchronize(stream));  // the staging vectors die here
    b.n_events_max = ev;
    b.text_total = txt;
    return true;
  }
  // run the batch; fills results / pages on the host (and the text, unless text_h is null: the
  // CLI streams it with a TextStream instead)
  bool run(Batch& b, const QueryDb& q, bool skip_codan, std::vector<uint8_t>* text_h,
           std::vector<pw_aln_result>& res_h, std::vector<pw_page>& pages_h) {
    if (b.gpu_packed && !b.desc.empty() && !gpu_pack(b, q)) return false;
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
    // every field is assigned below; PW_ARGS_POISON=1 (tests) fills the struct with 0xFF first so
    // that a field left unset shows up as a wrong report instead of as whatever the stack held
    pw_report_args a;
    memset(&a, (getenv("PW_ARGS_POISON") && atoi(getenv("PW_ARGS_POISON")) != 0) ? 0xFF : 0, sizeof a);
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
    a.max_rec_ops = 0;
    a.n_short = 0;
    for (const pw_aln_desc& d : b.desc) {
      a.max_rec_ops = d.n_ops > a.max_rec_ops ? d.n_ops : a.max_rec_ops;
      a.n_short += d.n_ops <= 64 ? 1u : 0u;
    }
    if (getenv("PW_NO_PAIRS") && atoi(getenv("PW_NO_PAIRS")) != 0) a.n_short = 0;  // (tests: one record per wave)
    // 16-byte event records when the query positions / indices fit (PW_HOT32=1 keeps 32-byte ones)
    a.hot_pbits = (getenv("PW_HOT32") && atoi(getenv("PW_HOT32")) != 0) ? 0u : pw_report_hot_pbits(q.max_len(), q.len.size());
    a.flags = 0;  // the CLI builds the next-stop table once per query set (Device::init)
    a.n_queries = (uint32_t)q.len.size();
    a.pad = 0;
    if (pw_report_events(&a, stream) != PW_OK) {
      fprintf(stderr, "pafreport: kernel launch failed\n");
      return false;
    }
    HIPCHK(hipMemcpyAsync(res_h.data(), res.p, na * sizeof(pw_aln_result), hipMemcpyDeviceToHost, stream));
    if (np) HIPCHK(hipMemcpyAsync(pages_h.data(), pages.p, np * sizeof(pw_page), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    if (!text_h) return true;
    // copy back the used part of the text (pages + arena)
    uint64_t used = 0;
    for (const pw_page& pg : pages_h)
      if (pg.len && pg.off + pg.len > used) used = pg.off + pg.len;
    if (used > tcap) used = tcap;
    text_h->resize(used);
    if (used) HIPCHK(hipMemcpy(text_h->data(), text.p, used, hipMemcpyDeviceToHost));
    return true;
  }
  ~Device() {
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// The report text of a finished batch, streamed to the host in the order the emit loop reads
// it: the page region [0, arena0) through two pinned windows (the DMA of window k + 1 runs while
// window k is written out), the arena (pages that overflowed, read out of order) as one host copy.
// Pages are PW_PAGE_BYTES-aligned and no longer than that, and the window is a multiple of it, so
// a page never straddles two windows.
struct TextStream {
  static constexpr uint64_t kWin = 32ull << 20;
  uint8_t* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipStream_t st = nullptr;
  uint64_t base[2] = {0, 0};
  int cur = 0;
  bool waited = false;
  const uint8_t* dev = nullptr;
  uint64_t region_end = 0, arena0 = 0;
  std::vector<uint8_t> arena;
  std::vector<uint8_t> img[2];  // emit_parallel's output images (kept across batches: faulted in once)
  bool ok = false;
  bool init() {  // (reports its own failure)
    if (ok) return true;
    for (int k = 0; k < 2; k++)
      if (hipHostMalloc((void**)&buf[k], kWin, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
        fprintf(stderr, "pafreport: pinned host buffers could not be allocated\n");
        return false;
      }
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
      fprintf(stderr, "pafreport: HIP stream creation failed\n");
      return false;
    }
    ok = true;
    return true;
  }
  void fetch(int k) {
    const uint64_t n = base[k] < region_end ? std::min(kWin, region_end - base[k]) : 0;
    if (n) (void)hipMemcpyAsync(buf[k], dev + base[k], n, hipMemcpyDeviceToHost, st);
    (void)hipEventRecord(ev[k], st);
  }
  // start streaming the text of a finished batch (pages on the host already)
  bool begin(const uint8_t* text_dev, const std::vector<pw_page>& pages, uint64_t n_chunks) {
    dev = text_dev;
    arena0 = n_chunks * (uint64_t)PW_PAGE_BYTES;
    region_end = 0;
    uint64_t aend = arena0;
    for (const pw_page& pg : pages) {
      if (!pg.len) continue;
      if (pg.off < arena0) region_end = std::max(region_end, pg.off + pg.len);
      else aend = std::max(aend, pg.off + pg.len);
    }
    arena.resize(aend - arena0);
    if (!arena.empty() && hipMemcpy(arena.data(), dev + arena0, arena.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return false;
    cur = 0;
    waited = false;
    base[0] = 0;
    base[1] = kWin;
    fetch(0);
    fetch(1);
    return true;
  }
  const uint8_t* at(uint64_t off, size_t) {
    if (off >= arena0) return arena.data() + (off - arena0);
    while (off >= base[cur] + kWin) {  // window cur is done: refill it two windows ahead
      if (!waited) (void)hipEventSynchronize(ev[cur]);
      base[cur] += 2 * kWin;
      fetch(cur);
      cur ^= 1;
      waited = false;
    }
    if (!waited) {
      (void)hipEventSynchronize(ev[cur]);
      waited = true;
    }
    return buf[cur] + (off - base[cur]);
  }
  void end() {  // nothing in flight after the batch (the buffers are reused)
    if (st) (void)hipStreamSynchronize(st);
  }
  ~TextStream() {
    end();
    for (int k = 0; k < 2; k++) {
      if (buf[k]) (void)hipHostFree(buf[k]);
      if (ev[k]) (void)hipEventDestroy(ev[k]);
    }
    if (st) (void)hipStreamDestroy(st);
  }
};

// Print what the reference prints for one log item; returns -1 to continue, else the exit code
// the reference ends with at this item.
// Write the first `nlines` event lines of a record (all of them when nlines == n_events): the
// bytes from text_off to text_end, crossing pages in chunk order (pwasm_amd.h, text pages).
// Where write_lines reads report text: a whole host copy (batch API), or a stream of pinned
// windows copied from the device while the emit loop writes (CLI, TextStream below).
struct TextSrc {
  const uint8_t* host = nullptr;
  struct TextStream* stream = nullptr;
  const uint8_t* at(uint64_t off, size_t n) const;
};
const uint8_t* TextSrc::at(uint64_t off, size_t n) const { return host ? host + off : stream->at(off, n); }

void write_lines(const TextSrc& text, const pw_page* pages, const pw_aln_result& r, uint32_t nlines, FILE* out) {
  if (r.n_events == 0 || nlines == 0) return;
  uint32_t seen = 0;
  for (uint32_t c = r.page_first;; c++) {
    const uint64_t lo = c == r.page_first ? r.text_off : pages[c].off;
    const uint64_t hi = c == r.page_last ? r.text_end : pages[c].off + pages[c].len;
    size_t n = (size_t)(hi - lo);
    const uint8_t* p = text.at(lo, n);
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

int emit_item(const Batch& b, const LogItem& it, const TextSrc& text, const pw_aln_result* res, const pw_page* pages,
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
  const char* lstr = b.buf.data() + rh.line_off;
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
  if (nlines == r.n_events) {
    if (rh.w_msg < 0) return -1;
    fflush(out);  // -w: rseq / taseq setGap failed after the report block (pafreport.cpp:394-404)
    fputs(b.msgs[rh.w_msg].c_str(), err);
    return 1;
  }
  fflush(out);
  fputs(post.c_str(), err);
  return 1;
}

// Print what the reference prints for this batch; returns -1 to continue, else an exit code.
int emit(const Batch& b, const TextSrc& text, const pw_aln_result* res, const pw_page* pages, FILE* out) {
  for (const LogItem& it : b.log) {
    const int rc = emit_item(b, it, text, res, pages, out, stderr);
    if (rc >= 0) return rc;
  }
  return -1;
}

// Parallel emit of a batch into a regular output file (-o): when no item of the batch ends the
// run or prints a partial record, every stdout byte's file offset is known up front (headers on
// the host, lines in the device text pages), so the batch is written as pieces — each record's
// header, then its page spans — by `nt` threads with pwritev at their offsets, window by window of
// the page region as the pinned TextStream windows arrive (the DMA of window k + 2 runs while
// window k + 1 is written); stderr lines are printed in item order by this thread.  The FILE's
// position is moved past the batch afterwards.  Returns -1 (continue) when done, -2 when the batch
// needs the sequential emit (a fatal item, a partial record, a -w message), -3 on a write error.
int emit_parallel(const Batch& b, TextStream& ts, const pw_aln_result* res, const pw_page* pages, FILE* out, int nt) {
  for (const LogItem& it : b.log) {
    if (it.kind == 2) return -2;
    if (it.kind != 1) continue;
    const RecHost& rh = b.recs[it.idx];
    const pw_aln_result& r = res[it.idx];
    if (rh.pre_msg >= 0 || r.err != 0 || rh.cs_msg >= 0 || rh.post_msg >= 0 || rh.w_msg >= 0 ||
        (rh.qlen < 9 && r.n_events > 0))
      return -2;
  }
  if (fflush(out) != 0) return -3;
  const int fd = fileno(out);
  const off_t base = lseek(fd, 0, SEEK_CUR);
  if (base < 0) return -2;
  // pieces in output order: a host source (headers, arena pages) or a page-region offset
  struct Piece {
    const uint8_t* host;
    uint64_t src, len, dst;
    int64_t win;  // page-region window of the source (-1: on the host)
  };
  std::vector<Piece> pc;
  pc.reserve(b.log.size() * 3);
  uint64_t dst = 0;
  for (const LogItem& it : b.log) {
    if (it.kind == 0) continue;
    const RecHost& rh = b.recs[it.idx];
    const pw_aln_result& r = res[it.idx];
    pc.push_back({(const uint8_t*)b.hdr.data() + rh.hdr_off, 0, rh.hdr_len, dst, -1});
    dst += rh.hdr_len;
    if (r.n_events == 0) continue;
    for (uint32_t c = r.page_first;; c++) {
      const uint64_t lo = c == r.page_first ? r.text_off : pages[c].off;
      const uint64_t hi = c == r.page_last ? r.text_end : pages[c].off + pages[c].len;
      if (hi > lo) {
        if (lo >= ts.arena0) pc.push_back({ts.arena.data() + (lo - ts.arena0), 0, hi - lo, dst, -1});
        else pc.push_back({nullptr, lo, hi - lo, dst, (int64_t)(lo / TextStream::kWin)});
        dst += hi - lo;
      }
      if (c == r.page_last) break;
    }
  }
  // host pieces go with the window of the next page-region piece (page-region sources increase
  // along the list; pages never straddle a window)
  int64_t next = 0;
  for (const Piece& p : pc) next = std::max(next, p.win);
  for (size_t i = pc.size(); i-- > 0;) {
    if (pc[i].win >= 0) next = pc[i].win;
    else pc[i].win = next;
  }
  for (size_t i = 1; i < pc.size(); i++)
    if (pc[i].win < pc[i - 1].win) return -2;  // (not monotone: cannot happen; keep the sequential path)
  for (const LogItem& it : b.log) {  // stderr, in item order
    if (it.kind == 0) {
      fputs(b.msgs[it.idx].c_str(), stderr);
      continue;
    }
    const RecHost& rh = b.recs[it.idx];
    for (int k = 0; k < rh.n_softclip; k++)
      fprintf(stderr, "Warning: soft clipping shouldn't be found in this application!\n%s\n",
              b.buf.data() + rh.line_off);
  }
  // Per window: the pieces are copied by up to nt threads into one contiguous host image of the
  // window's destination range, and that image goes out as one large pwrite on a writer thread
  // while the next window is copied (two images alternate).  Writers of one file serialise on its
  // inode lock, so many small concurrent pwritev calls (a piece is a ~60-byte header or a record's
  // ~2 KB of lines) ran at ~3.3 GB/s where one large pwrite reaches the file system's ~10 GB/s
  // (tools/gpu_e2e3.sh, round 5).
  const int64_t nwin = pc.empty() ? 0 : pc.back().win + 1;
  std::atomic<bool> bad{false};
  std::vector<uint8_t>* img = ts.img;
  std::thread wr[2];
  auto write_img = [&](int k, uint64_t d0, uint64_t n) {
    uint64_t done = 0;
    while (done < n) {
      const ssize_t w = pwrite(fd, img[k].data() + done, (size_t)(n - done), base + (off_t)(d0 + done));
      if (w <= 0) {
        bad = true;
        return;
      }
      done += (uint64_t)w;
    }
  };
  // A window's pieces are cut into groups of at most kImg destination bytes, so an image never
  // holds more than that (host pieces after the last page-region piece all join the last window:
  // a batch of mostly arena text would otherwise make one image of its whole output); a single
  // piece larger than kImg is written straight from its source.
  uint64_t kImg = 2 * TextStream::kWin;
  if (const char* e = getenv("PW_EMIT_IMG_BYTES")) kImg = std::max<uint64_t>(1, strtoull(e, nullptr, 10));  // (tests)
  int ik = 0;  // the image the next group is copied into (the two alternate)
  size_t i0 = 0;
  for (int64_t w = 0; w < nwin && !bad; w++) {
    size_t i1 = i0;
    while (i1 < pc.size() && pc[i1].win == w) i1++;
    const int slot = (int)(w & 1);
    const uint64_t wlo = (uint64_t)w * TextStream::kWin;
    const bool dma = wlo < ts.region_end;
    if (dma) {
      if (ts.base[slot] != wlo) {
        bad = true;
        break;  // (windows are consumed in order)
      }
      (void)hipEventSynchronize(ts.ev[slot]);
    }
    const uint8_t* wb = ts.buf[slot];
    for (size_t g0 = i0; g0 < i1 && !bad;) {
      if (pc[g0].len > kImg) {  // one large piece: written from its source, before wb is refilled
        const uint8_t* src = pc[g0].host ? pc[g0].host : wb + (pc[g0].src - wlo);
        for (uint64_t done = 0; done < pc[g0].len;) {
          const ssize_t n = pwrite(fd, src + done, (size_t)(pc[g0].len - done), base + (off_t)(pc[g0].dst + done));
          if (n <= 0) {
            bad = true;
            break;
          }
          done += (uint64_t)n;
        }
        g0++;
        continue;
      }
      size_t g1 = g0 + 1;
      while (g1 < i1 && pc[g1].len <= kImg && pc[g1].dst + pc[g1].len - pc[g0].dst <= kImg) g1++;
      if (wr[ik].joinable()) wr[ik].join();  // image `ik` is free again
      const uint64_t d0 = pc[g0].dst, d1 = pc[g1 - 1].dst + pc[g1 - 1].len;
      if (img[ik].size() < d1 - d0) img[ik].resize(d1 - d0);
      uint8_t* ib = img[ik].data();
      const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(nt, 1), (d1 - d0) >> 20));
      auto work = [&](int t) {  // the pieces whose destination starts in this thread's byte range
        const uint64_t a = d0 + (d1 - d0) * (uint64_t)t / (uint64_t)T;
        const uint64_t z = d0 + (d1 - d0) * (uint64_t)(t + 1) / (uint64_t)T;
        size_t j = (size_t)(std::lower_bound(pc.begin() + (long)g0, pc.begin() + (long)g1, a,
                                             [](const Piece& p, uint64_t v) { return p.dst < v; }) -
                            pc.begin());
        for (; j < g1 && pc[j].dst < z; j++)
          memcpy(ib + (pc[j].dst - d0), pc[j].host ? pc[j].host : wb + (pc[j].src - wlo), pc[j].len);
      };
      std::vector<std::thread> th;
      for (int t = 1; t < T; t++) th.emplace_back(work, t);
      work(0);
      for (auto& x : th) x.join();
      wr[ik] = std::thread(write_img, ik, d0, d1 - d0);
      ik ^= 1;
      g0 = g1;
    }
    if (dma) {  // this window's buffer takes window w + 2
      ts.base[slot] += 2 * TextStream::kWin;
      ts.fetch(slot);
    }
    i0 = i1;
  }
  for (auto& x : wr)
    if (x.joinable()) x.join();
  if (bad) return -3;
  if (fseeko(out, base + (off_t)dst, SEEK_SET) != 0) return -3;
  return -1;
}

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
static double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The CLI's host and device state (one allocation, so that the executable can leave it to the
// process exit: freeing the batches' host vectors and the device buffers took 0.8 s after a
// 16 GB cfg3 report — tools/gpu_e2e3.sh, round 5).
struct CliState {
  QueryDb qdb;
  Device dev;
  Packer pk;
  std::unique_ptr<ChunkReader> rd;
  Batch bb[2];
  TextStream tstream;
  std::vector<pw_aln_result> res_h;
  std::vector<pw_page> pages_h;
};

static int run_cli(int argc, char** argv, bool leave_state);

extern "C" int pw_pafreport_main(int argc, char** argv) { return run_cli(argc, argv, false); }

// (PW_PROFILE_HOST: wall-clock epochs at main's entry and just before the process exits, so the
// caller can attribute its own wall time: process start = entry - spawn, exit = reaped - exit)
static double epoch_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

extern "C" int pw_pafreport_main_exit(int argc, char** argv) {
  const bool prof = getenv("PW_PROFILE_HOST") != nullptr;
  if (prof) fprintf(stderr, "[cli] main_entry_epoch %.6f\n", epoch_s());
  const int rc = run_cli(argc, argv, true);  // (output files closed; the rest goes with the process)
  if (prof) fprintf(stderr, "[cli] exit_epoch %.6f\n", epoch_s());
  fflush(stdout);
  fflush(stderr);
  _exit(rc);
}

static int run_cli(int argc, char** argv, bool leave_state) {
  // (PW_PROFILE_HOST: the destructors' time at the end — declared first, so destroyed last)
  struct TearTimer {
    double t = 0;
    ~TearTimer() {
      if (t > 0) fprintf(stderr, "[cli] teardown %.3f s\n", mono_s() - t);
    }
  } tear;
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
  // the HIP runtime / context comes up on its own thread while the FASTA and the first batch are
  // read and packed (about 0.1 s of device initialisation hidden)
  struct Warm {
    std::thread t;
    Warm() : t([] {
      int n = 0;
      if (hipGetDeviceCount(&n) == hipSuccess && n > 0) (void)hipFree(nullptr);
    }) {}
    void join() {
      if (t.joinable()) t.join();
    }
    ~Warm() { join(); }
  } warm;
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
    setvbuf(out.f, nullptr, _IOFBF, 8u << 20);  // the report is written in large blocks
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
  const bool prof = getenv("PW_PROFILE_HOST") != nullptr;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = prof ? now() : 0;
  CliState* state = new CliState;
  std::unique_ptr<CliState, void (*)(CliState*)> state_owner(
      state, leave_state ? +[](CliState*) {} : +[](CliState* p) { delete p; });
  QueryDb& qdb = state->qdb;
  std::string err;
  if (!qdb.load(fa, err)) {
    fputs(err.c_str(), stderr);
    return 1;
  }
  const double t_fasta = prof ? now() : 0;
  if (!fullgenome && !gene && fsize > 120000) fullgenome = true;
  bool skip_codan = fullgenome || force_noncoding;
  if (!skip_codan && !force_coding && fsize > 120000) skip_codan = true;
  FileCloser fmsa;
  if (args.set['w'] && args.val['w'][0]) {  // pafreport.cpp:263-273
    if (fullgenome) {
      fprintf(stderr, "%s Error: can only generate MSA for -G mode!\n", USAGE);
      return 1;
    }
    fmsa.f = fopen(args.val['w'], "w");
    if (!fmsa.f) {
      fprintf(stderr, "Cannot open file %s for writing!\n", args.val['w']);
      return 1;
    }
  }
  Device& dev = state->dev;
  Packer& pk = state->pk;
  pk.qdb = &qdb;
  pk.nt = host_threads();
  pk.opt.fullgenome = fullgenome;
  pk.opt.skip_codan = skip_codan;
  pk.opt.verbose = verbose;
  pk.opt.single_query_gene = (qdb.ids.size() == 1 && !fullgenome);
  pk.opt.msa = fmsa.f != nullptr;
  // cs strings are packed on the GPU unless -w needs the op stream on the host
  // (the query run's MSA is built there) or PW_PACK_HOST=1 asks for the host packer
  pk.opt.gpu_pack = !pk.opt.msa && !(getenv("PW_PACK_HOST") && atoi(getenv("PW_PACK_HOST")) != 0);
  // Pipeline: while the GPU runs batch k and its report is written, batch k + 1 is read and
  // packed (by pk.nt threads); nothing past a fatal batch is packed.
  state->rd = std::make_unique<ChunkReader>(in.f);
  ChunkReader& rd = *state->rd;
  Batch* bb = state->bb;
  TextStream& tstream = state->tstream;
  std::vector<pw_aln_result>& res_h = state->res_h;
  std::vector<pw_page>& pages_h = state->pages_h;
  size_t kChunk = 256u << 20;  // input bytes per batch (PW_CHUNK_BYTES: tests force many batches)
  if (const char* e = getenv("PW_CHUNK_BYTES"))
    if (atoll(e) > 0) kChunk = (size_t)atoll(e);
  auto pack_next = [&](Batch& B) -> bool {
    B.clear();
    if (!rd.next(B, kChunk)) return false;
    pk.pack(B);
    return true;
  };
  // -o into a regular file: batches without a fatal item are written by pk.nt threads at known
  // offsets (emit_parallel); PW_SERIAL_EMIT=1 keeps the sequential stdio emit
  bool par_emit = false;
  if (out.f != stdout && !(getenv("PW_SERIAL_EMIT") && atoi(getenv("PW_SERIAL_EMIT")) != 0)) {
    struct stat os;
    par_emit = fstat(fileno(out.f), &os) == 0 && S_ISREG(os.st_mode);
  }
  int cur = 0;
  // the device side comes up beside the first batch's pack: the HIP runtime (warm-up thread), then
  // the queries, their next-stop tables and the pinned text windows
  bool dev_ok = false;
  double t_warm = 0, t_dinit = 0, t_tsinit = 0;  // (PW_PROFILE_HOST: when each step of dev_up ended)
  std::thread dev_up([&] {
    warm.join();
    if (prof) t_warm = now();
    // the pinned text windows (hipHostMalloc, ~6-9 ms) on a thread of their own beside the queries'
    // upload and stop tables (each prints its own failure)
    bool ts_ok = false;
    std::thread ts([&] {
      ts_ok = tstream.init();
      if (prof) t_tsinit = now();
    });
    dev_ok = dev.init(qdb, skip_codan);
    if (prof) t_dinit = now();
    ts.join();
    dev_ok = dev_ok && ts_ok;
  });
  bool have = pack_next(bb[0]);
  const double t_pack0 = prof ? now() : 0;
  dev_up.join();
  if (!dev_ok) return 2;
  if (prof) {
    fprintf(stderr, "[cli] fasta %.3f s, first batch read + pack %.3f s, device init (after warm-up) %.3f s\n",
            t_fasta - t_start, t_pack0 - t_fasta, now() - t_pack0);
    // (the device side's own steps from t_start, overlapped with the above: not summed into the total)
    fprintf(stderr, "[cli-dev] hip runtime up at %.3f s, queries + stop tables at %.3f s, pinned windows (beside them) at %.3f s\n",
            t_warm - t_start, t_dinit - t_start, t_tsinit - t_start);
  }
  while (have) {
    Batch& B = bb[cur];
    const bool more = !B.fatal;
    std::future<bool> nxt;
    if (more) {
      const int o = cur ^ 1;
      nxt = std::async(std::launch::async, [&, o] { return pack_next(bb[o]); });
    }
    const double t_r0 = prof ? now() : 0;
    bool ran = dev.run(B, qdb, skip_codan, nullptr, res_h, pages_h);
    ran = ran && tstream.begin(dev.text.p, pages_h, pw_report_page_count(B.n_events_max));
    const double t_r1 = prof ? now() : 0;
    TextSrc src;
    src.stream = &tstream;
    int rc = 2;
    if (ran) {
      rc = par_emit ? emit_parallel(B, tstream, res_h.data(), pages_h.data(), out.f, pk.nt) : -2;
      if (rc == -3) {
        fprintf(stderr, "pafreport: error writing the report\n");
        rc = 2;
      } else if (rc == -2) {
        rc = emit(B, src, res_h.data(), pages_h.data(), out.f);
      }
    }
    tstream.end();
    if (prof)
      fprintf(stderr, "[cli] batch: gpu run + result copies %.3f s, emit (text streamed) %.3f s\n", t_r1 - t_r0,
              now() - t_r1);
    if (rc >= 0) {
      if (more) nxt.wait();
      fflush(out.f);
      return rc;
    }
    have = more && nxt.get();
    cur ^= 1;
  }
  fflush(out.f);
  if (prof) fprintf(stderr, "[cli] total %.3f s\n", now() - t_start);
  // -D dumps refMSA on stderr first (pafreport.cpp:443-446; without -w refMSA is NULL there, D7)
  if (fmsa.f && pk.run.qi >= 0) {  // refMSA->writeMSA(fmsa), pafreport.cpp:447-450
    const int qi = pk.run.qi;
    fflush(stderr);
    const int rc = pw::write_run_msa(fmsa.f, debug ? stderr : nullptr, qdb.ids[(size_t)qi].c_str(), qdb.seq.data() + qdb.off[(size_t)qi],
                                 qdb.len[(size_t)qi], pk.run);
    if (rc != 0) return rc;
  }
  if (prof) {
    const double t = now();
    if (out.f && out.f != stdout) {
      fclose(out.f);
      out.f = nullptr;
    }
    fprintf(stderr, "[cli] close output %.3f s\n", now() - t);
    tear.t = mono_s();
  }
  return 0;
}

// ================================================================= batch API (bench / tests)
struct pw_batch {
  QueryDb q;
  Batch b;
  Packer pk;
  bool skip_codan = false;
  uint64_t alg_in = 0;
  // per-genome tables (target sequence names in order of first appearance), built on demand
  bool g_ready = false;
  std::vector<uint32_t> gid;
  std::vector<int32_t> taln;
  std::string gnames;
  uint32_t ngen = 0;
};

extern "C" pw_batch* pw_batch_from_files_shard(const char* fasta, const char* paf, uint32_t flags, uint32_t shard,
                                               uint32_t nshards, char* errbuf, size_t errlen) {
  auto fail = [&](const std::string& m) -> pw_batch* {
    if (errbuf && errlen) snprintf(errbuf, errlen, "%s", m.c_str());
    return nullptr;
  };
  if (nshards == 0 || shard >= nshards) return fail("bad shard");
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
  bt->pk.nt = host_threads();
  bt->pk.opt.fullgenome = full;
  bt->pk.opt.skip_codan = skip;
  bt->pk.opt.single_query_gene = (bt->q.ids.size() == 1 && !full);
  bt->pk.opt.shard = shard;
  bt->pk.opt.nshards = nshards;
  bt->pk.opt.msa = (flags & 16u) != 0 && !full;
  FILE* f = fopen(paf, "rb");
  if (!f) {
    delete bt;
    return fail(strf("cannot open %s", paf));
  }
  ChunkReader rd(f);
  const auto t0 = std::chrono::steady_clock::now();
  if (rd.next(bt->b, SIZE_MAX / 4)) {  // the whole file is one batch
    if (getenv("PW_PROFILE_HOST"))
      fprintf(stderr, "[read] %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    bt->pk.pack(bt->b);
  }
  fclose(f);
  bt->alg_in = alg_bytes(bt->b, bt->q, skip);
  return bt;
}

extern "C" pw_batch* pw_batch_from_files(const char* fasta, const char* paf, uint32_t flags, char* errbuf,
                                         size_t errlen) {
  return pw_batch_from_files_shard(fasta, paf, flags, 0, 1, errbuf, errlen);
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
  TextSrc src;
  src.host = text_host;
  int rc = emit(bt->b, src, res_host, pages_host, f);
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
    TextSrc src;
    src.host = text_host;
    const int32_t st = emit_item(bt->b, it, src, res_host, pages_host, o, e);
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

extern "C" int pw_batch_write_msa(const pw_batch* bt, const char* path) {
  if (!bt || !path || !bt->pk.opt.msa) return PW_E_ARG;
  FILE* f = fopen(path, "w");
  if (!f) return PW_E_IO;
  int rc = 0;
  const pw::MsaRun& run = bt->pk.run;
  if (run.qi >= 0)
    rc = pw::write_run_msa(f, nullptr, bt->q.ids[(size_t)run.qi].c_str(), bt->q.seq.data() + bt->q.off[(size_t)run.qi],
                           bt->q.len[(size_t)run.qi], run);
  if (fclose(f) != 0 && rc == 0) rc = PW_E_IO;
  return rc;
}

extern "C" uint32_t pw_batch_genomes(pw_batch* bt, uint64_t* names_bytes) {
  if (!bt) return 0;
  if (!bt->g_ready) {
    const Batch& b = bt->b;
    std::unordered_map<std::string_view, uint32_t> m;
    bt->gid.resize(b.recs.size());
    bt->taln.resize(b.recs.size());
    for (size_t i = 0; i < b.recs.size(); i++) {
      const RecHost& r = b.recs[i];
      const std::string_view nm(b.buf.data() + r.line_off + r.tname_off, r.tname_len);
      auto it = m.find(nm);
      uint32_t g;
      if (it == m.end()) {
        g = (uint32_t)m.size();
        m.emplace(nm, g);
        bt->gnames.append(nm.data(), nm.size());
        bt->gnames.push_back('\0');
      } else {
        g = it->second;
      }
      bt->gid[i] = g;
      bt->taln[i] = r.t_aln;
    }
    bt->ngen = (uint32_t)m.size();
    bt->g_ready = true;
  }
  if (names_bytes) *names_bytes = bt->gnames.size();
  return bt->ngen;
}

extern "C" int pw_batch_genomes_get(const pw_batch* bt, uint32_t* genome_of, int32_t* t_aln, char* names) {
  if (!bt || !bt->g_ready) return PW_E_ARG;
  if (genome_of && !bt->gid.empty()) memcpy(genome_of, bt->gid.data(), bt->gid.size() * 4);
  if (t_aln && !bt->taln.empty()) memcpy(t_aln, bt->taln.data(), bt->taln.size() * 4);
  if (names && !bt->gnames.empty()) memcpy(names, bt->gnames.data(), bt->gnames.size());
  return PW_OK;
}

// k-way merge of PWI1 item streams (each sorted by global input line) up to the first item
// with a status >= 0.
extern "C" int pw_items_merge(const char* const* paths, uint32_t n, const char* out_path, const char* err_path) {
  struct Src {
    FILE* f = nullptr;
    bool ok = false;
    uint64_t line = 0;
    int32_t st = -1;
    uint32_t no = 0, ne = 0;
    bool next() {
      unsigned char h[20];
      ok = fread(h, 1, 20, f) == 20;
      if (ok) {
        memcpy(&line, h, 8);
        memcpy(&st, h + 8, 4);
        memcpy(&no, h + 12, 4);
        memcpy(&ne, h + 16, 4);
      }
      return ok;
    }
  };
  std::vector<Src> src(n);
  int ret = 0;
  FILE* out = out_path ? fopen(out_path, "wb") : stdout;
  FILE* err = err_path ? fopen(err_path, "wb") : stderr;
  if (!out || !err) ret = PW_E_IO;
  for (uint32_t i = 0; i < n && ret == 0; i++) {
    src[i].f = fopen(paths[i], "rb");
    char mg[4];
    if (!src[i].f || fread(mg, 1, 4, src[i].f) != 4 || memcmp(mg, "PWI1", 4) != 0) ret = PW_E_IO;
    else src[i].next();
  }
  std::vector<char> buf(1 << 20);
  auto copy = [&](FILE* from, FILE* to, uint64_t bytes) {
    while (bytes > 0) {
      const size_t k = (size_t)std::min<uint64_t>(bytes, buf.size());
      if (fread(buf.data(), 1, k, from) != k) return false;
      fwrite(buf.data(), 1, k, to);
      bytes -= k;
    }
    return true;
  };
  while (ret == 0) {
    int best = -1;
    for (uint32_t i = 0; i < n; i++)
      if (src[i].ok && (best < 0 || src[i].line < src[(size_t)best].line)) best = (int)i;
    if (best < 0) break;
    Src& s = src[(size_t)best];
    if (!copy(s.f, out, s.no)) {
      ret = PW_E_IO;
      break;
    }
    fflush(out);
    if (!copy(s.f, err, s.ne)) {
      ret = PW_E_IO;
      break;
    }
    if (s.st >= 0) {
      ret = s.st;
      break;
    }
    s.next();
  }
  for (auto& s : src)
    if (s.f) fclose(s.f);
  if (out && out != stdout) fclose(out);
  else if (out) fflush(out);
  if (err && err != stderr) fclose(err);
  return ret;
}

// ----------------------------------------------------------------- multi-GPU host path
// Byte-range split of the PAF: the lines that START in [lo, hi) (a line starts at byte 0 or after a
// '\n'), cut into lines as ChunkReader does, each routed to the rank that owns its target genome
// (the classify() shard rule: crc32 of column 6 mod nshards; fewer than six tabs -> 0; comment
// lines -> nobody, though they are counted: every line keeps its index in the range).
struct pw_split {
  uint64_t n_lines = 0;
  uint32_t nshards = 1;
  std::vector<char> data;  // the range's bytes
  // per host thread (a sub-range cut after a '\n'): its lines (start, length, owner; owner
  // nshards = a comment line, nobody's) and per owner its bytes / lines
  struct Part {
    std::vector<uint64_t> start;
    std::vector<uint32_t> len;
    std::vector<uint32_t> owner;
    std::vector<uint64_t> nbytes, nlines;
    uint64_t first = 0;  // index in the range of its first line
  };
  std::vector<Part> parts;
};

// Two passes: pw_paf_split reads the range (host threads) and finds every line and its owner;
// pw_split_get copies one owner's lines straight into the caller's buffers (host threads, each at
// its part's offset) — no per-owner strings and no merge pass.
extern "C" pw_split* pw_paf_split(const char* paf, uint64_t lo, uint64_t hi, uint32_t nshards, char* errbuf,
                                  size_t errlen) {
  auto fail = [&](const std::string& m) -> pw_split* {
    if (errbuf && errlen) snprintf(errbuf, errlen, "%s", m.c_str());
    return nullptr;
  };
  if (!paf || nshards == 0 || hi < lo) return fail("bad arguments");
  const int fd = open(paf, O_RDONLY);
  if (fd < 0) return fail(strf("cannot open %s", paf));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail(strf("cannot stat %s", paf));
  }
  const uint64_t size = (uint64_t)st.st_size;
  if (hi > size) hi = size;
  if (lo > hi) lo = hi;
  // [start, end): from the first line start >= lo to the first line start >= hi
  auto line_start_at = [&](uint64_t x) -> uint64_t {
    if (x == 0) return 0;
    if (x >= size) return size;
    char buf[1 << 16];
    uint64_t p = x - 1;  // a line starts at x iff byte x-1 is '\n'
    while (p < size) {
      const ssize_t k = pread(fd, buf, sizeof buf, (off_t)p);
      if (k <= 0) return size;
      const char* q = (const char*)memchr(buf, '\n', (size_t)k);
      if (q) return p + (uint64_t)(q - buf) + 1;
      p += (uint64_t)k;
    }
    return size;
  };
  const uint64_t start = line_start_at(lo), end = line_start_at(hi);
  pw_split* sp = new pw_split();
  sp->nshards = nshards;
  const size_t n = (size_t)(end - start);
  sp->data.resize(n + 1);
  const int nt = std::max(1, std::min<int>(host_threads(), (int)(n >> 20) + 1));
  {  // the range, read by the host threads in slices
    std::atomic<bool> bad{false};
    parallel_for(nt, [&](int t) {
      const size_t a = n * (size_t)t / (size_t)nt, z = n * (size_t)(t + 1) / (size_t)nt;
      for (size_t got = a; got < z;) {
        const ssize_t k = pread(fd, sp->data.data() + got, z - got, (off_t)(start + got));
        if (k <= 0) {
          bad = true;
          return;
        }
        got += (size_t)k;
      }
    });
    close(fd);
    if (bad) {
      delete sp;
      return fail(strf("cannot read %s", paf));
    }
  }
  // threads take sub-ranges cut after a '\n' (line splitting is local to such a cut)
  std::vector<size_t> cut((size_t)nt + 1, n);
  cut[0] = 0;
  const char* s = sp->data.data();
  for (int t = 1; t < nt; t++) {
    size_t x = n * (size_t)t / (size_t)nt;
    if (x < cut[(size_t)t - 1]) x = cut[(size_t)t - 1];
    const char* q = x < n ? (const char*)memchr(s + x, '\n', n - x) : nullptr;
    cut[(size_t)t] = q ? (size_t)(q - s) + 1 : n;
  }
  sp->parts.resize((size_t)nt);
  parallel_for(nt, [&](int t) {
    pw_split::Part& pt = sp->parts[(size_t)t];
    pt.nbytes.assign(nshards, 0);
    pt.nlines.assign(nshards, 0);
    const size_t a = cut[(size_t)t], b = cut[(size_t)t + 1];
    const bool has_cr = memchr(s + a, '\r', b - a) != nullptr;
    size_t p = a;
    while (p < b) {
      size_t e;
      if (!has_cr) {
        const char* q = (const char*)memchr(s + p, '\n', b - p);
        e = q ? (size_t)(q - s) : b;
      } else {
        e = p;
        while (e < b && s[e] != '\n' && s[e] != '\r') e++;
      }
      if (e == b && e == p) break;
      const char* l = s + p;
      const size_t ln = e - p;
      uint32_t owner = 0;
      if (ln > 0 && l[0] == '#') {
        owner = nshards;  // (a comment line: counted, nobody's)
      } else if (nshards > 1) {
        const char* t5 = nullptr;
        size_t t5n = 0;
        int tabs = 0;
        for (size_t k = 0; k < ln; k++)
          if (l[k] == '\t') {
            tabs++;
            if (tabs == 5) t5 = l + k + 1;
            if (tabs == 6) {
              t5n = (size_t)(l + k - t5);
              break;
            }
          }
        owner = tabs >= 6 ? crc32_ieee(t5, t5n) % nshards : 0u;
      }
      pt.start.push_back(p);
      pt.len.push_back((uint32_t)ln);
      pt.owner.push_back(owner);
      if (owner < nshards) {
        pt.nbytes[owner] += ln + 1;
        pt.nlines[owner]++;
      }
      size_t nx = e + 1;
      if (e < b && s[e] == '\r' && e + 1 < b && s[e + 1] == '\n') nx = e + 2;
      p = nx;
    }
  });
  uint64_t base = 0;
  for (auto& pt : sp->parts) {
    pt.first = base;
    base += pt.start.size();
  }
  sp->n_lines = base;
  return sp;
}
extern "C" uint64_t pw_split_lines(const pw_split* sp) { return sp ? sp->n_lines : 0; }
extern "C" uint64_t pw_split_bytes(const pw_split* sp, uint32_t owner) {
  uint64_t v = 0;
  if (sp && owner < sp->nshards)
    for (const auto& pt : sp->parts) v += pt.nbytes[owner];
  return v;
}
extern "C" uint64_t pw_split_count(const pw_split* sp, uint32_t owner) {
  uint64_t v = 0;
  if (sp && owner < sp->nshards)
    for (const auto& pt : sp->parts) v += pt.nlines[owner];
  return v;
}
extern "C" int pw_split_get(const pw_split* sp, uint32_t owner, char* bytes, uint32_t* local_lines) {
  if (!sp || owner >= sp->nshards) return PW_E_ARG;
  const size_t np = sp->parts.size();
  std::vector<uint64_t> bo(np + 1, 0), lo(np + 1, 0);  // each part's offsets in the outputs
  for (size_t t = 0; t < np; t++) {
    bo[t + 1] = bo[t] + sp->parts[t].nbytes[owner];
    lo[t + 1] = lo[t] + sp->parts[t].nlines[owner];
  }
  parallel_for((int)np, [&](int t) {
    const pw_split::Part& pt = sp->parts[(size_t)t];
    uint64_t b = bo[(size_t)t], k = lo[(size_t)t];
    for (size_t i = 0; i < pt.start.size(); i++) {
      if (pt.owner[i] != owner) continue;
      if (bytes) {
        memcpy(bytes + b, sp->data.data() + pt.start[i], pt.len[i]);
        bytes[b + pt.len[i]] = '\n';
      }
      b += (uint64_t)pt.len[i] + 1;
      if (local_lines) local_lines[k] = (uint32_t)(pt.first + i);
      k++;
    }
  });
  return PW_OK;
}
extern "C" void pw_split_free(pw_split* sp) { delete sp; }

// A batch from lines already in memory (the lines a rank received in the exchange): text holds
// n_lines lines, each ended by '\n', with their global input lines in line_no (ascending).
extern "C" pw_batch* pw_batch_from_buffer(const char* fasta, const char* text, uint64_t len, const uint64_t* line_no,
                                          uint64_t n_lines, uint32_t flags, pw_batch* prev, char* errbuf,
                                          size_t errlen) {
  auto fail = [&](const std::string& m) -> pw_batch* {
    if (errbuf && errlen) snprintf(errbuf, errlen, "%s", m.c_str());
    return nullptr;
  };
  if (!fasta || (len && !text) || (n_lines && !line_no)) return fail("bad arguments");
  const double t0 = now_s();
  pw_batch* bt = new pw_batch();
  std::string err;
  if (!bt->q.load(fasta, err)) {
    delete bt;
    return fail(err);
  }
  const double t1 = now_s();
  struct stat st;
  const long long fsize = (stat(fasta, &st) == 0) ? (long long)st.st_size : -1;
  bool gene = flags & 1u, full = flags & 2u, fc = flags & 4u, fn = flags & 8u;
  if (!full && !gene && fsize > 120000) full = true;
  bool skip = full || fn;
  if (!skip && !fc && fsize > 120000) skip = true;
  bt->skip_codan = skip;
  bt->pk.qdb = &bt->q;
  bt->pk.nt = host_threads();
  bt->pk.opt.fullgenome = full;
  bt->pk.opt.skip_codan = skip;
  bt->pk.opt.single_query_gene = (bt->q.ids.size() == 1 && !full);
  bt->pk.opt.msa = false;
  // PW_BATCH_GPU_PACK: the cs strings stay text for pw_runner_run to pack on the GPU (the CLI's
  // default; PW_PACK_HOST=1 keeps the host packer)
  bt->pk.opt.gpu_pack = (flags & PW_BATCH_GPU_PACK) && !(getenv("PW_PACK_HOST") && atoi(getenv("PW_PACK_HOST")) != 0);
  if (prev) {  // the next batch of the same input: the q~t pairs seen so far move over
    bt->pk.alnpairs = std::move(prev->pk.alnpairs);
    bt->pk.n_lines = prev->pk.n_lines;
  }
  Batch& b = bt->b;
  b.buf.resize((size_t)len + 1);
  b.buf[(size_t)len] = '\0';
  {  // copy + line split by host threads over byte ranges that start at line starts
    char* s = b.buf.data();
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)host_threads(), len >> 22));
    std::vector<uint64_t> cut((size_t)T + 1, len);
    cut[0] = 0;
    for (int t = 1; t < T; t++) {
      uint64_t c = std::max(cut[t - 1], len * (uint64_t)t / (uint64_t)T);
      if (c > 0 && c < len) {  // the line start at or after c
        const char* q = (const char*)memchr(text + c - 1, '\n', (size_t)(len - c + 1));
        c = q ? (uint64_t)(q - text) + 1 : len;
      }
      cut[t] = c;
    }
    std::vector<std::vector<LineRef>> part((size_t)T);
    auto work = [&](int t) {
      const uint64_t a = cut[t], z = cut[t + 1];
      if (z <= a) return;
      memcpy(s + a, text + a, (size_t)(z - a));
      auto& ls = part[t];
      ls.reserve((size_t)((z - a) / 256 + 16));
      for (uint64_t p = a; p < z;) {
        const char* q = (const char*)memchr(s + p, '\n', (size_t)(z - p));
        const uint64_t e = q ? (uint64_t)(q - s) : z;
        ls.push_back({p, (uint32_t)(e - p)});
        s[e] = '\0';  // (e == len: the terminator already there)
        p = e + 1;
      }
    };
    if (T <= 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++) th.emplace_back(work, t);
      for (auto& x : th) x.join();
    }
    size_t nl = 0;
    for (auto& v : part) nl += v.size();
    b.lines.reserve(nl);
    for (auto& v : part) b.lines.append(v.data(), v.size());
  }
  if (b.lines.size() != n_lines) {
    delete bt;
    return fail(strf("line count mismatch (%zu vs %llu)", b.lines.size(), (unsigned long long)n_lines));
  }
  b.line_no.resize((size_t)n_lines);
  if (n_lines) memcpy(b.line_no.data(), line_no, (size_t)n_lines * 8);
  const double t2 = now_s();
  if (n_lines) bt->pk.pack(b);
  const double t3 = now_s();
  bt->alg_in = alg_bytes(b, bt->q, skip);
  if (host_prof())
    fprintf(stderr, "[from_buffer] %llu lines: queries %.3f s, copy + split %.3f s, pack %.3f s, alg bytes %.3f s\n",
            (unsigned long long)n_lines, t1 - t0, t2 - t1, t3 - t2, now_s() - t3);
  return bt;
}

// Output items of a finished batch (the log items up to and including the first one that ends the
// run, as pw_batch_write_items): their global line, status (-1 = continue, else the exit code) and
// the bytes each writes to stdout / stderr.
extern "C" uint64_t pw_batch_item_count(const pw_batch* bt) { return bt ? bt->b.log.size() : 0; }

namespace {
constexpr char kSoftclipMsg[] = "Warning: soft clipping shouldn't be found in this application!\n";
// A record item that prints its header, all its lines and nothing on stderr but soft-clip warnings
// (every item of a clean batch): its bytes are known without formatting it.  Anything else
// (messages, errors, partial records) goes through emit_item.
bool item_plain(const Batch& b, const LogItem& it, const pw_aln_result* res) {
  if (it.kind != 1) return false;
  const RecHost& rh = b.recs[it.idx];
  const pw_aln_result& r = res[it.idx];
  return rh.pre_msg < 0 && r.err == PW_REC_OK && rh.cs_msg < 0 && rh.post_msg < 0 && rh.w_msg < 0 &&
         !(rh.qlen < 9 && r.n_events > 0);
}
// the event-line bytes write_lines prints for all of a record's lines (page spans in chunk order)
template <class F>
void for_spans(const pw_aln_result& r, const pw_page* pages, F&& f) {
  if (r.n_events == 0) return;
  for (uint32_t c = r.page_first;; c++) {
    const uint64_t lo = c == r.page_first ? r.text_off : pages[c].off;
    const uint64_t hi = c == r.page_last ? r.text_end : pages[c].off + pages[c].len;
    if (hi > lo) f(lo, hi - lo);
    if (c == r.page_last) break;
  }
}
void plain_sizes(const Batch& b, const LogItem& it, const pw_aln_result* res, const pw_page* pages, uint64_t& out,
                 uint64_t& err) {
  const RecHost& rh = b.recs[it.idx];
  out = rh.hdr_len;
  for_spans(res[it.idx], pages, [&](uint64_t, uint64_t n) { out += n; });
  err = rh.n_softclip ? (uint64_t)rh.n_softclip * (sizeof(kSoftclipMsg) - 1 + strlen(b.buf.data() + rh.line_off) + 1) : 0;
}
// any item through emit_item into counting / memory streams (the rare items that are not plain)
int item_slow(const Batch& b, const LogItem& it, const uint8_t* text_host, const pw_aln_result* res, const pw_page* pages,
              std::string* out, std::string* err, uint64_t* out_n, uint64_t* err_n) {
  TextSrc src;
  src.host = text_host;
  char *ob = nullptr, *eb = nullptr;
  size_t on = 0, en = 0;
  FILE* o = open_memstream(&ob, &on);
  FILE* e = open_memstream(&eb, &en);
  if (!o || !e) {
    if (o) fclose(o);
    if (e) fclose(e);
    free(ob);
    free(eb);
    return INT_MIN;
  }
  const int st = emit_item(b, it, src, res, pages, o, e);
  fclose(o);
  fclose(e);
  if (out) out->assign(ob, on);
  if (err) err->assign(eb, en);
  if (out_n) *out_n = on;
  if (err_n) *err_n = en;
  free(ob);
  free(eb);
  return st;
}
}  // namespace

extern "C" int pw_batch_items(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                              const pw_page* pages_host, uint64_t* line, int32_t* status, uint64_t* out_len,
                              uint64_t* err_len, uint64_t* n_items) {
  if (!bt || !n_items) return PW_E_ARG;
  uint64_t k = 0;
  for (const LogItem& it : bt->b.log) {
    int32_t st = -1;
    uint64_t on = 0, en = 0;
    if (item_plain(bt->b, it, res_host)) {
      plain_sizes(bt->b, it, res_host, pages_host, on, en);
    } else {
      st = item_slow(bt->b, it, text_host, res_host, pages_host, nullptr, nullptr, &on, &en);
      if (st == INT_MIN) return PW_E_NOMEM;
    }
    if (line) line[k] = it.line;
    if (status) status[k] = st;
    if (out_len) out_len[k] = on;
    if (err_len) err_len[k] = en;
    k++;
    if (st >= 0) break;
  }
  *n_items = k;
  return PW_OK;
}

namespace {

// Plain flags and the back-to-back stdout / stderr offsets (ooff / eoff: n + 1 entries) of the items
// [first, first + n) of a finished batch: one sequential pass (about 12 ns an item).
int plan_items(const Batch& b, uint64_t first, uint64_t n, const uint8_t* text, const pw_aln_result* res,
               const pw_page* pages, std::vector<uint8_t>& plain, std::vector<uint64_t>& ooff,
               std::vector<uint64_t>& eoff) {
  plain.assign((size_t)n, 0);
  ooff.assign((size_t)n + 1, 0);
  eoff.assign((size_t)n + 1, 0);
  for (uint64_t j = 0; j < n; j++) {
    const LogItem& it = b.log[(size_t)(first + j)];
    uint64_t on = 0, en = 0;
    plain[j] = item_plain(b, it, res) ? 1 : 0;
    if (plain[j]) plain_sizes(b, it, res, pages, on, en);
    else if (item_slow(b, it, text, res, pages, nullptr, nullptr, &on, &en) == INT_MIN)
      return PW_E_NOMEM;
    ooff[j + 1] = ooff[j] + on;
    eoff[j + 1] = eoff[j] + en;
  }
  return PW_OK;
}

// Item j's stdout bytes at o and its stderr bytes at e (null: dropped).
int render_item(const Batch& b, const LogItem& it, bool plain, const uint8_t* text, const pw_aln_result* res,
                const pw_page* pages, uint8_t* o, char* e, std::string& so, std::string& se) {
  if (plain) {
    const RecHost& rh = b.recs[it.idx];
    memcpy(o, b.hdr.data() + rh.hdr_off, rh.hdr_len);
    o += rh.hdr_len;
    for_spans(res[it.idx], pages, [&](uint64_t lo, uint64_t n) {
      memcpy(o, text + lo, n);
      o += n;
    });
    if (rh.n_softclip && e) {
      const char* ln = b.buf.data() + rh.line_off;
      const size_t ll = strlen(ln);
      for (int q = 0; q < rh.n_softclip; q++) {
        memcpy(e, kSoftclipMsg, sizeof(kSoftclipMsg) - 1);
        e += sizeof(kSoftclipMsg) - 1;
        memcpy(e, ln, ll);
        e += ll;
        *e++ = '\n';
      }
    }
    return PW_OK;
  }
  if (item_slow(b, it, text, res, pages, &so, &se, nullptr, nullptr) == INT_MIN) return PW_E_NOMEM;
  memcpy(o, so.data(), so.size());
  if (e && !se.empty()) memcpy(e, se.data(), se.size());
  return PW_OK;
}

// The items [j0, j1) of a plan rendered back to back: item j's stdout bytes at out + ooff[j] - ooff[j0],
// its stderr bytes at err + eoff[j] - eoff[j0] (null: dropped); host threads over item ranges of
// about equal bytes.
int render_items(const Batch& b, uint64_t first, const std::vector<uint8_t>& plain, const std::vector<uint64_t>& ooff,
                 const std::vector<uint64_t>& eoff, uint64_t j0, uint64_t j1, const uint8_t* text,
                 const pw_aln_result* res, const pw_page* pages, uint8_t* out, char* err) {
  std::atomic<int> rc{PW_OK};
  auto work = [&](uint64_t a, uint64_t z) {
    std::string so, se;
    for (uint64_t j = a; j < z; j++) {
      const int r = render_item(b, b.log[(size_t)(first + j)], plain[j] != 0, text, res, pages,
                                out + (ooff[j] - ooff[j0]), err ? err + (eoff[j] - eoff[j0]) : nullptr, so, se);
      if (r != PW_OK) {
        rc = r;
        return;
      }
    }
  };
  const uint64_t n = j1 - j0, bytes = ooff[j1] - ooff[j0];
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)host_threads(), n / 64, bytes >> 18}));
  if (T <= 1) {
    work(j0, j1);
  } else {  // cuts at equal byte shares
    std::vector<uint64_t> cut((size_t)T + 1, j1);
    cut[0] = j0;
    for (int t = 1; t < T; t++)
      cut[t] = (uint64_t)(std::lower_bound(ooff.begin() + (ptrdiff_t)j0, ooff.begin() + (ptrdiff_t)j1,
                                           ooff[j0] + bytes * (uint64_t)t / (uint64_t)T) - ooff.begin());
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      if (cut[t + 1] > cut[t]) th.emplace_back(work, cut[t], cut[t + 1]);
    for (auto& x : th) x.join();
  }
  return rc.load();
}

// A file range assembled in images (64 MB) and written with one pwrite per image from a
// writer thread while host threads fill the next image: writers of one file serialise on its inode
// lock, so one large pwrite reaches the file system's rate and many concurrent smaller ones do not
// (the CLI's emit path does the same).  The two images are kept per calling thread
// across calls (no page faults on every window).
struct ImageWriter {
  static uint64_t img_bytes() {  // 64 MB (PW_EMIT_IMG_BYTES: tests)
    const char* e = getenv("PW_EMIT_IMG_BYTES");
    return e ? std::max<uint64_t>(1, strtoull(e, nullptr, 10)) : (64ull << 20);
  }
  int fd;
  int ik = 0;
  std::thread wr;
  std::atomic<int> rc{PW_OK};
  double waited = 0;  // seconds spent waiting for the writer thread
  explicit ImageWriter(int f) : fd(f) {}
  ~ImageWriter() { join(); }
  void join() {
    if (wr.joinable()) {
      const double t = now_s();
      wr.join();
      waited += now_s() - t;
    }
  }
  uint8_t* next(uint64_t n) {  // the image to fill (n bytes)
    static thread_local std::unique_ptr<uint8_t[]> pool[2];
    static thread_local uint64_t pcap[2] = {0, 0};
    if (pcap[ik] < n) {
      pool[ik].reset();
      pcap[ik] = 0;
      pool[ik].reset(new (std::nothrow) uint8_t[n]);
      if (!pool[ik]) return nullptr;
      pcap[ik] = n;
    }
    return pool[ik].get();
  }
  void submit(const uint8_t* p, uint64_t n, uint64_t off) {  // write the filled image at off
    join();
    if (rc.load() != PW_OK) return;
    wr = std::thread([this, p, n, off]() {
      for (uint64_t done = 0; done < n;) {
        const ssize_t w = pwrite(fd, p + done, (size_t)(n - done), (off_t)(off + done));
        if (w <= 0) {
          rc = PW_E_IO;
          return;
        }
        done += (uint64_t)w;
      }
    });
    ik ^= 1;
  }
  int finish() {
    join();
    return rc.load();
  }
};

}  // namespace

// Write the stdout bytes of the batch's items [first, first + n_items) at out_off[k - first] of fd
// (pwrite: ranks write disjoint ranges of one file) and their stderr bytes back to back into
// err_buf.  Runs of items whose destinations follow each other (a rank's whole window with one
// rank) go out as 64 MB images through ImageWriter; scattered destinations (ranks' lines
// interleaved, PW_MGPU_WRITE=pwrite) are assembled per host thread into buffers of up to 8 MB, one
// pwrite each (a per-item pwrite was the multi-GPU driver's largest host cost: 5.2 s for 3 M records).
extern "C" int pw_batch_write_range(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                                    const pw_page* pages_host, int fd, uint64_t first, const uint64_t* out_off,
                                    uint64_t n_items, char* err_buf, uint64_t err_cap) {
  if (!bt || (n_items && !out_off) || first > bt->b.log.size() || n_items > bt->b.log.size() - first)
    return PW_E_ARG;
  const Batch& b = bt->b;
  const double t0 = now_s();
  std::vector<uint8_t> plain;
  std::vector<uint64_t> ooff, eoff;
  if (int r = plan_items(b, first, n_items, text_host, res_host, pages_host, plain, ooff, eoff)) return r;
  if (err_buf && eoff[n_items] > err_cap) return PW_E_ARG;
  const double t1 = now_s();
  // runs of items whose destinations follow each other, cut at the image size
  struct Seg {
    uint64_t j0, j1, d0, n;
  };
  std::vector<Seg> segs;
  const uint64_t kImg = ImageWriter::img_bytes();
  uint64_t runs = 0;  // contiguity breaks + 1
  for (uint64_t j = 0; j < n_items; j++) {
    const uint64_t on = ooff[j + 1] - ooff[j];
    const bool brk = segs.empty() || out_off[j] != segs.back().d0 + segs.back().n;
    runs += brk;
    if (brk || (segs.back().n && segs.back().n + on > kImg)) segs.push_back({j, j, out_off[j], 0});
    segs.back().j1 = j + 1;
    segs.back().n += on;
  }
  if (runs && runs * 64 <= n_items) {  // long runs (one rank's window): images
    ImageWriter iw(fd);
    double fill = 0;
    int r = PW_OK;
    for (const Seg& sg : segs) {
      uint8_t* img = iw.next(sg.n);
      if (!img) {
        r = PW_E_NOMEM;
        break;
      }
      const double f0 = now_s();
      r = render_items(b, first, plain, ooff, eoff, sg.j0, sg.j1, text_host, res_host, pages_host, img,
                       err_buf ? err_buf + eoff[sg.j0] : nullptr);
      fill += now_s() - f0;
      if (r != PW_OK) break;
      iw.submit(img, sg.n, sg.d0);
    }
    const int w = iw.finish();
    if (host_prof())
      fprintf(stderr, "[host write_range] %llu items, %.1f MB in %zu images: plan %.3f s, fill %.3f s, writer wait %.3f s, total %.3f s\n",
              (unsigned long long)n_items, ooff[n_items] / 1e6, segs.size(), t1 - t0, fill, iw.waited, now_s() - t0);
    return r != PW_OK ? r : w;
  }
  constexpr uint64_t kBuf = 8ull << 20;
  std::atomic<int> rc{PW_OK};
  auto work = [&](uint64_t j0, uint64_t j1) {
    std::vector<uint8_t> buf;
    buf.reserve(1u << 20);
    uint64_t d0 = 0;  // destination of buf[0]
    auto flush = [&]() {
      for (uint64_t done = 0; done < buf.size();) {
        const ssize_t w = pwrite(fd, buf.data() + done, buf.size() - done, (off_t)(d0 + done));
        if (w <= 0) {
          rc = PW_E_IO;
          break;
        }
        done += (uint64_t)w;
      }
      buf.clear();
    };
    std::string so, se;
    for (uint64_t j = j0; j < j1 && rc.load() == PW_OK; j++) {
      const uint64_t on = ooff[j + 1] - ooff[j];
      if (!buf.empty() && (out_off[j] != d0 + buf.size() || buf.size() >= kBuf)) flush();
      if (buf.empty()) d0 = out_off[j];
      const size_t at = buf.size();
      buf.resize(at + on);
      const int r = render_item(b, b.log[(size_t)(first + j)], plain[j] != 0, text_host, res_host, pages_host,
                                buf.data() + at, err_buf ? err_buf + eoff[j] : nullptr, so, se);
      if (r != PW_OK) {
        rc = r;
        break;
      }
    }
    if (!buf.empty() && rc.load() == PW_OK) flush();
  };
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)host_threads(), n_items / 4096));
  if (T <= 1) {
    work(0, n_items);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back(work, n_items * (uint64_t)t / (uint64_t)T, n_items * (uint64_t)(t + 1) / (uint64_t)T);
    for (auto& x : th) x.join();
  }
  return rc.load();
}

// The stdout bytes of the items [first, first + n_items) back to back into out_buf and their stderr
// bytes into err_buf (the multi-GPU driver's exchange write: a rank renders its items of a window,
// the ranks exchange them so that each holds one contiguous byte range of the file, and each range
// goes out with large pwrites — pw_gather_write).
extern "C" int pw_batch_render_range(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                                     const pw_page* pages_host, uint64_t first, uint64_t n_items, uint8_t* out_buf,
                                     uint64_t out_cap, char* err_buf, uint64_t err_cap) {
  if (!bt || first > bt->b.log.size() || n_items > bt->b.log.size() - first || (n_items && !out_buf && out_cap))
    return PW_E_ARG;
  const Batch& b = bt->b;
  std::vector<uint8_t> plain;
  std::vector<uint64_t> ooff, eoff;
  if (int r = plan_items(b, first, n_items, text_host, res_host, pages_host, plain, ooff, eoff)) return r;
  if (ooff[n_items] > out_cap || (err_buf && eoff[n_items] > err_cap)) return PW_E_ARG;
  return render_items(b, first, plain, ooff, eoff, 0, n_items, text_host, res_host, pages_host, out_buf, err_buf);
}

// Spans src[src_off[k], + len[k]) for k = 0..n-1, in order, written contiguously to fd from
// file_off: host threads assemble 64 MB images of the range, a writer thread pwrites each in one
// call while the next is assembled (ImageWriter).
extern "C" int pw_gather_write(int fd, uint64_t file_off, const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                               uint64_t n) {
  if (n && (!src || !src_off || !len)) return PW_E_ARG;
  std::vector<uint64_t> dst((size_t)n + 1, 0);
  for (uint64_t k = 0; k < n; k++) dst[k + 1] = dst[k] + len[k];
  const uint64_t total = dst[n];
  if (total == 0) return PW_OK;
  ImageWriter iw(fd);
  const uint64_t kImg = ImageWriter::img_bytes();
  const double t0 = now_s();
  for (uint64_t x = 0; x < total;) {  // one image per kImg bytes of the range
    const uint64_t bn = std::min<uint64_t>(kImg, total - x);
    uint8_t* img = iw.next(bn);
    if (!img) {
      iw.finish();
      return PW_E_NOMEM;
    }
    auto fill = [&](uint64_t a, uint64_t z) {  // image bytes [a, z) from the spans
      uint64_t k = (uint64_t)(std::upper_bound(dst.begin(), dst.end(), x + a) - dst.begin()) - 1;
      for (uint64_t f = a; f < z;) {
        while (dst[k + 1] <= x + f) k++;
        const uint64_t in = x + f - dst[k], c = std::min<uint64_t>(len[k] - in, z - f);
        memcpy(img + f, src + src_off[k] + in, (size_t)c);
        f += c;
      }
    };
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)host_threads(), bn >> 20));
    if (T <= 1) {
      fill(0, bn);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++) th.emplace_back(fill, bn * (uint64_t)t / (uint64_t)T, bn * (uint64_t)(t + 1) / (uint64_t)T);
      for (auto& y : th) y.join();
    }
    iw.submit(img, bn, file_off + x);
    x += bn;
  }
  const int r = iw.finish();
  if (host_prof())
    fprintf(stderr, "[host gather_write] %.1f MB: writer wait %.3f s, total %.3f s\n", total / 1e6, iw.waited, now_s() - t0);
  return r;
}

// Cuts of a rank's received lines ('\n'-ended, n bytes) into batches of at most `target` bytes (at
// least one line) ending at line ends: out[4k .. 4k + 3] = byte lo, hi, line lo, hi of batch k;
// returns the number of batches (cap: the entries out holds; more -> 0).  The lines of each batch
// are counted by host threads (memchr).
extern "C" uint64_t pw_batch_cuts(const uint8_t* text, uint64_t n, uint64_t target, uint64_t* out, uint64_t cap) {
  if (!out || (n && !text)) return 0;
  if (target == 0) target = 1;
  std::vector<uint64_t> b;  // batch ends
  for (uint64_t b0 = 0; b0 < n;) {
    uint64_t b1;
    if (b0 + target > n) {
      b1 = n;
    } else {  // the last '\n' in [b0, b0 + target - 1), else the end of the first line
      const void* q = target > 1 ? memrchr(text + b0, '\n', (size_t)(target - 1)) : nullptr;
      if (q) {
        b1 = (uint64_t)((const uint8_t*)q - text) + 1;
      } else {
        const void* f = memchr(text + b0, '\n', (size_t)(n - b0));
        b1 = f ? (uint64_t)((const uint8_t*)f - text) + 1 : n;
      }
    }
    b.push_back(b1);
    b0 = b1;
  }
  if (b.size() > cap) return 0;
  std::vector<uint64_t> lines(b.size(), 0);
  parallel_for((int)b.size(), [&](int k) {
    const uint64_t lo = k ? b[(size_t)k - 1] : 0, hi = b[(size_t)k];
    uint64_t c = 0;
    for (const uint8_t* p = text + lo; p < text + hi;) {
      const void* f = memchr(p, '\n', (size_t)(text + hi - p));
      if (!f) break;
      c++;
      p = (const uint8_t*)f + 1;
    }
    lines[(size_t)k] = c;
  });
  uint64_t l0 = 0;
  for (size_t k = 0; k < b.size(); k++) {
    out[4 * k] = k ? b[k - 1] : 0;
    out[4 * k + 1] = b[k];
    out[4 * k + 2] = l0;
    l0 += lines[k];
    out[4 * k + 3] = l0;
  }
  return b.size();
}

extern "C" int pw_batch_write_at(const pw_batch* bt, const uint8_t* text_host, const pw_aln_result* res_host,
                                 const pw_page* pages_host, int fd, const uint64_t* out_off, uint64_t n_items,
                                 char* err_buf, uint64_t err_cap) {
  return pw_batch_write_range(bt, text_host, res_host, pages_host, fd, 0, out_off, n_items, err_buf, err_cap);
}

// Batches are freed by a reaper thread: releasing one returns ~1 GB of buffers to the system (about
// 75 ms of unmapping at cfg3's 256 MB batches), which the multi-GPU driver's window loop otherwise
// waited for once per batch.  PW_BATCH_FREE_SYNC=1 frees on the caller.  The reaper is detached: a
// batch still queued at exit is left to process teardown.
namespace {
struct BatchReaper {
  std::mutex m;
  std::condition_variable cv;
  std::vector<pw_batch*> q;
  bool started = false;
  void put(pw_batch* bt) {
    std::unique_lock<std::mutex> lk(m);
    if (!started) {
      started = true;
      std::thread([this]() {
        for (;;) {
          std::vector<pw_batch*> batch;
          {
            std::unique_lock<std::mutex> l2(m);
            cv.wait(l2, [this]() { return !q.empty(); });
            batch.swap(q);
          }
          for (pw_batch* b : batch) delete b;
        }
      }).detach();
    }
    q.push_back(bt);
    cv.notify_one();
  }
};
BatchReaper* reaper() {
  static BatchReaper* r = new BatchReaper;  // (never destroyed: the detached thread may outlive statics)
  return r;
}
}  // namespace

// ----------------------------------------------------------------- batch runner
// The CLI's device state (Device: queries and next-stop table uploaded once, device buffers grown
// and reused across batches, GPU cs packing) behind the C ABI for the multi-GPU driver: a batch
// runs on the runner's stream, its results / pages come back to host vectors here, and the used
// text is copied into the caller's (pinned) buffer by pw_runner_fetch.
struct pw_runner {
  Device dev;
  bool skip_codan = false;
  size_t q_len = 0, q_n = 0;
  std::vector<pw_aln_result> res;
  std::vector<pw_page> pages;
  uint64_t used = 0;
  bool have = false;  // a finished batch whose outputs are here
  DevBuf<uint32_t> gof;
  DevBuf<int32_t> taln;
  DevBuf<pw_genome_row> grows;
};

extern "C" pw_runner* pw_runner_create(const pw_batch* bt, char* errbuf, size_t errlen) {
  if (!bt) {
    if (errbuf && errlen) snprintf(errbuf, errlen, "bad arguments");
    return nullptr;
  }
  pw_runner* r = new pw_runner();
  r->skip_codan = bt->skip_codan;
  r->q_len = bt->q.seq.size();
  r->q_n = bt->q.len.size();
  if (!r->dev.init(bt->q, bt->skip_codan)) {  // (Device::init prints the cause)
    delete r;
    if (errbuf && errlen) snprintf(errbuf, errlen, "device initialisation failed");
    return nullptr;
  }
  return r;
}

extern "C" int pw_runner_run(pw_runner* r, pw_batch* bt, uint64_t* n_pages, uint64_t* text_used) {
  if (!r || !bt || !n_pages || !text_used) return PW_E_ARG;
  // (the runner's query set: the batch must come from the same FASTA and mode)
  if (bt->skip_codan != r->skip_codan || bt->q.seq.size() != r->q_len || bt->q.len.size() != r->q_n) return PW_E_ARG;
  r->have = false;
  if (!r->dev.run(bt->b, bt->q, bt->skip_codan, nullptr, r->res, r->pages)) return PW_E_HIP;
  const uint64_t tcap = pw_report_text_bytes(bt->b.n_events_max, bt->b.text_total);
  uint64_t used = 0;
  if (bt->b.desc.empty()) {  // (no pass ran: the pages Device::run sized are not written)
    for (pw_page& pg : r->pages) pg = pw_page{0, 0, 0};
  } else {
    for (const pw_page& pg : r->pages)
      if (pg.len && pg.off + pg.len > used) used = pg.off + pg.len;
  }
  r->used = used < tcap ? used : tcap;
  r->have = true;
  *n_pages = r->pages.size();
  *text_used = r->used;
  return PW_OK;
}

extern "C" int pw_runner_fetch(pw_runner* r, pw_aln_result* res, uint64_t n_res, pw_page* pages, uint64_t n_pages,
                               uint8_t* text, uint64_t text_cap) {
  if (!r || !r->have || n_res != r->res.size() || n_pages != r->pages.size() || text_cap < r->used ||
      (n_res && !res) || (n_pages && !pages) || (r->used && !text))
    return PW_E_ARG;
  if (n_res) memcpy(res, r->res.data(), n_res * sizeof(pw_aln_result));
  if (n_pages) memcpy(pages, r->pages.data(), n_pages * sizeof(pw_page));
  // (on the runner's stream; every path reaches ~57 GB/s alone on the box: tools/d2h_probe.py)
  if (r->used && (hipMemcpyAsync(text, r->dev.text.p, r->used, hipMemcpyDeviceToHost, r->dev.stream) != hipSuccess ||
                  hipStreamSynchronize(r->dev.stream) != hipSuccess))
    return PW_E_HIP;
  return PW_OK;
}

extern "C" int pw_runner_genome_rows(pw_runner* r, const uint32_t* genome_of, const int32_t* t_aln, uint32_t n_alns,
                                     uint32_t n_genomes, pw_genome_row* rows) {
  if (!r || !r->have || n_alns != r->res.size() || (n_alns && (!genome_of || !t_aln)) || (n_genomes && !rows))
    return PW_E_ARG;
  if (n_genomes == 0) return PW_OK;
  hipStream_t st = r->dev.stream;
  if (!r->gof.ensure(n_alns + 1) || !r->taln.ensure(n_alns + 1) || !r->grows.ensure(n_genomes)) return PW_E_NOMEM;
  if (n_alns && (hipMemcpyAsync(r->gof.p, genome_of, (size_t)n_alns * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
                 hipMemcpyAsync(r->taln.p, t_aln, (size_t)n_alns * 4, hipMemcpyHostToDevice, st) != hipSuccess))
    return PW_E_HIP;
  const int rc = pw_genome_table(r->dev.res.p, r->gof.p, r->taln.p, n_alns, r->grows.p, n_genomes, st);
  if (rc != PW_OK) return rc;
  if (hipMemcpyAsync(rows, r->grows.p, (size_t)n_genomes * sizeof(pw_genome_row), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return PW_E_HIP;
  return PW_OK;
}

extern "C" void pw_runner_free(pw_runner* r) { delete r; }

extern "C" void pw_batch_free(pw_batch* bt) {
  if (!bt) return;
  static const bool sync = getenv("PW_BATCH_FREE_SYNC") && atoi(getenv("PW_BATCH_FREE_SYNC")) != 0;
  if (sync) delete bt;
  else reaper()->put(bt);
}

extern "C" const char* pw_version(void) { return "pwasm_amd 0.1 (gfx950)"; }
