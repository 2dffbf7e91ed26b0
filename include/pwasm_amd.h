/*
 * pwasm_amd.h — C-ABI of the MI355X-native pafreport hot path (libpwasm_amd.so).
 *
 * The reference (gpertea/pwasm) has no FFI: its hot path is a set of C++ member functions
 * called from pafreport's per-record loop.  Each entry point below replaces one of them;
 * INTEGRATION.md shows the binding a maintainer would add to pafreport.cpp / GapAssem.cpp.
 *
 * Conventions: plain pointers + sizes, no torch or HIP C++ types in signatures (a stream is a
 * `void*` holding a hipStream_t; NULL = the default stream); device buffers are caller-owned;
 * every function returns 0 on success or a negative PW_E* status; launches are asynchronous
 * on the given stream and never allocate or synchronise (graph-capture safe).
 */
#ifndef PWASM_AMD_H
#define PWASM_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PW_ABI_VERSION 1

/* ---------------------------------------------------------------- status codes */
#define PW_OK 0
#define PW_E_ARG (-1)     /* bad argument / shape */
#define PW_E_HIP (-2)     /* HIP runtime error */
#define PW_E_IO (-3)      /* host I/O */
#define PW_E_NOMEM (-4)   /* host allocation */
#define PW_E_NODEV (-5)   /* no gfx950 device */

/* ---------------------------------------------------------------- packed cs op stream
 * The CPU pre-pass (pw_pack_cs) turns a short-form cs string into 32-bit ops:
 * bits 31..30 = type, bits 29..0 = length.  `:0` ops are dropped (they change nothing,
 * pafreport.cpp:541-546).  Literal bytes go to a side array, upper-cased:
 *   SUB: 2 bytes {target base, query base}   ('*tq', pafreport.cpp:547-578)
 *   INS: len bytes (target-only bases)        ('-acg', pafreport.cpp:579-601 -> event 'I')
 *   DEL: none (bases are taken from the query) ('+acg', pafreport.cpp:602-619 -> event 'D') */
#define PW_OP_MATCH 0u
#define PW_OP_SUB 1u
#define PW_OP_INS 2u
#define PW_OP_DEL 3u
#define PW_OP_TYPE(w) ((uint32_t)(w) >> 30)
#define PW_OP_LEN(w) ((uint32_t)(w)&0x3FFFFFFFu)
#define PW_OP(type, len) (((uint32_t)(type) << 30) | ((uint32_t)(len)&0x3FFFFFFFu))

/* One PAF record (= one PAFAlignment, pafreport.cpp:134-158), 32 bytes, device-resident. */
typedef struct pw_aln_desc {
  uint32_t op_begin;   /* first op in ops[] */
  uint32_t n_ops;      /* ops of this record */
  uint32_t lit_begin;  /* first literal byte in lits[] */
  uint32_t ref;        /* bits 0..29 query index; bit 30 = the query and this record's literal
                          bytes are all A/C/G/T; bit 31 = reverse strand ('-') */
  int32_t offset;      /* start on the aligned-strand query (pafreport.cpp:486-490) */
  int32_t t_len;       /* tseq length implied by the cs string */
  uint64_t ev_begin;   /* first event slot of this record (prefix of pw_cs_totals.n_events_max) */
} pw_aln_desc;
#define PW_REF_REVERSE 0x80000000u
#define PW_REF_ACGT 0x40000000u
#define PW_REF_QMASK 0x3FFFFFFFu

/* Text pages.  The event lines of 64 consecutive event slots (one chunk) form one page, written
 * at text[page.off, page.off + page.len).  A page normally lives at chunk * PW_PAGE_BYTES; a
 * page that does not fit is placed in the arena after the page area.  A record's lines are the
 * bytes from text_off (in page page_first) to text_end (in page page_last), crossing the pages
 * in between in chunk order (pw_batch_write_report stitches them). */
#define PW_PAGE_EVENTS 64
#define PW_PAGE_BYTES 8192
typedef struct pw_page {
  uint64_t off;  /* first byte of the page's lines in text[] */
  uint32_t len;  /* bytes of lines */
  uint32_t pad;
} pw_page;

/* Per-record result written by pw_report_events, 48 bytes. */
typedef struct pw_aln_result {
  uint64_t text_off;   /* first byte of the record's first event line in text[] */
  uint64_t text_end;   /* one past the last byte of its last event line */
  uint32_t page_first; /* pages holding those two lines */
  uint32_t page_last;
  uint32_t text_len;   /* bytes of event lines (header excluded) */
  uint32_t n_events;   /* TDiffInfo records after S-merging */
  int32_t err;         /* PW_REC_* */
  int32_t err_a;       /* MISMATCH: q_pos          MODSEQ: modseq index */
  int32_t err_b;       /* MISMATCH: query char     MODSEQ: evtsub index */
  int32_t err_c;       /* MISMATCH: aligned-strand query char; MODSEQ: output line index */
} pw_aln_result;

#define PW_REC_OK 0
#define PW_REC_MISMATCH 1 /* "Error: base mismatch ..." (pafreport.cpp:551-554) */
#define PW_REC_MODSEQ 2   /* "Error: modseq[%d] not matching ..." (pafreport.cpp:812-813) */
#define PW_REC_OVERFLOW 3 /* event slots or text capacity exceeded (caller sizing bug) */
#define PW_REC_LAYOUT 4   /* descriptor violates the pw_report_args contract (qoff / ev_begin) */

/* Arguments of pw_report_events (all pointers are device pointers).  qseq and lits must stay
 * readable for PW_DEV_PAD bytes past their last element (16-byte LDS staging loads).
 * Contract checked per record on the device (violations -> PW_REC_LAYOUT, no events):
 *   qoff[q] is a multiple of 16 and < 2^36 (64 GiB of concatenated queries);
 *   desc[].ev_begin is non-decreasing: record i owns slots [ev_begin(i), ev_begin(i+1)), the
 *   last record [ev_begin, n_ev_slots) (the prefix sum of pw_cs_totals.n_events_max). */
#define PW_DEV_PAD 256
typedef struct pw_report_args {
  const pw_aln_desc* desc;  /* [n_alns] */
  const uint32_t* ops;      /* packed ops */
  const uint8_t* lits;      /* literal bytes */
  const uint8_t* qseq;      /* forward upper-case query sequences, concatenated */
  const uint64_t* qoff;     /* [n_queries] start of each query in qseq */
  const int32_t* qlen;      /* [n_queries] */
  const int32_t* next_stop; /* [sum qlen] from pw_stop_table_build; may be NULL if skip_codan */
  uint8_t* text;            /* text pages + arena, text_total bytes (pw_report_text_bytes) */
  pw_aln_result* results;   /* [n_alns] */
  uint64_t text_total;      /* capacity of text */
  uint32_t n_alns;
  uint32_t skip_codan;      /* 1 = no codon impact column (pafreport.cpp:259-262, 915) */
  void* workspace;          /* device scratch, 64-byte aligned, >= pw_report_workspace_bytes() */
  uint64_t workspace_bytes;
  uint64_t n_ev_slots;      /* event slots of the batch = sum of pw_cs_totals.n_events_max
                               (< 2^32 - 2^16, else PW_E_ARG: cut larger inputs into batches) */
  pw_page* pages;           /* [pw_report_page_count(n_ev_slots)] */
  uint32_t max_rec_ops;     /* largest desc[].n_ops of the batch, or 0 = unknown.  Records of more
                               than PW_BLOCK_OPS ops are decoded as blocks of PW_BLOCK_OPS ops by
                               several wavefronts (block carries from a pre-pass); a value
                               <= PW_BLOCK_OPS lets the pass skip that pre-pass. */
  uint32_t n_short;         /* records of at most 64 ops, or 0 = unknown: when they are most of the
                               batch, index decoding takes two records per wavefront */
  uint32_t hot_pbits;       /* 0, or P in 1..31 when every query is shorter than 2^P bases and every
                               query index (desc[].ref & PW_REF_QMASK) < 2^(32 - P): the pass then
                               keeps 16 instead of 32 bytes per event between its kernels (an event
                               that violates it ends its record with PW_REC_LAYOUT) */
  uint32_t flags;           /* PW_REPORT_* */
  uint32_t n_queries;       /* queries of qoff / qlen (read with PW_REPORT_BUILD_NEXT_STOP) */
  uint32_t pad;
} pw_report_args;
/* The pass builds next_stop itself (pw_stop_table_build's table for n_queries queries, by workgroups
 * of its first kernel running beside the decode: no second stream, no event); next_stop is then
 * written, and must not be read by other work until the pass completes. */
#define PW_REPORT_BUILD_NEXT_STOP 1u
#define PW_BLOCK_OPS 2048

/* Pages of a batch with n_ev_slots event slots, and the text capacity that always suffices:
 * the page area plus an arena of text_bound bytes (sum of pw_cs_totals.text_bound). */
uint64_t pw_report_page_count(uint64_t n_ev_slots);
uint64_t pw_report_text_bytes(uint64_t n_ev_slots, uint64_t text_bound);

/* pw_report_args.hot_pbits for queries of at most max_qlen bases and n_queries query indices:
 * the smallest P with max_qlen < 2^P, when the query index fits the other 32 - P bits, else 0
 * (32-byte event records). */
uint32_t pw_report_hot_pbits(uint64_t max_qlen, uint64_t n_queries);

/* Device workspace pw_report_events needs for a batch of n_alns records with n_events_max event
 * slots (pw_cs_totals.n_events_max summed over the batch; pw_batch_view.n_events_max). */
uint64_t pw_report_workspace_bytes(uint64_t n_events_max, uint64_t n_alns);

/* ---------------------------------------------------------------- device entry points */

/* Replaces PAFAlignment::PAFAlignment (decode, pafreport.cpp:477-643) +
 * PAFAlignment::printDiffInfo's event loop (classify, codon, format; pafreport.cpp:893-954)
 * for a whole batch of records: a wavefront per record decodes the op stream into event
 * descriptors, then wavefronts of 64 consecutive events render the report lines. */
int pw_report_events(const pw_report_args* args, void* stream);

/* As pw_report_events, but next_stop may still be being built on another stream: the pass waits
 * for the HIP event next_stop_ready (a hipEvent_t recorded after pw_stop_table_build there; NULL =
 * already complete in stream order) only before its first kernel that reads next_stop, so the table
 * build overlaps the decode kernels.  The caller keeps the table alive and unmodified until the pass
 * completes. */
int pw_report_events_after(const pw_report_args* args, void* stream, void* next_stop_ready);

/* Per-query stop-codon lookahead used by the codon pass (replaces the forward scan of
 * predictImpact, pafreport.cpp:854-870): next_stop[off+j] = smallest k >= j, k = j mod 3,
 * k+2 < len, translateCodon(q+k) == '.', else INT32_MAX. */
int pw_stop_table_build(const uint8_t* qseq, const uint64_t* qoff, const int32_t* qlen, uint32_t n_queries,
                        int32_t* next_stop, void* stream);

/* ---------------------------------------------------------------- GapAssem column consensus
 * Packed MSA layout (GASeq rows, GapAssem.h:35-138): row r has its bases in
 * seq[row_off[r] .. +row_len[r]) and the int16 gaps before each base (GASeq::ofs) at the same
 * indices; col0[r] = offset - minoffset (GapAssem.cpp:568); clip_l/clip_r are the clip lengths
 * already oriented by revcompl (GapAssem.cpp:557-564).  Rows are cut into 256-base chunks;
 * pw_msa_slots() assigns each row ceil(len/256)+1 slots (the last one is the row's end).
 * seq / ofs of every row are readable up to the next multiple of 4 elements past its end (the
 * stagers start rows 8-element aligned and zero-pad between them). */
typedef struct pw_msa_args {
  const uint8_t* seq;       /* bases of all rows */
  const int16_t* ofs;       /* gaps before each base */
  const uint64_t* row_off;  /* [n_rows] first base of each row */
  const int32_t* row_len;   /* [n_rows] */
  const int32_t* col0;      /* [n_rows] offset - minoffset */
  const int32_t* clip_l;    /* [n_rows] oriented left clip */
  const int32_t* clip_r;    /* [n_rows] oriented right clip */
  const int64_t* slot_base; /* [n_rows + 1] from pw_msa_slots */
  int32_t* scratch;         /* [pw_msa_scratch_words(n_slots, n_rows)] (chunk sums, checkpoints,
                               slot -> row, per-chunk gap lists, per-row counted extents) */
  int32_t* counts;          /* [n_cols][6] A,C,G,T,N,- (GAlnColumn::counts order) */
  uint8_t* consensus;       /* [n_cols] bestChar() per column ('-' for gap), 0 = no coverage */
  int32_t* minmax;          /* [4]: mincol, maxcol, first out-of-range row, first zero column */
  uint64_t n_slots;
  uint32_t n_rows;
  int32_t n_cols;           /* GSeqAlign::length */
} pw_msa_args;

/* Host helper: fills slot_base[n_rows + 1], returns n_slots. */
uint64_t pw_msa_slots(const int32_t* row_len_host, uint32_t n_rows, int64_t* slot_base_host);
/* int32 words of pw_msa_args.scratch for a layout of n_slots slots and n_rows rows. */
uint64_t pw_msa_scratch_words(uint64_t n_slots, uint32_t n_rows);

/* Replaces GSeqAlign::buildMSA -> GASeq::toMSA -> GAlnColumn::addNuc/addGap and
 * GAlnColumn::bestChar (GapAssem.cpp:551-591, 1048-1069, 1088-1106; GapAssem.h:295-337).
 * minmax: INT_MAX / -1 sentinels when nothing is set.  = pw_msa_count + pw_msa_call. */
int pw_msa_columns(const pw_msa_args* args, void* stream);

/* The two halves of pw_msa_columns, for rows sharded over GPUs: pw_msa_count
 * fills counts[n_cols][6] and minmax[0..2] from this shard's rows (buildMSA's toMSA/addNuc/
 * addGap scatter); after the shards' counts are summed (all-reduce) and minmax[0] / [1]
 * reduced with min / max, pw_msa_call writes bestChar for every column and minmax[3]. */
int pw_msa_count(const pw_msa_args* args, void* stream);
int pw_msa_call(const pw_msa_args* args, void* stream);
/* pw_msa_call over columns [col_lo, col_hi) only (the zero-coverage scan too); counts_lo = the
 * counts of column col_lo onwards ([col_hi - col_lo][6]) or NULL for args->counts. */
int pw_msa_call_cols(const pw_msa_args* args, int32_t col_lo, int32_t col_hi, const int32_t* counts_lo, void* stream);

/* GSeqAlign::refineMSA after buildMSA (GapAssem.cpp:1143-1181): the consensus string over
 * [mincol, maxcol] ('-' -> '*'; with remove_gaps = MSAColumns::removeConsGaps the gap columns
 * are dropped) and, with remove_gaps, every row's removeColumn / removeBase edits and
 * removeClipGaps (GapAssem.cpp:755-779, 122-131, 522-549).  Needs the scratch of the
 * pw_msa_count call that produced args->counts; rows must have ofs >= 0 when remove_gaps. */
typedef struct pw_msa_refine_args {
  int32_t* gap_prefix;        /* [n_cols] scratch: consensus-gap columns in [mincol, c] */
  int32_t* tile_gaps;         /* [pw_msa_refine_tiles(n_cols)] scratch */
  uint8_t* cons_out;          /* [n_cols] the consensus (GSeqAlign::consensus) */
  int32_t* cons_len;          /* [1] its length */
  const int32_t* row_offset;  /* [n_rows] GASeq::offset (remove_gaps) */
  int16_t* ofs_out;           /* [bases] GASeq::ofs after refineMSA, same indexing as ofs */
  int32_t* offset_out;        /* [n_rows] GASeq::offset after refineMSA */
  int64_t* numgaps_out;       /* [n_rows] in: GASeq::numgaps; out: after refineMSA */
  uint32_t remove_gaps;
  uint32_t keep_clip_gaps;    /* 1: stop after the removeColumn edits (offset', ofs', numgaps');
                                 the caller runs refineClipping / removeClipGaps per row on the
                                 host (pw_ga_row_finish) */
} pw_msa_refine_args;
uint64_t pw_msa_refine_tiles(int32_t n_cols);
int pw_msa_refine(const pw_msa_args* args, const pw_msa_refine_args* refine, void* stream);
/* buildMSA + refineMSA of one shard holding every row (GapAssem.cpp:1088-1106, 1143-1181):
 * = pw_msa_columns then pw_msa_refine, the same results; without remove_gaps the consensus string
 * and its length are written by the counting pass itself (gap_prefix / tile_gaps untouched). */
int pw_msa_columns_refine(const pw_msa_args* args, const pw_msa_refine_args* refine, void* stream);

/* ---------------------------------------------------------------- GapAssem over RCCL
 * One process per GPU; the 128-byte id travels over any side channel (torch.distributed in
 * pwasm_amd/gapassem.py).  librccl is loaded on first use.
 * pw_msa_counts_allreduce: after every rank's pw_msa_count on its rows (rows row_base.. of the
 *   layout), sums counts[n_cols][6] and reduces minmax[0] min / [1] max / [2] min (as a global
 *   row index) on all ranks in place — one grouped RCCL call set on `stream`; follow with
 *   pw_msa_call.  The merged histograms are bit-identical to a single-GPU count.
 * pw_msa_counts_reduce_scatter: rank r receives the summed counts of columns
 *   [r * cols_per_rank, (r + 1) * cols_per_rank) in counts_part; counts holds nranks *
 *   cols_per_rank columns (zero past n_cols). */
#define PW_COMM_ID_BYTES 128
int pw_comm_unique_id(uint8_t* id);
int pw_comm_init(void** comm, int nranks, const uint8_t* id, int rank);
int pw_comm_destroy(void* comm);
int pw_msa_counts_allreduce(const pw_msa_args* args, uint32_t row_base, void* comm, void* stream);
int pw_msa_counts_reduce_scatter(const int32_t* counts, int32_t* counts_part, uint64_t cols_per_rank, void* comm,
                                 void* stream);
/* Column-sharded bestChar, after every rank's pw_msa_count on its rows: the
 * histograms reduce-scattered by column range (rank r: columns [r * cols_per_rank, ...) into
 * counts_part; args->counts holds nranks * cols_per_rank columns, zero past n_cols), the bounds
 * reduced as in pw_msa_counts_allreduce, bestChar + the zero-coverage scan of the rank's range only
 * (pw_msa_call_cols), then the consensus ranges all-gathered in place (args->consensus holds
 * nranks * cols_per_rank bytes) and minmax[3] reduced MIN.  Every rank then holds what an
 * all-reduce + pw_msa_call leaves, except the full counts (its own range is in counts_part). */
int pw_msa_call_sharded(const pw_msa_args* args, uint32_t row_base, int32_t* counts_part, uint64_t cols_per_rank,
                        int rank, int nranks, void* comm, void* stream);

/* Host per-row steps of GSeqAlign::refineMSA after the consensus (the GapAssem C++ API,
 * pwasm_gapassem.hpp, and the multi-GPU driver call these on the rows they own).
 * pw_ga_row_remove_columns: removeColumn(alpos) (GapAssem.cpp:755-779 -> GASeq::removeBase
 *   :122-131) for the non-decreasing layout positions alpos[0..n) of the removed consensus-gap
 *   columns (the k-th at column c_k: alpos = c_k - k + minoffset), in one pass over the row —
 *   exact for any gap values, including deleted bases (ofs < 0) where the closed form of
 *   pw_msa_refine does not apply.
 * pw_ga_row_finish: refineClipping (X-drop, :182-349), removeClipGaps (:522-549) when
 *   PW_GA_REMOVE_GAPS, and the second refineClipping(skipDels) when gaps were removed
 *   (:1163-1181).  cpos_base = minoffset + mincol.  Returns 0, or 1 after a GError the
 *   reference exits on; msgbuf receives what the reference prints for the row (its warnings,
 *   then the GError message), NUL-terminated and cut at msglen. */
typedef struct pw_ga_row {
  const uint8_t* seq; /* [seqlen] bases as stored */
  int16_t* ofs;       /* [seqlen] gap before each base (negative = deleted base), edited */
  int32_t seqlen;
  int32_t offset;     /* in / out */
  int32_t numgaps;    /* in / out */
  int32_t clp5, clp3; /* in / out */
  int32_t revcompl;
  const char* id;     /* for messages */
} pw_ga_row;
#define PW_GA_REMOVE_GAPS 1u /* MSAColumns::removeConsGaps */
#define PW_GA_REFINE_CLIP 2u /* MSAColumns::refineClipping */
int pw_ga_row_remove_columns(pw_ga_row* row, const int32_t* alpos, uint64_t n);
int pw_ga_row_finish(pw_ga_row* row, const uint8_t* cons, int32_t cons_len, int32_t cpos_base, uint32_t flags,
                     char* msgbuf, size_t msglen);
/* Both for n rows in one call: rows with replay[k] != 0 get pw_ga_row_remove_columns(alpos) first,
 * then every row pw_ga_row_finish; messages back to back in msgbuf (row k: [msg_off[k],
 * msg_off[k+1]), msg_off has n + 1 entries), failed[k] = 1 after a GError, after which it stops.
 * Returns the rows processed (or a negative PW_E_* status).  If the messages exceed msg_cap no row
 * is left edited (all restored to their input state) and msg_off[returned] > msg_cap is the size to
 * call again with. */
int64_t pw_ga_rows_finish(pw_ga_row* rows, uint64_t n, const uint8_t* replay, const int32_t* alpos, uint64_t n_alpos,
                          const uint8_t* cons, int32_t cons_len, int32_t cpos_base, uint32_t flags, char* msgbuf,
                          uint64_t msg_cap, uint64_t* msg_off, int32_t* failed);

/* ---------------------------------------------------------------- host pre-pass + CLI */

/* Pack one cs string (CPU pre-pass).  offset/qlen/reverse locate it on the query.  Appends
 * to caller arrays (capacity in *_cap, counts in/out in *_n).  Returns 0, or a PW_CS_* code
 * with *err_pos = byte offset in cs where the reference would stop (pafreport.cpp:536-626). */
#define PW_CS_OK 0
#define PW_CS_PARSE 1     /* CS_ERROR (pafreport.cpp:542) */
#define PW_CS_SPLICED 2   /* '~' (pafreport.cpp:620-622) */
#define PW_CS_UNHANDLED 3 /* unknown op char (pafreport.cpp:623-624) */
#define PW_CS_EMPTY 4     /* zero-length indel */
#define PW_CS_BOUNDS 5    /* reads past the query */
#define PW_CS_NOSPACE 6   /* caller arrays too small */
typedef struct pw_cs_totals {
  int32_t q_total, t_total; /* qpos / tpos after the last packed op */
  uint32_t n_ops, n_lits;   /* appended */
  uint32_t n_events_max;    /* upper bound of events (indels + substitutions) */
  uint64_t text_bound;      /* upper bound of report bytes for these events */
} pw_cs_totals;
int pw_pack_cs(const char* cs, int32_t offset, int32_t qlen, uint32_t* ops, size_t ops_cap, uint8_t* lits,
               size_t lits_cap, pw_cs_totals* totals, int32_t* err_pos);

/* The same packing for a whole batch on the GPU (pw_pack.hip): record i's cs
 * field is cs_text[cs_off[i], cs_off[i+1]) (device arrays; offset / qlen as for pw_pack_cs).  Its
 * op words go to ops[cs_off[i] ..] and its literal bytes to lits[cs_off[i] ..] (a record never
 * has more ops or literal bytes than cs characters, so the field offsets are a valid layout),
 * its totals to out[i].  A record that is not well-formed cs — or breaks a bounds check, or holds
 * one op longer than 256 characters — gets PW_PACK_HOST and nothing else is defined for it: pack
 * it with pw_pack_cs, which gives the reference's error.  PW_PACK_ACGT: every literal byte is
 * A/C/G/T (the host's PW_REF_ACGT also needs the query to be). */
#define PW_PACK_HOST 1u
#define PW_PACK_ACGT 2u
typedef struct pw_cs_rec {
  int32_t q_total, t_total;
  uint32_t n_ops, n_lits, n_events_max;
  uint32_t flags;        /* PW_PACK_* */
  uint64_t text_bound;
} pw_cs_rec;
int pw_pack_cs_batch(const uint8_t* cs_text, const uint64_t* cs_off, const int32_t* offset, const int32_t* qlen,
                     uint32_t n, uint32_t* ops, uint8_t* lits, pw_cs_rec* out, void* stream);

/* GSeqAlign::refineMSA consensus of a packed layout file (PWL1, tests/pwl_format.md) on the HIP
 * path, written as a PWC1 result; flags bit0 = MSAColumns::removeConsGaps, bit1 = disable
 * MSAColumns::refineClipping.  Returns the reference's exit code (0, 1 bad index / GError, 5 zero
 * coverage) or 2 for I/O / device errors.  Result rows: {offset, numgaps, clp5, clp3, ofs[]}. */
int pw_gapassem_run(const char* layout_path, const char* out_path, uint32_t flags);
/* pw_gapassem_run through the GapAssem C++ API (pwasm_gapassem.hpp), then, for each non-NULL
 * path, GSeqAlign::writeACE / writeInfo (contig "contig1") and writeMSA (GapAssem.cpp:1200-1367,
 * 1039-1046).  Clipped rows are refined (refineClipping) unless flags bit1. */
int pw_gapassem_run_ex(const char* layout_path, const char* out_path, uint32_t flags, const char* ace_path,
                       const char* info_path, const char* msa_path);

/* The `pafreport` CLI (pafreport.cpp:175-460) on the HIP path; returns the process exit code
 * the reference would produce (it prints exactly what the reference prints). */
int pw_pafreport_main(int argc, char** argv);
/* The same, for an executable's main(): the output files are closed, then the process ends with
 * that exit code (_exit) without freeing the run's host and device state.  Never returns. */
int pw_pafreport_main_exit(int argc, char** argv);

/* Host batch (the CLI's pre-pass), exposed so bench.py / tests can stage a batch on the
 * device themselves.  Array pointers stay valid until pw_batch_free. */
typedef struct pw_batch pw_batch;
typedef struct pw_batch_view {
  const pw_aln_desc* desc;
  const uint32_t* ops;
  const uint8_t* lits;
  const uint8_t* qseq;
  const uint64_t* qoff;
  const int32_t* qlen;
  uint64_t n_alns, n_ops, n_lits, qseq_len, n_queries, text_total, n_events_max;  /* text_total = text bound */
  uint64_t alg_bytes_in; /* algorithmic input bytes of one pass */
  uint32_t skip_codan;
} pw_batch_view;
/* flags: bit0 = -G, bit1 = -F, bit2 = -C, bit3 = -N (same defaults as the CLI), bit4 = -w (keep the
 * gap lists and the last query run for pw_batch_write_msa) */
pw_batch* pw_batch_from_files(const char* fasta, const char* paf, uint32_t flags, char* errbuf, size_t errlen);
int pw_batch_view_get(const pw_batch* b, pw_batch_view* out);
/* Render the report (headers + event text) for results of a finished batch into `path`
 * (host copies of text, results and pages). */
int pw_batch_write_report(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host,
                          const pw_page* pages_host, const char* path);
/* Shard output for a multi-GPU run: the same bytes as pw_batch_write_report, cut
 * into items tagged with their 0-based input line ("PWI1", then per item {u64 line, i32 status
 * (-1 = continue, else the exit code the reference ends with), u32 n_stdout, u32 n_stderr,
 * stdout bytes, stderr bytes}).  Merging the items of all shards by global line, up to the
 * first item with status >= 0, reproduces the single-process output (pwasm_amd/shard.py). */
int pw_batch_write_items(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host,
                         const pw_page* pages_host, const char* path);
/* pw_batch_from_buffer flag: keep the cs strings as text for pw_runner_run to pack on the GPU
 * (pw_pack_cs_batch, as the CLI does); without it the host packs the op words and literals. */
#define PW_BATCH_GPU_PACK 32u
/* Frees the batch: its memory is returned by a background thread (PW_BATCH_FREE_SYNC=1: on the
 * caller), so the call returns at once; the batch and its array pointers are invalid after it. */
void pw_batch_free(pw_batch* b);
/* `pafreport -w`: the multi-FASTA MSA of the batch's last query run (refMSA->writeMSA,
 * pafreport.cpp:382-421, 447-450; GapAssem.cpp:645-753, 1006-1046) from its gap lists — the
 * query's gap profile is the elementwise max of the alignments' query gaps and target-only
 * bases are left-packed in it.  Needs flags bit4, and gene mode: in full-genome
 * mode (-F, or auto for a FASTA over 120000 bytes) it returns PW_E_ARG, as the reference refuses
 * -w there ("can only generate MSA for -G mode", pafreport.cpp:263-268). */
int pw_batch_write_msa(const pw_batch* b, const char* path);

/* ---------------------------------------------------------------- multi-GPU
 * Shard by target genome: rank `shard` of `nshards` packs only the PAF lines whose target name
 * (column 6) has crc32 % nshards == shard (lines with fewer than 7 columns: shard 0; comment
 * lines: nowhere).  Gene-mode q~t dedupe (pafreport.cpp:319-334) is keyed by the target, so it
 * stays shard-local; every item keeps its global input line.  pw_batch_from_files(...) ==
 * pw_batch_from_files_shard(..., 0, 1, ...). */
pw_batch* pw_batch_from_files_shard(const char* fasta, const char* paf, uint32_t flags, uint32_t shard,
                                    uint32_t nshards, char* errbuf, size_t errlen);
/* Merge the PWI1 item streams of all shards (pw_batch_write_items) by global input line up to
 * the first item that ends the run; stdout bytes to out_path (NULL = stdout), stderr bytes to
 * err_path (NULL = stderr).  Returns the exit code the single-process run ends with (>= 0) or a
 * negative PW_E_* status. */
int pw_items_merge(const char* const* paths, uint32_t n, const char* out_path, const char* err_path);

/* Scalable host path of the multi-GPU driver (pwasm_amd/mgpu.py):
 * pw_paf_split: rank r reads only the PAF lines that START in bytes [lo, hi) of the file (a line
 *   starts at byte 0 or after a '\n'; lines are cut as the CLI cuts them: \n, \r or \r\n) and
 *   routes each to the rank owning its target genome (the shard rule above); every line, comments
 *   included, keeps its index in the range, so global line = (lines of the ranges before) + index.
 *   Getters: lines in the range; per owner the bytes (its lines, each ended by '\n') and the count.
 * pw_batch_from_buffer: a batch from received lines (n_lines lines ended by '\n' in text, global
 *   input lines in line_no, ascending) — the pre-pass of pw_batch_from_files without the file.  prev
 *   (or NULL): the batch of the lines before these; its gene-mode q~t dedupe state moves over
 *   (pafreport.cpp:319-334), so a rank's lines can be packed batch by batch.
 * pw_batch_items / pw_batch_write_at: the batch's output items (log items up to the first that
 *   ends the run, as in pw_batch_write_items): global line, status (-1 = continue, else the exit
 *   code), stdout / stderr byte counts; then the stdout bytes of the first n_items written with
 *   pwrite at out_off[k] of fd (ranks write disjoint ranges of one output file, the offsets from an
 *   exclusive scan of all ranks' per-line byte counts) and their stderr bytes, back to back, into
 *   err_buf (capacity err_cap). */
typedef struct pw_split pw_split;
pw_split* pw_paf_split(const char* paf, uint64_t lo, uint64_t hi, uint32_t nshards, char* errbuf, size_t errlen);
uint64_t pw_split_lines(const pw_split* sp);
uint64_t pw_split_bytes(const pw_split* sp, uint32_t owner);
uint64_t pw_split_count(const pw_split* sp, uint32_t owner);
int pw_split_get(const pw_split* sp, uint32_t owner, char* bytes, uint32_t* local_lines);
void pw_split_free(pw_split* sp);
pw_batch* pw_batch_from_buffer(const char* fasta, const char* text, uint64_t len, const uint64_t* line_no,
                               uint64_t n_lines, uint32_t flags, pw_batch* prev, char* errbuf, size_t errlen);
uint64_t pw_batch_item_count(const pw_batch* b);
int pw_batch_items(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host, const pw_page* pages_host,
                   uint64_t* line, int32_t* status, uint64_t* out_len, uint64_t* err_len, uint64_t* n_items);
int pw_batch_write_at(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host,
                      const pw_page* pages_host, int fd, const uint64_t* out_off, uint64_t n_items, char* err_buf,
                      uint64_t err_cap);
/* pw_batch_write_range: as pw_batch_write_at for the items [first, first + n_items) (out_off[0] is
 * item first's offset) — the multi-GPU driver writes a batch window by window of global lines. */
int pw_batch_write_range(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host,
                         const pw_page* pages_host, int fd, uint64_t first, const uint64_t* out_off, uint64_t n_items,
                         char* err_buf, uint64_t err_cap);
/* pw_batch_render_range: the stdout bytes of the items [first, first + n_items) back to back into
 * out_buf (capacity out_cap: the sum of their pw_batch_items stdout counts) and their stderr bytes
 * into err_buf.  pw_gather_write: the spans src[src_off[k], + len[k]) in order, written
 * contiguously into fd from file_off (host threads, large pwrites).  Together the multi-GPU
 * driver's exchange write: ranks render their items of a window, exchange them (all-to-all) so
 * that each holds one contiguous byte range of the window, and write that range. */
int pw_batch_render_range(const pw_batch* b, const uint8_t* text_host, const pw_aln_result* res_host,
                          const pw_page* pages_host, uint64_t first, uint64_t n_items, uint8_t* out_buf, uint64_t out_cap,
                          char* err_buf, uint64_t err_cap);
int pw_gather_write(int fd, uint64_t file_off, const uint8_t* src, const uint64_t* src_off, const uint64_t* len,
                    uint64_t n);
/* pw_batch_cuts: a rank's received lines ('\n'-ended, n bytes) cut into batches of at most target
 * bytes (at least one line) at line ends: out[4k .. 4k + 3] = byte lo, hi, line lo, hi of batch k;
 * returns the batch count (0 when more than cap). */
uint64_t pw_batch_cuts(const uint8_t* text, uint64_t n, uint64_t target, uint64_t* out, uint64_t cap);

/* Batch runner (the multi-GPU driver's per-rank device state): the CLI's device
 * session behind the ABI — the batch's query set and next-stop table uploaded once on the current
 * device (pw_runner_create), then per batch of that query set pw_runner_run: the cs strings packed
 * on the GPU (batches made with PW_BATCH_GPU_PACK; the host descriptors are completed from the
 * packer's totals), the report pass on the runner's stream, results and pages copied back; it
 * returns the page count and the used text bytes, and pw_runner_fetch copies the results
 * (n_res = the batch's records), the pages and the text (text_cap >= text_used) out.
 * pw_runner_genome_rows: the batch's per-genome rows (pw_batch_genomes_get's genome_of / t_aln) from
 * the results still on the device.  Errors: PW_E_ARG (wrong sizes, another query set), PW_E_HIP. */
typedef struct pw_runner pw_runner;
pw_runner* pw_runner_create(const pw_batch* b, char* errbuf, size_t errlen);
int pw_runner_run(pw_runner* r, pw_batch* b, uint64_t* n_pages, uint64_t* text_used);
int pw_runner_fetch(pw_runner* r, pw_aln_result* res, uint64_t n_res, pw_page* pages, uint64_t n_pages, uint8_t* text,
                    uint64_t text_cap);
void pw_runner_free(pw_runner* r);

/* Per-genome coverage / event tables: genome = target sequence (PAF column 6).  Host: number of
 * distinct targets of a batch (+ bytes of their NUL-terminated names), then per record its
 * genome index (first-appearance order) and aligned target bases.  Device: one row per genome
 * from the per-record results of pw_report_events (rows are overwritten).  The multi-GPU driver
 * all-gathers the rows of every rank (RCCL) before rank 0 writes the merged table. */
typedef struct pw_genome_row {
  uint32_t records;   /* alignments to this target */
  uint32_t events;    /* report event lines */
  uint64_t t_bases;   /* aligned target bases (sum of tend - tstart) */
} pw_genome_row;
uint32_t pw_batch_genomes(pw_batch* b, uint64_t* names_bytes);
int pw_batch_genomes_get(const pw_batch* b, uint32_t* genome_of, int32_t* t_aln, char* names);
int pw_genome_table(const pw_aln_result* results, const uint32_t* genome_of, const int32_t* t_aln, uint32_t n_alns,
                    pw_genome_row* rows, uint32_t n_genomes, void* stream);
/* (the batch runner above: the rows of its last batch, into host memory) */
int pw_runner_genome_rows(pw_runner* r, const uint32_t* genome_of, const int32_t* t_aln, uint32_t n_alns,
                          uint32_t n_genomes, pw_genome_row* rows);

const char* pw_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PWASM_AMD_H */
