// pw_msa_layout.h — internal: the `pafreport -w` MSA of one query run (pafreport.cpp:382-421,
// 447-450), shared by the CLI pre-pass (pw_host.cpp) and the layout writer (pw_msa_layout.cpp).
#pragma once
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

namespace pw {

// One alignment of the run: what GSeqAlign(rseq, taseq) + addAlign needs from its PAF record.
struct MsaRec {
  int32_t offset;      // start on the aligned-strand query (pafreport.cpp:486-490)
  int32_t r_alnstart;  // taseq offset in the layout (pafreport.cpp:383)
  int32_t t_len;       // tseq length
  uint8_t reverse;
  uint32_t op_begin, n_ops, lit_begin, n_lits;  // the packed cs ops / literals (tseq rebuilt from them)
  uint32_t gap_off, n_rg, n_tg;                 // rgaps then tgaps, (pos, len) pairs (CIGAR, :645-718)
  uint32_t lab_off, lab_len;                    // tlabel (the taseq name, :366-376)
};

// The alignments of the current query run.  pafreport keeps one refseq GASeq per query switch
// (rseqs is never filled, :341-351), so only the last run of consecutive records of one query
// reaches writeMSA (refMSA, :447-448).
struct MsaRun {
  int qi = -1;
  std::vector<MsaRec> recs;
  std::vector<uint32_t> ops;
  std::vector<uint8_t> lits;
  std::vector<int32_t> gaps;
  std::string labels;
  void clear() {
    qi = -1;
    recs.clear();
    ops.clear();
    lits.clear();
    gaps.clear();
    labels.clear();
  }
};

// Write refMSA->writeMSA(f) (GapAssem.cpp:1039-1046) for the run: the query row then every
// target row in input order, 60 columns per line.  q / qlen: the forward upper-case query.
// Returns 0, or 1 after printing the reference's message for an error (stderr).
int write_run_msa(FILE* f, FILE* dbg, const char* qid, const uint8_t* q, int qlen, const MsaRun& run);

}  // namespace pw
