// pw_tables.h — byte tables shared by the HIP kernels (device copy in __constant__ memory,
// staged into LDS per workgroup) and the host pre-pass.
//
//  comp[256]   IUPAC complement (gclib gdna IUPAC_DEFS -> IUPAC_COMP, identity otherwise);
//              used by revCompl (pafreport.cpp:469-472) and GASeq::reverseComplement.
//  nt[256]     4-bit IUPAC nucleotide mask of toupper(c) (A=1 C=2 G=4 T=8, 0 = not a nucleotide).
//  codon[4096] translateCodon (gclib codons.cpp; call sites pafreport.cpp:824-825,855,865,898)
//              indexed by nt[c0]<<8 | nt[c1]<<4 | nt[c2]: NCBI table 1, stop '.', 'X' when any
//              base is not a nucleotide; degenerate codons give the amino acid common to all
//              expansions, Asx 'B' / Glx 'Z' for RAY / SAR (parity unpinned off ACGT).
//  status      the hpolyCheck/mmotifCheck status words, indexed by status id (0 = unknown)
//  codon64[64] fast path of codon[] for three bases of {A,C,G,T,a,c,g,t}, indexed by the 2-bit
//              code (c >> 1) & 3 of each base (A=0 C=1 T=2 G=3, either case).
#pragma once
#include <stdint.h>

namespace pw {

struct Tables {
  uint8_t nt[256];
  uint8_t comp[256];
  uint8_t codon[4096];
  uint8_t codon64[64];
  uint8_t status[8][12];  // printDiffInfo status words (pafreport.cpp:904-917), length in [11]
};

constexpr char kAA64[65] = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV.Y.YSSSS.CWCLFLF";
constexpr char kIupacDefs[] = "AaCcTtGgUuMmRrWwSsYyKkVvHhDdBbNnXx-*";
constexpr char kIupacComp[] = "TtGgAaCcAaKkYyWwSsRrMmBbDdHhVvNnXx-*";

constexpr uint8_t nt_mask_upper(int c) {
  switch (c) {
    case 'A': return 1;
    case 'C': return 2;
    case 'G': return 4;
    case 'T': return 8;
    case 'R': return 5;
    case 'Y': return 10;
    case 'S': return 6;
    case 'W': return 9;
    case 'K': return 12;
    case 'M': return 3;
    case 'B': return 14;
    case 'D': return 13;
    case 'H': return 11;
    case 'V': return 7;
    case 'N': return 15;
    default: return 0;
  }
}

constexpr uint8_t codon_of_masks(int m0, int m1, int m2) {
  if (!m0 || !m1 || !m2) return 'X';
  char aa = 0;
  bool mixed = false;
  for (int a = 0; a < 4; a++)
    if (m0 >> a & 1)
      for (int b = 0; b < 4; b++)
        if (m1 >> b & 1)
          for (int c = 0; c < 4; c++)
            if (m2 >> c & 1) {
              char x = kAA64[16 * a + 4 * b + c];
              if (aa == 0) aa = x;
              else if (aa != x) mixed = true;
            }
  if (!mixed) return (uint8_t)aa;
  if (m0 == 5 && m1 == 1 && (m2 & ~10) == 0) return 'B';
  if (m0 == 6 && m1 == 1 && (m2 & ~5) == 0) return 'Z';
  return 'X';
}

constexpr Tables build_tables() {
  Tables t{};
  for (int c = 0; c < 256; c++) {
    int u = (c >= 'a' && c <= 'z') ? c - 32 : c;
    t.nt[c] = nt_mask_upper(u);
    t.comp[c] = (uint8_t)c;
  }
  for (int i = 0; kIupacDefs[i]; i++) t.comp[(uint8_t)kIupacDefs[i]] = (uint8_t)kIupacComp[i];
  for (int i = 0; i < 4096; i++) t.codon[i] = codon_of_masks(i >> 8, (i >> 4) & 15, i & 15);
  constexpr int kCodeToAcgt[4] = {0, 1, 3, 2};  // fast code A,C,T,G -> kAA64 index A,C,G,T
  for (int i = 0; i < 64; i++)
    t.codon64[i] = (uint8_t)kAA64[16 * kCodeToAcgt[i >> 4] + 4 * kCodeToAcgt[(i >> 2) & 3] + kCodeToAcgt[i & 3]];
  constexpr const char* kStatus[6] = {"[unknown]", "homopolymer", "motif CCTGG", "motif CCAGG", "motif GATC",
                                      "motif GTAC"};
  for (int i = 0; i < 6; i++) {
    int n = 0;
    while (kStatus[i][n]) {
      t.status[i][n] = (uint8_t)kStatus[i][n];
      n++;
    }
    t.status[i][11] = (uint8_t)n;
  }
  return t;
}

}  // namespace pw
