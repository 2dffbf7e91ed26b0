// gapassem_main.cpp — `gapassem_consensus <layout.pwl> <out.pwc> [--remove-gaps]
// [--no-refine-clipping] [--ace F] [--info F] [--msa F]`: GSeqAlign::refineMSA of a packed layout
// on the HIP path through the GapAssem C++ API, plus writeACE / writeInfo / writeMSA (same CLI and
// outputs as oracle/gapassem_oracle.c, for the parity tests and bench).
#include <stdio.h>
#include <string.h>

#include "pwasm_amd.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr,
            "usage: gapassem_consensus <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping] [--ace F] "
            "[--info F] [--msa F]\n");
    return 2;
  }
  uint32_t flags = 0;
  const char *ace = nullptr, *info = nullptr, *msa = nullptr;
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--remove-gaps")) flags |= 1u;
    else if (!strcmp(argv[i], "--no-refine-clipping")) flags |= 2u;
    else if (!strcmp(argv[i], "--ace") && i + 1 < argc) ace = argv[++i];
    else if (!strcmp(argv[i], "--info") && i + 1 < argc) info = argv[++i];
    else if (!strcmp(argv[i], "--msa") && i + 1 < argc) msa = argv[++i];
  }
  return pw_gapassem_run_ex(argv[1], argv[2], flags, ace, info, msa);
}
