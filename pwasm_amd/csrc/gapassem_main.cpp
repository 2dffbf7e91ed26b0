// gapassem_main.cpp — `gapassem_consensus <layout.pwl> <out.pwc> [--remove-gaps]
// [--no-refine-clipping]`: GSeqAlign::refineMSA consensus of a packed layout on the HIP path
// (same CLI and output as oracle/gapassem_oracle.c, for the parity tests and bench).
#include <stdio.h>
#include <string.h>

#include "pwasm_amd.h"

extern "C" int pw_gapassem_run(const char* layout_path, const char* out_path, uint32_t flags);

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: gapassem_consensus <layout.pwl> <out.pwc> [--remove-gaps] [--no-refine-clipping]\n");
    return 2;
  }
  uint32_t flags = 0;
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--remove-gaps")) flags |= 1u;
    else if (!strcmp(argv[i], "--no-refine-clipping")) flags |= 2u;
  }
  return pw_gapassem_run(argv[1], argv[2], flags);
}
