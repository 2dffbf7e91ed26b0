// pafreport_main.cpp — the `pafreport` executable: a thin main() over the C-ABI entry point
// pw_pafreport_main (same flags, report format and exit codes as pafreport.cpp:175-460).
#include <stdio.h>
#include <unistd.h>

#include "pwasm_amd.h"

int main(int argc, char** argv) {
  const int rc = pw_pafreport_main(argc, argv);  // (its output files are closed when it returns)
  fflush(stdout);
  fflush(stderr);
  // skip the HIP runtime's exit-time teardown (~0.1 s): the device memory and the context go with
  // the process either way
  _exit(rc);
}
