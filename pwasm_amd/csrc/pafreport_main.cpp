// pafreport_main.cpp — the `pafreport` executable: a thin main() over the C-ABI entry point
// pw_pafreport_main (same flags, report format and exit codes as pafreport.cpp:175-460).
#include <stdio.h>

#include "pwasm_amd.h"

int main(int argc, char** argv) {
  const int rc = pw_pafreport_main(argc, argv);
  fflush(stdout);
  return rc;
}
