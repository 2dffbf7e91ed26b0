// pafreport_main.cpp — the `pafreport` executable: a thin main() over the C-ABI entry point
// pw_pafreport_main_exit (same flags, report format and exit codes as pafreport.cpp:175-460; the
// process ends as soon as the output files are closed — the batches' memory and the HIP runtime's
// state are left to the exit).
#include "pwasm_amd.h"

int main(int argc, char** argv) { return pw_pafreport_main_exit(argc, argv); }
