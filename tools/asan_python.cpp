// A Python interpreter whose executable carries the AddressSanitizer + UBSan
// runtimes (linked statically, so they are first in the process and export the
// __asan_* / __ubsan_* symbols), for running the CPU test tier against the
// sanitized extension ddp_practice_amd/_C_asan.so (build.py DPA_SANITIZE=1).
// Built and driven by scripts/asan_check.sh; never used on a GPU box.
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
