#!/bin/bash
# Host-code sanitizer run (CPU only, this container): the extension's host C++
# (DDP reducer + autograd hooks, watchdog thread, communicator objects, bindings)
# under AddressSanitizer + UndefinedBehaviorSanitizer, exercised by the CPU test
# tier's DDP / reducer / watchdog / aux tests over gloo (multi-process).
#   bash scripts/asan_check.sh [pytest args...]   -> log in profiles/asan_cpu_tests.log
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
DPA_SANITIZE=1 python -m ddp_practice_amd.build || exit 1
mkdir -p build
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
clang=/opt/rocm/lib/llvm/bin/clang++
$clang -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -I"$PYINC" tools/asan_python.cpp \
  -o build/asan_python $(python3-config --ldflags --embed) || exit 1
export DPA_EXT_SO=$ROOT/ddp_practice_amd/_C_asan.so
# leaks: CPython and torch keep allocations until exit by design; the interest here
# is invalid accesses, use-after-free, races on object lifetimes and UB
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:print_summary=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# time budgets in the tests (watchdogs) stretch for the sanitized interpreter
export DPA_TEST_TIME_SCALE=4
TESTS=${*:-tests/test_ddp_cpu.py tests/test_aux_cpu.py tests/test_amp_optim_cpu.py tests/test_data_cpu.py tests/test_resnet_cpu.py tests/test_bench_cpu.py tests/test_comm_selftest_cpu.py tests/test_bntap_cpu.py tests/test_ext_digest_cpu.py}
./build/asan_python -c "import ctypes, sys; from ddp_practice_amd import _ext; C = _ext.load(); \
print('extension:', C.__file__, '| asan runtime:', hasattr(ctypes.CDLL(None), '__asan_init'))" \
  2>&1 | tee profiles/asan_cpu_tests.log
./build/asan_python -m pytest $TESTS -x -q -p no:cacheprovider 2>&1 | tee -a profiles/asan_cpu_tests.log
