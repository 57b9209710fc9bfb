#!/bin/bash
# Host-code sanitizer run (CPU only, no GPU): builds libclay_amd_asan.so (ASan + UBSan on
# code.cpp / plan.cpp / the engine's host side) and liboracle_asan.so, then runs the CPU
# suites that exercise the planner, validation and the oracle under them.
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
make -s -C clay_amd/csrc asan
make -s -C oracle asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n 1)
export CLAY_AMD_LIB="$R/clay_amd/libclay_amd_asan.so" CLAY_ORACLE_LIB="$R/oracle/liboracle_asan.so"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_planner_cpu.py tests/test_reference_properties.py \
    tests/test_oracle_kats.py tests/test_golden.py tests/test_abi_cpu.py "$@"
