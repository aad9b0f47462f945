#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against a host-ASan + UBSan build of libmbik.so
# (the C ABI's host side: plan building, describe_topology, argument checks; hipcc with each
# -fsanitize= after -Xarch_host, device code unchanged).  Output: build/san/libmbik_asan.so,
# the pytest summary on stdout.    tools/san/cpu_suite_asan.sh
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/san
python3 -m many_bone_ik_amd.build --variant build/san/libmbik_asan.so -O1 -g -Xarch_host -fsanitize=address \
  -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -shared-libsan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
MBIK_LIB_OVERRIDE=$PWD/build/san/libmbik_asan.so LD_PRELOAD="$RT${LD_PRELOAD:+ $LD_PRELOAD}" \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider
