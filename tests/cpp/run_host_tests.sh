#!/bin/bash
# Build and run tests/cpp/test_capi_host.cpp against (1) the normal library and (2) a build whose
# host code runs under AddressSanitizer + UndefinedBehaviorSanitizer.  Running needs the GPU box.
# usage: tests/cpp/run_host_tests.sh [outdir] [build|run|all]
#   build: compile both test binaries and the sanitized library (here, on the CPU: hipcc
#          cross-compiles gfx950); run: execute them (GPU box; outdir must travel, e.g. abv/host);
#   all (default): both.
set -e
cd "$(dirname "$0")/../.."
out=${1:-/tmp/deoss_hosttests}
phase=${2:-all}
mkdir -p $out
INC="-I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__"
LIBS="-L oracle -loracle_merkle -L /opt/rocm/lib -lamdhip64 -lpthread -Wl,-rpath,$PWD/oracle:/opt/rocm/lib"
if [ "$phase" != run ]; then
  make -s -C oracle
  # (1) plain
  g++ -O2 -std=c++17 $INC tests/cpp/test_capi_host.cpp -L deoss_amd -ldeoss_merkle -Wl,-rpath,$PWD/deoss_amd $LIBS \
    -o $out/test_plain
  # (2) sanitized host code
  hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -I include \
    -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
    -o $out/libdeoss_merkle_asan.so deoss_amd/csrc/merkle_capi.hip -L /opt/rocm/lib -lrccl
  # same compiler (ROCm clang) as the library's host code, so both use clang's sanitizer runtime
  /opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer $INC \
    tests/cpp/test_capi_host.cpp -L $out -ldeoss_merkle_asan -Wl,-rpath,$PWD/$out -Wl,-rpath,$out $LIBS -o $out/test_asan
fi
if [ "$phase" != build ]; then
  $out/test_plain $out
  # DEOSS_TEST_QUICK_EXIT: skip the HIP/HSA exit-time teardown after PASS (see the end of the test:
  # ASan's device allocator CHECKs on quarantined device chunks recycled after HSA unloads)
  DEOSS_TEST_QUICK_EXIT=1 ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 $out/test_asan $out
fi
