#!/bin/bash
# Run the oracle test suite (and an fjp_ref stress run) against the ThreadSanitizer and the
# AddressSanitizer+UBSan builds of the CPU oracles (oracle/Makefile targets tsan, asan).
# Host code only -- GPU sanitizers are not available on this pool.
set -e
cd "$(dirname "$0")/.."
make -s -C oracle all tsan asan
export AKKA_AMD_NO_TORCH=1
TSAN=$(gcc -print-file-name=libtsan.so)
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
echo "== ThreadSanitizer"
AGX_FJP_LIB=libfjp_ref.tsan.so AGX_BSP_LIB=libbsp_ref.tsan.so LD_PRELOAD=$TSAN \
  TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0" \
  python -m pytest -q -p no:cacheprovider tests/test_oracle_golden.py tests/test_fjp_baseline.py
echo "== AddressSanitizer + UBSan"
AGX_FJP_LIB=libfjp_ref.asan.so AGX_BSP_LIB=libbsp_ref.asan.so LD_PRELOAD="$ASAN $UBSAN" \
  ASAN_OPTIONS="detect_leaks=0 halt_on_error=1 exitcode=67" UBSAN_OPTIONS="halt_on_error=1" \
  python -m pytest -q -p no:cacheprovider tests/test_oracle_golden.py tests/test_fjp_baseline.py
echo "sanitizers clean"
