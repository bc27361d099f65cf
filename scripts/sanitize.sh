#!/bin/bash
# SURVEY §5 "Race detection / sanitizers": the CPU golden model and the engine's host code under
# AddressSanitizer + UndefinedBehaviorSanitizer (every report fatal), driven by the CPU test-suite.
# CPU only (GPU sanitizers are not available on this pool).  Output: profiles/r02/sanitize.log
set -eo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
python3 -c "from testground_amd.build import build_engine_host_asan as b; print(b())"
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
echo "== oracle (libtgoracle_asan.so) under the CPU parity and model tests"
LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" TGORACLE_LIB=oracle/build/libtgoracle_asan.so \
  python3 -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_oracle.py tests/test_golden.py \
  tests/test_window_model.py tests/test_shard_gloo.py tests/test_config_semantics.py tests/test_gossip.py \
  tests/test_sidecar.py tests/test_runner.py tests/test_bridge.py tests/test_metrics.py
echo "== engine host code (libtgsim_asan.so) under the C-ABI tests"
LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" TGSIM_LIB=testground_amd/build_asan/libtgsim_asan.so \
  python3 -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_abi.py
