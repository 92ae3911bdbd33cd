#!/usr/bin/env bash
# Host-code sanitizer runs of the native extension (_kwcore), SURVEY §5.2:
#  * ASan + UBSan over every test that drives the C++ decoder, pipeline,
#    pod cache and notifier core;
#  * TSan over the tests that run the decode worker pool (DecodePool), the
#    end-to-end service and the TLS record layer's CryptoPool / writer threads.
# The interpreter is not instrumented: the sanitizer runtime is preloaded and
# the instrumented build is loaded via $K8S_WATCHER_KWCORE_SO (ops/native.py).
# Never run on the GPU box (GPU sanitizers are not available there; this is
# host code anyway).
set -euo pipefail
cd "$(dirname "$0")/.."
python -m k8s_watcher_amd.ops.native address
python -m k8s_watcher_amd.ops.native thread
SO=$(python -c "import sysconfig; print('_kwcore' + sysconfig.get_config_var('EXT_SUFFIX'))")
mkdir -p build
echo "== ASan+UBSan"
K8S_WATCHER_KWCORE_SO=build/sanitize-address/$SO \
LD_PRELOAD="$(g++ -print-file-name=libasan.so):$(g++ -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  timeout -k 10 900 python -m pytest -q -p no:cacheprovider --timeout 300 \
  tests/test_native_parity.py tests/test_native_pipeline.py tests/test_podcache.py tests/test_notifier.py \
  tests/test_spool.py tests/test_notifier_tls.py tests/test_watch_list.py tests/test_e2e_slice.py tests/test_reflector.py tests/test_http_metrics.py tests/test_reader_hub.py tests/test_reader_hub_tls.py tests/test_native_sink.py \
  tests/test_validate.py tests/test_pyrepr.py tests/test_native_relist.py tests/test_relist_storm.py tests/test_memory.py \
  tests/test_partitioned_apply.py tests/test_cluster_replay.py tests/test_tls13.py \
  2>&1 | tee build/asan.log | tail -3
echo "== TSan"
K8S_WATCHER_KWCORE_SO=build/sanitize-thread/$SO \
LD_PRELOAD="$(g++ -print-file-name=libtsan.so)" TSAN_OPTIONS=report_signal_unsafe=0:halt_on_error=1 \
  timeout -k 10 900 python -m pytest -q -s -p no:cacheprovider --timeout 300 \
  tests/test_native_pipeline.py tests/test_e2e_slice.py tests/test_reflector.py tests/test_native_parity.py \
  tests/test_notifier.py tests/test_notifier_tls.py tests/test_spool.py tests/test_leader.py tests/test_reader_hub.py tests/test_reader_hub_tls.py tests/test_native_sink.py \
  tests/test_sharding.py::test_discover_scope_two_shards_exactly_once tests/test_sharding.py::test_deleted_namespace_drains_then_synthesizes_deleted \
  tests/test_native_relist.py tests/test_relist_storm.py tests/test_partitioned_apply.py tests/test_tls13.py \
  2>&1 | tee build/tsan.log | tail -3
if grep -q "WARNING: ThreadSanitizer\|ERROR: AddressSanitizer\|runtime error:" build/asan.log build/tsan.log; then
  echo "sanitizer reports found (build/asan.log, build/tsan.log)"; exit 1
fi
echo "sanitizers clean"
