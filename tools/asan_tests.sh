#!/bin/bash
# Parser hardening run: the host library built with -fsanitize=address,undefined, loaded
# through MIVC_HOST_LIB into an uninstrumented Python (libasan preloaded), running the
# CPU tests of every parser a worker exposes to network-fetched data plus the fuzz tests.
# Host code only (no GPU): python -m govideocompressor_amd._build asan first.
set -euo pipefail
cd "$(dirname "$0")/.."
lib=$(python -c "from govideocompressor_amd import _build; print(_build.build_host(8, sanitize=True))")
asan=$(g++ -print-file-name=libasan.so)
ubsan=$(g++ -print-file-name=libubsan.so)
export MIVC_HOST_LIB=$lib
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# -s: a sanitizer report goes to stderr just before the process exits; pytest capture would eat it
LD_PRELOAD="$asan $ubsan" python -m pytest -s -q -p no:warnings -p no:cacheprovider \
  tests/test_fuzz_parsers.py tests/test_parser_ranges.py tests/test_host_codec.py tests/test_decode_parse.py tests/test_cabac.py \
  tests/test_h264_bframes.py tests/test_hevc_codec.py tests/test_mp4_tracks.py tests/test_mp4_hevc.py \
  tests/test_segment_media.py "$@"
