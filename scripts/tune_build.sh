#!/bin/bash
# Build libgcmx.so variants with different tuning knobs into gcm_amd/lib/tune/<name>/.
cd "$(dirname "$0")/../gcm_amd/csrc"
build() {  # name, flags
  make -s OUT=../lib/tune/$1 TUNE="$2" ../lib/tune/$1/libgcmx.so >/dev/null 2>&1 && echo "built $1" || echo "FAILED $1"
}
build v0 "" &
build march_mw3 "-DGCMX_MARCH_MINWAVES=3" &
build march_mw2 "-DGCMX_MARCH_MINWAVES=2" &
build march_c32 "-DGCMX_MARCH_CHUNK=32" &
wait
build march_c128 "-DGCMX_MARCH_CHUNK=128" &
build fused_c32 "-DGCMX_FUSED_CHUNK=32" &
build fused_c128 "-DGCMX_FUSED_CHUNK=128" &
build fused_mw2 "-DGCMX_FUSED_MINWAVES=2" &
wait
