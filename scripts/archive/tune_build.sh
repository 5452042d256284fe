#!/bin/bash
# Build libgcmx.so variants with different tuning knobs into gcm_amd/lib/tune/<name>/.
cd "$(dirname "$0")/../gcm_amd/csrc"
rm -rf ../lib/tune
build() {  # name, flags
  make -s OUT=../lib/tune/$1 TUNE="$2" ../lib/tune/$1/libgcmx.so >/dev/null 2>&1 && echo "built $1" || echo "FAILED $1"
}
build base "" &
build wt4 "-DGCMX_FUSED_WAVETILE=1 -DGCMX_FUSED_MINWAVES=4" &
build wt3 "-DGCMX_FUSED_WAVETILE=1 -DGCMX_FUSED_MINWAVES=3" &
build wt2 "-DGCMX_FUSED_WAVETILE=1 -DGCMX_FUSED_MINWAVES=2" &
wait
