#!/bin/bash
# Build libgcmx.so variants for A/B timing: each argument is NAME=FLAGS, e.g.
#   scripts/ab_build.sh base= noasm="-DGCMX_ASM_MINMAX=0"
# Output: gcm_amd/lib/tune/NAME/libgcmx.so (git-ignored; removed after use).
set -e
cd "$(dirname "$0")/../gcm_amd/csrc"
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  make -s OUT=../lib/tune/$name TUNE="$flags" ../lib/tune/$name/libgcmx.so -j8 >/dev/null
  echo "built $name: $flags"
done
