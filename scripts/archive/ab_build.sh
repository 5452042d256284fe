#!/bin/bash
# Build libgcmx.so variants for A/B timing: each argument is NAME=FLAGS, e.g.
#   scripts/ab_build.sh base= noasm="-DGCMX_ASM_MINMAX=0"
# Only kernels_xyz.hip is rebuilt per variant (the rest is the regular build's
# objects).  Output: gcm_amd/lib/tune/NAME/libgcmx.so (git-ignored).
set -e
cd "$(dirname "$0")/../gcm_amd/csrc"
make -s -j8 >/dev/null 2>&1
for spec in "$@"; do
  name="${spec%%=*}"; flags="${spec#*=}"
  rm -rf ../lib/tune/$name
  ( make -s OUT=../lib/tune/$name TUNE="$flags" tune >/dev/null 2>../lib/tune_$name.err \
      && echo "built $name: $flags" || { echo "FAILED $name"; tail -5 ../lib/tune_$name.err; } ) &
done
wait
